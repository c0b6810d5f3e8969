# Round 6 BatchNorm chunk A/B: GPU suite, then the wide and deep S=(3,4,5)+BN population steps under
# rocprofv3 --kernel-trace --stats (BN kernel times per call), chunks per shape (new) vs 512 pixels (old).
export GENTUN_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/ > gpurun_out/bn_tests.log 2>&1 || { tail -30 gpurun_out/bn_tests.log; exit 1; }
tail -1 gpurun_out/bn_tests.log
SPACE=deep KERNELS=64,128,256 BN=1 WARM=0 bash tools/gpu.sh prof widebn -- python3 tools/probe_pop.py 5 5 1 1 2000 || exit 1
SPACE=deep BN=1 WARM=0 bash tools/gpu.sh prof deepbn -- python3 tools/probe_pop.py 5 5 1 1 2000 || exit 1
for i in 1 2; do
  for mode in new old; do
    SPACE=deep KERNELS=64,128,256 BN=1 BNCHUNK=$mode timeout -k 10 200 python3 tools/probe_pop.py 5 5 1 1 4000 > gpurun_out/bnab.log 2>&1 || { tail -5 gpurun_out/bnab.log; exit 1; }
    echo "wide $mode $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bnab.log)" | tee -a gpurun_out/bnab.txt
    SPACE=deep BN=1 BNCHUNK=$mode timeout -k 10 200 python3 tools/probe_pop.py 5 5 1 1 4000 > gpurun_out/bnab.log 2>&1 || { tail -5 gpurun_out/bnab.log; exit 1; }
    echo "deep $mode $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bnab.log)" | tee -a gpurun_out/bnab.txt
  done
done
