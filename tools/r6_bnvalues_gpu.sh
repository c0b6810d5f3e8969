# Round 6: BatchNorm chunk budget sweep (values per workgroup, cnn_kernels.BN_CHUNK_VALUES), alternating on one box.
export GENTUN_NO_AUTOBUILD=1
: > gpurun_out/bnvalues.txt
for i in 1 2; do
  for v in 16384 8192 4096 32768; do
    SPACE=deep KERNELS=64,128,256 BN=1 BNVALUES=$v timeout -k 10 200 python3 tools/probe_pop.py 5 5 1 1 4000 > gpurun_out/bv.log 2>&1 || { tail -5 gpurun_out/bv.log; exit 1; }
    echo "wide $v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bv.log)" | tee -a gpurun_out/bnvalues.txt
    SPACE=deep BN=1 BNVALUES=$v timeout -k 10 200 python3 tools/probe_pop.py 5 5 1 1 4000 > gpurun_out/bv.log 2>&1 || { tail -5 gpurun_out/bv.log; exit 1; }
    echo "deep $v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bv.log)" | tee -a gpurun_out/bnvalues.txt
  done
done
