# wgrad geometry A/B at bench-sized launches (25 / 30 groups): stage-2 splits and column slices
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_hip_fp32.py tests/test_hip_kernels.py > gpurun_out/r4c9_tests.log 2>&1 || { tail -30 gpurun_out/r4c9_tests.log; exit 1; }
tail -1 gpurun_out/r4c9_tests.log
for P in 5 6; do
  for v in "8 0" "10 0" "16 0" "8 2" "12 0" "8 0"; do
    set -- $v
    GENTUN_F32_SPLITS16=$1 GENTUN_WGRAD_NZ=$2 DTYPE=fp32 RESET=all timeout -k 10 200 python -u tools/probe_pop.py $P $P 1 1 \
      > gpurun_out/r4c9_run.log 2>&1 || { tail -5 gpurun_out/r4c9_run.log; exit 1; }
    echo "P=$P splits16=$1 nz=$2 $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c9_run.log)"
  done
done
for v in "6 6 1" "6 3 2" "10 5 2" "10 10 1"; do
  set -- $v
  DTYPE=fp32 RESET=all timeout -k 10 200 python -u tools/probe_pop.py $1 $2 $3 1 \
    > gpurun_out/r4c9_run.log 2>&1 || { tail -5 gpurun_out/r4c9_run.log; exit 1; }
  echo "P=$1 pop_batch=$2 streams=$3 $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c9_run.log)"
done
# conv tile threshold at small / mid launches: Q=5 (P=1), Q=10 (P=2)
for P in 1 2; do
  for wg in 300 512 1000 2000 512; do
    GENTUN_CONV_SMALLQ_WG=$wg DTYPE=fp32 RESET=all timeout -k 10 200 python -u tools/probe_pop.py $P $P 1 1 \
      > gpurun_out/r4c9_run.log 2>&1 || { tail -5 gpurun_out/r4c9_run.log; exit 1; }
    echo "P=$P smallq_wg=$wg $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c9_run.log)"
  done
done
