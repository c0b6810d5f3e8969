# small-launch tiles + wgrad streams: tests, then A/B on the probe (Q=2 reference folds, Q=10, Q=25)
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_hip_train.py tests/test_hip_kernels.py tests/test_hip_fp32.py > gpurun_out/r4c6_tests.log 2>&1 \
  || { tail -30 gpurun_out/r4c6_tests.log; exit 1; }
tail -1 gpurun_out/r4c6_tests.log
for spec in "kernels 2" "all 2" "all 5"; do
  set -- $spec
  for v in "1 2" "0 1" "1 1" "1 3"; do
    set -- $spec $v
    GENTUN_CONV_SMALLQ=$3 GENTUN_WGRAD_STREAMS=$4 DTYPE=fp32 RESET=$1 timeout -k 10 200 python -u tools/probe_pop.py $2 $2 1 1 \
      > gpurun_out/r4c6_run.log 2>&1 || { tail -5 gpurun_out/r4c6_run.log; exit 1; }
    echo "RESET=$1 P=$2 smallq=$3 wstreams=$4 $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c6_run.log)"
  done
done
