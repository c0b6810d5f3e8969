# 8-slice 4-wave wgrad for tiny launches + head_fwd label-chain hoist: tests, then A/B at small launches
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_hip_duo.py \
  tests/test_hip_kernels.py tests/test_hip_train.py > gpurun_out/r4c24_tests.log 2>&1 || { tail -30 gpurun_out/r4c24_tests.log; exit 1; }
tail -1 gpurun_out/r4c24_tests.log
for spec in "kernels 2" "all 1" "all 5"; do
  set -- $spec
  for v in 32 0 32 0; do
    GENTUN_WGRAD_NZ8=$v DTYPE=fp32 RESET=$1 timeout -k 10 200 python -u tools/probe_pop.py $2 $2 1 1 \
      > gpurun_out/r4c24_run.log 2>&1 || { tail -5 gpurun_out/r4c24_run.log; exit 1; }
    echo "RESET=$1 P=$2 nz8_below=$v $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c24_run.log)"
  done
done
