# wgrad half-split staging (GT_WGRAD_HALVES): tests, then same-box A/B vs a build without it
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_hip_fp32.py tests/test_hip_train.py tests/test_hip_dp.py > gpurun_out/r4c12_tests.log 2>&1 \
  || { tail -30 gpurun_out/r4c12_tests.log; exit 1; }
tail -1 gpurun_out/r4c12_tests.log
for i in 1 2 3; do
  for lib in "" ab_libs/nohalves.so; do
    GENTUN_HIP_LIB=$lib DTYPE=fp32 RESET=all timeout -k 10 200 python -u tools/probe_pop.py 5 5 1 1 \
      > gpurun_out/r4c12_run.log 2>&1 || { tail -5 gpurun_out/r4c12_run.log; exit 1; }
    echo "P=5 lib=${lib:-tree} $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c12_run.log)"
  done
done
for lib in "" ab_libs/nohalves.so; do
  GENTUN_HIP_LIB=$lib G=25 DBGS=0 ONLY=s2 timeout -k 10 200 python -u tools/bench_conv.py 10 2>&1 | grep conv_wgrad | cut -c1-220
done
