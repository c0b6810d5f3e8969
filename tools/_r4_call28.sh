set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_hip_fp32.py \
  tests/test_hip_train.py tests/test_hip_duo.py tests/test_hip_dp.py > gpurun_out/r4c28_tests.log 2>&1 || { tail -30 gpurun_out/r4c28_tests.log; exit 1; }
tail -1 gpurun_out/r4c28_tests.log
for i in 1 2; do
  DTYPE=fp32 RESET=all timeout -k 10 200 python -u tools/probe_pop.py 5 5 1 1 > gpurun_out/r4c28_run.log 2>&1 || { tail -5 gpurun_out/r4c28_run.log; exit 1; }
  echo "P=5 $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c28_run.log)"
done
