# fold-job reuse: tests, then A/B on the reference-fold probe and a fresh Q=2 timeline
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_hip_train.py tests/test_hip_dp.py tests/test_hip_step_parity.py > gpurun_out/r4c7_tests.log 2>&1 \
  || { tail -30 gpurun_out/r4c7_tests.log; exit 1; }
tail -1 gpurun_out/r4c7_tests.log
for v in 1 0 1 0; do
  GENTUN_FOLD_REUSE=$v DTYPE=fp32 RESET=kernels timeout -k 10 200 python -u tools/probe_pop.py 2 2 1 1 \
    > gpurun_out/r4c7_run.log 2>&1 || { tail -5 gpurun_out/r4c7_run.log; exit 1; }
  echo "RESET=kernels P=2 reuse=$v $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c7_run.log)"
done
RESET=kernels P=2 SAMPLES=10000 TAG=_k2b DUMP=2 bash tools/gpu.sh timeline > /dev/null && head -4 gpurun_out/timeline/summary_k2b.txt
