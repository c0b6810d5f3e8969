# adam band tests + inactive-node test, then Q=2 (reference folds) and Q=10 timelines
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_hip_kernels.py -k adam_segments tests/test_hip_train.py > gpurun_out/r4c5_tests.log 2>&1 \
  || { tail -30 gpurun_out/r4c5_tests.log; exit 1; }
tail -2 gpurun_out/r4c5_tests.log
RESET=kernels P=2 SAMPLES=10000 TAG=_k2 DUMP=2 bash tools/gpu.sh timeline > /dev/null && head -24 gpurun_out/timeline/summary_k2.txt
RESET=all P=2 SAMPLES=10000 TAG=_a2 DUMP=1 bash tools/gpu.sh timeline > /dev/null && head -24 gpurun_out/timeline/summary_a2.txt
