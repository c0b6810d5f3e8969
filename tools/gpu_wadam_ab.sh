#!/bin/bash
# dense wgrad + Adam load hoist (A/B build ab/wadam1.so): kernel tests on it, then fp32 P=5 timelines
# with the default build and the A/B build (same box)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
AB=$PWD/gentun_amd/_native/ab/wadam1.so
mkdir -p gpurun_out/wadam
GENTUN_HIP_LIB=$AB timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_hip_kernels.py tests/test_hip_fp32.py tests/test_hip_train.py \
  > gpurun_out/wadam/tests.log 2>&1 || { tail -30 gpurun_out/wadam/tests.log; exit 1; }
tail -1 gpurun_out/wadam/tests.log
P=5 bash tools/gpu_timeline.sh > /dev/null && cp gpurun_out/timeline/summary.txt gpurun_out/wadam/default.txt || exit 1
GENTUN_HIP_LIB=$AB P=5 bash tools/gpu_timeline.sh > /dev/null && cp gpurun_out/timeline/summary.txt gpurun_out/wadam/hoist.txt || exit 1
for f in default hoist; do echo "== $f"; grep -E "steps analysed|dense_wgrad_adam" gpurun_out/wadam/$f.txt; done
