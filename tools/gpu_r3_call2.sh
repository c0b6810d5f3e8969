#!/bin/bash
# dense head A/B (bitwise test + timing sweep), then the secondary bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
mkdir -p gpurun_out/dense3
timeout -k 10 200 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_dense_stream.py > gpurun_out/dense3/tests.log 2>&1 || { tail -20 gpurun_out/dense3/tests.log; exit 1; }
tail -1 gpurun_out/dense3/tests.log
for cfg in "0 2" "1 1" "1 2" "1 4"; do
  set -- $cfg
  GENTUN_DENSE_STREAM=$1 GENTUN_DENSE_UT=$2 timeout -k 10 120 python3 -u tools/bench_dense.py 25 20 >> gpurun_out/dense3/sweep.log 2>&1 || { tail -5 gpurun_out/dense3/sweep.log; exit 1; }
done
cat gpurun_out/dense3/sweep.log
bash tools/gpu_r3_secondary.sh
