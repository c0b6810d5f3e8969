#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_hip_fp32.py \
  tests/test_hip_kernels.py tests/test_hip_train.py tests/test_hip_step_parity.py > gpurun_out/dense_w1_tests.log 2>&1; rc=$?
grep -E "dense|passed|failed|FAILED|Error" gpurun_out/dense_w1_tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
for P in 3 16; do
  DTYPE=fp32 timeout -k 10 200 python -u tools/probe_pop.py $P $P 1 1 > gpurun_out/dw.log 2>&1 || { tail -5 gpurun_out/dw.log; exit 1; }
  grep '^{' gpurun_out/dw.log | cut -c1-160
done
