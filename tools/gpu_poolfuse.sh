#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_hip_train.py \
  tests/test_hip_step_parity.py > gpurun_out/poolfuse_tests.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/poolfuse_tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
for f in 0 1; do
  for P in 3 16; do
    GENTUN_POOL_FUSE=$f DTYPE=fp32 timeout -k 10 200 python -u tools/probe_pop.py $P $P 1 1 > gpurun_out/pf.log 2>&1 || { tail -5 gpurun_out/pf.log; exit 1; }
    echo "fuse=$f $(grep '^{' gpurun_out/pf.log | cut -c1-160)"
  done
done
