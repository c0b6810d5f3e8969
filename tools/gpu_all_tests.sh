#!/bin/bash
# every GPU test (one pytest process), then smoke()
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
timeout -k 10 1000 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/ \
  > gpurun_out/gpu_tests.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/gpu_tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
tail -2 gpurun_out/smoke.log | cut -c1-300
exit $rc
