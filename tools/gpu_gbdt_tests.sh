#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gbdt_gpu.py \
  > gpurun_out/gbdt_tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|assert|passed|failed" gpurun_out/gbdt_tests.log | head -40
exit $rc
