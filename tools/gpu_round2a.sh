#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest tests/test_hip_step_parity.py -x -v -s --timeout 300 --timeout-method thread -k fifty > gpurun_out/parity2.log 2>&1
rc=$?; grep -E "parity|passed|failed|Error" gpurun_out/parity2.log | tail -8
true
exit $rc
