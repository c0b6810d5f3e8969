#!/bin/bash
# fp32 + bf16 kernel tests and the smoke entry point on one MI355X
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest tests/test_hip_fp32.py tests/test_hip_kernels.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/fp32_tests.log 2>&1
rc=$?
tail -5 gpurun_out/fp32_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as e; e.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?
tail -3 gpurun_out/smoke.log
exit $rc
