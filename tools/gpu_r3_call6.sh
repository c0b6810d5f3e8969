#!/bin/bash
# GPU suite (fp32 batch invariance), Q-curve (both fold protocols), driver-equivalent headline
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/ > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
bash tools/gpu_qcurve3.sh || exit $?
bash tools/gpu_headline3.sh
