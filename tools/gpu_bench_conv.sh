#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1 DBGS=${DBGS:-0}
timeout -k 10 300 python -u -m pytest tests/test_hip_fp32.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fp32_tests.log 2>&1 || { tail -30 gpurun_out/fp32_tests.log; exit 1; }
tail -2 gpurun_out/fp32_tests.log
: > gpurun_out/bench_conv.log
for G in ${GS:-80}; do for P in ${PS:-"0 0" "1 0"}; do
  set -- $P
  G=$G F32P=$1 F32P_GRID=$2 ONLY="${ONLY:-}" timeout -k 10 300 python -u tools/bench_conv.py 10 >> gpurun_out/bench_conv.log 2>&1 || exit $?
done; done
