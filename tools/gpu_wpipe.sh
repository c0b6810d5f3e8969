#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_fp32.py > gpurun_out/wpipe_tests.log 2>&1; rc=$?
tail -1 gpurun_out/wpipe_tests.log
[ $rc -eq 0 ] || exit $rc
DTYPE=fp32 DBGS=0 F32P=0 timeout -k 10 300 python -u tools/bench_conv.py 10 > gpurun_out/wp.log 2>&1 || { tail -5 gpurun_out/wp.log; exit 1; }
grep '^{' gpurun_out/wp.log | grep wgrad | cut -c60-200
for P in 3 16; do
  DTYPE=fp32 timeout -k 10 200 python -u tools/probe_pop.py $P $P 1 1 > gpurun_out/wp.log 2>&1 || { tail -5 gpurun_out/wp.log; exit 1; }
  grep '^{' gpurun_out/wp.log | cut -c1-160
done
