#!/bin/bash
# fp32 kernel tests (wide shapes) + deep-space population throughput (fp32), with / without BN.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest -v -s --timeout 120 --timeout-method thread tests/test_hip_fp32.py \
  > gpurun_out/fp32_tests_wide.log 2>&1; rc=$?
grep -E "\[fp32\]|passed|failed" gpurun_out/fp32_tests_wide.log
[ $rc -eq 0 ] || exit 1
export SPACE=deep DTYPE=fp32
for cfg in "20,50,100 0 3" "20,50,100 1 3" "20,50,100 0 16" "64,128,256 0 1" "64,128,256 1 1" "64,128,256 0 3"; do
  set -- $cfg
  echo "== kernels $1 bn $2 P=$3"
  KERNELS=$1 BN=$2 timeout -k 10 300 python -u tools/probe_pop.py $3 $3 1 1 > gpurun_out/dp.log 2>&1 || { tail -5 gpurun_out/dp.log; exit 1; }
  grep '^{' gpurun_out/dp.log | cut -c1-240
done
