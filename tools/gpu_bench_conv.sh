#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1 DBGS=${DBGS:-0}
: > gpurun_out/bench_conv.log
for G in ${GS:-80 10}; do for TH in ${THS:-0 4}; do
  G=$G F32_TH=$TH timeout -k 10 300 python -u tools/bench_conv.py 10 | sed "s/^{/{\"th\": $TH, /" >> gpurun_out/bench_conv.log 2>&1 || exit $?
done; done
