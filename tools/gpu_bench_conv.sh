#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
timeout -k 10 400 python -u tools/bench_conv.py 10 > gpurun_out/bench_conv.log 2>&1
rc=$?; tail -3 gpurun_out/bench_conv.log; exit $rc
