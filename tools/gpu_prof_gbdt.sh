#!/bin/bash
# Kernel + runtime-API statistics of the GBDT GPU path (1M x 256, 2 candidates, 10 rounds)
set -o pipefail
mkdir -p gpurun_out/prof_gbdt
export GENTUN_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 tools/bench_gbdt.py --pop 2 --rounds 10 > gpurun_out/prof_gbdt/plain.log 2>&1 || { tail -5 gpurun_out/prof_gbdt/plain.log; exit 1; }
grep "{" gpurun_out/prof_gbdt/plain.log
rm -rf /tmp/pg
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --stats -d /tmp/pg -o run --output-format csv -- python3 tools/bench_gbdt.py --pop 2 --rounds 10 > gpurun_out/prof_gbdt/run.log 2>&1 || { tail -5 gpurun_out/prof_gbdt/run.log; exit 1; }
find /tmp/pg -name "*stats.csv" -exec cp {} gpurun_out/prof_gbdt/ \;
for f in gpurun_out/prof_gbdt/*stats.csv; do echo "== $f"; head -12 $f | cut -c1-200; done
