#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/prof_gbdt2
export GENTUN_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for d in 6 10; do
  GENTUN_GBDT_TIMING=1 timeout -k 10 200 python3 tools/probe_gbdt.py 1000000 256 $d 5 > gpurun_out/prof_gbdt2/plain_$d.log 2>&1 || { tail -5 gpurun_out/prof_gbdt2/plain_$d.log; exit 1; }
  grep "{\|gbdt_hip" gpurun_out/prof_gbdt2/plain_$d.log | tail -2
done
rm -rf /tmp/pg2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pg2 -o run --output-format csv -- python3 tools/probe_gbdt.py 1000000 256 10 5 > gpurun_out/prof_gbdt2/run.log 2>&1 || { tail -5 gpurun_out/prof_gbdt2/run.log; exit 1; }
find /tmp/pg2 -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_gbdt2/ \;
head -12 gpurun_out/prof_gbdt2/run_kernel_stats.csv | cut -c1-60,200-330
