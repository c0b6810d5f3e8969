#!/bin/bash
# kernel stats of deep-space (S=(3,4,5), kernels (20,50,100)) fp32 + BN population steps
set -o pipefail
mkdir -p gpurun_out/deep
export GENTUN_NO_AUTOBUILD=1 SPACE=deep BN=${BN:-1} DTYPE=fp32
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf /tmp/pd
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pd -o run --output-format csv -- python3 tools/probe_pop.py ${P:-3} ${P:-3} 1 1 2000 > gpurun_out/deep/run.log 2>&1 || { tail -5 gpurun_out/deep/run.log; exit 1; }
s=$(find /tmp/pd -name "*kernel_stats.csv" | head -1)
cp "$s" gpurun_out/deep/kernel_stats.csv
head -25 gpurun_out/deep/kernel_stats.csv | cut -d, -f1-5 | cut -c1-160
tail -2 gpurun_out/deep/run.log | cut -c1-300
