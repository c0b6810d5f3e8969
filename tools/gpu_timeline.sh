#!/bin/bash
# Kernel trace of population steps (16 S=(3,5) candidates x 5 folds) -> tools/timeline.py summary
set -o pipefail
mkdir -p gpurun_out/timeline
export GENTUN_NO_AUTOBUILD=1 WARM=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf /tmp/tl
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/tl -o run --output-format csv -- python3 tools/probe_pop.py ${P:-16} 16 1 1 ${SAMPLES:-2000} > gpurun_out/timeline/run.log 2>&1 || { tail -5 gpurun_out/timeline/run.log; exit 1; }
f=$(find /tmp/tl -name "*kernel_trace.csv" | head -1)
python3 tools/timeline.py "$f" > gpurun_out/timeline/summary.txt
head -40 gpurun_out/timeline/summary.txt
