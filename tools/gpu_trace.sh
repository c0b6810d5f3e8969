#!/bin/bash
# Kernel trace (start/end per dispatch) of a short population run, for timeline analysis.
mkdir -p gpurun_out/trace
export GENTUN_NO_AUTOBUILD=1 WARM=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf /tmp/trace
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/trace -o run --output-format csv -- python3 tools/probe_pop.py 16 16 1 1 4000 > gpurun_out/trace/probe.log 2>&1 || { tail -20 gpurun_out/trace/probe.log; exit 1; }
f=$(find /tmp/trace -name "*kernel_trace.csv" | head -1)
python3 tools/timeline.py "$f" > gpurun_out/trace/timeline.txt
gzip -c "$f" > gpurun_out/trace/kernel_trace.csv.gz
cat gpurun_out/trace/timeline.txt
