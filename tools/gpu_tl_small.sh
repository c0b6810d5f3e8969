#!/bin/bash
# kernel timelines of small population steps (Q = 2: reference folds, P=2; Q = 10: concurrent folds, P=2)
export GENTUN_NO_AUTOBUILD=1 WARM=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/tl_small; rm -rf /tmp/tl2 /tmp/tl10
RESET=kernels timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/tl2 -o run --output-format csv -- python3 tools/probe_pop.py 2 2 1 1 2000 > gpurun_out/tl_small/q2.log 2>&1 || { tail -5 gpurun_out/tl_small/q2.log; exit 1; }
python3 tools/timeline.py "$(find /tmp/tl2 -name '*kernel_trace.csv' | head -1)" > gpurun_out/tl_small/q2.txt
RESET=all timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/tl10 -o run --output-format csv -- python3 tools/probe_pop.py 2 2 1 1 2000 > gpurun_out/tl_small/q10.log 2>&1 || { tail -5 gpurun_out/tl_small/q10.log; exit 1; }
python3 tools/timeline.py "$(find /tmp/tl10 -name '*kernel_trace.csv' | head -1)" > gpurun_out/tl_small/q10.txt
head -30 gpurun_out/tl_small/q2.txt; head -30 gpurun_out/tl_small/q10.txt
rm -f gpurun_out/probe_spread4.log
for kw in '{"noise": 0.35}' '{"noise": 0.35, "distractors": 0}'; do
  timeout -k 10 200 python3 -u tools/probe_spread.py 12 compound "$kw" >> gpurun_out/probe_spread4.log 2>&1 || { tail -5 gpurun_out/probe_spread4.log; exit 1; }
done
timeout -k 10 200 python3 -u tools/probe_spread.py 12 relation '{"noise": 0.35, "distractors": 1}' >> gpurun_out/probe_spread4.log 2>&1 || { tail -5 gpurun_out/probe_spread4.log; exit 1; }
grep summary gpurun_out/probe_spread4.log
