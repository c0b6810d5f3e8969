#!/bin/bash
# kernel timeline + stats at the bench round size (P=5 -> 25 groups), then the torch-ops comparator bench
set -o pipefail
mkdir -p gpurun_out/timeline
export GENTUN_NO_AUTOBUILD=1 WARM=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf /tmp/tl
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /tmp/tl -o run --output-format csv -- python3 tools/probe_pop.py 5 5 1 1 4000 > gpurun_out/timeline/run.log 2>&1 || { tail -5 gpurun_out/timeline/run.log; exit 1; }
f=$(find /tmp/tl -name "*kernel_trace.csv" | head -1)
python3 tools/timeline.py "$f" > gpurun_out/timeline/summary_p5.txt
s=$(find /tmp/tl -name "*kernel_stats.csv" | head -1)
cp "$s" gpurun_out/timeline/kernel_stats_p5.csv
head -30 gpurun_out/timeline/summary_p5.txt
[ -z "$TORCHCMP" ] && exit 0
timeout -k 10 900 python -u bench.py --gpus 1 --backend torch --per-gpu 2 --steps 1 --warmup 0 \
  > gpurun_out/bench_torch.json 2> gpurun_out/bench_torch.err || { tail -20 gpurun_out/bench_torch.err; exit 1; }
cat gpurun_out/bench_torch.json
