#!/bin/bash
# split-K reduction by the last wgrad workgroup: tests, per-kernel stats, bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1 WARM=0
mkdir -p gpurun_out/wred
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_hip_fp32.py tests/test_hip_train.py tests/test_hip_step_parity.py tests/test_hip_kernels.py \
  > gpurun_out/wred/tests.log 2>&1 || { tail -30 gpurun_out/wred/tests.log; exit 1; }
tail -1 gpurun_out/wred/tests.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in 1 0; do
  rm -rf /tmp/wr$v
  GENTUN_WGRAD_REDUCE=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /tmp/wr$v -o run --output-format csv -- python3 tools/probe_pop.py 5 5 1 1 2000 > gpurun_out/wred/run$v.log 2>&1 || { tail -5 gpurun_out/wred/run$v.log; exit 1; }
  find /tmp/wr$v -name "*kernel_stats.csv" -exec cp {} gpurun_out/wred/kernel_stats_$v.csv \;
  echo "reduce=$v"; grep -E "adam_segments|wgrad_fast_f32" gpurun_out/wred/kernel_stats_$v.csv | cut -d, -f1-4
done
: > gpurun_out/wred/bench.log
for v in 1 0; do
  GENTUN_WGRAD_REDUCE=$v timeout -k 10 400 python -u bench.py --gpus 1 --per-gpu 5 --steps 3 --warmup 1 > gpurun_out/wred/b$v.json 2> gpurun_out/wred/b$v.err || { tail -20 gpurun_out/wred/b$v.err; exit 1; }
  echo "reduce=$v $(cut -c1-200 gpurun_out/wred/b$v.json)" >> gpurun_out/wred/bench.log
done
cat gpurun_out/wred/bench.log
