#!/bin/bash
# stage-2 3x3 fp32 conv: 8-row (default) vs 4-row bands (GENTUN_F32_S2=3)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
mkdir -p gpurun_out
GENTUN_F32_S2=3 timeout -k 10 300 python -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread tests/test_hip_fp32.py -k "16-16-50-50 or dgrad" > gpurun_out/th4_tests.log 2>&1 || { tail -30 gpurun_out/th4_tests.log; exit 1; }
tail -1 gpurun_out/th4_tests.log
: > gpurun_out/th4_conv.log
for v in 0 3; do for G in 25 80; do
  GENTUN_F32_S2=$v ONLY=s2_n G=$G DBGS=0 F32P=0 timeout -k 10 300 python -u tools/bench_conv.py 10 2>&1 | grep '^{' | sed "s/^/s2=$v /" >> gpurun_out/th4_conv.log || exit 1
done; done
cut -c1-160 gpurun_out/th4_conv.log
: > gpurun_out/th4_bench.log
for v in 3 0; do
  GENTUN_F32_S2=$v timeout -k 10 400 python -u bench.py --gpus 1 --per-gpu 5 --steps 4 --warmup 1 > gpurun_out/th4_bench_$v.json 2> gpurun_out/th4_bench_$v.err || { tail -20 gpurun_out/th4_bench_$v.err; exit 1; }
  echo "s2=$v $(cut -c1-200 gpurun_out/th4_bench_$v.json)" >> gpurun_out/th4_bench.log
done
cat gpurun_out/th4_bench.log
