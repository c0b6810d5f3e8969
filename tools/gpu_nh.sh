#!/bin/bash
# fp32 stage-2 3x3 conv without the column halo (3 workgroups per CU) vs the default
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -x -q -s --timeout 300 --timeout-method thread tests/test_hip_fp32.py tests/test_hip_train.py tests/test_hip_step_parity.py \
  > gpurun_out/nh_tests.log 2>&1 || { grep -E "rel.err|FAIL|Error" gpurun_out/nh_tests.log | tail -30; exit 1; }
grep -E "passed|failed" gpurun_out/nh_tests.log | tail -1
grep -E "\[fp32\] conv.*(16x16 50->50|k3 H16)" gpurun_out/nh_tests.log | head -4
: > gpurun_out/nh_conv.log
for v in 1 0; do for G in 25 80; do
  GENTUN_F32_NH=$v ONLY=s2_n G=$G DBGS=0,1 F32P=0 timeout -k 10 300 python -u tools/bench_conv.py 10 2>&1 | grep '^{' | grep -v wgrad | sed "s/^/nh=$v /" >> gpurun_out/nh_conv.log || exit 1
done; done
cut -c1-170 gpurun_out/nh_conv.log | sed 's/"f32p": "0", "grid": "0", "dtype": "fp32", //'
: > gpurun_out/nh_bench.log
for v in 1 0; do
  GENTUN_F32_NH=$v timeout -k 10 400 python -u bench.py --gpus 1 --per-gpu 5 --steps 3 --warmup 1 > gpurun_out/nh_bench_$v.json 2> gpurun_out/nh_bench_$v.err || { tail -20 gpurun_out/nh_bench_$v.err; exit 1; }
  echo "nh=$v $(cut -c1-200 gpurun_out/nh_bench_$v.json)" >> gpurun_out/nh_bench.log
done
cat gpurun_out/nh_bench.log
