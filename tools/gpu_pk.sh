#!/bin/bash
# packed last co tile: fp32 kernel tests + e2e parity, conv microbench A/B, bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_hip_fp32.py tests/test_hip_train.py tests/test_hip_step_parity.py \
  > gpurun_out/gpu_tests_pk.log 2>&1 || { tail -30 gpurun_out/gpu_tests_pk.log; exit 1; }
tail -2 gpurun_out/gpu_tests_pk.log
: > gpurun_out/pk_conv.log
for pk in 1 0; do
  GENTUN_CONV_PK=$pk G=25 DBGS=0 F32P=0 timeout -k 10 300 python -u tools/bench_conv.py 10 2>&1 | grep '^{' | sed "s/^/pk=$pk /" >> gpurun_out/pk_conv.log || exit 1
done
echo conv done
[ -n "$NOBENCH" ] && exit 0
: > gpurun_out/pk_bench.log
for pk in 1 0; do
  GENTUN_CONV_PK=$pk timeout -k 10 400 python -u bench.py --gpus 1 --per-gpu 5 --steps 4 --warmup 1 > gpurun_out/pk_bench_$pk.json 2> gpurun_out/pk_bench_$pk.err || { tail -20 gpurun_out/pk_bench_$pk.err; exit 1; }
  echo "pk=$pk $(cut -c1-300 gpurun_out/pk_bench_$pk.json)" >> gpurun_out/pk_bench.log; echo "bench pk=$pk done"
done
