#!/bin/bash
# stage-3 (deep space) fp32 specialisations: kernel tests, profile, deep bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -x -q -s --timeout 300 --timeout-method thread tests/test_hip_fp32.py tests/test_hip_bn.py tests/test_hip_train.py tests/test_hip_step_parity.py \
  > gpurun_out/gpu_tests_s3.log 2>&1 || { tail -30 gpurun_out/gpu_tests_s3.log; exit 1; }
tail -2 gpurun_out/gpu_tests_s3.log
grep -E "\[fp32\] conv.*8x8" gpurun_out/gpu_tests_s3.log || true
tools/gpu_prof_deep.sh || exit 1
timeout -k 10 600 python -u bench.py --gpus 1 --space deep --batch-norm --per-gpu 3 --steps 3 --warmup 1 > gpurun_out/bench_deep.json 2> gpurun_out/bench_deep.err || { tail -20 gpurun_out/bench_deep.err; exit 1; }
cut -c1-400 gpurun_out/bench_deep.json
