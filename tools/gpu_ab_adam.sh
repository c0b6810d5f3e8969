#!/bin/bash
# correctness of the per-layer optimizer overlap, then bench A/B (same seed, same candidates)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_hip_train.py tests/test_hip_step_parity.py \
  > gpurun_out/gpu_tests_adam.log 2>&1 || { tail -30 gpurun_out/gpu_tests_adam.log; exit 1; }
tail -2 gpurun_out/gpu_tests_adam.log
: > gpurun_out/ab_adam.log
run() {  # name env... -- bench args
  name=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --gpus 1 --warmup 1 $BARGS > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || { tail -20 gpurun_out/ab_$name.err; exit 1; }
  echo "$name $(cut -c1-330 gpurun_out/ab_$name.json)" >> gpurun_out/ab_adam.log; echo "$name done"
}
BARGS="--per-gpu 6 --steps 4"
run ovl1 GENTUN_ADAM_OVERLAP=1
run ovl0 GENTUN_ADAM_OVERLAP=0
BARGS="--per-gpu 6 --steps 4 --streams 2"
run ovl1_s2 GENTUN_ADAM_OVERLAP=1
