#!/bin/bash
# MNIST-shaped RR-GA bench (the reference's tests/test_mnist.py config: 28x28x1, population 20, RR-GA
# pC 0.2 / pM 0.8, 5-fold, epochs (20,4,1), batch 32, fp32): padded fast kernels vs the generic kernels
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export GENTUN_NO_AUTOBUILD=1
out=gpurun_out/r5/mnist_bench; mkdir -p $out
( while sleep 50; do date >> $out/heartbeat; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 ${T1:-560} python3 -u bench.py --gpus 1 --input-shape 28,28,1 --population 20 --steps ${S1:-8} --warmup 2 \
  --json-out $out/padded.json > $out/padded.out 2> $out/padded.err || { tail -5 $out/padded.err; exit 1; }
cat $out/padded.json
timeout -k 10 ${T2:-400} python3 -u bench.py --gpus 1 --input-shape 28,28,1 --population 20 --pad-images 0 --steps ${S2:-2} \
  --warmup 1 --json-out $out/generic.json > $out/generic.out 2> $out/generic.err || { tail -5 $out/generic.err; exit 1; }
cat $out/generic.json
