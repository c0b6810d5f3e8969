#!/bin/bash
# BASELINE config 4 shapes on one GPU: S=(3,4,5) (20,50,100) + BN and the wide (64,128,256) + BN space,
# bench.py rounds (3 timed after 1 warm-up), each under its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export GENTUN_NO_AUTOBUILD=1
out=gpurun_out/r5/deep_bench; mkdir -p $out
( while sleep 50; do date >> $out/heartbeat; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 400 python3 -u bench.py --gpus 1 --space deep --batch-norm --steps 3 --warmup 1 \
  > $out/deep.json 2> $out/deep.err || { tail -5 $out/deep.err; exit 1; }
cut -c1-200 $out/deep.json
timeout -k 10 700 python3 -u bench.py --gpus 1 --space deep --kernels 64,128,256 --batch-norm --per-gpu 3 --steps 3 \
  --warmup 1 > $out/wide.json 2> $out/wide.err || { tail -5 $out/wide.err; exit 1; }
cut -c1-200 $out/wide.json
