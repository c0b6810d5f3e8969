#!/bin/bash
# secondary bench lines at HEAD: bf16 fast mode; deep S=(3,4,5) fp32 + BN with more timed rounds
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
mkdir -p gpurun_out/sec
timeout -k 10 600 python -u bench.py --gpus 1 --dtype bf16 --steps 4 --warmup 1 > gpurun_out/sec/bf16.json 2> gpurun_out/sec/bf16.err || { tail -20 gpurun_out/sec/bf16.err; exit 1; }
cut -c1-300 gpurun_out/sec/bf16.json
timeout -k 10 900 python -u bench.py --gpus 1 --space deep --batch-norm --per-gpu 3 --steps 6 --warmup 1 > gpurun_out/sec/deep.json 2> gpurun_out/sec/deep.err || { tail -20 gpurun_out/sec/deep.err; exit 1; }
cut -c1-300 gpurun_out/sec/deep.json
