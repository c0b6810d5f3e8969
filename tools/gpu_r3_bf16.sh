#!/bin/bash
# bf16 fast-mode bench line at HEAD (secondary; fp32 stays the headline)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
mkdir -p gpurun_out/bf16
( while sleep 50; do date >> gpurun_out/bf16/heartbeat; done ) & hb=$!
trap 'kill $hb' EXIT
timeout -k 10 600 python3 -u bench.py --gpus 1 --dtype bf16 --steps 4 --warmup 1 --json-out gpurun_out/bf16/bench.json \
  > gpurun_out/bf16/bench.out 2> gpurun_out/bf16/bench.err || { tail -5 gpurun_out/bf16/bench.err; exit 1; }
cat gpurun_out/bf16/bench.json
