#!/bin/bash
# fp32 wgrad splits per width (partials bytes vs workgroups) at the bench round size
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
mkdir -p gpurun_out
: > gpurun_out/splits_bench.log
for sp in "16:8,32:32" "16:4,32:16" "16:4,32:32" "16:8,32:16"; do
  GENTUN_WGRAD_SPLITS_W=$sp timeout -k 10 400 python -u bench.py --gpus 1 --per-gpu 5 --steps 3 --warmup 1 > gpurun_out/sp.json 2> gpurun_out/sp.err || { tail -20 gpurun_out/sp.err; exit 1; }
  echo "splits=$sp $(cut -c1-200 gpurun_out/sp.json)" >> gpurun_out/splits_bench.log; echo "$sp done"
done
cat gpurun_out/splits_bench.log
