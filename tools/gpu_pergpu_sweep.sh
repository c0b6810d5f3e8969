#!/bin/bash
# bench.py candidates-per-round sweep (same seed; 24 timed candidates each)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
mkdir -p gpurun_out
: > gpurun_out/pergpu_sweep.log
for cfg in ${CFGS:-"3 8" "4 6" "6 4"}; do
  set -- $cfg
  timeout -k 10 400 python -u bench.py --gpus 1 --per-gpu $1 --steps $2 --warmup 1 > gpurun_out/pg_$1.json 2> gpurun_out/pg_$1.err || { tail -20 gpurun_out/pg_$1.err; exit 1; }
  echo "per_gpu=$1 $(cat gpurun_out/pg_$1.json)" >> gpurun_out/pergpu_sweep.log
  echo "per_gpu=$1 done"
done
