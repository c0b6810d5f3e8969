#!/bin/bash
mkdir -p gpurun_out
export GENTUN_NO_AUTOBUILD=1 SPACE=deep
for st in GENTUN_WGRAD_TARGET=50 GENTUN_WGRAD_TARGET=25 GENTUN_WGRAD_TARGET=12 GENTUN_WGRAD_TARGET=100 GENTUN_WGRAD_SPLITS_W=16:2 GENTUN_WGRAD_TARGET=50; do
  env $st timeout -k 10 200 python tools/probe_pop.py 16 16 1 1 10000 > gpurun_out/dsweep.log 2>&1 || { echo "FAIL $st"; tail -5 gpurun_out/dsweep.log; exit 1; }
  echo "$st -> $(grep -o '"ms_per_cand_step": [0-9.]*' gpurun_out/dsweep.log)"
done
