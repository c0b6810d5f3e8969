#!/bin/bash
# Population-step throughput under tuning overrides (one probe per setting; SETTINGS="ENV=VAL ..." entries separated by ';')
mkdir -p gpurun_out
export GENTUN_NO_AUTOBUILD=1
IFS=';' read -ra SET <<< "$SETTINGS"
for st in "${SET[@]}"; do
  env $st timeout -k 10 200 python tools/probe_pop.py 16 16 1 ${EP:-2} 10000 > gpurun_out/sweep.log 2>&1 || { echo "FAIL $st"; tail -5 gpurun_out/sweep.log; exit 1; }
  echo "$st -> $(grep -o '"ms_per_cand_step": [0-9.]*' gpurun_out/sweep.log)"
done
