#!/bin/bash
# A/B of the population step: ab_old/ (previous commit, built) vs the tree.
mkdir -p gpurun_out
export GENTUN_NO_AUTOBUILD=1
EP=${EP:-3}
for i in 1 2 3; do
  (cd ab_old && timeout -k 10 200 python tools/probe_pop.py 16 16 1 $EP 10000) > gpurun_out/ab_old_$i.log 2>&1 || { tail -20 gpurun_out/ab_old_$i.log; exit 1; }
  timeout -k 10 200 python tools/probe_pop.py 16 16 1 $EP 10000 > gpurun_out/ab_new_$i.log 2>&1 || { tail -20 gpurun_out/ab_new_$i.log; exit 1; }
  GENTUN_W1_STREAM=0 timeout -k 10 200 python tools/probe_pop.py 16 16 1 $EP 10000 > gpurun_out/ab_new1s_$i.log 2>&1 || { tail -20 gpurun_out/ab_new1s_$i.log; exit 1; }
  echo "old: $(grep -o '"ms_per_cand_step": [0-9.]*' gpurun_out/ab_old_$i.log)  new: $(grep -o '"ms_per_cand_step": [0-9.]*' gpurun_out/ab_new_$i.log)  new-1side: $(grep -o '"ms_per_cand_step": [0-9.]*' gpurun_out/ab_new1s_$i.log)"
done
