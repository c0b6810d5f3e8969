#!/bin/bash
# Same-box A/B of the population step: build/ab_head (tree of the last commit + its HIP library) vs this tree.
mkdir -p gpurun_out
export GENTUN_NO_AUTOBUILD=1
R=$PWD
for i in 1 2 3; do
  (cd build/ab_head && timeout -k 10 200 python tools/probe_pop.py 16 16 1 ${EP:-2} 10000) > gpurun_out/ab_old_$i.log 2>&1 || { tail -20 gpurun_out/ab_old_$i.log; exit 1; }
  timeout -k 10 200 python tools/probe_pop.py 16 16 1 ${EP:-2} 10000 > gpurun_out/ab_new_$i.log 2>&1 || { tail -20 gpurun_out/ab_new_$i.log; exit 1; }
  echo "old: $(grep -o '"ms_per_cand_step": [0-9.]*' gpurun_out/ab_old_$i.log)  new: $(grep -o '"ms_per_cand_step": [0-9.]*' gpurun_out/ab_new_$i.log)"
done
