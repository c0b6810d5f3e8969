#!/bin/bash
# Q-curve (groups per launch = 5 x candidates) of the fp32 population step + bf16-vs-fp32 fitness delta.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1 DTYPE=fp32
for P in 2 4 8 16; do
  echo "== Q=$((5 * P)) (P=$P candidates x 5 folds), fp32, concurrent folds, 1 epoch of 8000 rows"
  timeout -k 10 200 python -u tools/probe_pop.py $P $P 1 1 > gpurun_out/qc.log 2>&1 || { tail -5 gpurun_out/qc.log; exit 1; }
  grep '^{' gpurun_out/qc.log | cut -c1-220
done
timeout -k 10 600 python -u tools/fitness_delta.py 16 > gpurun_out/fitness_delta.log 2>&1 || { tail -5 gpurun_out/fitness_delta.log; exit 1; }
grep -E "delta|summary" gpurun_out/fitness_delta.log
