#!/bin/bash
# Q-curve at HEAD: groups per launch vs per-group throughput, both fold protocols
# (all: P candidates x 5 concurrent folds = 5P groups; kernels: P groups per launch, folds in sequence)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1 DTYPE=fp32
mkdir -p gpurun_out/qc3
for spec in "all 1" "all 2" "all 4" "all 5" "all 8" "all 16" "kernels 2" "kernels 5" "kernels 10" "kernels 16"; do
  set -- $spec
  RESET=$1 timeout -k 10 200 python -u tools/probe_pop.py $2 $2 1 1 > gpurun_out/qc3/run.log 2>&1 || { tail -5 gpurun_out/qc3/run.log; exit 1; }
  echo "== RESET=$1 P=$2 $(grep '^{' gpurun_out/qc3/run.log | cut -c1-200)" | tee -a gpurun_out/qc3/qcurve.txt
done
