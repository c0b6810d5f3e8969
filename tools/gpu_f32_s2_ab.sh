#!/bin/bash
# A/B of the fp32 stage-2 conv tiles (GENTUN_F32_S2): microbench + population step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1 DTYPE=fp32
for v in 0 1 2; do
  echo "== GENTUN_F32_S2=$v"
  GENTUN_F32_S2=$v ONLY=s2_ DBGS=0 F32P=0 timeout -k 10 200 python -u tools/bench_conv.py 10 > gpurun_out/s2ab.log 2>&1 || { tail -5 gpurun_out/s2ab.log; exit 1; }
  grep '^{' gpurun_out/s2ab.log | grep -v wgrad | cut -c1-220
  for P in 3 16; do
    GENTUN_F32_S2=$v timeout -k 10 200 python -u tools/probe_pop.py $P $P 1 1 > gpurun_out/s2ab.log 2>&1 || { tail -5 gpurun_out/s2ab.log; exit 1; }
    grep '^{' gpurun_out/s2ab.log | cut -c1-200
  done
done
