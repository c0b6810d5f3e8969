#!/bin/bash
# Forward conv microbench: one-tile kernel (epi 1) vs pipelined kernel (epi 2) at several tiles per workgroup.
mkdir -p gpurun_out
export GENTUN_NO_AUTOBUILD=1 GENTUN_BENCH_G=40
for cfg in "1 0" "2 0" "2 2" "2 4" "2 8"; do
  set -- $cfg
  for sh in 1 4; do
    GENTUN_EPI_BF16=$1 GENTUN_CONV_PIPE=1 GENTUN_CONV_PIPE_IPT=$2 GENTUN_BENCH_ONLY=conv_fwd:$sh timeout -k 10 120 python tools/bench_kernels.py 20 > gpurun_out/bkp.log 2>&1 || { tail -20 gpurun_out/bkp.log; exit 1; }
    echo "epi=$1 ipt=$2 $(grep -h '"conv_fwd"' gpurun_out/bkp.log | cut -c1-100)"
  done
done
