#!/bin/bash
# 4- vs 8-wave workgroups of the fast conv shapes: conv tests at both, per-shape microbench, population probe.
mkdir -p gpurun_out
export GENTUN_NO_AUTOBUILD=1 GENTUN_BENCH_G=40
for n in 4 8; do
GENTUN_CONV_NWV=$n timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread -k "conv" > gpurun_out/pytest_nwv$n.log 2>&1 || { tail -30 gpurun_out/pytest_nwv$n.log; exit 1; }
tail -1 gpurun_out/pytest_nwv$n.log
done
for sh in 0 1 3 4; do
  for k in conv_fwd conv_dgrad; do
    for n in 4 8; do
      GENTUN_EPI_BF16=$([ $k = conv_fwd ] && echo 1 || echo 0) GENTUN_CONV_NWV=$n GENTUN_BENCH_ONLY=$k:$sh timeout -k 10 120 python tools/bench_kernels.py 20 > gpurun_out/bkn.log 2>&1 || { tail -20 gpurun_out/bkn.log; exit 1; }
      echo "nwv=$n $(grep -h "\"$k\"" gpurun_out/bkn.log | cut -c1-90)"
    done
  done
done
for i in 1 2; do
for n in 0 4; do
  GENTUN_CONV_NWV=$n timeout -k 10 200 python tools/probe_pop.py 16 16 1 3 10000 > gpurun_out/nwv_$n.log 2>&1 || { tail -20 gpurun_out/nwv_$n.log; exit 1; }
  echo "nwv=$n $(grep -o '"ms_per_cand_step": [0-9.]*' gpurun_out/nwv_$n.log)"
done
done
