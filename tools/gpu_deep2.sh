#!/bin/bash
# Kernel tests, small-image conv microbench (images per workgroup 1/2/4), deep-space throughput.
mkdir -p gpurun_out
export GENTUN_NO_AUTOBUILD=1
timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py tests/test_hip_train.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -n 60 gpurun_out/pytest_gpu.log; exit 1; }
tail -n 2 gpurun_out/pytest_gpu.log
for n in 1 2 4; do
  GENTUN_CONV_IMGS=$n GENTUN_BENCH_G=40 GENTUN_BENCH_ONLY=conv_fwd:5 timeout -k 10 120 python tools/bench_kernels.py 20 > gpurun_out/bk_imgs$n.log 2>&1 || { tail -20 gpurun_out/bk_imgs$n.log; exit 1; }
  echo "imgs=$n $(grep -h '"us"' gpurun_out/bk_imgs$n.log | cut -c1-120)"
done
for n in 1 2 4; do
  GENTUN_CONV_IMGS=$n SPACE=deep timeout -k 10 300 python tools/probe_pop.py 16 16 1 1 10000 > gpurun_out/deep_probe_$n.log 2>&1 || { tail -20 gpurun_out/deep_probe_$n.log; exit 1; }
  echo "imgs=$n $(grep -o '"ms_per_cand_step": [0-9.]*' gpurun_out/deep_probe_$n.log)"
done
