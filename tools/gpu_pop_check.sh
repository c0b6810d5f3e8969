#!/bin/bash
# HIP kernel + training tests, then 3 population-step throughput probes (16 S=(3,5) candidates, EP epochs)
mkdir -p gpurun_out
export GENTUN_NO_AUTOBUILD=1
timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py tests/test_hip_train.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -n 40 gpurun_out/pytest_gpu.log; exit 1; }
tail -n 1 gpurun_out/pytest_gpu.log
for i in 1 2 3; do
  timeout -k 10 200 python tools/probe_pop.py 16 16 1 ${EP:-2} 10000 > gpurun_out/pop_$i.log 2>&1 || { tail -20 gpurun_out/pop_$i.log; exit 1; }
  grep -o '"ms_per_cand_step": [0-9.]*' gpurun_out/pop_$i.log
done
