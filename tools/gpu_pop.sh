#!/bin/bash
# Population executor: GPU tests, then throughput probes. Each GPU step has its own limit.
mkdir -p gpurun_out
export GENTUN_NO_AUTOBUILD=1
timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py tests/test_hip_train.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -n 60 gpurun_out/pytest_gpu.log; exit 1; }
tail -n 2 gpurun_out/pytest_gpu.log
for cfg in "8 8 1" "8 4 2" "16 16 1" "16 8 2"; do
  timeout -k 10 200 python tools/probe_pop.py $cfg 1 10000 >> gpurun_out/pop.log 2>&1 || { tail -20 gpurun_out/pop.log; exit 1; }
done
grep '{' gpurun_out/pop.log
