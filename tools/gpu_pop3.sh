#!/bin/bash
# GPU tests (kernels + training), then population throughput A/B of the
# dense-W1 optimizer stream (own stream vs the wgrad side stream).
mkdir -p gpurun_out
export GENTUN_NO_AUTOBUILD=1
timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py tests/test_hip_train.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -n 60 gpurun_out/pytest_gpu.log; exit 1; }
tail -n 2 gpurun_out/pytest_gpu.log
timeout -k 10 200 python tools/probe_pop.py 16 16 1 1 10000 > gpurun_out/pop.log 2>&1 || { tail -20 gpurun_out/pop.log; exit 1; }
GENTUN_W1_STREAM=0 timeout -k 10 200 python tools/probe_pop.py 16 16 1 1 10000 >> gpurun_out/pop.log 2>&1 || { tail -20 gpurun_out/pop.log; exit 1; }
timeout -k 10 200 python tools/probe_pop.py 16 16 1 1 10000 >> gpurun_out/pop.log 2>&1 || { tail -20 gpurun_out/pop.log; exit 1; }
grep '{' gpurun_out/pop.log
