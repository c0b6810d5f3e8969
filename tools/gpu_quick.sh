#!/bin/bash
# Quick GPU check: tests, kernel microbench, learning curve, full bench. Each GPU step has its own limit.
mkdir -p gpurun_out
export GENTUN_NO_AUTOBUILD=1
timeout -k 10 400 python -m pytest tests/ -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1 || { tail -n 40 gpurun_out/pytest_gpu.log; exit 1; }
tail -n 2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/bench_kernels.py 50 > gpurun_out/bench_kernels.log 2>&1 || exit 1
timeout -k 10 300 python tools/probe_learning.py > gpurun_out/learn_deep.log 2>&1 || exit 1
timeout -k 10 800 python bench.py --steps 1 --warmup 0 > gpurun_out/bench_full.log 2>&1 || exit 1
tail -n 1 gpurun_out/bench_full.log
