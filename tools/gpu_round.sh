#!/bin/bash
# Standard GPU validation round: tests, kernel microbench, profile, bench. Each GPU step has its own limit.
mkdir -p gpurun_out
export GENTUN_NO_AUTOBUILD=1
timeout -k 10 400 python -m pytest tests/ -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/round.log
timeout -k 10 300 python tools/bench_kernels.py 50 > gpurun_out/bench_kernels.log 2>&1 || exit 1
timeout -k 10 300 python tools/probe_concurrency.py 4 1 4000 > gpurun_out/concurrency.log 2>&1 || exit 1
tools/gpu_prof.sh hip -- python3 tools/probe_steps.py hip 101-0101110011 1 4000 > gpurun_out/prof_hip.log 2>&1 || exit 1
timeout -k 10 800 python bench.py --steps 1 --warmup 0 > gpurun_out/bench_full.log 2>&1 || exit 1
