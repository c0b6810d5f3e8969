#!/bin/bash
# Baseline GPU check: gpu tests, concurrency probe, per-step profile, 1-step bench. Each GPU step has its own limit.
mkdir -p gpurun_out
export GENTUN_NO_AUTOBUILD=1
timeout -k 10 400 python -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -n 40 gpurun_out/pytest_gpu.log; exit 1; }
tail -n 2 gpurun_out/pytest_gpu.log
timeout -k 10 200 python tools/probe_steps.py hip 101-0101110011 1 10000 > gpurun_out/steps_hip.log 2>&1 || exit 1
timeout -k 10 200 python tools/probe_steps.py hip 111-1111111111 1 10000 >> gpurun_out/steps_hip.log 2>&1 || exit 1
timeout -k 10 300 python tools/probe_concurrency.py 8 1 10000 > gpurun_out/concurrency.log 2>&1 || exit 1
cat gpurun_out/steps_hip.log gpurun_out/concurrency.log | grep '{'
tools/gpu_prof.sh hip -- python3 tools/probe_steps.py hip 101-0101110011 1 4000 > gpurun_out/prof_hip.log 2>&1 || exit 1
timeout -k 10 800 python bench.py --steps 1 --warmup 0 > gpurun_out/bench_full.log 2>&1 || exit 1
tail -n 1 gpurun_out/bench_full.log
