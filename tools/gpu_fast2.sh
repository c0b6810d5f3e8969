#!/bin/bash
mkdir -p gpurun_out
export GENTUN_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_k.log 2>&1 || { tail -n 40 gpurun_out/pytest_k.log; exit 1; }
tail -n 1 gpurun_out/pytest_k.log
GENTUN_BENCH_G=40 GENTUN_EPI_BF16=1 timeout -k 10 200 python tools/bench_kernels.py 20 > gpurun_out/bk_e1.log 2>&1 || exit 1
GENTUN_BENCH_G=40 GENTUN_EPI_BF16=0 timeout -k 10 200 python tools/bench_kernels.py 20 > gpurun_out/bk_e0.log 2>&1 || exit 1
