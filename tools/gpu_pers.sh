#!/bin/bash
mkdir -p gpurun_out
export GENTUN_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_k.log 2>&1 || { tail -n 60 gpurun_out/pytest_k.log; exit 1; }
tail -n 2 gpurun_out/pytest_k.log
for p in 0 1; do GENTUN_BENCH_G=40 GENTUN_CONV_PERS=$p timeout -k 10 200 python tools/bench_kernels.py 20 > gpurun_out/bkp_$p.log 2>&1 || exit 1; done
