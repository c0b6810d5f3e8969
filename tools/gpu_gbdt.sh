#!/bin/bash
# GBDT GPU path: tests, then the 1M x 256 GA throughput bench (BASELINE cfg 5 per GPU)
mkdir -p gpurun_out
export GENTUN_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest tests/test_gbdt_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gbdt_tests.log 2>&1 || { tail -30 gpurun_out/gbdt_tests.log; exit 1; }
tail -1 gpurun_out/gbdt_tests.log
timeout -k 10 400 python tools/bench_gbdt.py --pop ${POP:-8} --rounds ${ROUNDS:-50} > gpurun_out/bench_gbdt.log 2>&1 || { tail -10 gpurun_out/bench_gbdt.log; exit 1; }
grep "{" gpurun_out/bench_gbdt.log
