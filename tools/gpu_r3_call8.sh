#!/bin/bash
# wide deep-space kernels: fp32 numerics tests first, GPU suite, kernel stats + population probe
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_fp32.py > gpurun_out/fp32_tests.log 2>&1 || { tail -30 gpurun_out/fp32_tests.log; exit 1; }
tail -1 gpurun_out/fp32_tests.log
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/ > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
KERNELS=64,128,256 P=3 bash tools/gpu_prof_deep.sh > gpurun_out/deep_stats.txt || { tail gpurun_out/deep_stats.txt; exit 1; }
head -14 gpurun_out/deep/kernel_stats.csv | cut -d, -f1-5 | cut -c1-140
SPACE=deep KERNELS=64,128,256 BN=1 DTYPE=fp32 timeout -k 10 300 python3 -u tools/probe_pop.py 3 3 1 1 10000 2>&1 | grep '^{' | tee gpurun_out/deep/probe_wide.json
SPACE=deep BN=1 DTYPE=fp32 timeout -k 10 300 python3 -u tools/probe_pop.py 3 3 1 1 10000 2>&1 | grep '^{' | tee gpurun_out/deep/probe_deep.json
