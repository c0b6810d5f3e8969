#!/bin/bash
# GPU suite (wide conv tile kernels), wide deep-space kernel stats + population probe, GA20 part 1
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/ > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
KERNELS=64,128,256 P=3 bash tools/gpu_prof_deep.sh > gpurun_out/deep_stats.txt || { tail gpurun_out/deep_stats.txt; exit 1; }
head -12 gpurun_out/deep/kernel_stats.csv | cut -d, -f1-5 | cut -c1-140
SPACE=deep KERNELS=64,128,256 BN=1 DTYPE=fp32 timeout -k 10 300 python3 -u tools/probe_pop.py 3 3 1 1 10000 2>&1 | grep '^{' | tee gpurun_out/deep/probe_wide.json
BUDGET=${BUDGET:-780} bash tools/gpu_ga20.sh
