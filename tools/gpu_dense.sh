#!/bin/bash
# dense fwd / dgrad pipelining: kernel tests, per-kernel time at the bench round size, short bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1 WARM=0
mkdir -p gpurun_out/dense
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_hip_fp32.py tests/test_hip_kernels.py tests/test_hip_train.py tests/test_hip_step_parity.py \
  > gpurun_out/dense/tests.log 2>&1 || { tail -30 gpurun_out/dense/tests.log; exit 1; }
tail -1 gpurun_out/dense/tests.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf /tmp/dn
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /tmp/dn -o run --output-format csv -- python3 tools/probe_pop.py 5 5 1 1 2000 > gpurun_out/dense/run.log 2>&1 || { tail -5 gpurun_out/dense/run.log; exit 1; }
find /tmp/dn -name "*kernel_stats.csv" -exec cp {} gpurun_out/dense/kernel_stats.csv \;
grep -E "dense" gpurun_out/dense/kernel_stats.csv | cut -d, -f1-4
timeout -k 10 400 python -u bench.py --gpus 1 --per-gpu 5 --steps 3 --warmup 1 > gpurun_out/dense/bench.json 2> gpurun_out/dense/bench.err || { tail -20 gpurun_out/dense/bench.err; exit 1; }
cut -c1-200 gpurun_out/dense/bench.json
