#!/bin/bash
# BatchNorm statistics from the fp32 conv epilogue: tests (fp32 BN parity, fused pool), deep bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
mkdir -p gpurun_out/bns
timeout -k 10 600 python -u -m pytest -m gpu -x -q -s --timeout 300 --timeout-method thread tests/test_hip_bn.py tests/test_hip_step_parity.py tests/test_hip_train.py tests/test_batchnorm.py \
  > gpurun_out/bns/tests.log 2>&1 || { grep -E "parity|FAIL|Error|assert" gpurun_out/bns/tests.log | tail -30; exit 1; }
grep -E "passed|failed" gpurun_out/bns/tests.log | tail -1
grep -E "\[parity\].*bn True" gpurun_out/bns/tests.log | head -4
: > gpurun_out/bns/bench.log
for v in 1 0; do
  GENTUN_BN_EPI_STATS=$v timeout -k 10 600 python -u bench.py --gpus 1 --space deep --batch-norm --per-gpu 3 --steps 3 --warmup 1 > gpurun_out/bns/b$v.json 2> gpurun_out/bns/b$v.err || { tail -20 gpurun_out/bns/b$v.err; exit 1; }
  echo "epi_stats=$v $(cut -c1-200 gpurun_out/bns/b$v.json)" >> gpurun_out/bns/bench.log
done
cat gpurun_out/bns/bench.log
