#!/bin/bash
# BatchNorm: kernel tests, step parity with BN, deep-space learning with / without BN.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export GENTUN_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -s tests/test_hip_step_parity.py \
  -k "batchnorm or True" > gpurun_out/bn_parity.log 2>&1; rc=$?
grep -E "parity|passed|failed" gpurun_out/bn_parity.log
[ $rc -le 1 ] || exit 1
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -s tests/test_hip_bn.py \
  > gpurun_out/bn_tests.log 2>&1; rc=$?
grep -E "\[bn\]|passed|failed" gpurun_out/bn_tests.log
[ $rc -le 1 ] || exit 1
timeout -k 10 900 python -u tools/probe_deep.py 3000 6 > gpurun_out/deep_bn.log 2>&1 || { tail -20 gpurun_out/deep_bn.log; exit 1; }
grep '{' gpurun_out/deep_bn.log
