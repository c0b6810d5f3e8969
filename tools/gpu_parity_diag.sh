#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -m gpu -q --timeout 200 --timeout-method thread tests/test_hip_fp32.py -k "dgrad or conv_fwd" -s > gpurun_out/diag_fp32.log 2>&1; echo "fp32 rc=$?"
grep -E "\[fp32\] conv|passed|failed" gpurun_out/diag_fp32.log | tail -40
for pk in 1 0; do for m in "" 1; do
  GENTUN_CONV_PK=$pk GENTUN_PARITY_MASKS=$m timeout -k 10 300 python -u -m pytest -m gpu -q --timeout 200 --timeout-method thread tests/test_hip_step_parity.py -k "one_step_gradients_match" -s > gpurun_out/diag_par_$pk$m.log 2>&1; echo "parity pk=$pk masks=$m rc=$?"
  grep -E "\[parity\]" gpurun_out/diag_par_$pk$m.log
done; done
