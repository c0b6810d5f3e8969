# per-layer conv Adam on the W1 optimizer stream (GENTUN_ADAM_OVERLAP=1) vs one launch after the backward (0)
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_hip_train.py -k "adam_overlap" \
  > gpurun_out/r4c30_test.log 2>&1 || { tail -30 gpurun_out/r4c30_test.log; exit 1; }
grep -E "passed|failed" gpurun_out/r4c30_test.log | tail -3
for v in "all 5 0" "all 5 1" "all 5 0" "all 5 1" "kernels 2 0" "kernels 2 1" "all 2 0" "all 2 1"; do
  set -- $v
  GENTUN_ADAM_OVERLAP=$3 DTYPE=fp32 RESET=$1 timeout -k 10 200 python -u tools/probe_pop.py $2 $2 1 1 \
    > gpurun_out/r4c30_run.log 2>&1 || { tail -5 gpurun_out/r4c30_run.log; exit 1; }
  echo "RESET=$1 P=$2 adam_overlap=$3 $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c30_run.log)"
done
