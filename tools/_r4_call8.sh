# split-K dense forward from the W1 master: tests, then A/B (GENTUN_DENSE_SK) on the probe
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_hip_dense_stream.py tests/test_hip_train.py tests/test_hip_dp.py tests/test_hip_step_parity.py \
  > gpurun_out/r4c8_tests.log 2>&1 || { tail -30 gpurun_out/r4c8_tests.log; exit 1; }
tail -1 gpurun_out/r4c8_tests.log
for spec in "kernels 2" "all 5" "all 2"; do
  set -- $spec
  for v in 1 0 1 0; do
    GENTUN_DENSE_SK=$v DTYPE=fp32 RESET=$1 timeout -k 10 200 python -u tools/probe_pop.py $2 $2 1 1 \
      > gpurun_out/r4c8_run.log 2>&1 || { tail -5 gpurun_out/r4c8_run.log; exit 1; }
    echo "RESET=$1 P=$2 dense_sk=$v $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c8_run.log)"
  done
done
P=5 TAG=_p5sk DUMP=1 bash tools/gpu.sh timeline > /dev/null && head -22 gpurun_out/timeline/summary_p5sk.txt
for wg in 512 2000 100000 512; do
  GENTUN_CONV_SMALLQ_WG=$wg DTYPE=fp32 RESET=all timeout -k 10 200 python -u tools/probe_pop.py 5 5 1 1 \
    > gpurun_out/r4c8_run.log 2>&1 || { tail -5 gpurun_out/r4c8_run.log; exit 1; }
  echo "RESET=all P=5 smallq_wg=$wg $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c8_run.log)"
done
