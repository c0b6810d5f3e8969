# step PMC profile at the bench round size (25 groups), and the separate-vs-fused wgrad split reduction A/B
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_hip_kernels.py tests/test_hip_train.py tests/test_hip_dense_stream.py > gpurun_out/r4c11_tests.log 2>&1 \
  || { tail -30 gpurun_out/r4c11_tests.log; exit 1; }
tail -1 gpurun_out/r4c11_tests.log
P=5 OUT=profstep_p5 bash tools/gpu.sh profstep || exit 1
for spec in "kernels 2" "all 5" "all 2"; do
  set -- $spec
  for v in 1 0 1 0; do
    GENTUN_WGRAD_REDUCE=$v DTYPE=fp32 RESET=$1 timeout -k 10 200 python -u tools/probe_pop.py $2 $2 1 1 \
      > gpurun_out/r4c11_run.log 2>&1 || { tail -5 gpurun_out/r4c11_run.log; exit 1; }
    echo "RESET=$1 P=$2 wgrad_reduce=$v $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c11_run.log)"
  done
done
