# part-major order for the 5x5 s2 input-conv dgrad too (GT_S2_PARTS=2 build) vs the tree (3x3 only)
set -o pipefail
GENTUN_HIP_LIB=ab_libs/parts2.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_hip_fp32.py tests/test_hip_train.py > gpurun_out/r4c22_tests.log 2>&1 || { tail -30 gpurun_out/r4c22_tests.log; exit 1; }
tail -1 gpurun_out/r4c22_tests.log
for lib in "" ab_libs/parts2.so; do
  GENTUN_HIP_LIB=$lib G=25 DBGS=0 ONLY=s2_in timeout -k 10 200 python -u tools/bench_conv.py 10 > gpurun_out/r4c22_conv.log 2>&1 || { tail -5 gpurun_out/r4c22_conv.log; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/r4c22_conv.log'):
    if l.startswith('{'):
        d = json.loads(l); print('${lib:-tree}', d['kernel'], d['shape'], d['us'])"
done
for i in 1 2; do
  for lib in "" ab_libs/parts2.so; do
    GENTUN_HIP_LIB=$lib DTYPE=fp32 RESET=all timeout -k 10 200 python -u tools/probe_pop.py 5 5 1 1 \
      > gpurun_out/r4c22_run.log 2>&1 || { tail -5 gpurun_out/r4c22_run.log; exit 1; }
    echo "P=5 ${lib:-tree} $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c22_run.log)"
  done
done
