# two-part staging of the stage-2 3x3 conv: tests, microbench and step A/B (tree / split off / kk-major build)
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_hip_fp32.py \
  tests/test_hip_train.py tests/test_hip_duo.py > gpurun_out/r4c20_tests.log 2>&1 || { tail -30 gpurun_out/r4c20_tests.log; exit 1; }
tail -1 gpurun_out/r4c20_tests.log
for v in "tree 1" "tree 0" "ab_libs/noparts.so 1"; do
  set -- $v
  lib=$1; [ "$lib" = tree ] && lib=""
  GENTUN_HIP_LIB=$lib GENTUN_S2_SPLIT=$2 G=25 DBGS=0 ONLY=s2_n timeout -k 10 200 python -u tools/bench_conv.py 10 > gpurun_out/r4c20_conv.log 2>&1 || { tail -5 gpurun_out/r4c20_conv.log; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/r4c20_conv.log'):
    if l.startswith('{'):
        d = json.loads(l); print('$1 split=$2', d['kernel'], d['shape'], d['us'])"
done
for i in 1 2; do
  for v in "tree 1" "tree 0" "ab_libs/noparts.so 1"; do
    set -- $v
    lib=$1; [ "$lib" = tree ] && lib=""
    GENTUN_HIP_LIB=$lib GENTUN_S2_SPLIT=$2 DTYPE=fp32 RESET=all timeout -k 10 200 python -u tools/probe_pop.py 5 5 1 1 \
      > gpurun_out/r4c20_run.log 2>&1 || { tail -5 gpurun_out/r4c20_run.log; exit 1; }
    echo "P=5 $1 split=$2 $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c20_run.log)"
  done
done
