# bank-paired reduction order of the stage-2 3x3 conv: tests, microbench + step A/B vs the kk-major build
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_hip_fp32.py \
  tests/test_hip_train.py tests/test_hip_duo.py > gpurun_out/r4c21_tests.log 2>&1 || { tail -30 gpurun_out/r4c21_tests.log; exit 1; }
tail -1 gpurun_out/r4c21_tests.log
for lib in "" ab_libs/kkmajor.so; do
  GENTUN_HIP_LIB=$lib G=25 DBGS=0 ONLY=s2_n timeout -k 10 200 python -u tools/bench_conv.py 10 > gpurun_out/r4c21_conv.log 2>&1 || { tail -5 gpurun_out/r4c21_conv.log; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/r4c21_conv.log'):
    if l.startswith('{'):
        d = json.loads(l); print('${lib:-tree}', d['kernel'], d['shape'], d['us'])"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for lib in "" ab_libs/kkmajor.so; do
  rm -rf /tmp/pmcb; GENTUN_HIP_LIB=$lib G=25 DBGS=0 ONLY=s2_n timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d /tmp/pmcb -o run --output-format csv -- python3 tools/bench_conv.py 3 > gpurun_out/r4c21_pmc.log 2>&1 || { tail -5 gpurun_out/r4c21_pmc.log; exit 1; }
  echo "lib=${lib:-tree}"; python3 tools/pmc_summary.py /tmp/pmcb | grep conv_fast | cut -c1-300
done
cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
  for lib in "" ab_libs/kkmajor.so; do
    GENTUN_HIP_LIB=$lib DTYPE=fp32 RESET=all timeout -k 10 200 python -u tools/probe_pop.py 5 5 1 1 \
      > gpurun_out/r4c21_run.log 2>&1 || { tail -5 gpurun_out/r4c21_run.log; exit 1; }
    echo "P=5 ${lib:-tree} $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c21_run.log)"
  done
done
