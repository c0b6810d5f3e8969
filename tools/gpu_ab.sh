#!/bin/bash
# GPU kernel + training tests, per-kernel microbench (new vs ab_old/), then an
# A/B of the population step: ab_old/ (previous commit, built) vs the tree.
mkdir -p gpurun_out
export GENTUN_NO_AUTOBUILD=1
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py tests/test_hip_train.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -n 60 gpurun_out/pytest_gpu.log; exit 1; }
tail -n 2 gpurun_out/pytest_gpu.log
fi
GENTUN_BENCH_G=40 timeout -k 10 200 python tools/bench_kernels.py 20 > gpurun_out/bk_new.log 2>&1 || { tail -20 gpurun_out/bk_new.log; exit 1; }
(cd ab_old && GENTUN_BENCH_G=40 timeout -k 10 200 python tools/bench_kernels.py 20) > gpurun_out/bk_old.log 2>&1 || { tail -20 gpurun_out/bk_old.log; exit 1; }
EP=${EP:-3}
for i in 1 2 3; do
  (cd ab_old && timeout -k 10 200 python tools/probe_pop.py 16 16 1 $EP 10000) > gpurun_out/ab_old_$i.log 2>&1 || { tail -20 gpurun_out/ab_old_$i.log; exit 1; }
  timeout -k 10 200 python tools/probe_pop.py 16 16 1 $EP 10000 > gpurun_out/ab_new_$i.log 2>&1 || { tail -20 gpurun_out/ab_new_$i.log; exit 1; }
  echo "old: $(grep -o '"ms_per_cand_step": [0-9.]*' gpurun_out/ab_old_$i.log)  new: $(grep -o '"ms_per_cand_step": [0-9.]*' gpurun_out/ab_new_$i.log)"
done
if [ -n "$DEEP" ]; then
  (cd ab_old && SPACE=deep timeout -k 10 300 python tools/probe_pop.py 16 16 1 1 10000) > gpurun_out/ab_deep_old.log 2>&1 || { tail -20 gpurun_out/ab_deep_old.log; exit 1; }
  SPACE=deep timeout -k 10 300 python tools/probe_pop.py 16 16 1 1 10000 > gpurun_out/ab_deep_new.log 2>&1 || { tail -20 gpurun_out/ab_deep_new.log; exit 1; }
  echo "deep old: $(grep -o '"ms_per_cand_step": [0-9.]*' gpurun_out/ab_deep_old.log)  new: $(grep -o '"ms_per_cand_step": [0-9.]*' gpurun_out/ab_deep_new.log)"
fi
