#!/bin/bash
# A/B of the population step: build/ab_old/libgentun_hip.so (previous commit's
# kernels, same C ABI, loaded through GENTUN_HIP_LIB) vs the tree's library.
# usage: [TESTS="tests/..."] [EP=3] [SPACE=deep] tools/gpu_ab2.sh
mkdir -p gpurun_out
export GENTUN_NO_AUTOBUILD=1
if [ -n "$TESTS" ]; then
timeout -k 10 400 python -u -m pytest $TESTS -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -n 60 gpurun_out/pytest_gpu.log; exit 1; }
tail -n 2 gpurun_out/pytest_gpu.log
fi
EP=${EP:-2}
for i in 1 2 3; do
  GENTUN_HIP_LIB=build/ab_old/libgentun_hip.so timeout -k 10 200 python tools/probe_pop.py 16 16 1 $EP 10000 > gpurun_out/ab_old_$i.log 2>&1 || { tail -20 gpurun_out/ab_old_$i.log; exit 1; }
  timeout -k 10 200 python tools/probe_pop.py 16 16 1 $EP 10000 > gpurun_out/ab_new_$i.log 2>&1 || { tail -20 gpurun_out/ab_new_$i.log; exit 1; }
  echo "old: $(grep -o '"ms_per_cand_step": [0-9.]*' gpurun_out/ab_old_$i.log)  new: $(grep -o '"ms_per_cand_step": [0-9.]*' gpurun_out/ab_new_$i.log)"
done
