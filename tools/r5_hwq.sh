#!/bin/bash
# GPU_MAX_HW_QUEUES=3 crash (verdict r4 6a): torch-only graph probe with 1, 2, 3 side streams, then the
# population probe; stops at the first crash (run LAST in a gpurun call).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export GENTUN_NO_AUTOBUILD=1
mkdir -p gpurun_out/r5; log=gpurun_out/r5/hwq_probe.log; : > $log
for k in 1 2 3; do
  GPU_MAX_HW_QUEUES=3 timeout -k 10 120 python -X faulthandler tools/probe_hwq.py $k >> $log 2>&1
  rc=$?; echo "torch graph, $k side streams, GPU_MAX_HW_QUEUES=3: exit $rc" | tee -a $log
  [ $rc -ne 0 ] && { tail -30 $log; exit 0; }
done
GPU_MAX_HW_QUEUES=3 DTYPE=fp32 RESET=all timeout -k 10 240 python -X faulthandler tools/probe_pop.py 5 5 1 1 2000 >> $log 2>&1
echo "population probe, GPU_MAX_HW_QUEUES=3: exit $?" | tee -a $log
tail -30 $log
