#!/bin/bash
# fp32 batch invariance at the bench's settings; kernel stats of the wide deep space; PMC of the headline step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
mkdir -p gpurun_out/inv
timeout -k 10 240 python3 -u tools/probe_invariance.py 2000 6 1 > gpurun_out/inv/inv.log 2>&1 || { tail -5 gpurun_out/inv/inv.log; exit 1; }
grep '^{' gpurun_out/inv/inv.log
KERNELS=64,128,256 P=3 bash tools/gpu_prof_deep.sh || exit $?
P=5 OUT=prof_r3 bash tools/gpu_prof_head.sh || exit $?
