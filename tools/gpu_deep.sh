#!/bin/bash
# Deep S=(3,4,5) search space: population throughput and per-kernel profile.
mkdir -p gpurun_out
export GENTUN_NO_AUTOBUILD=1 SPACE=deep
timeout -k 10 300 python tools/probe_pop.py 16 16 1 1 10000 > gpurun_out/deep_probe.log 2>&1 || { tail -20 gpurun_out/deep_probe.log; exit 1; }
grep '{' gpurun_out/deep_probe.log
WARM=0 bash tools/gpu_prof.sh deep -- python3 tools/probe_pop.py 16 16 1 1 4000 > gpurun_out/prof_deep.log 2>&1 || { tail -20 gpurun_out/prof_deep.log; exit 1; }
