#!/bin/bash
# kernel timeline of the deep-wide population step: S=(3,4,5), kernels (64,128,256), fp32 + BatchNorm, 1 candidate x 5 folds
export GENTUN_NO_AUTOBUILD=1 WARM=0 SPACE=deep KERNELS=64,128,256 BN=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/tl_deep; rm -rf /tmp/tld
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/tld -o run --output-format csv -- python3 tools/probe_pop.py ${P:-1} ${P:-1} 1 1 2000 > gpurun_out/tl_deep/run.log 2>&1 || { tail -5 gpurun_out/tl_deep/run.log; exit 1; }
python3 tools/timeline.py "$(find /tmp/tld -name '*kernel_trace.csv' | head -1)" > gpurun_out/tl_deep/summary.txt
head -40 gpurun_out/tl_deep/summary.txt
