#!/bin/bash
# usage: tools/gpu_pmc.sh NAME "COUNTERS" -- cmd...   (PMC pass with kernel-trace only; keeps the CSV summaries)
set -e
name=$1; shift; counters=$1; shift; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf /tmp/pmc_$name
timeout -k 10 600 rocprofv3 --kernel-trace --pmc $counters -d /tmp/pmc_$name -o run --output-format csv -- "$@"
mkdir -p gpurun_out/pmc_$name
python3 tools/pmc_summary.py /tmp/pmc_$name > gpurun_out/pmc_$name/summary.txt
cat gpurun_out/pmc_$name/summary.txt | head -40
