#!/bin/bash
# usage: tools/gpu_prof.sh NAME -- cmd...   (runs rocprofv3 kernel-trace+stats, keeps only the stats CSVs)
set -e
name=$1; shift; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf /tmp/prof_$name
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_$name -o run --output-format csv -- "$@"
mkdir -p gpurun_out/prof_$name
find /tmp/prof_$name -name "*stats.csv" -exec cp {} gpurun_out/prof_$name/ \;
ls gpurun_out/prof_$name
