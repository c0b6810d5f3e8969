#!/bin/bash
# headline bench at the driver's settings (K=20 timed rounds after W=5) + kernel stats / PMC of the bench round size
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
mkdir -p gpurun_out
timeout -k 10 1000 python -u bench.py --gpus 1 --steps ${K:-20} --warmup ${W:-5} > gpurun_out/headline.json 2> gpurun_out/headline.err || { tail -20 gpurun_out/headline.err; exit 1; }
cat gpurun_out/headline.json
