#!/bin/bash
# s2 wgrad NZ x splits sweep at G = 10 / 25, then the GBDT device path (tests, level timing, kernel stats)
# and the GBDT tournament-GA bench (BASELINE config 5)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
bash tools/gpu_wgrad_sweep.sh > gpurun_out/wgrad_sweep_summary.txt 2>&1 || { tail -5 gpurun_out/wgrad_sweep_summary.txt; exit 1; }
cat gpurun_out/wgrad_sweep_summary.txt
bash tools/gpu_gbdt3.sh || exit $?
( while sleep 50; do date >> gpurun_out/gbdt3/heartbeat; done ) & hb=$!
trap 'kill $hb' EXIT
timeout -k 10 ${GA_TIME:-600} python3 -u tools/bench_gbdt.py --pop 10 --gens 3 > gpurun_out/gbdt3/ga.json 2> gpurun_out/gbdt3/ga.err || { tail -5 gpurun_out/gbdt3/ga.err; exit 1; }
cat gpurun_out/gbdt3/ga.json
