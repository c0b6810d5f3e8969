#!/bin/bash
# GPU suite; dense head re-measure; s2 wgrad NZ x splits sweep at G = 10 / 25; GBDT device path
# (tests, level timing, kernel stats) and the GBDT tournament-GA bench (BASELINE config 5)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/ > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
mkdir -p gpurun_out/dense3
rm -f gpurun_out/dense3/sweep2.log
for ut in 2 4; do
  GENTUN_DENSE_UT=$ut timeout -k 10 120 python3 -u tools/bench_dense.py 25 20 >> gpurun_out/dense3/sweep2.log 2>&1 || { tail -5 gpurun_out/dense3/sweep2.log; exit 1; }
done
grep '^{' gpurun_out/dense3/sweep2.log
bash tools/gpu_wgrad_sweep.sh > gpurun_out/wgrad_sweep_summary.txt 2>&1 || { tail -5 gpurun_out/wgrad_sweep_summary.txt; exit 1; }
cat gpurun_out/wgrad_sweep_summary.txt
bash tools/gpu_gbdt3.sh || exit $?
( while sleep 50; do date >> gpurun_out/gbdt3/heartbeat; done ) & hb=$!
trap 'kill $hb' EXIT
timeout -k 10 ${GA_TIME:-540} python3 -u tools/bench_gbdt.py --pop 10 --gens 3 > gpurun_out/gbdt3/ga.json 2> gpurun_out/gbdt3/ga.err || { tail -5 gpurun_out/gbdt3/ga.err; exit 1; }
cat gpurun_out/gbdt3/ga.json
