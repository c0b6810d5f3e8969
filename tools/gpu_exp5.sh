#!/bin/bash
# round 3: eval-batch tests, streams-at-small-P probe, compound dataset spread
export GENTUN_NO_AUTOBUILD=1
mkdir -p gpurun_out; rm -f gpurun_out/streams.log gpurun_out/probe_spread3.log
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_hip_dp.py > gpurun_out/hip_train_tests.log 2>&1 || { tail -30 gpurun_out/hip_train_tests.log; exit 1; }
tail -2 gpurun_out/hip_train_tests.log
for cfg in "5 5 1" "5 3 2" "2 2 1" "2 1 2" "10 5 2" "10 10 1"; do
  set -- $cfg
  echo "== P=$1 pop_batch=$2 streams=$3 RESET=all" >> gpurun_out/streams.log
  WARM=1 timeout -k 10 120 python3 -u tools/probe_pop.py $1 $2 $3 1 10000 >> gpurun_out/streams.log 2>&1 || { tail -5 gpurun_out/streams.log; exit 1; }
done
for cfg in "5 5 1" "5 3 2" "5 1 5"; do
  set -- $cfg
  echo "== P=$1 pop_batch=$2 streams=$3 RESET=kernels" >> gpurun_out/streams.log
  RESET=kernels WARM=1 timeout -k 10 120 python3 -u tools/probe_pop.py $1 $2 $3 1 10000 >> gpurun_out/streams.log 2>&1 || { tail -5 gpurun_out/streams.log; exit 1; }
done
grep -A1 "==" gpurun_out/streams.log | grep -o '"P".*cand_per_hour_full_protocol": [0-9.]*'
timeout -k 10 200 python3 -u tools/probe_spread.py 12 compound '{}' >> gpurun_out/probe_spread3.log 2>&1 || { tail -5 gpurun_out/probe_spread3.log; exit 1; }
timeout -k 10 200 python3 -u tools/probe_spread.py 12 compound '{"dist": [6, 8], "distractors": 0}' >> gpurun_out/probe_spread3.log 2>&1 || { tail -5 gpurun_out/probe_spread3.log; exit 1; }
grep summary gpurun_out/probe_spread3.log
