#!/bin/bash
# round 3: wgrad column slices (tests + small-Q probe), overlap A/B at small Q, variant dataset spread
export GENTUN_NO_AUTOBUILD=1
mkdir -p gpurun_out; rm -f gpurun_out/exp7.log gpurun_out/probe_spread5.log
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_duo.py > gpurun_out/duo_tests.log 2>&1 || { tail -30 gpurun_out/duo_tests.log; exit 1; }
tail -1 gpurun_out/duo_tests.log
for nz in 1 0; do for ov in 1 0; do
  echo "== Q=2 kernels NZ=$nz OVERLAP=$ov" >> gpurun_out/exp7.log
  GENTUN_WGRAD_NZ=$nz GENTUN_OVERLAP=$ov RESET=kernels WARM=1 timeout -k 10 120 python3 -u tools/probe_pop.py 2 2 1 1 10000 >> gpurun_out/exp7.log 2>&1 || { tail -5 gpurun_out/exp7.log; exit 1; }
  echo "== Q=10 all NZ=$nz OVERLAP=$ov" >> gpurun_out/exp7.log
  GENTUN_WGRAD_NZ=$nz GENTUN_OVERLAP=$ov RESET=all WARM=1 timeout -k 10 120 python3 -u tools/probe_pop.py 2 2 1 1 10000 >> gpurun_out/exp7.log 2>&1 || { tail -5 gpurun_out/exp7.log; exit 1; }
done; done
echo "== Q=25 all NZ=0 OVERLAP=1" >> gpurun_out/exp7.log
RESET=all WARM=1 timeout -k 10 120 python3 -u tools/probe_pop.py 5 5 1 1 10000 >> gpurun_out/exp7.log 2>&1 || { tail -5 gpurun_out/exp7.log; exit 1; }
grep -o '== .*\|"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/exp7.log
for kw in '{}' '{"tick": 8, "noise": 0.7}'; do
  timeout -k 10 200 python3 -u tools/probe_spread.py 12 variant "$kw" >> gpurun_out/probe_spread5.log 2>&1 || { tail -5 gpurun_out/probe_spread5.log; exit 1; }
done
grep summary gpurun_out/probe_spread5.log
