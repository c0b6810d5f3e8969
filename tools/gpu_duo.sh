#!/bin/bash
# duo conv kernel: bit-identity tests, then per-kernel timing duo on / off at G=25 and G=80; dataset spread probes
export GENTUN_NO_AUTOBUILD=1
mkdir -p gpurun_out; rm -f gpurun_out/duo_conv.log gpurun_out/probe_spread2.log
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_duo.py > gpurun_out/duo_tests.log 2>&1 || { tail -30 gpurun_out/duo_tests.log; exit 1; }
tail -3 gpurun_out/duo_tests.log
for G in 25 80; do
  for D in 0 1; do
    DUO=$D G=$G DBGS=0,1,6 timeout -k 10 200 python3 -u tools/bench_conv.py 10 >> gpurun_out/duo_conv.log 2>&1 || { tail -5 gpurun_out/duo_conv.log; exit 1; }
  done
done
python3 - <<'PY'
import json
rows=[json.loads(l) for l in open("gpurun_out/duo_conv.log") if l.startswith("{")]
for r in rows:
    if r["kernel"]!="conv_wgrad":
        print(r["G"], r["duo"], r["kernel"], r["shape"], "dbg", r["dbg"], r["us"])
PY
timeout -k 10 200 python3 -u tools/probe_spread.py 12 relation '{}' >> gpurun_out/probe_spread2.log 2>&1 || { tail -5 gpurun_out/probe_spread2.log; exit 1; }
timeout -k 10 200 python3 -u tools/probe_spread.py 12 relation '{"distractors": 3, "noise": 1.5}' >> gpurun_out/probe_spread2.log 2>&1 || { tail -5 gpurun_out/probe_spread2.log; exit 1; }
grep summary gpurun_out/probe_spread2.log
