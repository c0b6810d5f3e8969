#!/bin/bash
export GENTUN_NO_AUTOBUILD=1
mkdir -p gpurun_out; rm -f gpurun_out/regepi_conv.log
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_duo.py > gpurun_out/duo_tests.log 2>&1 || { tail -30 gpurun_out/duo_tests.log; exit 1; }
tail -1 gpurun_out/duo_tests.log
for G in 10 25 80; do for R in 0 1; do
  REGEPI=$R DUO=0 G=$G DBGS=0 timeout -k 10 200 python3 -u tools/bench_conv.py 10 >> gpurun_out/regepi_conv.log 2>&1 || { tail -5 gpurun_out/regepi_conv.log; exit 1; }
done; done
python3 - <<'PY'
import json
rows=[json.loads(l) for l in open("gpurun_out/regepi_conv.log") if l.startswith("{")]
d={}
for r in rows:
    if r["kernel"]=="conv_wgrad" or "s1_in" in r["shape"] and r["kernel"]=="conv_dgrad": continue
    d.setdefault((r["G"], r["kernel"], r["shape"]), {})[r["regepi"]]=r["us"]
for k,v in sorted(d.items()):
    print(k, v.get("0"), v.get("1"))
PY
