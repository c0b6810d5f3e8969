#!/bin/bash
export GENTUN_NO_AUTOBUILD=1
mkdir -p gpurun_out; rm -f gpurun_out/wgrad_sweep.log
for G in 10 25; do for NZ in 1 2 4; do for SP in 8 16 32; do
  GENTUN_WGRAD_NZ=$NZ GENTUN_WGRAD_SPLITS_W=16:$SP G=$G DBGS=0 ONLY=s2 timeout -k 10 120 python3 -u tools/bench_conv.py 10 2>&1 | grep conv_wgrad | sed "s/^/NZ=$NZ SP=$SP /" >> gpurun_out/wgrad_sweep.log || { tail -5 gpurun_out/wgrad_sweep.log; exit 1; }
done; done; done
python3 - <<'PY'
import json
for l in open("gpurun_out/wgrad_sweep.log"):
    tag, js = l.split(" {", 1)[0], "{" + l.split(" {", 1)[1]
    r = json.loads(js)
    print(tag, r["G"], r["shape"], r["us"])
PY
