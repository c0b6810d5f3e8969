#!/bin/bash
# GPU suite (branch-free staging numerics), per-launch conv / wgrad times at G = 10 / 25, s2 wgrad NZ A/B,
# timeline at the bench round size, driver-equivalent headline
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/ > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
mkdir -p gpurun_out/conv4; rm -f gpurun_out/conv4/*.log
for G in 10 25; do
  REGEPI=1 DUO=0 G=$G DBGS=0 timeout -k 10 200 python3 -u tools/bench_conv.py 10 >> gpurun_out/conv4/conv.log 2>&1 || { tail -5 gpurun_out/conv4/conv.log; exit 1; }
  for NZ in 1 2; do
    GENTUN_WGRAD_NZ=$NZ REGEPI=1 DUO=0 G=$G DBGS=0 ONLY=s2 timeout -k 10 120 python3 -u tools/bench_conv.py 10 2>&1 | grep conv_wgrad | sed "s/^/NZ=$NZ /" >> gpurun_out/conv4/nz.log || { tail -5 gpurun_out/conv4/nz.log; exit 1; }
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/conv4/conv.log"):
    if l.startswith("{"):
        r = json.loads(l); print(r["G"], r["kernel"], r["shape"], r["us"])
for l in open("gpurun_out/conv4/nz.log"):
    tag, js = l.split(" ", 1); r = json.loads(js); print(tag, r["G"], r["shape"], r["us"])
PY
P=5 SAMPLES=2000 bash tools/gpu_timeline.sh > /dev/null || exit $?
head -20 gpurun_out/timeline/summary.txt
bash tools/gpu_headline3.sh
