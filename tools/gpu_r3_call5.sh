#!/bin/bash
# same-box A/B: branch-free staging loads (default build) vs per-chunk branches (ab/branchy.so):
# per-launch conv / wgrad at G = 25 and the population step at P = 5; then the GBDT chunk-rows A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
mkdir -p gpurun_out/ab5; rm -f gpurun_out/ab5/*.log
for round in 1 2; do
for lib in default branchy; do
  if [ $lib = branchy ]; then export GENTUN_HIP_LIB=gentun_amd/_native/ab/branchy.so; else unset GENTUN_HIP_LIB; fi
  REGEPI=1 DUO=0 G=25 DBGS=0 timeout -k 10 200 python3 -u tools/bench_conv.py 10 2>/dev/null | grep '^{' | sed "s/^/$lib /" >> gpurun_out/ab5/conv.log || { echo conv failed; exit 1; }
  timeout -k 10 200 python3 -u tools/probe_pop.py 5 5 1 2 10000 2>/dev/null | grep '^{' | sed "s/^/$lib /" >> gpurun_out/ab5/pop.log || { echo pop failed; exit 1; }
done
done
unset GENTUN_HIP_LIB
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/ab5/conv.log"):
    lib, js = l.split(" ", 1); r = json.loads(js)
    d[(r["kernel"], r["shape"], lib)].append(r["us"])
keys = sorted({(k[0], k[1]) for k in d})
for k in keys:
    print(k, "default", d[k + ("default",)], "branchy", d[k + ("branchy",)])
for l in open("gpurun_out/ab5/pop.log"):
    lib, js = l.split(" ", 1); r = json.loads(js); print(lib, r["ms_per_step"], r["cand_per_hour_full_protocol"])
PY
bash tools/gpu_gbdt_chunk.sh
