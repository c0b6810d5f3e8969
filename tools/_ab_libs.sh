set -o pipefail
export GENTUN_NO_AUTOBUILD=1
mkdir -p gpurun_out/abl
: > gpurun_out/abl/conv.log
for r in 1 2; do for lib in ${LIBS:-base ro ro_pf3 ro_pf4}; do
  GENTUN_HIP_LIB=ab_libs/$lib.so G=25 DBGS=0 ONLY="${ONLY:-_n}" timeout -k 10 120 python -u tools/bench_conv.py 10 2>/dev/null | grep -v wgrad | sed "s/^/$lib /" >> gpurun_out/abl/conv.log || exit 1
done; done
for r in 1 2; do for lib in ${LIBS:-base ro ro_pf3 ro_pf4}; do
  GENTUN_HIP_LIB=ab_libs/$lib.so timeout -k 10 200 python tools/probe_pop.py 5 5 1 1 10000 > gpurun_out/abl/pop.log 2>&1 || { tail -5 gpurun_out/abl/pop.log; exit 1; }
  echo "$lib $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abl/pop.log)" | tee -a gpurun_out/abl/pop_summary.txt
done; done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/abl/conv.log"):
    lib, js = l.split(" ", 1)
    r = json.loads(js)
    d[(r["kernel"], r["shape"], lib)].append(r["us"])
for k in sorted(d):
    print("%-11s %-18s %-8s %s" % (k[0], k[1], k[2], " ".join("%.1f" % v for v in d[k])))
PY
