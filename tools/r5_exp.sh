#!/bin/bash
# Round-5 GPU experiments (run through gpurun from the repo root). Every step under its own limit,
# chained so the first failure ends the call.
#   TESTS="tests/x.py ..."  GPU tests first (default: the fp32 / kernel / train suites; TESTS=none skips)
#   LIBS="a b"              ab_libs/<name>.so kernel libraries compared (conv microbench + population step)
#   CONV_ONLY=, CONV_DBGS=0 conv microbench filter / dbg modes; POP=5 population-step groups; REPS=2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export GENTUN_NO_AUTOBUILD=1
out=gpurun_out/r5/${TAG:-x}; mkdir -p $out
( while sleep 50; do date >> $out/heartbeat; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
tests=${TESTS:-tests/test_hip_fp32.py tests/test_hip_kernels.py tests/test_hip_train.py}
if [ "$tests" != "none" ]; then
  timeout -k 10 ${TTIME:-500} python -u -m pytest -m gpu -x -q --timeout 150 --timeout-method thread $tests \
    > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
  tail -1 $out/tests.log
fi
for r in $(seq ${REPS:-2}); do
  for lib in ${LIBS:-}; do
    if [ -n "${CONV:-1}" ] && [ "${CONV:-1}" != "0" ]; then
      GENTUN_HIP_LIB=ab_libs/$lib.so G=${G:-25} DBGS=${CONV_DBGS:-0} ONLY="${CONV_ONLY:-}" timeout -k 10 200 \
        python -u tools/bench_conv.py 10 2>/dev/null | sed "s/^/$lib /" >> $out/conv.log || { echo "conv $lib failed"; exit 1; }
    fi
    if [ "${POP:-5}" != "0" ]; then
      GENTUN_HIP_LIB=ab_libs/$lib.so DTYPE=fp32 RESET=${RESET:-all} timeout -k 10 200 \
        python tools/probe_pop.py ${POP:-5} ${POP:-5} 1 1 10000 > $out/pop_$lib.log 2>&1 || { tail -5 $out/pop_$lib.log; exit 1; }
      echo "$lib P=${POP:-5} $(grep -o '"ms_per_step": [0-9.]*' $out/pop_$lib.log)" | tee -a $out/pop_summary.txt
    fi
  done
done
if [ -s $out/conv.log ]; then
python3 - "$out/conv.log" <<'PY' | tee $out/conv_summary.txt
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    lib, js = l.split(" ", 1)
    r = json.loads(js)
    d[(r["kernel"], r["shape"], r["dbg"], lib)].append(r["us"])
for k in sorted(d):
    print("%-11s %-18s dbg%-2d %-10s %s" % (k[0], k[1], k[2], k[3], " ".join("%.1f" % v for v in d[k])))
PY
fi
