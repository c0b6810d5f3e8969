#!/bin/bash
# GBDT histogram A/B on one box: GPU tests (default library), then for every ab_libs/<name>.so in
# LIBS (plus the in-tree library, "tree") a rocprofv3 --stats run of one cv call (tools/probe_gbdt.py
# 1M x 256, depth 10), REPS times alternating; BENCH=1 adds the tournament-GA bench on the tree lib.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export GENTUN_NO_AUTOBUILD=1
root=$PWD
out=$root/gpurun_out/r5/gbdt_ab${TAG:-}; mkdir -p $out
( while sleep 50; do date >> $out/heartbeat; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
if [ "${TESTS:-1}" != "0" ]; then
  timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 150 --timeout-method thread tests/test_gbdt_gpu.py \
    > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
  tail -1 $out/tests.log
fi
export TMPDIR=/tmp
for r in $(seq ${REPS:-2}); do
  for lib in ${LIBS:-} tree; do
    d=/tmp/gbab_${lib}_$r; rm -rf $d
    if [ $lib = tree ]; then unset GENTUN_HIP_LIB; else export GENTUN_HIP_LIB=$root/ab_libs/$lib.so; fi
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- \
      python3 $root/tools/probe_gbdt.py ${ROWS:-1000000} 256 ${DEPTH:-10} ${ROUNDS:-3}) > $out/run_${lib}_$r.log 2>&1 \
      || { tail -5 $out/run_${lib}_$r.log; exit 1; }
    f=$(find $d -name "*kernel_stats.csv" | head -1); cp $f $out/stats_${lib}_$r.csv
    python3 - $out/stats_${lib}_$r.csv "$lib" "$(grep '{' $out/run_${lib}_$r.log | tail -1)" <<'PY' | tee -a $out/summary.txt
import csv, json, sys
hist = [r for r in csv.DictReader(open(sys.argv[1])) if "hist_kernel" in r["Name"]]
js = json.loads(sys.argv[3])
print("%-8s hist %7.1f us/call (%d calls)  ms_per_tree %.3f  rmse %.6f" % (
    sys.argv[2], float(hist[0]["AverageNs"]) / 1e3, int(hist[0]["Calls"]), js["ms_per_tree"], js["test_rmse"]))
PY
  done
done
unset GENTUN_HIP_LIB
if [ -n "${BENCH:-}" ]; then
  timeout -k 10 700 python -u tools/bench_gbdt.py --pop ${POP:-10} --gens ${GENS:-3} --rounds 5000 --esr 100 \
    > $out/bench_gbdt.log 2>&1 || { tail -10 $out/bench_gbdt.log; exit 1; }
  grep "{" $out/bench_gbdt.log | cut -c1-400
fi
