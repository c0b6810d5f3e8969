#!/bin/bash
# rocprofv3 --stats of the population step (probe_pop P P 1 1 SAMPLES) for each ab_libs/<lib>.so in LIBS;
# prints the per-call time of the kernels matching KPAT (regex).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export GENTUN_NO_AUTOBUILD=1 TMPDIR=/tmp
root=$PWD; out=$root/gpurun_out/r5/prof${TAG:-}; mkdir -p $out
for lib in ${LIBS:-}; do
  d=/tmp/pl_$lib; rm -rf $d
  (cd /tmp && GENTUN_HIP_LIB=$root/ab_libs/$lib.so DTYPE=fp32 RESET=all WARM=0 timeout -k 10 240 rocprofv3 --kernel-trace --stats \
    -d $d -o run --output-format csv -- python3 $root/tools/probe_pop.py ${P:-5} ${P:-5} 1 1 ${SAMPLES:-2000}) \
    > $out/run_$lib.log 2>&1 || { tail -5 $out/run_$lib.log; exit 1; }
  cp $(find $d -name "*kernel_stats.csv" | head -1) $out/stats_$lib.csv
  python3 - $out/stats_$lib.csv "$lib" "${KPAT:-.}" <<'PY' | tee -a $out/summary.txt
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    if re.search(sys.argv[3], r["Name"]):
        print("%-10s %-60s %6s calls %9.1f us" % (sys.argv[2], r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
