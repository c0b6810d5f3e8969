#!/bin/bash
# GBDT histogram chunk rows A/B (GENTUN_GBDT_CHUNK): level timing + test RMSE (must not change: exact int64
# sums), kernel stats at the best setting, GPU GBDT tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
mkdir -p gpurun_out/gbdtc; rm -f gpurun_out/gbdtc/ab.log
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gbdt_gpu.py > gpurun_out/gbdtc/tests.log 2>&1 || { tail -20 gpurun_out/gbdtc/tests.log; exit 1; }
tail -1 gpurun_out/gbdtc/tests.log
for ch in 16384 32768 65536 131072; do
  for d in 6 10; do
    GENTUN_GBDT_CHUNK=$ch timeout -k 10 200 python3 tools/probe_gbdt.py 1000000 256 $d 5 > gpurun_out/gbdtc/p.log 2>&1 || { tail -5 gpurun_out/gbdtc/p.log; exit 1; }
    echo "chunk=$ch $(grep '{' gpurun_out/gbdtc/p.log | tail -1)" | tee -a gpurun_out/gbdtc/ab.log
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf /tmp/pgc
GENTUN_GBDT_CHUNK=${BEST:-65536} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pgc -o run --output-format csv -- python3 tools/probe_gbdt.py 1000000 256 10 5 > gpurun_out/gbdtc/run.log 2>&1 || { tail -5 gpurun_out/gbdtc/run.log; exit 1; }
find /tmp/pgc -name "*kernel_stats.csv" -exec cp {} gpurun_out/gbdtc/ \;
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/gbdtc/run_kernel_stats.csv")))
for r in rows[:10]:
    print(r["Name"].split("(")[0].replace("(anonymous namespace)::", "")[:40], r["Calls"], r["AverageNs"], r["Percentage"])
PY
