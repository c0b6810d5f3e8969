#!/bin/bash
# round 3 GBDT: GPU tests (exactness vs CPU engine), per-level timing and kernel stats after the reduce fix
set -o pipefail
mkdir -p gpurun_out/gbdt3
export GENTUN_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gbdt_gpu.py > gpurun_out/gbdt3/tests.log 2>&1 || { tail -20 gpurun_out/gbdt3/tests.log; exit 1; }
tail -1 gpurun_out/gbdt3/tests.log
for d in 6 10; do
  timeout -k 10 200 python3 tools/probe_gbdt.py 1000000 256 $d 5 > gpurun_out/gbdt3/plain_$d.log 2>&1 || { tail -5 gpurun_out/gbdt3/plain_$d.log; exit 1; }
  grep "{" gpurun_out/gbdt3/plain_$d.log | tail -1
done
rm -rf /tmp/pg3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pg3 -o run --output-format csv -- python3 tools/probe_gbdt.py 1000000 256 10 5 > gpurun_out/gbdt3/run.log 2>&1 || { tail -5 gpurun_out/gbdt3/run.log; exit 1; }
find /tmp/pg3 -name "*kernel_stats.csv" -exec cp {} gpurun_out/gbdt3/ \;
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/gbdt3/run_kernel_stats.csv")))
for r in rows[:8]:
    print(r["Name"].split("(")[0].replace("(anonymous namespace)::", "")[:40], r["Calls"], r["AverageNs"], r["Percentage"])
PY
