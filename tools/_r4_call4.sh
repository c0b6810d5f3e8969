set -o pipefail
export GENTUN_NO_AUTOBUILD=1
mkdir -p gpurun_out/r4c4
timeout -k 10 300 python -u -m pytest -s -q --timeout 200 --timeout-method thread tests/test_hip_fp32.py -k s2in tests/test_hip_dp.py > gpurun_out/r4c4/tests.log 2>&1 || { tail -30 gpurun_out/r4c4/tests.log; exit 1; }
grep -E "\[fp32\]|\[dp\]|passed|failed" gpurun_out/r4c4/tests.log
for i in 1 2; do for ct in 0 1; do
  GENTUN_S2IN_CT1=$ct timeout -k 10 200 python tools/probe_pop.py 5 5 1 1 10000 > gpurun_out/r4c4/pop_ct$ct.log 2>&1 || { tail -5 gpurun_out/r4c4/pop_ct$ct.log; exit 1; }
  echo "ct1=$ct $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4c4/pop_ct$ct.log)"
done; done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf /tmp/pmcclk
G=25 DBGS=0 ONLY=s2_n timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES -d /tmp/pmcclk -o run --output-format csv -- python3 tools/bench_conv.py 5 > gpurun_out/r4c4/pmcclk.log 2>&1 || { tail -5 gpurun_out/r4c4/pmcclk.log; exit 1; }
python3 tools/pmc_summary.py /tmp/pmcclk > gpurun_out/r4c4/pmcclk.txt 2>&1; head -20 gpurun_out/r4c4/pmcclk.txt
find /tmp/pmcclk -name "*counter_collection.csv" -exec cp {} gpurun_out/r4c4/counters.csv \;
