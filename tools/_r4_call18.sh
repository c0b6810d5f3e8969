# GBDT constant-hessian count histograms: GPU tests, hist A/B under rocprof, and the tournament-GA bench (r3 settings)
set -o pipefail
( while sleep 50; do date >> gpurun_out/heartbeat; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 400 python -u -m pytest tests/test_gbdt_gpu.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r4c18_tests.log 2>&1 || { tail -30 gpurun_out/r4c18_tests.log; exit 1; }
tail -1 gpurun_out/r4c18_tests.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for hc in 1 0; do
  rm -rf /tmp/pg$hc; mkdir -p gpurun_out/gbdt_hc$hc
  GENTUN_GBDT_HCONST=$hc GENTUN_GBDT_TIMING=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pg$hc -o run --output-format csv -- \
    python3 tools/probe_gbdt.py 1000000 256 10 5 > gpurun_out/gbdt_hc$hc/run.log 2>&1 || { tail -5 gpurun_out/gbdt_hc$hc/run.log; exit 1; }
  find /tmp/pg$hc -name "*kernel_stats.csv" -exec cp {} gpurun_out/gbdt_hc$hc/ \;
  echo "hconst=$hc"; grep "{\|gbdt_hip" gpurun_out/gbdt_hc$hc/run.log | tail -2 | cut -c1-300
  head -4 gpurun_out/gbdt_hc$hc/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
done
timeout -k 10 700 python -u tools/bench_gbdt.py --pop 10 --gens 3 > gpurun_out/bench_gbdt_r4.log 2>&1 || { tail -10 gpurun_out/bench_gbdt_r4.log; exit 1; }
grep "{" gpurun_out/bench_gbdt_r4.log | cut -c1-400
