# Round 6: cost of the GPU auc per boosting round, 1M x 256, depth 10, 5 folds, binary:logistic:
# logloss vs auc runs under rocprofv3 --kernel-trace --stats.
export GENTUN_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for m in logloss auc; do
  rm -rf /tmp/pa_$m; mkdir -p gpurun_out/auc_$m
  OBJ=binary:logistic METRIC=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pa_$m -o run --output-format csv -- \
    python3 tools/probe_gbdt.py 1000000 256 10 10 > gpurun_out/auc_$m/run.log 2>&1 || { tail -5 gpurun_out/auc_$m/run.log; exit 1; }
  find /tmp/pa_$m -name "*kernel_stats.csv" -exec cp {} gpurun_out/auc_$m/ \;
  grep "{" gpurun_out/auc_$m/run.log
done
grep -h "auc\|radix\|metric_kernel\|onesweep\|histogram" gpurun_out/auc_*/run_kernel_stats.csv | cut -d, -f1-4
