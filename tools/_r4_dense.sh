set -o pipefail
export GENTUN_NO_AUTOBUILD=1
mkdir -p gpurun_out/dense
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_hip_dense_stream.py tests/test_hip_step_parity.py tests/test_hip_train.py > gpurun_out/dense/tests.log 2>&1 || { tail -30 gpurun_out/dense/tests.log; exit 1; }
tail -1 gpurun_out/dense/tests.log
for r in 1 2; do for d2 in 0 1; do
  GENTUN_DENSE_DGRAD2=$d2 timeout -k 10 200 python tools/probe_pop.py 5 5 1 1 10000 > gpurun_out/dense/pop.log 2>&1 || { tail -5 gpurun_out/dense/pop.log; exit 1; }
  echo "dgrad2=$d2 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dense/pop.log)"
done; done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for d2 in 0 1; do
  rm -rf /tmp/dn$d2
  GENTUN_DENSE_DGRAD2=$d2 WARM=0 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /tmp/dn$d2 -o run --output-format csv -- python3 tools/probe_pop.py 5 5 1 1 2000 > gpurun_out/dense/prof$d2.log 2>&1 || { tail -5 gpurun_out/dense/prof$d2.log; exit 1; }
  find /tmp/dn$d2 -name "*kernel_stats.csv" -exec cp {} gpurun_out/dense/kernel_stats_d2_$d2.csv \;
  grep -E "dense|head" gpurun_out/dense/kernel_stats_d2_$d2.csv | cut -d, -f1-4
done
