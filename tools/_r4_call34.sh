# native step program (GENTUN_GRAPH=0, GENTUN_NATIVE_STEPS=1) vs captured graph vs Python eager: tests, population step, bench.py
set -o pipefail
( while true; do sleep 50; echo hb > gpurun_out/heartbeat; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_hip_train.py -k "native_step or graph_equals or adam_overlap" \
  > gpurun_out/r4c34_test.log 2>&1 || { tail -30 gpurun_out/r4c34_test.log; exit 1; }
grep -E "passed|failed" gpurun_out/r4c34_test.log | tail -2
for v in "all 5 1 1 8" "all 5 0 1 8" "all 5 0 0 8" "kernels 2 1 1 4" "kernels 2 0 1 4" "all 2 1 1 8" "all 2 0 1 8"; do
  set -- $v
  GENTUN_GRAPH=$3 GENTUN_NATIVE_STEPS=$4 DTYPE=fp32 RESET=$1 timeout -k 10 200 python -u tools/probe_pop.py $2 $2 1 $5 \
    > gpurun_out/r4c34_run.log 2>&1 || { tail -5 gpurun_out/r4c34_run.log; exit 1; }
  echo "RESET=$1 P=$2 graph=$3 native=$4 epochs=$5 $(grep -o '"enqueue_s": [0-9.]*, "ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c34_run.log)"
done
for g in 1 0 1 0; do
  GENTUN_GRAPH=$g timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 8 --warmup 2 > gpurun_out/r4c34_g$g.json 2> gpurun_out/r4c34_g$g.err \
    || { tail -5 gpurun_out/r4c34_g$g.err; exit 1; }
  echo "bench graph=$g native=1 $(grep -o '"value": [0-9.]*, "unit": "[a-z/]*", "n_gpus": 1, "steps": 8, "warmup": 2, "ms_per_step": [0-9.]*' gpurun_out/r4c34_g$g.json)"
done
