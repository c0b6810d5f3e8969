# bench.py same-box A/B: captured step graph (GENTUN_GRAPH=1) vs eager launches (0)
set -o pipefail
( while true; do sleep 50; echo hb > gpurun_out/heartbeat; done ) & HB=$!
trap "kill $HB" EXIT
for g in 1 0 1 0; do
  GENTUN_GRAPH=$g timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 8 --warmup 2 > gpurun_out/r4c33_g$g.json 2> gpurun_out/r4c33_g$g.err \
    || { tail -5 gpurun_out/r4c33_g$g.err; exit 1; }
  echo "graph=$g $(grep -o '"value": [0-9.]*, "unit": "[a-z/]*", "n_gpus": 1, "steps": 8, "warmup": 2, "ms_per_step": [0-9.]*' gpurun_out/r4c33_g$g.json)"
done
