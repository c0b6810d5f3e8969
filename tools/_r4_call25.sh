# deep S=(3,4,5) (20,50,100) + BN bench at this tree (3 timed rounds)
set -o pipefail
( while sleep 50; do date >> gpurun_out/heartbeat; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
mkdir -p gpurun_out/deep
timeout -k 10 900 python3 -u bench.py --gpus 1 --space deep --batch-norm --steps 3 --warmup 1 \
  --json-out gpurun_out/deep/bench.json > gpurun_out/deep/bench.out 2> gpurun_out/deep/bench.err \
  || { tail -5 gpurun_out/deep/bench.err; exit 1; }
cut -c1-500 gpurun_out/deep/bench.json
