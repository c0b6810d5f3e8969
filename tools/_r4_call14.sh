# wide deep space (64,128,256)+BN: 3 timed rounds + step PMC profile (heartbeat: the first round is silent for minutes)
set -o pipefail
( while sleep 50; do date >> gpurun_out/heartbeat; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
mkdir -p gpurun_out/wide
timeout -k 10 1000 python3 -u bench.py --gpus 1 --space deep --kernels 64,128,256 --batch-norm --per-gpu 3 --steps 3 --warmup 1 \
  --json-out gpurun_out/wide/bench.json > gpurun_out/wide/bench.out 2> gpurun_out/wide/bench.err \
  || { tail -5 gpurun_out/wide/bench.err; exit 1; }
cut -c1-600 gpurun_out/wide/bench.json
SPACE=deep KERNELS=64,128,256 BN=1 P=3 OUT=profstep_wide bash tools/gpu.sh profstep
