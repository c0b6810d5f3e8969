# driver-equivalent headline bench, then the wide deep space (64,128,256)+BN: 3 timed rounds + step PMC profile
set -o pipefail
STEPS=20 WARMUP=5 TAG=_r4a bash tools/gpu.sh headline || exit 1
mkdir -p gpurun_out/wide
timeout -k 10 900 python3 -u bench.py --gpus 1 --space deep --kernels 64,128,256 --batch-norm --steps 3 --warmup 1 \
  --json-out gpurun_out/wide/bench.json > gpurun_out/wide/bench.out 2> gpurun_out/wide/bench.err \
  || { tail -5 gpurun_out/wide/bench.err; exit 1; }
cut -c1-600 gpurun_out/wide/bench.json
SPACE=deep KERNELS=64,128,256 BN=1 P=3 OUT=profstep_wide bash tools/gpu.sh profstep
