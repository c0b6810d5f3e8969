# config-3 share on one GPU (about 2 candidates per rank per generation: 10 groups concurrent folds, 2 reference
( while sleep 50; do date >> gpurun_out/heartbeat; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
# folds), then the Q-curve republished at this tree
set -o pipefail
mkdir -p gpurun_out/c3share
timeout -k 10 400 python3 -u bench.py --gpus 1 --per-gpu 2 --steps 4 --warmup 1 \
  > gpurun_out/c3share/all.json 2> gpurun_out/c3share/all.err || { tail -5 gpurun_out/c3share/all.err; exit 1; }
cut -c1-400 gpurun_out/c3share/all.json
timeout -k 10 500 python3 -u bench.py --gpus 1 --per-gpu 2 --steps 3 --warmup 1 --fold-reset kernels \
  > gpurun_out/c3share/kernels.json 2> gpurun_out/c3share/kernels.err || { tail -5 gpurun_out/c3share/kernels.err; exit 1; }
cut -c1-400 gpurun_out/c3share/kernels.json
bash tools/gpu.sh qcurve
