#!/bin/bash
# round 3 secondary lines: reference fold semantics (--fold-reset kernels, whole-generation rounds)
# and the population-batched stock-PyTorch comparator (TorchPopJob), each with warm-up rounds
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
mkdir -p gpurun_out/sec3
( while sleep 50; do date >> gpurun_out/sec3/heartbeat; done ) & hb=$!
trap 'kill $hb' EXIT
if [ -z "${SKIP_KERNELS:-}" ]; then
timeout -k 10 ${KTIME:-560} python3 -u bench.py --gpus 1 --fold-reset kernels --steps ${KSTEPS:-3} --warmup 1 \
  --json-out gpurun_out/sec3/kernels.json > gpurun_out/sec3/kernels.out 2> gpurun_out/sec3/kernels.err || { tail -5 gpurun_out/sec3/kernels.err; exit 1; }
cat gpurun_out/sec3/kernels.json
fi
if [ -z "${SKIP_TORCH:-}" ]; then
timeout -k 10 ${TTIME:-560} python3 -u bench.py --gpus 1 --backend torch --steps ${TSTEPS:-2} --warmup 1 \
  --json-out gpurun_out/sec3/torch.json > gpurun_out/sec3/torch.out 2> gpurun_out/sec3/torch.err || { tail -5 gpurun_out/sec3/torch.err; exit 1; }
cat gpurun_out/sec3/torch.json
fi
