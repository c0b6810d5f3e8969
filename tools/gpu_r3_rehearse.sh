#!/bin/bash
# 2-rank bench rehearsal on one GPU (gloo control plane, HIP compute): the torchrun path the driver's
# scaling run takes (RCCL there), at this round's bench defaults
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
( while sleep 50; do date >> gpurun_out/rehearse_hb; done ) & hb=$!
trap 'kill $hb' EXIT
GENTUN_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/rehearse2.json 2> gpurun_out/rehearse2.err || { tail -20 gpurun_out/rehearse2.err; exit 1; }
cut -c1-600 gpurun_out/rehearse2.json
