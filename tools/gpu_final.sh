#!/bin/bash
# end-of-round check: full GPU suite, smoke, 2-rank bench rehearsal on the one GPU (gloo control plane)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/ \
  > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log | cut -c1-200
GENTUN_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --per-gpu 2 --steps 1 --warmup 0 > gpurun_out/rehearse2.json 2> gpurun_out/rehearse2.err || { tail -20 gpurun_out/rehearse2.err; exit 1; }
cut -c1-400 gpurun_out/rehearse2.json
