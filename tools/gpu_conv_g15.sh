#!/bin/bash
# conv phase breakdown at the bench launch size (G=15) and at G=80, fp32; then the torch-ops comparator
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
mkdir -p gpurun_out
: > gpurun_out/bench_conv_g15.log
for G in 15 80; do
  G=$G DBGS=0,1,2,4,7 F32P=0 timeout -k 10 300 python -u tools/bench_conv.py 10 >> gpurun_out/bench_conv_g15.log 2>&1 || exit $?
done
echo conv done
if [ -n "$TORCHCMP" ]; then
timeout -k 10 900 python -u bench.py --gpus 1 --backend torch --per-gpu 2 --steps 2 --warmup 0 \
  > gpurun_out/bench_torch.json 2> gpurun_out/bench_torch.err || { tail -20 gpurun_out/bench_torch.err; exit 1; }
cat gpurun_out/bench_torch.json
fi
