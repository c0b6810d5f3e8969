#!/bin/bash
# Round-6 final benches on one GPU, each under its own limit:
#   bash tools/r6_bench.sh headline   driver-equivalent headline (20 timed rounds after 5 warm-up) + deep (20,50,100)+BN
#   bash tools/r6_bench.sh wide       wide (64,128,256)+BN, 3 timed rounds after 1 warm-up
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export GENTUN_NO_AUTOBUILD=1
out=gpurun_out/r6bench; mkdir -p $out
( while sleep 50; do date >> $out/heartbeat; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
case "${1:-}" in
headline)
  timeout -k 10 620 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $out/headline.json 2> $out/headline.err \
    || { tail -5 $out/headline.err; exit 1; }
  cut -c1-300 $out/headline.json
  timeout -k 10 400 python3 -u bench.py --gpus 1 --space deep --batch-norm --steps 3 --warmup 1 \
    > $out/deep.json 2> $out/deep.err || { tail -5 $out/deep.err; exit 1; }
  cut -c1-200 $out/deep.json ;;
wide)
  timeout -k 10 900 python3 -u bench.py --gpus 1 --space deep --kernels 64,128,256 --batch-norm --per-gpu 3 --steps 3 \
    --warmup 1 > $out/wide.json 2> $out/wide.err || { tail -5 $out/wide.err; exit 1; }
  cut -c1-200 $out/wide.json ;;
*) sed -n 2,4p "$0"; exit 2 ;;
esac
