#!/bin/bash
# Round 6: non-default architectures on the fast path vs the generic kernels (bench.py, short runs).
# usage (GPU box): bash tools/r6_generality.sh   -> gpurun_out/r6/gen_*.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export GENTUN_NO_AUTOBUILD=1
mkdir -p gpurun_out/r6
( while sleep 50; do date >> gpurun_out/heartbeat; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
run() {   # name, extra args
  local name=$1; shift
  timeout -k 10 ${TIME:-420} python3 -u bench.py --gpus 1 --steps ${STEPS:-4} --warmup ${WARMUP:-1} "$@" \
    > gpurun_out/r6/gen_$name.json 2> gpurun_out/r6/gen_$name.err || { tail -3 gpurun_out/r6/gen_$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[2], d['value'], d['config']['model'], d['config']['fast_path'])" gpurun_out/r6/gen_$name.json $name
}
for cfg in ${CFGS:-"k16_32:--kernels 16,32" "ks3:--kernel-size 3" "k32_64:--kernels 32,64" "mnist_bn:--input-shape 28,28,1 --batch-norm"}; do
  name=${cfg%%:*}; args=${cfg#*:}; args=${args//_/ }
  run ${name}_fast $args || exit 1
  run ${name}_generic $args --generic-kernels || exit 1
done
