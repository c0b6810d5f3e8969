#!/bin/bash
# bench.py rounds of ~5 candidates (the driver's per-step size): one job (pop_batch 16) vs two concurrent
# jobs on the evaluator's 2 streams (pop_batch 3), same seed / same candidates; STEPS timed after WARMUP.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export GENTUN_NO_AUTOBUILD=1
out=gpurun_out/r5/popbatch; mkdir -p $out
( while sleep 50; do date >> $out/heartbeat; done ) & HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for r in $(seq ${REPS:-1}); do
  for pb in ${PBS:-16 3}; do
    timeout -k 10 400 python3 -u bench.py --steps ${STEPS:-4} --warmup ${WARMUP:-1} --pop-batch $pb \
      > $out/pb${pb}_$r.json 2> $out/pb${pb}_$r.err || { tail -5 $out/pb${pb}_$r.err; exit 1; }
    echo "pop_batch $pb: $(python3 -c "import json,sys; d=json.load(open('$out/pb${pb}_$r.json')); print(d['value'], d['ms_per_step'])")" | tee -a $out/summary.txt
  done
done
