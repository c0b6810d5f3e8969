#!/bin/bash
# bench.py on one MI355X: K timed rounds after W warm-up rounds
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
K=${K:-3}; W=${W:-1}
timeout -k 10 ${TLIM:-900} python -u bench.py --gpus 1 --steps $K --warmup $W $EXTRA > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; tail -4 gpurun_out/bench.err; cat gpurun_out/bench.json; exit $rc
