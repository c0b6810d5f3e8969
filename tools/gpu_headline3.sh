#!/bin/bash
# driver-equivalent headline: python bench.py --gpus 1 --steps 20 --warmup 5 (defaults: population 32 total, balanced rounds, hard data)
export GENTUN_NO_AUTOBUILD=1
mkdir -p gpurun_out/headline3
( while sleep 50; do date >> gpurun_out/headline3/heartbeat; done ) & hb=$!
timeout -k 10 700 python3 -u bench.py --gpus 1 --steps ${STEPS:-20} --warmup ${WARMUP:-5} ${EXTRA:-} > gpurun_out/headline3/bench${TAG:-}.json 2> gpurun_out/headline3/bench${TAG:-}.err
rc=$?
kill $hb
tail -3 gpurun_out/headline3/bench${TAG:-}.err; cat gpurun_out/headline3/bench${TAG:-}.json
exit $rc
