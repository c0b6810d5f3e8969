#!/bin/bash
# 20-generation RR-GA search, pop 32, fp32 full protocol, hard data, split over calls (checkpointed per generation)
export GENTUN_NO_AUTOBUILD=1
mkdir -p gpurun_out/ga20
if [ -d profiles/ga20_ckpt ] && [ ! -d gpurun_out/ga20/ckpt ]; then cp -r profiles/ga20_ckpt gpurun_out/ga20/ckpt; fi
( while sleep 50; do date >> gpurun_out/ga20/heartbeat; done ) & hb=$!
timeout -k 10 1080 python3 -u tools/ga_run.py --gens 20 --ckpt gpurun_out/ga20/ckpt --resume --time-budget ${BUDGET:-900} > gpurun_out/ga20/run${TAG:-}.json 2> gpurun_out/ga20/run${TAG:-}.err
rc=$?
kill $hb
grep "\[ga_run\]" gpurun_out/ga20/run${TAG:-}.err | tail -25; cat gpurun_out/ga20/run${TAG:-}.json
exit $rc
