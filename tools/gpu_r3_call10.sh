#!/bin/bash
# (1) same-box A/B of the S=(3,5) s2 input-conv dgrad with one co tile per wave (ab/s2in_ct1.so) vs the
#     packed-tile default: numerics test, per-launch time, population step;
# (2) wide deep space: PMC profile of its population step, then its bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
# the 20-generation search first: resume from profiles/ga20_ckpt (generations 19-20)
TAG=_part2 BUDGET=600 bash tools/gpu_ga20.sh > gpurun_out/ga20_part2.txt 2>&1 || { tail -5 gpurun_out/ga20_part2.txt; exit 1; }
tail -3 gpurun_out/ga20_part2.txt | cut -c1-400
mkdir -p gpurun_out/ct1; rm -f gpurun_out/ct1/*.log
GENTUN_HIP_LIB=gentun_amd/_native/ab/s2in_ct1.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_fp32.py -k "dgrad_fanout" > gpurun_out/ct1/tests.log 2>&1 || { tail -20 gpurun_out/ct1/tests.log; exit 1; }
tail -1 gpurun_out/ct1/tests.log
for round in 1 2; do
for lib in default ct1; do
  if [ $lib = ct1 ]; then export GENTUN_HIP_LIB=gentun_amd/_native/ab/s2in_ct1.so; else unset GENTUN_HIP_LIB; fi
  REGEPI=1 DUO=0 G=25 DBGS=0 ONLY=s2_in timeout -k 10 200 python3 -u tools/bench_conv.py 10 2>/dev/null | grep '"conv_dgrad"' | sed "s/^/$lib /" >> gpurun_out/ct1/conv.log || { echo conv failed; exit 1; }
  timeout -k 10 200 python3 -u tools/probe_pop.py 5 5 1 2 10000 2>/dev/null | grep '^{' | sed "s/^/$lib /" >> gpurun_out/ct1/pop.log || { echo pop failed; exit 1; }
done
done
unset GENTUN_HIP_LIB
cut -c1-200 gpurun_out/ct1/conv.log; cut -c1-160 gpurun_out/ct1/pop.log
SPACE=deep KERNELS=64,128,256 BN=1 DTYPE=fp32 P=3 OUT=prof_wide bash tools/gpu_prof_head.sh > gpurun_out/prof_wide.txt 2>&1 || { tail -20 gpurun_out/prof_wide.txt; exit 1; }
mkdir -p gpurun_out/wide
( while sleep 50; do date >> gpurun_out/wide/heartbeat; done ) & hb=$!
trap 'kill $hb' EXIT
timeout -k 10 720 python3 -u bench.py --gpus 1 --space deep --kernels 64,128,256 --batch-norm --per-gpu 2 --steps 2 --warmup 1 \
  --json-out gpurun_out/wide/bench.json > gpurun_out/wide/bench.out 2> gpurun_out/wide/bench.err || { tail -5 gpurun_out/wide/bench.err; exit 1; }
cat gpurun_out/wide/bench.json
# deep (20,50,100) + BN bench line at HEAD (round 2: 385.2)
timeout -k 10 400 python3 -u bench.py --gpus 1 --space deep --batch-norm --per-gpu 3 --steps 3 --warmup 1 \
  --json-out gpurun_out/wide/bench_deep.json > gpurun_out/wide/bench_deep.out 2> gpurun_out/wide/bench_deep.err || { tail -5 gpurun_out/wide/bench_deep.err; exit 1; }
cat gpurun_out/wide/bench_deep.json
