#!/bin/bash
# Round-4 GPU experiments (A/B runs, searches), one function per gpurun call; every
# profiles/*_r4* file names the experiment that produced it: bash tools/r4_experiments.sh NAME
#   NAME: call4 call5 call6 call7 call8 call9 call10 call11 call12 call13 call14 call15 call16 call17 call18 call19 call20 call21 call22 call23 call24 call25 call26 call27 call28 call29 call30 call31 call32 call33 call34 dense ga_deep call35 call36 call37 call38 call39 call40 call41 call42
# Run from the repository root on the GPU box (tools/gpu.sh has the shared tasks).
set -o pipefail

exp_call4() {
  export GENTUN_NO_AUTOBUILD=1
  mkdir -p gpurun_out/r4c4
  timeout -k 10 300 python -u -m pytest -s -q --timeout 200 --timeout-method thread tests/test_hip_fp32.py -k s2in tests/test_hip_dp.py > gpurun_out/r4c4/tests.log 2>&1 || { tail -30 gpurun_out/r4c4/tests.log; exit 1; }
  grep -E "\[fp32\]|\[dp\]|passed|failed" gpurun_out/r4c4/tests.log
  for i in 1 2; do for ct in 0 1; do
    GENTUN_S2IN_CT1=$ct timeout -k 10 200 python tools/probe_pop.py 5 5 1 1 10000 > gpurun_out/r4c4/pop_ct$ct.log 2>&1 || { tail -5 gpurun_out/r4c4/pop_ct$ct.log; exit 1; }
    echo "ct1=$ct $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r4c4/pop_ct$ct.log)"
  done; done
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  rm -rf /tmp/pmcclk
  G=25 DBGS=0 ONLY=s2_n timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES -d /tmp/pmcclk -o run --output-format csv -- python3 tools/bench_conv.py 5 > gpurun_out/r4c4/pmcclk.log 2>&1 || { tail -5 gpurun_out/r4c4/pmcclk.log; exit 1; }
  python3 tools/pmc_summary.py /tmp/pmcclk > gpurun_out/r4c4/pmcclk.txt 2>&1; head -20 gpurun_out/r4c4/pmcclk.txt
  find /tmp/pmcclk -name "*counter_collection.csv" -exec cp {} gpurun_out/r4c4/counters.csv \;
}

exp_call5() {
  # adam band tests + inactive-node test, then Q=2 (reference folds) and Q=10 timelines
  timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_hip_kernels.py -k adam_segments tests/test_hip_train.py > gpurun_out/r4c5_tests.log 2>&1 \
    || { tail -30 gpurun_out/r4c5_tests.log; exit 1; }
  tail -2 gpurun_out/r4c5_tests.log
  RESET=kernels P=2 SAMPLES=10000 TAG=_k2 DUMP=2 bash tools/gpu.sh timeline > /dev/null && head -24 gpurun_out/timeline/summary_k2.txt
  RESET=all P=2 SAMPLES=10000 TAG=_a2 DUMP=1 bash tools/gpu.sh timeline > /dev/null && head -24 gpurun_out/timeline/summary_a2.txt
}

exp_call6() {
  # small-launch tiles + wgrad streams: tests, then A/B on the probe (Q=2 reference folds, Q=10, Q=25)
  timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
    tests/test_hip_train.py tests/test_hip_kernels.py tests/test_hip_fp32.py > gpurun_out/r4c6_tests.log 2>&1 \
    || { tail -30 gpurun_out/r4c6_tests.log; exit 1; }
  tail -1 gpurun_out/r4c6_tests.log
  for spec in "kernels 2" "all 2" "all 5"; do
    set -- $spec
    for v in "1 2" "0 1" "1 1" "1 3"; do
      set -- $spec $v
      GENTUN_CONV_SMALLQ=$3 GENTUN_WGRAD_STREAMS=$4 DTYPE=fp32 RESET=$1 timeout -k 10 200 python -u tools/probe_pop.py $2 $2 1 1 \
        > gpurun_out/r4c6_run.log 2>&1 || { tail -5 gpurun_out/r4c6_run.log; exit 1; }
      echo "RESET=$1 P=$2 smallq=$3 wstreams=$4 $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c6_run.log)"
    done
  done
}

exp_call7() {
  # fold-job reuse: tests, then A/B on the reference-fold probe and a fresh Q=2 timeline
  timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
    tests/test_hip_train.py tests/test_hip_dp.py tests/test_hip_step_parity.py > gpurun_out/r4c7_tests.log 2>&1 \
    || { tail -30 gpurun_out/r4c7_tests.log; exit 1; }
  tail -1 gpurun_out/r4c7_tests.log
  for v in 1 0 1 0; do
    GENTUN_FOLD_REUSE=$v DTYPE=fp32 RESET=kernels timeout -k 10 200 python -u tools/probe_pop.py 2 2 1 1 \
      > gpurun_out/r4c7_run.log 2>&1 || { tail -5 gpurun_out/r4c7_run.log; exit 1; }
    echo "RESET=kernels P=2 reuse=$v $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c7_run.log)"
  done
  RESET=kernels P=2 SAMPLES=10000 TAG=_k2b DUMP=2 bash tools/gpu.sh timeline > /dev/null && head -4 gpurun_out/timeline/summary_k2b.txt
}

exp_call8() {
  # split-K dense forward from the W1 master: tests, then A/B (GENTUN_DENSE_SK) on the probe
  timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
    tests/test_hip_dense_stream.py tests/test_hip_train.py tests/test_hip_dp.py tests/test_hip_step_parity.py \
    > gpurun_out/r4c8_tests.log 2>&1 || { tail -30 gpurun_out/r4c8_tests.log; exit 1; }
  tail -1 gpurun_out/r4c8_tests.log
  for spec in "kernels 2" "all 5" "all 2"; do
    set -- $spec
    for v in 1 0 1 0; do
      GENTUN_DENSE_SK=$v DTYPE=fp32 RESET=$1 timeout -k 10 200 python -u tools/probe_pop.py $2 $2 1 1 \
        > gpurun_out/r4c8_run.log 2>&1 || { tail -5 gpurun_out/r4c8_run.log; exit 1; }
      echo "RESET=$1 P=$2 dense_sk=$v $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c8_run.log)"
    done
  done
  P=5 TAG=_p5sk DUMP=1 bash tools/gpu.sh timeline > /dev/null && head -22 gpurun_out/timeline/summary_p5sk.txt
  for wg in 512 2000 100000 512; do
    GENTUN_CONV_SMALLQ_WG=$wg DTYPE=fp32 RESET=all timeout -k 10 200 python -u tools/probe_pop.py 5 5 1 1 \
      > gpurun_out/r4c8_run.log 2>&1 || { tail -5 gpurun_out/r4c8_run.log; exit 1; }
    echo "RESET=all P=5 smallq_wg=$wg $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c8_run.log)"
  done
}

exp_call9() {
  # wgrad geometry A/B at bench-sized launches (25 / 30 groups): stage-2 splits and column slices
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_hip_fp32.py tests/test_hip_kernels.py > gpurun_out/r4c9_tests.log 2>&1 || { tail -30 gpurun_out/r4c9_tests.log; exit 1; }
  tail -1 gpurun_out/r4c9_tests.log
  for P in 5 6; do
    for v in "8 0" "10 0" "16 0" "8 2" "12 0" "8 0"; do
      set -- $v
      GENTUN_F32_SPLITS16=$1 GENTUN_WGRAD_NZ=$2 DTYPE=fp32 RESET=all timeout -k 10 200 python -u tools/probe_pop.py $P $P 1 1 \
        > gpurun_out/r4c9_run.log 2>&1 || { tail -5 gpurun_out/r4c9_run.log; exit 1; }
      echo "P=$P splits16=$1 nz=$2 $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c9_run.log)"
    done
  done
  for v in "6 6 1" "6 3 2" "10 5 2" "10 10 1"; do
    set -- $v
    DTYPE=fp32 RESET=all timeout -k 10 200 python -u tools/probe_pop.py $1 $2 $3 1 \
      > gpurun_out/r4c9_run.log 2>&1 || { tail -5 gpurun_out/r4c9_run.log; exit 1; }
    echo "P=$1 pop_batch=$2 streams=$3 $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c9_run.log)"
  done
  # conv tile threshold at small / mid launches: Q=5 (P=1), Q=10 (P=2)
  for P in 1 2; do
    for wg in 300 512 1000 2000 512; do
      GENTUN_CONV_SMALLQ_WG=$wg DTYPE=fp32 RESET=all timeout -k 10 200 python -u tools/probe_pop.py $P $P 1 1 \
        > gpurun_out/r4c9_run.log 2>&1 || { tail -5 gpurun_out/r4c9_run.log; exit 1; }
      echo "P=$P smallq_wg=$wg $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c9_run.log)"
    done
  done
}

exp_call10() {
  # config-3 share on one GPU (about 2 candidates per rank per generation: 10 groups concurrent folds, 2 reference
  ( while sleep 50; do date >> gpurun_out/heartbeat; done ) & HB=$!
  trap 'kill $HB 2>/dev/null' EXIT
  # folds), then the Q-curve republished at this tree
  mkdir -p gpurun_out/c3share
  timeout -k 10 400 python3 -u bench.py --gpus 1 --per-gpu 2 --steps 4 --warmup 1 \
    > gpurun_out/c3share/all.json 2> gpurun_out/c3share/all.err || { tail -5 gpurun_out/c3share/all.err; exit 1; }
  cut -c1-400 gpurun_out/c3share/all.json
  timeout -k 10 500 python3 -u bench.py --gpus 1 --per-gpu 2 --steps 3 --warmup 1 --fold-reset kernels \
    > gpurun_out/c3share/kernels.json 2> gpurun_out/c3share/kernels.err || { tail -5 gpurun_out/c3share/kernels.err; exit 1; }
  cut -c1-400 gpurun_out/c3share/kernels.json
  bash tools/gpu.sh qcurve
}

exp_call11() {
  # step PMC profile at the bench round size (25 groups), and the separate-vs-fused wgrad split reduction A/B
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_hip_kernels.py tests/test_hip_train.py tests/test_hip_dense_stream.py > gpurun_out/r4c11_tests.log 2>&1 \
    || { tail -30 gpurun_out/r4c11_tests.log; exit 1; }
  tail -1 gpurun_out/r4c11_tests.log
  P=5 OUT=profstep_p5 bash tools/gpu.sh profstep || exit 1
  for spec in "kernels 2" "all 5" "all 2"; do
    set -- $spec
    for v in 1 0 1 0; do
      GENTUN_WGRAD_REDUCE=$v DTYPE=fp32 RESET=$1 timeout -k 10 200 python -u tools/probe_pop.py $2 $2 1 1 \
        > gpurun_out/r4c11_run.log 2>&1 || { tail -5 gpurun_out/r4c11_run.log; exit 1; }
      echo "RESET=$1 P=$2 wgrad_reduce=$v $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c11_run.log)"
    done
  done
}

exp_call12() {
  # wgrad half-split staging (GT_WGRAD_HALVES): tests, then same-box A/B vs a build without it
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_hip_fp32.py tests/test_hip_train.py tests/test_hip_dp.py > gpurun_out/r4c12_tests.log 2>&1 \
    || { tail -30 gpurun_out/r4c12_tests.log; exit 1; }
  tail -1 gpurun_out/r4c12_tests.log
  for i in 1 2 3; do
    for lib in "" ab_libs/nohalves.so; do
      GENTUN_HIP_LIB=$lib DTYPE=fp32 RESET=all timeout -k 10 200 python -u tools/probe_pop.py 5 5 1 1 \
        > gpurun_out/r4c12_run.log 2>&1 || { tail -5 gpurun_out/r4c12_run.log; exit 1; }
      echo "P=5 lib=${lib:-tree} $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c12_run.log)"
    done
  done
  for lib in "" ab_libs/nohalves.so; do
    GENTUN_HIP_LIB=$lib G=25 DBGS=0 ONLY=s2 timeout -k 10 200 python -u tools/bench_conv.py 10 2>&1 | grep conv_wgrad | cut -c1-220
  done
}

exp_call13() {
  # driver-equivalent headline bench, then the wide deep space (64,128,256)+BN: 3 timed rounds + step PMC profile
  STEPS=20 WARMUP=5 TAG=_r4a bash tools/gpu.sh headline || exit 1
  mkdir -p gpurun_out/wide
  timeout -k 10 900 python3 -u bench.py --gpus 1 --space deep --kernels 64,128,256 --batch-norm --steps 3 --warmup 1 \
    --json-out gpurun_out/wide/bench.json > gpurun_out/wide/bench.out 2> gpurun_out/wide/bench.err \
    || { tail -5 gpurun_out/wide/bench.err; exit 1; }
  cut -c1-600 gpurun_out/wide/bench.json
  SPACE=deep KERNELS=64,128,256 BN=1 P=3 OUT=profstep_wide bash tools/gpu.sh profstep
}

exp_call14() {
  # wide deep space (64,128,256)+BN: 3 timed rounds + step PMC profile (heartbeat: the first round is silent for minutes)
  ( while sleep 50; do date >> gpurun_out/heartbeat; done ) & HB=$!
  trap 'kill $HB 2>/dev/null' EXIT
  mkdir -p gpurun_out/wide
  timeout -k 10 1000 python3 -u bench.py --gpus 1 --space deep --kernels 64,128,256 --batch-norm --per-gpu 3 --steps 3 --warmup 1 \
    --json-out gpurun_out/wide/bench.json > gpurun_out/wide/bench.out 2> gpurun_out/wide/bench.err \
    || { tail -5 gpurun_out/wide/bench.err; exit 1; }
  cut -c1-600 gpurun_out/wide/bench.json
  SPACE=deep KERNELS=64,128,256 BN=1 P=3 OUT=profstep_wide bash tools/gpu.sh profstep
}

exp_call15() {
  # diagnostic: conv fwd / dgrad with L1-resident weights (dbg 8) vs normal, and MFMA-only (dbg 6), 25 groups
  G=25 DBGS=0,8,6,14 ONLY=s2_n timeout -k 10 200 python -u tools/bench_conv.py 10 > gpurun_out/r4c15.log 2>&1 || { tail -5 gpurun_out/r4c15.log; exit 1; }
  grep -v wgrad gpurun_out/r4c15.log | python3 -c "
  import sys, json
  for l in sys.stdin:
      if l.startswith('{'):
          d = json.loads(l); print(d['kernel'], d['shape'], 'dbg', d['dbg'], d['us'])"
}

exp_call16() {
  # register-held k-step offsets (GT_F32_KREG): fp32 tests, conv microbench and population step vs a build without
  timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_hip_fp32.py \
    > gpurun_out/r4c16_tests.log 2>&1 || { tail -30 gpurun_out/r4c16_tests.log; exit 1; }
  tail -1 gpurun_out/r4c16_tests.log
  for lib in "" ab_libs/nokreg.so; do
    GENTUN_HIP_LIB=$lib G=25 DBGS=0 timeout -k 10 200 python -u tools/bench_conv.py 10 > gpurun_out/r4c16_conv.log 2>&1 || { tail -5 gpurun_out/r4c16_conv.log; exit 1; }
    python3 -c "
  import sys, json
  for l in open('gpurun_out/r4c16_conv.log'):
      if l.startswith('{'):
          d = json.loads(l); print('${lib:-tree}', d['kernel'], d['shape'], d['us'])"
  done
  for i in 1 2; do
    for lib in "" ab_libs/nokreg.so; do
      GENTUN_HIP_LIB=$lib DTYPE=fp32 RESET=all timeout -k 10 200 python -u tools/probe_pop.py 5 5 1 1 \
        > gpurun_out/r4c16_run.log 2>&1 || { tail -5 gpurun_out/r4c16_run.log; exit 1; }
      echo "P=5 lib=${lib:-tree} $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c16_run.log)"
    done
  done
}

exp_call17() {
  # pairwise multi-input patch staging (GT_STAGE_PAIRS): tests, conv microbench, population step vs a build without
  timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_hip_fp32.py tests/test_hip_train.py tests/test_hip_kernels.py \
    > gpurun_out/r4c17_tests.log 2>&1 || { tail -30 gpurun_out/r4c17_tests.log; exit 1; }
  tail -1 gpurun_out/r4c17_tests.log
  for lib in "" ab_libs/nopairs.so; do
    GENTUN_HIP_LIB=$lib G=25 DBGS=0 timeout -k 10 200 python -u tools/bench_conv.py 10 > gpurun_out/r4c17_conv.log 2>&1 || { tail -5 gpurun_out/r4c17_conv.log; exit 1; }
    python3 -c "
  import sys, json
  for l in open('gpurun_out/r4c17_conv.log'):
      if l.startswith('{'):
          d = json.loads(l); print('${lib:-tree}', d['kernel'], d['shape'], d['us'])"
  done
  for i in 1 2; do
    for lib in "" ab_libs/nopairs.so; do
      GENTUN_HIP_LIB=$lib DTYPE=fp32 RESET=all timeout -k 10 200 python -u tools/probe_pop.py 5 5 1 1 \
        > gpurun_out/r4c17_run.log 2>&1 || { tail -5 gpurun_out/r4c17_run.log; exit 1; }
      echo "P=5 lib=${lib:-tree} $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c17_run.log)"
    done
  done
}

exp_call18() {
  # GBDT constant-hessian count histograms: GPU tests, hist A/B under rocprof, and the tournament-GA bench (r3 settings)
  ( while sleep 50; do date >> gpurun_out/heartbeat; done ) & HB=$!
  trap 'kill $HB 2>/dev/null' EXIT
  timeout -k 10 400 python -u -m pytest tests/test_gbdt_gpu.py -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/r4c18_tests.log 2>&1 || { tail -30 gpurun_out/r4c18_tests.log; exit 1; }
  tail -1 gpurun_out/r4c18_tests.log
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  for hc in 1 0; do
    rm -rf /tmp/pg$hc; mkdir -p gpurun_out/gbdt_hc$hc
    GENTUN_GBDT_HCONST=$hc GENTUN_GBDT_TIMING=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pg$hc -o run --output-format csv -- \
      python3 tools/probe_gbdt.py 1000000 256 10 5 > gpurun_out/gbdt_hc$hc/run.log 2>&1 || { tail -5 gpurun_out/gbdt_hc$hc/run.log; exit 1; }
    find /tmp/pg$hc -name "*kernel_stats.csv" -exec cp {} gpurun_out/gbdt_hc$hc/ \;
    echo "hconst=$hc"; grep "{\|gbdt_hip" gpurun_out/gbdt_hc$hc/run.log | tail -2 | cut -c1-300
    head -4 gpurun_out/gbdt_hc$hc/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
  done
  timeout -k 10 700 python -u tools/bench_gbdt.py --pop 10 --gens 3 > gpurun_out/bench_gbdt_r4.log 2>&1 || { tail -10 gpurun_out/bench_gbdt_r4.log; exit 1; }
  grep "{" gpurun_out/bench_gbdt_r4.log | cut -c1-400
}

exp_call19() {
  # A/B: main-stream priority (the data-gradient chain) and per-layer conv Adam on a third stream, 25 groups
  for v in "0 0 0" "-1 0 0" "0 0 1" "-1 0 0" "0 0 0"; do
    set -- $v
    MAIN_PRIO=$1 GENTUN_SIDE_PRIO=$2 GENTUN_ADAM_OVERLAP=$3 DTYPE=fp32 RESET=all timeout -k 10 200 python -u tools/probe_pop.py 5 5 1 1 \
      > gpurun_out/r4c19_run.log 2>&1 || { tail -5 gpurun_out/r4c19_run.log; exit 1; }
    echo "main_prio=$1 side_prio=$2 adam_overlap=$3 $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c19_run.log)"
  done
}

exp_call20() {
  # two-part staging of the stage-2 3x3 conv: tests, microbench and step A/B (tree / split off / kk-major build)
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_hip_fp32.py \
    tests/test_hip_train.py tests/test_hip_duo.py > gpurun_out/r4c20_tests.log 2>&1 || { tail -30 gpurun_out/r4c20_tests.log; exit 1; }
  tail -1 gpurun_out/r4c20_tests.log
  for v in "tree 1" "tree 0" "ab_libs/noparts.so 1"; do
    set -- $v
    lib=$1; [ "$lib" = tree ] && lib=""
    GENTUN_HIP_LIB=$lib GENTUN_S2_SPLIT=$2 G=25 DBGS=0 ONLY=s2_n timeout -k 10 200 python -u tools/bench_conv.py 10 > gpurun_out/r4c20_conv.log 2>&1 || { tail -5 gpurun_out/r4c20_conv.log; exit 1; }
    python3 -c "
  import json
  for l in open('gpurun_out/r4c20_conv.log'):
      if l.startswith('{'):
          d = json.loads(l); print('$1 split=$2', d['kernel'], d['shape'], d['us'])"
  done
  for i in 1 2; do
    for v in "tree 1" "tree 0" "ab_libs/noparts.so 1"; do
      set -- $v
      lib=$1; [ "$lib" = tree ] && lib=""
      GENTUN_HIP_LIB=$lib GENTUN_S2_SPLIT=$2 DTYPE=fp32 RESET=all timeout -k 10 200 python -u tools/probe_pop.py 5 5 1 1 \
        > gpurun_out/r4c20_run.log 2>&1 || { tail -5 gpurun_out/r4c20_run.log; exit 1; }
      echo "P=5 $1 split=$2 $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c20_run.log)"
    done
  done
}

exp_call21() {
  # bank-paired reduction order of the stage-2 3x3 conv: tests, microbench + step A/B vs the kk-major build
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_hip_fp32.py \
    tests/test_hip_train.py tests/test_hip_duo.py > gpurun_out/r4c21_tests.log 2>&1 || { tail -30 gpurun_out/r4c21_tests.log; exit 1; }
  tail -1 gpurun_out/r4c21_tests.log
  for lib in "" ab_libs/kkmajor.so; do
    GENTUN_HIP_LIB=$lib G=25 DBGS=0 ONLY=s2_n timeout -k 10 200 python -u tools/bench_conv.py 10 > gpurun_out/r4c21_conv.log 2>&1 || { tail -5 gpurun_out/r4c21_conv.log; exit 1; }
    python3 -c "
  import json
  for l in open('gpurun_out/r4c21_conv.log'):
      if l.startswith('{'):
          d = json.loads(l); print('${lib:-tree}', d['kernel'], d['shape'], d['us'])"
  done
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  for lib in "" ab_libs/kkmajor.so; do
    rm -rf /tmp/pmcb; GENTUN_HIP_LIB=$lib G=25 DBGS=0 ONLY=s2_n timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d /tmp/pmcb -o run --output-format csv -- python3 tools/bench_conv.py 3 > gpurun_out/r4c21_pmc.log 2>&1 || { tail -5 gpurun_out/r4c21_pmc.log; exit 1; }
    echo "lib=${lib:-tree}"; python3 tools/pmc_summary.py /tmp/pmcb | grep conv_fast | cut -c1-300
  done
  cd "$GRAFT_REPO_ROOT"
  for i in 1 2; do
    for lib in "" ab_libs/kkmajor.so; do
      GENTUN_HIP_LIB=$lib DTYPE=fp32 RESET=all timeout -k 10 200 python -u tools/probe_pop.py 5 5 1 1 \
        > gpurun_out/r4c21_run.log 2>&1 || { tail -5 gpurun_out/r4c21_run.log; exit 1; }
      echo "P=5 ${lib:-tree} $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c21_run.log)"
    done
  done
}

exp_call22() {
  # part-major order for the 5x5 s2 input-conv dgrad too (GT_S2_PARTS=2 build) vs the tree (3x3 only)
  GENTUN_HIP_LIB=ab_libs/parts2.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_hip_fp32.py tests/test_hip_train.py > gpurun_out/r4c22_tests.log 2>&1 || { tail -30 gpurun_out/r4c22_tests.log; exit 1; }
  tail -1 gpurun_out/r4c22_tests.log
  for lib in "" ab_libs/parts2.so; do
    GENTUN_HIP_LIB=$lib G=25 DBGS=0 ONLY=s2_in timeout -k 10 200 python -u tools/bench_conv.py 10 > gpurun_out/r4c22_conv.log 2>&1 || { tail -5 gpurun_out/r4c22_conv.log; exit 1; }
    python3 -c "
  import json
  for l in open('gpurun_out/r4c22_conv.log'):
      if l.startswith('{'):
          d = json.loads(l); print('${lib:-tree}', d['kernel'], d['shape'], d['us'])"
  done
  for i in 1 2; do
    for lib in "" ab_libs/parts2.so; do
      GENTUN_HIP_LIB=$lib DTYPE=fp32 RESET=all timeout -k 10 200 python -u tools/probe_pop.py 5 5 1 1 \
        > gpurun_out/r4c22_run.log 2>&1 || { tail -5 gpurun_out/r4c22_run.log; exit 1; }
      echo "P=5 ${lib:-tree} $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c22_run.log)"
    done
  done
}

exp_call23() {
  RESET=kernels P=2 SAMPLES=10000 TAG=_k2c DUMP=2 bash tools/gpu.sh timeline > /dev/null && head -4 gpurun_out/timeline/summary_k2c.txt
  P=5 TAG=_p5c DUMP=1 bash tools/gpu.sh timeline > /dev/null && head -4 gpurun_out/timeline/summary_p5c.txt
}

exp_call24() {
  # 8-slice 4-wave wgrad for tiny launches + head_fwd label-chain hoist: tests, then A/B at small launches
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_hip_duo.py \
    tests/test_hip_kernels.py tests/test_hip_train.py > gpurun_out/r4c24_tests.log 2>&1 || { tail -30 gpurun_out/r4c24_tests.log; exit 1; }
  tail -1 gpurun_out/r4c24_tests.log
  for spec in "kernels 2" "all 1" "all 5"; do
    set -- $spec
    for v in 32 0 32 0; do
      GENTUN_WGRAD_NZ8=$v DTYPE=fp32 RESET=$1 timeout -k 10 200 python -u tools/probe_pop.py $2 $2 1 1 \
        > gpurun_out/r4c24_run.log 2>&1 || { tail -5 gpurun_out/r4c24_run.log; exit 1; }
      echo "RESET=$1 P=$2 nz8_below=$v $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c24_run.log)"
    done
  done
}

exp_call25() {
  # deep S=(3,4,5) (20,50,100) + BN bench at this tree (3 timed rounds)
  ( while sleep 50; do date >> gpurun_out/heartbeat; done ) & HB=$!
  trap 'kill $HB 2>/dev/null' EXIT
  mkdir -p gpurun_out/deep
  timeout -k 10 900 python3 -u bench.py --gpus 1 --space deep --batch-norm --steps 3 --warmup 1 \
    --json-out gpurun_out/deep/bench.json > gpurun_out/deep/bench.out 2> gpurun_out/deep/bench.err \
    || { tail -5 gpurun_out/deep/bench.err; exit 1; }
  cut -c1-500 gpurun_out/deep/bench.json
}

exp_call26() {
  # wgrad band buffers at the bench size: single buffer (57 KB LDS: co-resides with a conv workgroup) vs double (115 KB)
  for v in 0 1 0 1; do
    GENTUN_WGRAD_NB=$v DTYPE=fp32 RESET=all timeout -k 10 200 python -u tools/probe_pop.py 5 5 1 1 \
      > gpurun_out/r4c26_run.log 2>&1 || { tail -5 gpurun_out/r4c26_run.log; exit 1; }
    echo "P=5 wgrad_nb=$v $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c26_run.log)"
  done
}

exp_call27() {
  # wgrad single band buffer across launch sizes (P = 2, 6, 8 concurrent folds; reference folds P = 2)
  for spec in "all 2" "all 6" "all 8" "kernels 2"; do
    set -- $spec
    for v in 0 1 0 1; do
      GENTUN_WGRAD_NB=$v DTYPE=fp32 RESET=$1 timeout -k 10 200 python -u tools/probe_pop.py $2 $2 1 1 \
        > gpurun_out/r4c27_run.log 2>&1 || { tail -5 gpurun_out/r4c27_run.log; exit 1; }
      echo "RESET=$1 P=$2 wgrad_nb=$v $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c27_run.log)"
    done
  done
}

exp_call28() {
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_hip_fp32.py \
    tests/test_hip_train.py tests/test_hip_duo.py tests/test_hip_dp.py > gpurun_out/r4c28_tests.log 2>&1 || { tail -30 gpurun_out/r4c28_tests.log; exit 1; }
  tail -1 gpurun_out/r4c28_tests.log
  for i in 1 2; do
    DTYPE=fp32 RESET=all timeout -k 10 200 python -u tools/probe_pop.py 5 5 1 1 > gpurun_out/r4c28_run.log 2>&1 || { tail -5 gpurun_out/r4c28_run.log; exit 1; }
    echo "P=5 $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c28_run.log)"
  done
}

exp_call29() {
  # stream layout at 25 groups with the single-buffer wgrads: wgrad streams 2 / 3, dense W1 optimizer on its own stream or not
  for v in "2 1" "3 1" "3 0" "2 0" "2 1" "3 0"; do
    set -- $v
    GENTUN_WGRAD_STREAMS=$1 GENTUN_W1_STREAM=$2 DTYPE=fp32 RESET=all timeout -k 10 200 python -u tools/probe_pop.py 5 5 1 1 \
      > gpurun_out/r4c29_run.log 2>&1 || { tail -5 gpurun_out/r4c29_run.log; exit 1; }
    echo "P=5 wgrad_streams=$1 w1_stream=$2 $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c29_run.log)"
  done
}

exp_call30() {
  # per-layer conv Adam on the W1 optimizer stream (GENTUN_ADAM_OVERLAP=1) vs one launch after the backward (0)
  timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_hip_train.py -k "adam_overlap" \
    > gpurun_out/r4c30_test.log 2>&1 || { tail -30 gpurun_out/r4c30_test.log; exit 1; }
  grep -E "passed|failed" gpurun_out/r4c30_test.log | tail -3
  for v in "all 5 0" "all 5 1" "all 5 0" "all 5 1" "kernels 2 0" "kernels 2 1" "all 2 0" "all 2 1"; do
    set -- $v
    GENTUN_ADAM_OVERLAP=$3 DTYPE=fp32 RESET=$1 timeout -k 10 200 python -u tools/probe_pop.py $2 $2 1 1 \
      > gpurun_out/r4c30_run.log 2>&1 || { tail -5 gpurun_out/r4c30_run.log; exit 1; }
    echo "RESET=$1 P=$2 adam_overlap=$3 $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c30_run.log)"
  done
}

exp_call31() {
  # captured step graph vs eager launches, multi-stream backward vs one stream (GENTUN_OVERLAP=0)
  for v in "all 5 1 1" "all 5 0 1" "all 5 1 0" "all 5 0 0" "kernels 2 1 1" "kernels 2 0 1" "kernels 2 1 0" "all 5 1 1" "all 5 0 1"; do
    set -- $v
    GRAPH=$3 GENTUN_OVERLAP=$4 DTYPE=fp32 RESET=$1 timeout -k 10 200 python -u tools/probe_pop.py $2 $2 1 1 \
      > gpurun_out/r4c31_run.log 2>&1 || { tail -5 gpurun_out/r4c31_run.log; exit 1; }
    echo "RESET=$1 P=$2 graph=$3 overlap=$4 $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c31_run.log)"
  done
}

exp_call32() {
  # captured step graph vs eager launches with the capture amortised over 8 epochs (probe_pop P P 1 EPOCHS)
  for v in "all 5 1 8" "all 5 0 8" "kernels 2 1 4" "kernels 2 0 4" "all 5 1 8" "all 5 0 8" "all 2 1 8" "all 2 0 8"; do
    set -- $v
    GENTUN_GRAPH=$3 DTYPE=fp32 RESET=$1 timeout -k 10 200 python -u tools/probe_pop.py $2 $2 1 $4 \
      > gpurun_out/r4c32_run.log 2>&1 || { tail -5 gpurun_out/r4c32_run.log; exit 1; }
    echo "RESET=$1 P=$2 graph=$3 epochs=$4 $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c32_run.log)"
  done
}

exp_call33() {
  # bench.py same-box A/B: captured step graph (GENTUN_GRAPH=1) vs eager launches (0)
  ( while true; do sleep 50; echo hb > gpurun_out/heartbeat; done ) & HB=$!
  trap "kill $HB" EXIT
  for g in 1 0 1 0; do
    GENTUN_GRAPH=$g timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 8 --warmup 2 > gpurun_out/r4c33_g$g.json 2> gpurun_out/r4c33_g$g.err \
      || { tail -5 gpurun_out/r4c33_g$g.err; exit 1; }
    echo "graph=$g $(grep -o '"value": [0-9.]*, "unit": "[a-z/]*", "n_gpus": 1, "steps": 8, "warmup": 2, "ms_per_step": [0-9.]*' gpurun_out/r4c33_g$g.json)"
  done
}

exp_call34() {
  # native step program (GENTUN_GRAPH=0, GENTUN_NATIVE_STEPS=1) vs captured graph vs Python eager: tests, population step, bench.py
  ( while true; do sleep 50; echo hb > gpurun_out/heartbeat; done ) & HB=$!
  trap "kill $HB" EXIT
  timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_hip_train.py -k "native_step or graph_equals or adam_overlap" \
    > gpurun_out/r4c34_test.log 2>&1 || { tail -30 gpurun_out/r4c34_test.log; exit 1; }
  grep -E "passed|failed" gpurun_out/r4c34_test.log | tail -2
  for v in "all 5 1 1 8" "all 5 0 1 8" "all 5 0 0 8" "kernels 2 1 1 4" "kernels 2 0 1 4" "all 2 1 1 8" "all 2 0 1 8"; do
    set -- $v
    GENTUN_GRAPH=$3 GENTUN_NATIVE_STEPS=$4 DTYPE=fp32 RESET=$1 timeout -k 10 200 python -u tools/probe_pop.py $2 $2 1 $5 \
      > gpurun_out/r4c34_run.log 2>&1 || { tail -5 gpurun_out/r4c34_run.log; exit 1; }
    echo "RESET=$1 P=$2 graph=$3 native=$4 epochs=$5 $(grep -o '"enqueue_s": [0-9.]*, "ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c34_run.log)"
  done
  for g in 1 0 1 0; do
    GENTUN_GRAPH=$g timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 8 --warmup 2 > gpurun_out/r4c34_g$g.json 2> gpurun_out/r4c34_g$g.err \
      || { tail -5 gpurun_out/r4c34_g$g.err; exit 1; }
    echo "bench graph=$g native=1 $(grep -o '"value": [0-9.]*, "unit": "[a-z/]*", "n_gpus": 1, "steps": 8, "warmup": 2, "ms_per_step": [0-9.]*' gpurun_out/r4c34_g$g.json)"
  done
}

exp_dense() {
  export GENTUN_NO_AUTOBUILD=1
  mkdir -p gpurun_out/dense
  timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_hip_dense_stream.py tests/test_hip_step_parity.py tests/test_hip_train.py > gpurun_out/dense/tests.log 2>&1 || { tail -30 gpurun_out/dense/tests.log; exit 1; }
  tail -1 gpurun_out/dense/tests.log
  for r in 1 2; do for d2 in 0 1; do
    GENTUN_DENSE_DGRAD2=$d2 timeout -k 10 200 python tools/probe_pop.py 5 5 1 1 10000 > gpurun_out/dense/pop.log 2>&1 || { tail -5 gpurun_out/dense/pop.log; exit 1; }
    echo "dgrad2=$d2 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dense/pop.log)"
  done; done
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  for d2 in 0 1; do
    rm -rf /tmp/dn$d2
    GENTUN_DENSE_DGRAD2=$d2 WARM=0 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /tmp/dn$d2 -o run --output-format csv -- python3 tools/probe_pop.py 5 5 1 1 2000 > gpurun_out/dense/prof$d2.log 2>&1 || { tail -5 gpurun_out/dense/prof$d2.log; exit 1; }
    find /tmp/dn$d2 -name "*kernel_stats.csv" -exec cp {} gpurun_out/dense/kernel_stats_d2_$d2.csv \;
    grep -E "dense|head" gpurun_out/dense/kernel_stats_d2_$d2.csv | cut -d, -f1-4
  done
}

exp_ga_deep() {
  # BASELINE config 4 search: S=(3,4,5) kernels (20,50,100) + BatchNorm, RR-GA pop 32, fp32 full protocol,
  # checkpointed per generation (resumed from ckpt_seed/ga_deep when present)
  CKPT=gpurun_out/ga_deep/ckpt SEED_CKPT=ckpt_seed/ga_deep GENS=${GENS:-12} BUDGET=${BUDGET:-840} TIME=1080 TAG=${TAG:-} \
    GA_ARGS="--space deep --batch-norm" bash tools/gpu.sh ga
}

exp_call35() {
  # the last stage's conv Adam + head Adam on the W1 stream once that stage's backward is done (GENTUN_ADAM_SPLIT=1) vs one update after the join
  timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_hip_train.py -k "adam_overlap" \
    > gpurun_out/r4c35_test.log 2>&1 || { tail -30 gpurun_out/r4c35_test.log; exit 1; }
  grep -E "passed|failed" gpurun_out/r4c35_test.log | tail -2
  for v in "all 5 0" "all 5 1" "all 5 0" "all 5 1" "kernels 2 0" "kernels 2 1" "all 2 0" "all 2 1"; do
    set -- $v
    GENTUN_ADAM_SPLIT=$3 DTYPE=fp32 RESET=$1 timeout -k 10 200 python -u tools/probe_pop.py $2 $2 1 4 \
      > gpurun_out/r4c35_run.log 2>&1 || { tail -5 gpurun_out/r4c35_run.log; exit 1; }
    echo "RESET=$1 P=$2 adam_split=$3 $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c35_run.log)"
  done
}

exp_call36() {
  # reference folds (reset kernels) at 2 candidates: one 2-group population job vs two 1-group jobs on two streams
  for v in "2 1 4 2" "1 2 4 2" "1 2 4 1" "2 1 4 2" "1 2 4 2"; do
    set -- $v
    GENTUN_WGRAD_STREAMS=$4 DTYPE=fp32 RESET=kernels timeout -k 10 200 python -u tools/probe_pop.py 2 $1 $2 $3 \
      > gpurun_out/r4c36_run.log 2>&1 || { tail -5 gpurun_out/r4c36_run.log; exit 1; }
    echo "RESET=kernels P=2 pop_batch=$1 job_streams=$2 wgrad_streams=$4 $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c36_run.log)"
  done
}

exp_call37() {
  # adam_segments tiles with 4 elements' loads in flight per thread (GT_ADAM_UNROLL=4, default) vs one (ab_libs/adam_u1.so)
  timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_kernels.py tests/test_hip_train.py tests/test_hip_fp32.py -k "adam or inactive or invariance or dense" \
    > gpurun_out/r4c37_test.log 2>&1 || { tail -30 gpurun_out/r4c37_test.log; exit 1; }
  tail -1 gpurun_out/r4c37_test.log
  for v in "u1 5" "u4 5" "u1 5" "u4 5" "u1 2" "u4 2"; do
    set -- $v
    lib=""; [ "$1" = "u1" ] && lib=ab_libs/adam_u1.so
    GENTUN_HIP_LIB=$lib DTYPE=fp32 RESET=all timeout -k 10 200 python -u tools/probe_pop.py $2 $2 1 4 \
      > gpurun_out/r4c37_run.log 2>&1 || { tail -5 gpurun_out/r4c37_run.log; exit 1; }
    echo "P=$2 adam=$1 $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c37_run.log)"
  done
  rm -rf /tmp/a37; cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  WARM=0 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /tmp/a37 -o run --output-format csv -- python3 tools/probe_pop.py 5 5 1 1 2000 > gpurun_out/r4c37_prof.log 2>&1 \
    || { tail -5 gpurun_out/r4c37_prof.log; exit 1; }
  find /tmp/a37 -name "*kernel_stats.csv" -exec cp {} gpurun_out/r4c37_kernel_stats.csv \;
  grep -E "adam" gpurun_out/r4c37_kernel_stats.csv | cut -c1-160
}

exp_call38() {
  # dense data gradient v2 with 4 k-steps in flight per wave (GT_DGRAD_BUF=4, default) vs 2 (ab_libs/dgrad_b2.so)
  timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_dense_stream.py tests/test_hip_train.py tests/test_hip_fp32.py tests/test_hip_dp.py \
    > gpurun_out/r4c38_test.log 2>&1 || { tail -30 gpurun_out/r4c38_test.log; exit 1; }
  tail -1 gpurun_out/r4c38_test.log
  for v in "b2 5" "b4 5" "b2 5" "b4 5" "b2 2" "b4 2"; do
    set -- $v
    lib=""; [ "$1" = "b2" ] && lib=ab_libs/dgrad_b2.so
    GENTUN_HIP_LIB=$lib DTYPE=fp32 RESET=all timeout -k 10 200 python -u tools/probe_pop.py $2 $2 1 4 \
      > gpurun_out/r4c38_run.log 2>&1 || { tail -5 gpurun_out/r4c38_run.log; exit 1; }
    echo "P=$2 dgrad=$1 $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c38_run.log)"
  done
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  for v in b2 b4; do
    lib=""; [ "$v" = "b2" ] && lib=ab_libs/dgrad_b2.so
    rm -rf /tmp/a38$v
    GENTUN_HIP_LIB=$lib WARM=0 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /tmp/a38$v -o run --output-format csv -- python3 tools/probe_pop.py 5 5 1 1 2000 > gpurun_out/r4c38_prof.log 2>&1 \
      || { tail -5 gpurun_out/r4c38_prof.log; exit 1; }
    find /tmp/a38$v -name "*kernel_stats.csv" -exec cp {} gpurun_out/r4c38_kernel_stats_$v.csv \;
    echo "$v: $(grep -E "dense_dgrad" gpurun_out/r4c38_kernel_stats_$v.csv | cut -c1-120)"
  done
}

exp_call39() {
  # wgrad streams 2 vs 3 at small launches (2 and 10 groups)
  for v in "kernels 2 2" "kernels 2 3" "kernels 2 2" "kernels 2 3" "all 2 2" "all 2 3" "all 2 2" "all 2 3"; do
    set -- $v
    GENTUN_WGRAD_STREAMS=$3 DTYPE=fp32 RESET=$1 timeout -k 10 200 python -u tools/probe_pop.py $2 $2 1 4 \
      > gpurun_out/r4c39_run.log 2>&1 || { tail -5 gpurun_out/r4c39_run.log; exit 1; }
    echo "RESET=$1 P=$2 wgrad_streams=$3 $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c39_run.log)"
  done
}

exp_call40() {
  # hardware queues per process (GPU_MAX_HW_QUEUES, HIP default 4) x wgrad streams
  for v in "4 2 all 5" "8 2 all 5" "8 3 all 5" "4 2 all 5" "8 2 all 5" "8 3 all 5" "4 2 kernels 2" "8 2 kernels 2" "8 3 kernels 2"; do
    set -- $v
    GPU_MAX_HW_QUEUES=$1 GENTUN_WGRAD_STREAMS=$2 DTYPE=fp32 RESET=$3 timeout -k 10 200 python -u tools/probe_pop.py $4 $4 1 4 \
      > gpurun_out/r4c40_run.log 2>&1 || { tail -5 gpurun_out/r4c40_run.log; exit 1; }
    echo "hwq=$1 wgrad_streams=$2 RESET=$3 P=$4 $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c40_run.log)"
  done
}

exp_call41() {
  # hardware queues per process below the default (GPU_MAX_HW_QUEUES 2 / 3 / 4)
  for v in "4 all 5" "3 all 5" "2 all 5" "4 all 5" "3 all 5" "2 all 5" "4 kernels 2" "3 kernels 2" "2 kernels 2"; do
    set -- $v
    GPU_MAX_HW_QUEUES=$1 DTYPE=fp32 RESET=$2 timeout -k 10 200 python -u tools/probe_pop.py $3 $3 1 4 \
      > gpurun_out/r4c41_run.log 2>&1 || { tail -5 gpurun_out/r4c41_run.log; exit 1; }
    echo "hwq=$1 RESET=$2 P=$3 $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c41_run.log)"
  done
}

exp_call42() {
  # side streams created once per process (GENTUN_STREAM_CACHE=1) vs fresh streams per job (0): tests, population step, bench.py
  ( while true; do sleep 50; echo hb > gpurun_out/heartbeat; done ) & HB=$!
  trap "kill $HB" EXIT
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_train.py \
    > gpurun_out/r4c42_test.log 2>&1 || { tail -30 gpurun_out/r4c42_test.log; exit 1; }
  tail -1 gpurun_out/r4c42_test.log
  for v in "0 all 5" "1 all 5" "0 kernels 2" "1 kernels 2"; do
    set -- $v
    GENTUN_STREAM_CACHE=$1 DTYPE=fp32 RESET=$2 timeout -k 10 200 python -u tools/probe_pop.py $3 $3 1 4 \
      > gpurun_out/r4c42_run.log 2>&1 || { tail -5 gpurun_out/r4c42_run.log; exit 1; }
    echo "cache=$1 RESET=$2 P=$3 $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c42_run.log)"
  done
  for c in 0 1 0 1; do
    GENTUN_STREAM_CACHE=$c timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 8 --warmup 2 > gpurun_out/r4c42_c$c.json 2> gpurun_out/r4c42_c$c.err \
      || { tail -5 gpurun_out/r4c42_c$c.err; exit 1; }
    echo "bench cache=$c $(grep -o '"value": [0-9.]*, "unit": "[a-z/]*", "n_gpus": 1, "steps": 8, "warmup": 2, "ms_per_step": [0-9.]*' gpurun_out/r4c42_c$c.json)"
  done
}

case "${1:-}" in
  call4) exp_call4 ;;
  call5) exp_call5 ;;
  call6) exp_call6 ;;
  call7) exp_call7 ;;
  call8) exp_call8 ;;
  call9) exp_call9 ;;
  call10) exp_call10 ;;
  call11) exp_call11 ;;
  call12) exp_call12 ;;
  call13) exp_call13 ;;
  call14) exp_call14 ;;
  call15) exp_call15 ;;
  call16) exp_call16 ;;
  call17) exp_call17 ;;
  call18) exp_call18 ;;
  call19) exp_call19 ;;
  call20) exp_call20 ;;
  call21) exp_call21 ;;
  call22) exp_call22 ;;
  call23) exp_call23 ;;
  call24) exp_call24 ;;
  call25) exp_call25 ;;
  call26) exp_call26 ;;
  call27) exp_call27 ;;
  call28) exp_call28 ;;
  call29) exp_call29 ;;
  call30) exp_call30 ;;
  call31) exp_call31 ;;
  call32) exp_call32 ;;
  call33) exp_call33 ;;
  call34) exp_call34 ;;
  dense) exp_dense ;;
  ga_deep) exp_ga_deep ;;
  call35) exp_call35 ;;
  call36) exp_call36 ;;
  call37) exp_call37 ;;
  call38) exp_call38 ;;
  call39) exp_call39 ;;
  call40) exp_call40 ;;
  call41) exp_call41 ;;
  call42) exp_call42 ;;
  *) sed -n 2,5p "$0"; exit 2 ;;
esac
