#!/bin/bash
# One entry point for every GPU-box task (run through gpurun from the repo root):
#
#   bash tools/gpu.sh tests [PYTEST_ARGS]     GPU test suite (one pytest process) + __graft_entry__.smoke()
#   bash tools/gpu.sh headline                driver-equivalent bench.py (STEPS=20 WARMUP=5 EXTRA= TAG=)
#   bash tools/gpu.sh timeline                kernel timeline of a population step (P=5 SAMPLES=2000 SPACE= KERNELS= BN=)
#   bash tools/gpu.sh prof NAME -- CMD...     rocprofv3 --kernel-trace --stats, keeps the stats CSVs
#   bash tools/gpu.sh pmc NAME "CTRS" -- CMD  one PMC pass (kernel-trace only) + tools/pmc_summary.py
#   bash tools/gpu.sh profstep                stats + 3 PMC passes of a population step -> tools/pmc_table.py (P= SPACE= KERNELS= BN= OUT=)
#   bash tools/gpu.sh conv                    conv microbench tools/bench_conv.py (GS="25" ONLY= DBGS=0), fp32 tests first
#   bash tools/gpu.sh ab                      tests + population-step A/B: ab_old/ (built previous tree) vs this tree
#   bash tools/gpu.sh qcurve                  groups per launch vs throughput, both fold protocols
#   bash tools/gpu.sh ga                      long RR-GA search with checkpoints (GENS= CKPT= BUDGET= GA_ARGS=)
#   bash tools/gpu.sh gbdt                    GBDT GPU tests, GA bench and kernel stats (POP= ROUNDS=)
#   bash tools/gpu.sh rehearse                2-rank torchrun bench on one GPU (gloo control plane)
#   bash tools/gpu.sh secondary               bench lines: reference fold semantics, torch comparator
#
# Every GPU step runs under its own `timeout -k 10`; steps are chained so the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export GENTUN_NO_AUTOBUILD=1
mkdir -p gpurun_out
task=${1:-}; shift || true

heartbeat() {   # a line every 50 s under gpurun_out/ so a long step is not taken for a hang
  ( while sleep 50; do date >> gpurun_out/heartbeat; done ) & HB=$!
  trap 'kill $HB 2>/dev/null' EXIT
}

rocprof_env() { cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$OLDPWD}"; }

case "$task" in
tests)
  timeout -k 10 1000 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/ "$@" \
    > gpurun_out/gpu_tests.log 2>&1; rc=$?
  grep -E "passed|failed|FAILED|Error" gpurun_out/gpu_tests.log | tail -8
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
  tail -3 gpurun_out/smoke.log | cut -c1-400
  exit $rc ;;
headline)
  heartbeat; mkdir -p gpurun_out/headline
  timeout -k 10 ${TIME:-700} python3 -u bench.py --gpus 1 --steps ${STEPS:-20} --warmup ${WARMUP:-5} ${EXTRA:-} \
    > gpurun_out/headline/bench${TAG:-}.json 2> gpurun_out/headline/bench${TAG:-}.err; rc=$?
  tail -3 gpurun_out/headline/bench${TAG:-}.err; cat gpurun_out/headline/bench${TAG:-}.json
  exit $rc ;;
timeline)
  rocprof_env; mkdir -p gpurun_out/timeline; rm -rf /tmp/tl
  WARM=0 timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/tl -o run --output-format csv -- \
    python3 tools/probe_pop.py ${P:-5} ${P:-5} 1 1 ${SAMPLES:-2000} > gpurun_out/timeline/run${TAG:-}.log 2>&1 \
    || { tail -5 gpurun_out/timeline/run${TAG:-}.log; exit 1; }
  TIMELINE_DUMP=${DUMP:-1} python3 tools/timeline.py "$(find /tmp/tl -name "*kernel_trace.csv" | head -1)" > gpurun_out/timeline/summary${TAG:-}.txt
  head -30 gpurun_out/timeline/summary${TAG:-}.txt ;;
prof)
  name=$1; shift; shift
  rocprof_env; rm -rf /tmp/prof_$name; mkdir -p gpurun_out/prof_$name
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_$name -o run --output-format csv -- "$@" \
    > gpurun_out/prof_$name/run.log 2>&1 || { tail -5 gpurun_out/prof_$name/run.log; exit 1; }
  find /tmp/prof_$name -name "*stats.csv" -exec cp {} gpurun_out/prof_$name/ \;
  head -16 gpurun_out/prof_$name/run_kernel_stats.csv 2>/dev/null | cut -d, -f1-4 ;;
pmc)
  name=$1; counters=$2; shift 3
  rocprof_env; rm -rf /tmp/pmc_$name; mkdir -p gpurun_out/pmc_$name
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $counters -d /tmp/pmc_$name -o run --output-format csv -- "$@" \
    > gpurun_out/pmc_$name/run.log 2>&1 || { tail -5 gpurun_out/pmc_$name/run.log; exit 1; }
  python3 tools/pmc_summary.py /tmp/pmc_$name > gpurun_out/pmc_$name/summary.txt
  head -30 gpurun_out/pmc_$name/summary.txt ;;
profstep)
  out=gpurun_out/${OUT:-profstep}; mkdir -p $out; rocprof_env; export WARM=0
  cmd="python3 tools/probe_pop.py ${P:-5} ${P:-5} 1 1 ${SAMPLES:-2000}"
  rm -rf /tmp/ps_stats
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /tmp/ps_stats -o run --output-format csv -- $cmd \
    > $out/stats_run.log 2>&1 || { tail -5 $out/stats_run.log; exit 1; }
  find /tmp/ps_stats -name "*kernel_stats.csv" -exec cp {} $out/kernel_stats.csv \;
  i=0
  for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
             "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
             "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
    i=$((i+1)); rm -rf /tmp/ps_pmc$i
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctr -d /tmp/ps_pmc$i -o run --output-format csv -- $cmd \
      > $out/pmc$i.log 2>&1 || { tail -5 $out/pmc$i.log; exit 1; }
    python3 tools/pmc_summary.py /tmp/ps_pmc$i > $out/pmc$i.txt
  done
  python3 tools/pmc_table.py $out > $out/table.txt; head -24 $out/table.txt ;;
conv)
  timeout -k 10 300 python -u -m pytest tests/test_hip_fp32.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/fp32_tests.log 2>&1 || { tail -30 gpurun_out/fp32_tests.log; exit 1; }
  tail -1 gpurun_out/fp32_tests.log
  : > gpurun_out/bench_conv${TAG:-}.log
  for G in ${GS:-25}; do
    G=$G DBGS=${DBGS:-0} ONLY="${ONLY:-}" timeout -k 10 300 python -u tools/bench_conv.py ${REPS:-10} \
      >> gpurun_out/bench_conv${TAG:-}.log 2>&1 || { tail -5 gpurun_out/bench_conv${TAG:-}.log; exit 1; }
  done
  cut -c1-160 gpurun_out/bench_conv${TAG:-}.log ;;
ab)
  if [ -z "${SKIP_TESTS:-}" ]; then
    timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread ${AB_TESTS:-tests/test_hip_fp32.py tests/test_hip_kernels.py tests/test_hip_train.py} \
      > gpurun_out/ab_tests.log 2>&1 || { tail -40 gpurun_out/ab_tests.log; exit 1; }
    tail -1 gpurun_out/ab_tests.log
  fi
  for i in $(seq ${REPS:-3}); do
    (cd ab_old && timeout -k 10 200 python tools/probe_pop.py ${P:-5} ${P:-5} 1 ${EP:-1} 10000) > gpurun_out/ab_old_$i.log 2>&1 \
      || { tail -20 gpurun_out/ab_old_$i.log; exit 1; }
    timeout -k 10 200 python tools/probe_pop.py ${P:-5} ${P:-5} 1 ${EP:-1} 10000 > gpurun_out/ab_new_$i.log 2>&1 \
      || { tail -20 gpurun_out/ab_new_$i.log; exit 1; }
    echo "old: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_old_$i.log)  new: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_new_$i.log)"
  done ;;
qcurve)
  mkdir -p gpurun_out/qc; : > gpurun_out/qc/qcurve.txt
  for spec in ${SPECS:-"all 1" "all 2" "all 4" "all 5" "all 8" "all 16" "kernels 2" "kernels 5" "kernels 10" "kernels 16"}; do
    set -- $spec
    DTYPE=fp32 RESET=$1 timeout -k 10 200 python -u tools/probe_pop.py $2 $2 1 1 > gpurun_out/qc/run.log 2>&1 \
      || { tail -5 gpurun_out/qc/run.log; exit 1; }
    echo "== RESET=$1 P=$2 $(grep '^{' gpurun_out/qc/run.log | cut -c1-200)" | tee -a gpurun_out/qc/qcurve.txt
  done ;;
ga)
  heartbeat; ck=${CKPT:-gpurun_out/ga/ckpt}; mkdir -p gpurun_out/ga "$(dirname "$ck")"
  if [ -n "${SEED_CKPT:-}" ] && [ -d "$SEED_CKPT" ] && [ ! -d "$ck" ]; then cp -r "$SEED_CKPT" "$ck"; fi
  timeout -k 10 ${TIME:-1080} python3 -u tools/ga_run.py --gens ${GENS:-20} --ckpt "$ck" --resume \
    --time-budget ${BUDGET:-900} ${GA_ARGS:-} > gpurun_out/ga/run${TAG:-}.json 2> gpurun_out/ga/run${TAG:-}.err; rc=$?
  grep "\[ga_run\]" gpurun_out/ga/run${TAG:-}.err | tail -25; cat gpurun_out/ga/run${TAG:-}.json
  exit $rc ;;
gbdt)
  timeout -k 10 300 python -u -m pytest tests/test_gbdt_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gbdt_tests.log 2>&1 || { tail -30 gpurun_out/gbdt_tests.log; exit 1; }
  tail -1 gpurun_out/gbdt_tests.log
  if [ -n "${BENCH:-}" ]; then
    timeout -k 10 600 python tools/bench_gbdt.py --pop ${POP:-8} --rounds ${ROUNDS:-50} ${GBDT_ARGS:-} > gpurun_out/bench_gbdt.log 2>&1 \
      || { tail -10 gpurun_out/bench_gbdt.log; exit 1; }
    grep "{" gpurun_out/bench_gbdt.log
  fi
  rocprof_env; rm -rf /tmp/pg; mkdir -p gpurun_out/prof_gbdt
  GENTUN_GBDT_TIMING=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pg -o run --output-format csv -- \
    python3 tools/probe_gbdt.py 1000000 256 ${DEPTH:-10} 5 > gpurun_out/prof_gbdt/run.log 2>&1 \
    || { tail -5 gpurun_out/prof_gbdt/run.log; exit 1; }
  find /tmp/pg -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_gbdt/ \;
  grep "{\|gbdt_hip" gpurun_out/prof_gbdt/run.log | tail -2
  head -12 gpurun_out/prof_gbdt/run_kernel_stats.csv | cut -d, -f1-4 ;;
rehearse)
  heartbeat
  GENTUN_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${N:-2} \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus ${N:-2} --steps ${STEPS:-2} --warmup 1 \
    > gpurun_out/rehearse.json 2> gpurun_out/rehearse.err || { tail -20 gpurun_out/rehearse.err; exit 1; }
  cut -c1-600 gpurun_out/rehearse.json ;;
secondary)
  heartbeat; mkdir -p gpurun_out/sec
  if [ -z "${SKIP_KERNELS:-}" ]; then
    timeout -k 10 ${KTIME:-560} python3 -u bench.py --gpus 1 --fold-reset kernels --steps ${KSTEPS:-3} --warmup 1 \
      --json-out gpurun_out/sec/kernels.json > gpurun_out/sec/kernels.out 2> gpurun_out/sec/kernels.err \
      || { tail -5 gpurun_out/sec/kernels.err; exit 1; }
    cat gpurun_out/sec/kernels.json
  fi
  if [ -z "${SKIP_TORCH:-}" ]; then
    timeout -k 10 ${TTIME:-560} python3 -u bench.py --gpus 1 --backend torch --steps ${TSTEPS:-2} --warmup 1 \
      --json-out gpurun_out/sec/torch.json > gpurun_out/sec/torch.out 2> gpurun_out/sec/torch.err \
      || { tail -5 gpurun_out/sec/torch.err; exit 1; }
    cat gpurun_out/sec/torch.json
  fi ;;
*)
  sed -n 2,17p "$0"; exit 2 ;;
esac
