#!/bin/bash
# Profile one population step workload (16 S=(3,5) candidates x 5 folds, 1 epoch on 2,000 samples):
#   1) rocprofv3 --kernel-trace --stats  -> per-kernel time
#   2-4) PMC passes (kernel-trace only, each its own run): SQ occupancy/LDS, MFMA/VALU/VMEM, HBM bytes
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
# env: P (candidates, default 16), DTYPE (fp32 / bf16, probe_pop.py), OUT (output dir under gpurun_out)
P=${P:-16}
OUT=${OUT:-prof_head}
mkdir -p gpurun_out/$OUT
export GENTUN_NO_AUTOBUILD=1 WARM=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CMD="python3 tools/probe_pop.py $P $P 1 1 2000"
rm -rf /tmp/ph_stats
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /tmp/ph_stats -o run --output-format csv -- $CMD \
  > gpurun_out/$OUT/stats_run.log 2>&1 || { echo "FAIL stats"; tail -5 gpurun_out/$OUT/stats_run.log; exit 1; }
find /tmp/ph_stats -name "*kernel_stats.csv" -exec cp {} gpurun_out/$OUT/kernel_stats.csv \;
head -20 gpurun_out/$OUT/kernel_stats.csv | cut -c1-160
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
P3="TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  rm -rf /tmp/ph_pmc$i
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P -d /tmp/ph_pmc$i -o run --output-format csv -- $CMD \
    > gpurun_out/$OUT/pmc$i.log 2>&1 || { echo "FAIL pmc$i"; tail -5 gpurun_out/$OUT/pmc$i.log; exit 1; }
  python3 tools/pmc_summary.py /tmp/ph_pmc$i > gpurun_out/$OUT/pmc$i.txt
  head -12 gpurun_out/$OUT/pmc$i.txt | cut -c1-400
done
