#!/bin/bash
# GBDT GPU path: kernel stats + PMC passes of one cv call (tools/probe_gbdt.py rows features depth rounds)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export GENTUN_NO_AUTOBUILD=1
out=gpurun_out/r5/gbdt${TAG:-}; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$OLDPWD}"
cmd="python3 tools/probe_gbdt.py ${ROWS:-1000000} 256 ${DEPTH:-10} ${ROUNDS:-3}"
rm -rf /tmp/gb_stats
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/gb_stats -o run --output-format csv -- $cmd \
  > $out/stats_run.log 2>&1 || { tail -5 $out/stats_run.log; exit 1; }
find /tmp/gb_stats -name "*kernel_stats.csv" -exec cp {} $out/kernel_stats.csv \;
grep "{" $out/stats_run.log | tail -1
head -8 $out/kernel_stats.csv | cut -d, -f1-4
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
           "TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1)); rm -rf /tmp/gb_pmc$i
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $ctr -d /tmp/gb_pmc$i -o run --output-format csv -- $cmd \
    > $out/pmc$i.log 2>&1 || { tail -5 $out/pmc$i.log; exit 1; }
  python3 tools/pmc_summary.py /tmp/gb_pmc$i > $out/pmc$i.txt
  grep -i "hist_kernel\|reduce_kernel\|partition" $out/pmc$i.txt | cut -c1-400
done
