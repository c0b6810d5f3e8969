#!/bin/bash
# PMC passes over conv kernels of the microbench at G=40 (one counter group per run).
mkdir -p gpurun_out
export GENTUN_NO_AUTOBUILD=1 GENTUN_BENCH_G=40
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU FETCH_SIZE GRBM_GUI_ACTIVE"
P3="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
for spec in ${SPECS:-conv_fwd:1 conv_fwd:4 conv_wgrad:1 conv_wgrad:4}; do
  for m in 0; do
    i=0
    for P in "$P1" "$P2" "$P3"; do
      i=$((i+1))
      n=${spec/:/_}_m${m}_p$i
      rm -rf /tmp/pmc_$n
      GENTUN_BENCH_ONLY=$spec GENTUN_CONV_MODES=$m timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P -d /tmp/pmc_$n -o run --output-format csv -- python3 tools/bench_kernels.py 5 > /tmp/pmc_$n.log 2>&1 || { echo "FAIL $n"; tail -5 /tmp/pmc_$n.log; exit 1; }
      python3 tools/pmc_summary.py /tmp/pmc_$n | grep -v "^void at::\|elementwise\|copyBuffer\|fill" > gpurun_out/pmc_$n.txt
    done
  done
done
ls gpurun_out
