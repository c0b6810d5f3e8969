#!/bin/bash
# PMC passes on one microbench kernel (SPEC=kernel:shape, EPI=epi_bf16).
mkdir -p gpurun_out/pmc2
export GENTUN_NO_AUTOBUILD=1 GENTUN_BENCH_G=40 GENTUN_EPI_BF16=${EPI:-1} GENTUN_BENCH_ONLY=${SPEC:-conv_fwd:4}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  rm -rf /tmp/pmc2_$i
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P -d /tmp/pmc2_$i -o run --output-format csv -- python3 tools/bench_kernels.py 5 > gpurun_out/pmc2/p$i.log 2>&1 || { echo "FAIL p$i"; tail -5 gpurun_out/pmc2/p$i.log; exit 1; }
  python3 tools/pmc_summary.py /tmp/pmc2_$i | grep -v "^void at::\|elementwise\|copyBuffer\|fill" > gpurun_out/pmc2/p$i.txt
  cat gpurun_out/pmc2/p$i.txt | cut -c1-700
done
