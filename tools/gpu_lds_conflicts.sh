#!/bin/bash
# LDS bank conflicts of the fp32 stage-2 conv by phase (dbg: 0 full, 2 skip epilogue stores, 1 skip MFMA loop)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export GENTUN_NO_AUTOBUILD=1 DTYPE=fp32 ONLY=s2_n F32P=0
for d in 0 2 1; do
  rm -rf /tmp/ldsc$d
  DBGS=$d timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE \
    -d /tmp/ldsc$d -o run --output-format csv -- python3 tools/bench_conv.py 3 > gpurun_out/ldsc$d.log 2>&1 || { tail -5 gpurun_out/ldsc$d.log; exit 1; }
  echo "== dbg $d"
  python3 tools/pmc_summary.py /tmp/ldsc$d | grep -i conv_fast | cut -c1-260
done
