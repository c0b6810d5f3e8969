#!/bin/bash
# population-step throughput: fp32 vs bf16, and the Q (groups per launch) curve in fp32
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
out=gpurun_out/probe_fp32.log
: > $out
for cfg in "bf16 16 16" "fp32 16 16" "fp32 8 8" "fp32 4 4" "fp32 2 2"; do
  set -- $cfg
  echo "== DTYPE=$1 P=$2 pb=$3" >> $out
  DTYPE=$1 timeout -k 10 300 python -u tools/probe_pop.py $2 $3 1 1 >> $out 2>&1 || exit $?
done
cd /tmp && export TMPDIR=/tmp
DTYPE=fp32 WARM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_fp32 -o run -- python3 $GRAFT_REPO_ROOT/tools/probe_pop.py 16 16 1 1 >> $GRAFT_REPO_ROOT/$out 2>&1
