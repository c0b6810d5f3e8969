#!/bin/bash
# every GPU test, then the fold-semantics throughput probe
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1
true
true
out=gpurun_out/probe_reset.log; : > $out
for cfg in ${RCFGS:-"2 all" "2 kernels" "16 all" "16 kernels"}; do
  set -- $cfg
  echo "== P=$1 RESET=$2" >> $out
  RESET=$2 timeout -k 10 300 python -u tools/probe_pop.py $1 $1 1 1 >> $out 2>&1 || exit $?
done
grep -E "^==|^\{" $out | cut -c1-200
