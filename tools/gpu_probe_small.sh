#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1 DTYPE=${DTYPE:-fp32}
out=gpurun_out/probe_small.log
: > $out
for cfg in ${CFGS:-"2 2 1" "2 1 2" "4 4 1" "4 2 2" "16 16 1"}; do
  set -- $cfg
  echo "== P=$1 pb=$2 streams=$3" >> $out
  timeout -k 10 300 python -u tools/probe_pop.py $1 $2 $3 1 >> $out 2>&1 || exit $?
done
grep -E "^==|^\{" $out | cut -c1-260
