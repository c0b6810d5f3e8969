#!/bin/bash
# kernel stats of a population job at bench round size (P candidates x 5 folds), fp32
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1 WARM=0 DTYPE=${DTYPE:-fp32}
P=${P:-2}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/prof_p$P -o run -- python3 $GRAFT_REPO_ROOT/tools/probe_pop.py $P $P 1 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_p$P.log 2>&1
rc=$?; grep '^{' $GRAFT_REPO_ROOT/gpurun_out/prof_p$P.log; exit $rc
