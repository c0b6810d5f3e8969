#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export GENTUN_NO_AUTOBUILD=1 DTYPE=fp32
for cfg in "8 0" "16 0" "16 1" "32 1"; do
  set -- $cfg
  for P in 3 16; do
    echo "== splits16=$1 nb=$2 P=$P"
    GENTUN_F32_SPLITS16=$1 GENTUN_WGRAD_NB=$2 timeout -k 10 200 python -u tools/probe_pop.py $P $P 1 1 2>&1 | grep '^{' | cut -c1-160 || exit 1
  done
done
