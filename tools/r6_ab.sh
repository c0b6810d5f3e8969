#!/bin/bash
# Same-box A/B of alternative kernel-library builds (ab_libs/<name>.so, tools/build_ab.sh):
#   LIBS="old new" TESTS="tests/test_hip_kernels.py -k wadam" REPS=3 bash tools/r6_ab.sh
# Each library first passes TESTS (if given), then population steps (tools/probe_pop.py P P 1 1 10000)
# alternate between the libraries REPS times; ms/step per run -> gpurun_out/r6ab/summary.txt.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export GENTUN_NO_AUTOBUILD=1
out=gpurun_out/r6ab${TAG:-}; mkdir -p $out; : > $out/summary.txt
if [ -n "${TESTS:-}" ]; then
  for lib in ${LIBS}; do
    GENTUN_HIP_LIB=ab_libs/$lib.so timeout -k 10 300 python -u -m pytest -m gpu -x -q --timeout 120 \
      --timeout-method thread $TESTS > $out/tests_$lib.log 2>&1 || { tail -30 $out/tests_$lib.log; exit 1; }
    echo "$lib tests: $(tail -1 $out/tests_$lib.log)" | tee -a $out/summary.txt
  done
fi
# VARIANTS (default: LIBS) entries are lib or lib@VAR=value (an environment switch of tools/probe_pop.py)
for i in $(seq ${REPS:-3}); do
  for spec in ${VARIANTS:-$LIBS}; do
    lib=${spec%%@*}; envs=""; [ "$spec" != "$lib" ] && envs=${spec#*@}
    env $envs GENTUN_HIP_LIB=ab_libs/$lib.so timeout -k 10 200 python tools/probe_pop.py ${P:-5} ${P:-5} 1 ${EP:-1} \
      ${N:-10000} > $out/pop.log 2>&1 || { tail -20 $out/pop.log; exit 1; }
    echo "$spec $(grep -o '"ms_per_step": [0-9.]*' $out/pop.log)" | tee -a $out/summary.txt
  done
done
