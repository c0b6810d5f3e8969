#!/bin/bash
# end-of-round checks at HEAD: GPU suite + smoke, timeline at the bench round size, driver-equivalent headline
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_all_tests.sh || exit $?
P=5 SAMPLES=2000 bash tools/gpu_timeline.sh > /dev/null || exit $?
head -20 gpurun_out/timeline/summary.txt
bash tools/gpu_headline3.sh
