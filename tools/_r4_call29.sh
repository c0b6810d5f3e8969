# stream layout at 25 groups with the single-buffer wgrads: wgrad streams 2 / 3, dense W1 optimizer on its own stream or not
set -o pipefail
for v in "2 1" "3 1" "3 0" "2 0" "2 1" "3 0"; do
  set -- $v
  GENTUN_WGRAD_STREAMS=$1 GENTUN_W1_STREAM=$2 DTYPE=fp32 RESET=all timeout -k 10 200 python -u tools/probe_pop.py 5 5 1 1 \
    > gpurun_out/r4c29_run.log 2>&1 || { tail -5 gpurun_out/r4c29_run.log; exit 1; }
  echo "P=5 wgrad_streams=$1 w1_stream=$2 $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c29_run.log)"
done
