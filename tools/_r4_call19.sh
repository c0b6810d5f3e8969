# A/B: main-stream priority (the data-gradient chain) and per-layer conv Adam on a third stream, 25 groups
set -o pipefail
for v in "0 0 0" "-1 0 0" "0 0 1" "-1 0 0" "0 0 0"; do
  set -- $v
  MAIN_PRIO=$1 GENTUN_SIDE_PRIO=$2 GENTUN_ADAM_OVERLAP=$3 DTYPE=fp32 RESET=all timeout -k 10 200 python -u tools/probe_pop.py 5 5 1 1 \
    > gpurun_out/r4c19_run.log 2>&1 || { tail -5 gpurun_out/r4c19_run.log; exit 1; }
  echo "main_prio=$1 side_prio=$2 adam_overlap=$3 $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c19_run.log)"
done
