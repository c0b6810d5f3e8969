# wgrad single band buffer across launch sizes (P = 2, 6, 8 concurrent folds; reference folds P = 2)
set -o pipefail
for spec in "all 2" "all 6" "all 8" "kernels 2"; do
  set -- $spec
  for v in 0 1 0 1; do
    GENTUN_WGRAD_NB=$v DTYPE=fp32 RESET=$1 timeout -k 10 200 python -u tools/probe_pop.py $2 $2 1 1 \
      > gpurun_out/r4c27_run.log 2>&1 || { tail -5 gpurun_out/r4c27_run.log; exit 1; }
    echo "RESET=$1 P=$2 wgrad_nb=$v $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c27_run.log)"
  done
done
