# captured step graph vs eager launches with the capture amortised over 8 epochs (probe_pop P P 1 EPOCHS)
set -o pipefail
for v in "all 5 1 8" "all 5 0 8" "kernels 2 1 4" "kernels 2 0 4" "all 5 1 8" "all 5 0 8" "all 2 1 8" "all 2 0 8"; do
  set -- $v
  GENTUN_GRAPH=$3 DTYPE=fp32 RESET=$1 timeout -k 10 200 python -u tools/probe_pop.py $2 $2 1 $4 \
    > gpurun_out/r4c32_run.log 2>&1 || { tail -5 gpurun_out/r4c32_run.log; exit 1; }
  echo "RESET=$1 P=$2 graph=$3 epochs=$4 $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c32_run.log)"
done
