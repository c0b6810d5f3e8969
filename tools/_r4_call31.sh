# captured step graph vs eager launches, multi-stream backward vs one stream (GENTUN_OVERLAP=0)
set -o pipefail
for v in "all 5 1 1" "all 5 0 1" "all 5 1 0" "all 5 0 0" "kernels 2 1 1" "kernels 2 0 1" "kernels 2 1 0" "all 5 1 1" "all 5 0 1"; do
  set -- $v
  GRAPH=$3 GENTUN_OVERLAP=$4 DTYPE=fp32 RESET=$1 timeout -k 10 200 python -u tools/probe_pop.py $2 $2 1 1 \
    > gpurun_out/r4c31_run.log 2>&1 || { tail -5 gpurun_out/r4c31_run.log; exit 1; }
  echo "RESET=$1 P=$2 graph=$3 overlap=$4 $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c31_run.log)"
done
