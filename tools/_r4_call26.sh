# wgrad band buffers at the bench size: single buffer (57 KB LDS: co-resides with a conv workgroup) vs double (115 KB)
set -o pipefail
for v in 0 1 0 1; do
  GENTUN_WGRAD_NB=$v DTYPE=fp32 RESET=all timeout -k 10 200 python -u tools/probe_pop.py 5 5 1 1 \
    > gpurun_out/r4c26_run.log 2>&1 || { tail -5 gpurun_out/r4c26_run.log; exit 1; }
  echo "P=5 wgrad_nb=$v $(grep -o '"ms_per_step": [0-9.]*, "ms_per_cand_step": [0-9.]*, "cand_per_hour_full_protocol": [0-9.]*' gpurun_out/r4c26_run.log)"
done
