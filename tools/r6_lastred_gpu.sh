# (The LASTRED switch was removed after this A/B: profiles/r6/last_wred_r6.txt.)
# Round 6: last weight gradient summed by Adam (LASTRED=1) vs a reduce launch (LASTRED=0): HIP training tests,
# then alternating population steps (25 and 10 groups) on one box.
export GENTUN_NO_AUTOBUILD=1
timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_hip_train.py tests/test_hip_step_parity.py tests/test_hip_dp.py tests/test_padded_geometry.py > gpurun_out/lr_tests.log 2>&1 || { tail -30 gpurun_out/lr_tests.log; exit 1; }
tail -1 gpurun_out/lr_tests.log
: > gpurun_out/lastred.txt
for i in 1 2 3; do
  for v in 1 0; do
    for P in 5 2; do
      LASTRED=$v timeout -k 10 200 python3 tools/probe_pop.py $P $P 1 1 10000 > gpurun_out/lr.log 2>&1 || { tail -5 gpurun_out/lr.log; exit 1; }
      echo "P=$P LASTRED=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/lr.log)" | tee -a gpurun_out/lastred.txt
    done
  done
done
