# diagnostic: conv fwd / dgrad with L1-resident weights (dbg 8) vs normal, and MFMA-only (dbg 6), 25 groups
set -o pipefail
G=25 DBGS=0,8,6,14 ONLY=s2_n timeout -k 10 200 python -u tools/bench_conv.py 10 > gpurun_out/r4c15.log 2>&1 || { tail -5 gpurun_out/r4c15.log; exit 1; }
grep -v wgrad gpurun_out/r4c15.log | python3 -c "
import sys, json
for l in sys.stdin:
    if l.startswith('{'):
        d = json.loads(l); print(d['kernel'], d['shape'], 'dbg', d['dbg'], d['us'])"
