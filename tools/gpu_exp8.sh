#!/bin/bash
export GENTUN_NO_AUTOBUILD=1
mkdir -p gpurun_out; rm -f gpurun_out/probe_spread6.log
for kw in '{"label_noise": 0.2}' '{"label_noise": 0.3, "noise": 0.7}'; do
  timeout -k 10 200 python3 -u tools/probe_spread.py 12 variant "$kw" >> gpurun_out/probe_spread6.log 2>&1 || { tail -5 gpurun_out/probe_spread6.log; exit 1; }
done
grep summary gpurun_out/probe_spread6.log
grep genes gpurun_out/probe_spread6.log | python3 -c "
import sys, json
for l in sys.stdin:
    d=json.loads(l); print(d['genes'], d['cat_acc_folds'], d['cat_acc'])
"
