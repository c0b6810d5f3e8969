#!/bin/bash
# Measurements for the BASELINE.md table: GA search (best fitness per generation),
# torch-ops comparator, deep S=(3,4,5) throughput. Each GPU step has its own limit.
mkdir -p gpurun_out
export GENTUN_NO_AUTOBUILD=1
timeout -k 10 200 python tools/probe_torch.py torch > gpurun_out/torch_probe.log 2>&1 || exit 1
SPACE=deep timeout -k 10 300 python tools/probe_pop.py 8 8 1 1 10000 > gpurun_out/deep_probe.log 2>&1 || exit 1
timeout -k 10 600 python -m gentun_amd cnn --pop 16 --gens 4 --seed 1 --events gpurun_out/ga_events.jsonl > gpurun_out/ga_search.log 2>&1 || exit 1
tail -n 1 gpurun_out/ga_search.log | cut -c1-1500
grep '{' gpurun_out/deep_probe.log; grep '{' gpurun_out/torch_probe.log
