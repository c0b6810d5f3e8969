"""Do candidates on separate HIP streams overlap? Time N identical fold-batched
jobs run (a) one after another and (b) concurrently on N streams.

usage: python tools/probe_concurrency.py [N] [epochs] [samples]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from gentun_amd.models import cnn_engine as E
from gentun_amd.models.genome import make_plan
from gentun_amd.utils.data import make_cifar_like, stratified_kfold

N = int(sys.argv[1]) if len(sys.argv) > 1 else 4
epochs = int(sys.argv[2]) if len(sys.argv) > 2 else 1
n = int(sys.argv[3]) if len(sys.argv) > 3 else 10000
dev = torch.device("cuda", 0)
x, y = make_cifar_like(n=n, seed=0)
folds = stratified_kfold(np.argmax(y, 1), 5, seed=0)
plan = make_plan({'S_1': '101', 'S_2': '0101110011'}, (3, 5), (32, 32, 3), (20, 50), ((5, 5), (5, 5)), 500, 10)
cfg = E.TrainConfig(epochs=(epochs,), learning_rate=(1e-3,), batch_size=32, dtype="bf16", loss="ce")
E.make_job("hip", plan, x, y, folds, cfg, dev).launch().finish()      # warm caches / allocator
torch.cuda.synchronize()

t = time.perf_counter()
for _ in range(N):
    E.make_job("hip", plan, x, y, folds, cfg, dev).launch().finish()
torch.cuda.synchronize()
serial = time.perf_counter() - t

streams = [torch.cuda.Stream(dev) for _ in range(N)]
t = time.perf_counter()
jobs = [E.make_job("hip", plan, x, y, folds, cfg, dev, stream=s) for s in streams]
tl = time.perf_counter()
for j in jobs:
    j.launch()
tq = time.perf_counter()
for j in jobs:
    j.finish()
torch.cuda.synchronize()
conc = time.perf_counter() - t
steps = jobs[0].steps_per_epoch * epochs
print(json.dumps({"N": N, "steps_per_job": steps, "serial_s": serial, "concurrent_s": conc,
                  "speedup": serial / conc, "host_build_s": tl - t, "host_enqueue_s": tq - tl,
                  "serial_ms_per_step": 1000 * serial / (N * steps),
                  "concurrent_ms_per_step": 1000 * conc / (N * steps)}), flush=True)
