"""Time / profile the fold-batched train step of one architecture.

usage: python tools/probe_steps.py [backend] [genes S1-S2] [epochs] [samples]
"""
import os, sys, time, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from gentun_amd.utils.data import make_cifar_like, stratified_kfold
from gentun_amd.models.genome import make_plan
from gentun_amd.models import cnn_engine as E

backend = sys.argv[1] if len(sys.argv) > 1 else "hip"
s1, s2 = (sys.argv[2] if len(sys.argv) > 2 else "101-0101110011").split("-")
epochs = int(sys.argv[3]) if len(sys.argv) > 3 else 1
n = int(sys.argv[4]) if len(sys.argv) > 4 else 10000
dev = torch.device("cuda", 0)
x, y = make_cifar_like(n=n, seed=0)
folds = stratified_kfold(np.argmax(y, 1), 5, seed=0)
plan = make_plan({'S_1': s1, 'S_2': s2}, (3, 5), (32, 32, 3), (20, 50), ((5, 5), (5, 5)), 500, 10)
cfg = E.TrainConfig(epochs=(epochs,), learning_rate=(1e-3,), batch_size=32, dtype="bf16", loss="ce")
job = E.make_job(backend, plan, x, y, folds, cfg, dev)
torch.cuda.synchronize()
t = time.perf_counter()
job.launch(); r = job.finish()
dt = time.perf_counter() - t
steps = job.steps_per_epoch * epochs
print(json.dumps({"backend": backend, "genes": [s1, s2], "steps": steps, "s": dt, "ms_per_step": 1000 * dt / steps,
                  "mflop_fwd_per_sample": plan.forward_flops() / 1e6,
                  "tflops_fwd_bwd": 3 * plan.forward_flops() * 32 * 5 * steps / dt / 1e12,
                  "cat_acc": r["categorical_accuracy"]}), flush=True)
