"""Host-launch overhead of the population train step: seconds per epoch at
P candidates, fold mode RESET (all / kernels) and k train steps per graph
replay (GENTUN_GRAPH_STEPS), one process for the whole sweep.

usage: python tools/probe_graph.py "1,2,5,10" "1,10,50" "all,kernels" [samples]
Prints one JSON line per configuration: wall s, host enqueue s, ms per step.
"""
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from gentun_amd.models import cnn_engine as E
from gentun_amd.models.genome import make_plan
from gentun_amd.utils.data import make_cifar_like, stratified_kfold

Ps = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "2,5").split(",")]
Ks = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "1,10").split(",")]
modes = (sys.argv[3] if len(sys.argv) > 3 else "all").split(",")
n = int(sys.argv[4]) if len(sys.argv) > 4 else 10000
dev = torch.device("cuda", 0)
x, y = make_cifar_like(n=n, seed=0)
folds = stratified_kfold(np.argmax(y, 1), 5, seed=0)
rnd = random.Random(0)
plans = []
for _ in range(max(Ps)):
    g = {"S_{}".format(s + 1): "".join(rnd.choice("01") for _ in range(k * (k - 1) // 2)) for s, k in enumerate((3, 5))}
    plans.append(make_plan(g, (3, 5), (32, 32, 3), (20, 50), ((5, 5),) * 2, 500, 10))

# warm-up: code objects, allocator
cfg0 = E.TrainConfig(epochs=(1,), learning_rate=(1e-3,), batch_size=32, dtype="fp32", reset="all")
E.make_population_job("hip", [(plans[0], folds[:1], [0])], x, y, cfg0, dev).launch().finish()
torch.cuda.synchronize()
for mode in modes:
    for P in Ps:
        for k in Ks:
            os.environ["GENTUN_GRAPH_STEPS"] = str(k)
            cfg = E.TrainConfig(epochs=(1,), learning_rate=(1e-3,), batch_size=32, dtype="fp32", reset=mode)
            torch.cuda.synchronize()
            t = time.perf_counter()
            job = E.make_population_job("hip", [(p, folds, list(range(5))) for p in plans[:P]], x, y, cfg, dev)
            job.launch()
            tl = time.perf_counter()
            res = job.finish()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
            jobs = job.jobs if hasattr(job, "jobs") else [job]
            steps = sum(j.steps_per_epoch for j in jobs)
            ph = E._sum_phases(jobs) or {}
            print(json.dumps({"mode": mode, "P": P, "groups_per_launch": P * (5 if mode == "all" else 1),
                              "graph_steps": jobs[0]._k_steps, "steps": steps, "s": round(dt, 3),
                              "enqueue_s": round(tl - t, 3), "ms_per_step": round(1000 * dt / steps, 3),
                              "train_ms_per_step": round(ph.get("train", 0.0) / steps, 3),
                              "cand_per_hour_full_protocol": round(3600 * P / (dt / steps * 6250 * (1 if mode == "all" else 5)), 1),
                              "cat_acc": [round(float(np.mean(r["categorical_accuracy"])), 3) for r in res]}), flush=True)
