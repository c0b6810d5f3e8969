"""Throughput of population-batched training: P random S=(3,5) candidates
split into jobs of ``pop_batch`` on ``streams`` streams, 1 epoch each.

usage: python tools/probe_pop.py [P] [pop_batch] [streams] [epochs] [samples]
Env: WINO=0/1 (Winograd stage-2 3x3 layers), WFRAG=0/1 (fragment-major conv weights), SHAPE=28,28,1 (MNIST-shaped: the reference default, stored zero-padded to 32 x 32 unless PAD=0),
SPACE=deep, KERNELS=, BN=1, DTYPE=, RESET=, GRAPH=0, WARM=0.
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
from gentun_amd.utils.data import make_cifar_like, make_mnist_like, stratified_kfold

P = int(sys.argv[1]) if len(sys.argv) > 1 else 8
pb = int(sys.argv[2]) if len(sys.argv) > 2 else 8
ns = int(sys.argv[3]) if len(sys.argv) > 3 else 1
epochs = int(sys.argv[4]) if len(sys.argv) > 4 else 1
n = int(sys.argv[5]) if len(sys.argv) > 5 else 10000
dev = torch.device("cuda", 0)
if os.environ.get("WINO") is not None:                # A/B: Winograd stage-2 3x3 layers on (1) / off (0)
    from gentun_amd.models import cnn_hip
    cnn_hip.WINOGRAD = os.environ["WINO"] != "0"
if os.environ.get("WFRAG") is not None:               # A/B: fragment-major conv weight planes on (1) / off (0)
    from gentun_amd.models import cnn_hip as _ch
    _ch.WFRAG = os.environ["WFRAG"] != "0"
if os.environ.get("BNVALUES"):                      # A/B: BatchNorm values per workgroup budget (cnn_kernels)
    from gentun_amd.ops import cnn_kernels as _K
    _K.BN_CHUNK_VALUES = int(os.environ["BNVALUES"])
if os.environ.get("BNCHUNK") == "old":             # A/B: BatchNorm chunks of 512 pixels for every shape (round 5)
    from gentun_amd.ops import cnn_kernels as _K
    _K.bn_chunk_px = lambda H, W, Cp: _K.BN_CHUNK_PX
if os.environ.get("GENTUN_WGRAD_NB"):                 # A/B: force the wgrad band buffers
    from gentun_amd.ops import cnn_kernels as K
    K.lib().gt_wgrad_set_nb(int(os.environ["GENTUN_WGRAD_NB"]))
shape = tuple(int(v) for v in os.environ.get("SHAPE", "32,32,3").split(","))
x, y = make_cifar_like(n=n, seed=0) if shape == (32, 32, 3) else make_mnist_like(n=n, seed=0)
assert tuple(x.shape[1:]) == shape, (x.shape, shape)
folds = stratified_kfold(np.argmax(y, 1), 5, seed=0)
rnd = random.Random(0)
plans = []
deep = os.environ.get("SPACE") == "deep"          # BASELINE cfg 4: S=(3,4,5), kernels (20,50,100)
nodes = (3, 4, 5) if deep else (3, 5)
kernels = (20, 50, 100) if deep else (20, 50)
if os.environ.get("KERNELS"):
    kernels = tuple(int(v) for v in os.environ["KERNELS"].split(","))
for _ in range(P):
    g = {"S_{}".format(s + 1): "".join(rnd.choice("01") for _ in range(k * (k - 1) // 2)) for s, k in enumerate(nodes)}
    plans.append(make_plan(g, nodes, shape, kernels, ((5, 5),) * len(nodes), 500, 10))
cfg = E.TrainConfig(epochs=(epochs,), learning_rate=(1e-3,), batch_size=32, dtype=os.environ.get("DTYPE", "fp32"),
                    loss="ce", reset=os.environ.get("RESET", "all"), batch_norm=os.environ.get("BN", "0") == "1",
                    use_graph=os.environ.get("GRAPH", "1") != "0", pad_images=os.environ.get("PAD", "1") != "0")
streams = [torch.cuda.Stream(dev, priority=int(os.environ.get("MAIN_PRIO", "0"))) for _ in range(ns)]
# warm-up (allocator, code objects); WARM=0 keeps profiles free of the small warm-up job
if os.environ.get("WARM", "1") != "0":
    E.make_population_job("hip", [(plans[0], folds, list(range(5)))], x, y, cfg, dev).launch().finish()
torch.cuda.synchronize()
t = time.perf_counter()
jobs = []
for i in range(0, P, pb):
    members = [(p, folds, list(range(5))) for p in plans[i:i + pb]]
    jobs.append(E.make_population_job("hip", members, x, y, cfg, dev, stream=streams[len(jobs) % ns]))
tb = time.perf_counter()
for j in jobs:
    j.launch()
tl = time.perf_counter()
res = [r for j in jobs for r in j.finish()]
torch.cuda.synchronize()
dt = time.perf_counter() - t
# one "step" = one optimizer step of every fold of every candidate (the
# sequential-fold job runs its folds' steps one fold at a time)
j0 = jobs[0]
steps = (j0.steps_per_epoch if hasattr(j0, "steps_per_epoch") else j0.jobs[0].steps_per_epoch) * epochs
print(json.dumps({"P": P, "pop_batch": pb, "streams": ns, "steps": steps, "s": round(dt, 3),
                  "build_s": round(tb - t, 3), "enqueue_s": round(tl - tb, 3),
                  "ms_per_step": round(1000 * dt / steps, 3), "ms_per_cand_step": round(1000 * dt / steps / P, 4),
                  "cand_per_hour_full_protocol": round(3600 * P / (dt / steps * 6250), 1),
                  "cat_acc": [round(float(np.mean(r["categorical_accuracy"])), 3) for r in res]}), flush=True)
