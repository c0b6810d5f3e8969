"""Measure per-step time of the torch-ops (comparator a) fold-batched train step."""
import os, sys, time, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from gentun_amd.utils.data import make_cifar_like, stratified_kfold
from gentun_amd.models.genome import make_plan
from gentun_amd.models import cnn_engine as E

backend = sys.argv[1] if len(sys.argv) > 1 else "torch"
dev = torch.device("cuda", 0)
x, y = make_cifar_like(n=10000, seed=0)
folds = stratified_kfold(np.argmax(y, 1), 5, seed=0)
res = {}
for genes in ({'S_1': '000', 'S_2': '0000000000'}, {'S_1': '101', 'S_2': '0101110011'}, {'S_1': '111', 'S_2': '1111111111'}):
    plan = make_plan(genes, (3, 5), (32, 32, 3), (20, 50), ((5, 5), (5, 5)), 500, 10)
    cfg = E.TrainConfig(epochs=(1,), learning_rate=(1e-3,), batch_size=32, dtype="bf16")
    job = E.make_job(backend, plan, x, y, folds, cfg, dev)
    job.launch(); job.finish()
    torch.cuda.synchronize()
    t = time.perf_counter()
    job = E.make_job(backend, plan, x, y, folds, cfg, dev)
    job.launch(); r = job.finish()
    dt = time.perf_counter() - t
    key = genes['S_1'] + '-' + genes['S_2']
    res[key] = {"epoch_s": dt, "ms_per_step": 1000 * dt / job.steps_per_epoch, "mflop": plan.forward_flops() / 1e6,
                "cat_acc": r["categorical_accuracy"]}
    print(key, json.dumps(res[key]), flush=True)
