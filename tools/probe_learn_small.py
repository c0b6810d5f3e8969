"""Small learning-speed probe: HIP vs torch executors on learnable data
(make_image_classification, 1280 samples, 2 folds = 20 steps per epoch),
val loss / categorical accuracy after E epochs.

usage: python tools/probe_learn_small.py [epochs...]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from gentun_amd.models import cnn_engine as E
from gentun_amd.models.genome import make_plan
from gentun_amd.utils.data import make_image_classification, stratified_kfold

dev = torch.device("cuda", 0)
x, y = make_image_classification(n=1280, shape=(32, 32, 3), classes=10, seed=3, noise=0.35, shift=3)
folds = stratified_kfold(np.argmax(y, 1), 2, seed=0)
genes = {'S_1': '000', 'S_2': '0000000000'}
plan = make_plan(genes, (3, 5), (32, 32, 3), (20, 50), ((5, 5), (5, 5)), 500, 10)
for ep in [int(a) for a in sys.argv[1:]] or [1, 3]:
    for backend in ("hip", "torch"):
        for seed in (0, 1):
            for lr in (1e-9, 1e-3):
                cfg = E.TrainConfig(epochs=(ep,), learning_rate=(lr,), batch_size=32, dtype="fp32",
                                    use_graph=backend == "hip", reset="all", seed=seed)
                job = E.make_job(backend, plan, x, y, folds, cfg, dev)
                job.launch()
                r = job.finish()
                print(json.dumps({"epochs": ep, "backend": backend, "seed": seed, "lr": lr,
                                  "val_loss": [round(v, 5) for v in r["val_loss"]],
                                  "cat": [round(v, 4) for v in r["categorical_accuracy"]]}), flush=True)
