"""Determinism probe of the HIP train step: graph vs graph vs eager, with the
weight-gradient side streams on and off. Prints one JSON line.

usage: [GENTUN_HIP_LIB=...] python tools/probe_determinism.py [reps]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from gentun_amd.models import cnn_engine as E
from gentun_amd.models.genome import make_plan
from gentun_amd.utils.data import make_image_classification, stratified_kfold

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
x, y = make_image_classification(n=600, shape=(32, 32, 3), classes=10, seed=3, noise=0.35, shift=3)
folds = stratified_kfold(np.argmax(y, 1), 3, seed=0)
plan = make_plan({'S_1': '101', 'S_2': '0101110011'}, (3, 5), (32, 32, 3), (20, 50), ((5, 5), (5, 5)), 500, 10)
dev = torch.device("cuda", 0)


def run(use_graph, overlap):
    cfg = E.TrainConfig(epochs=(1, 1), learning_rate=(1e-3, 1e-4), batch_size=32, dtype="bf16", loss="ce",
                        use_graph=use_graph)
    job = E.make_job("hip", plan, x, y, folds, cfg, dev)
    for obj in (job, getattr(job, "job", None), getattr(job, "impl", None)):
        if obj is not None and hasattr(obj, "overlap"):
            obj.overlap = overlap
    job.launch()
    r = job.finish()
    return r["val_loss"]


out = {}
for name, g, ov in [("graph", True, True), ("eager", False, True), ("graph_serial", True, False),
                    ("eager_serial", False, False)]:
    out[name] = [run(g, ov) for _ in range(reps)]
ref = out["graph"][0]
print(json.dumps({"lib": os.environ.get("GENTUN_HIP_LIB", "tree"),
                  "equal_to_graph0": {k: [v == ref for v in vs] for k, vs in out.items()},
                  "val_loss": {k: vs[0] for k, vs in out.items()}}))
