"""Validation-accuracy spread of random S=(3,5) candidates on a synthetic
dataset variant (is the bench task discriminative?).

usage: python tools/probe_spread.py P GENERATOR 'JSON kwargs' [epochs] [lr]
  GENERATOR: parts | glyph      e.g.  16 parts '{"distractors": 2}'
Full protocol by default: 5-fold CV on 10k samples, epochs (20,4,1), lr
(1e-3,1e-4,1e-5), batch 32, fp32, concurrent folds. Prints per-candidate
fold categorical accuracies and the spread summary as JSON lines.
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
from gentun_amd.utils import data as D

P = int(sys.argv[1]) if len(sys.argv) > 1 else 16
gen = sys.argv[2] if len(sys.argv) > 2 else "parts"
kw = json.loads(sys.argv[3]) if len(sys.argv) > 3 else {}
epochs = tuple(int(v) for v in (sys.argv[4] if len(sys.argv) > 4 else "20,4,1").split(","))
lrs = tuple(float(v) for v in (sys.argv[5] if len(sys.argv) > 5 else "1e-3,1e-4,1e-5").split(","))
dev = torch.device("cuda", 0)
t0 = time.perf_counter()
if gen == "variant":
    x, y = D.make_variant_classification(n=10000, shape=(32, 32, 3), seed=0, **kw)
elif gen == "compound":
    x, y = D.make_compound_classification(n=10000, shape=(32, 32, 3), seed=0, **kw)
elif gen == "relation":
    x, y = D.make_relation_classification(n=10000, shape=(32, 32, 3), seed=0, **kw)
elif gen == "parts":
    x, y = D.make_parts_classification(n=10000, shape=(32, 32, 3), seed=0, **kw)
else:
    x, y = D.make_glyph_classification(n=10000, shape=(32, 32, 3), seed=0, **kw)
tdata = time.perf_counter() - t0
folds = D.stratified_kfold(np.argmax(y, 1), 5, seed=0)
rnd = random.Random(1)
plans, genes = [], []
for _ in range(P):
    g = {"S_{}".format(s + 1): "".join(rnd.choice("01") for _ in range(k * (k - 1) // 2)) for s, k in enumerate((3, 5))}
    genes.append(g)
    plans.append(make_plan(g, (3, 5), (32, 32, 3), (20, 50), ((5, 5),) * 2, 500, 10))
cfg = E.TrainConfig(epochs=epochs, learning_rate=lrs, batch_size=32, dtype="fp32", reset="all")
t = time.perf_counter()
res = E.make_population_job("hip", [(p, folds, list(range(5))) for p in plans], x, y, cfg, dev).launch().finish()
dt = time.perf_counter() - t
accs = []
for g, r in zip(genes, res):
    ca = r["categorical_accuracy"]
    accs.append(float(np.mean(ca)))
    print(json.dumps({"genes": g, "cat_acc_folds": [round(v, 4) for v in ca], "cat_acc": round(accs[-1], 4),
                      "bin_acc": round(float(np.mean(r["binary_accuracy"])), 5),
                      "fold_collapse": int(sum(v < 0.15 for v in ca))}), flush=True)
a = np.asarray(accs)
print(json.dumps({"summary": True, "generator": gen, "kwargs": kw, "P": P, "epochs": epochs, "train_s": round(dt, 1),
                  "data_s": round(tdata, 1), "min": round(float(a.min()), 4), "max": round(float(a.max()), 4),
                  "mean": round(float(a.mean()), 4), "std": round(float(a.std()), 4),
                  "quartiles": [round(float(q), 4) for q in np.percentile(a, [25, 50, 75])]}), flush=True)
