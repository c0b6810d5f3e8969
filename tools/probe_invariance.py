"""Batch invariance at the bench's settings (fp32, bce_compat, hard data):
the first-generation candidates of the bench's seed trained as ONE
population job vs split into jobs of different sizes; prints the per-fold
val_loss / accuracies of each candidate under each split and whether they
are bit-identical. Env A/B: GENTUN_WGRAD_NZ (forced column slices), ...

usage: python tools/probe_invariance.py [n_samples] [ncand] [epochs]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from gentun_amd import GeneticCnnIndividual
from gentun_amd.models import cnn_engine as E
from gentun_amd.models.genome import make_plan
from gentun_amd.utils import rng as grng
from gentun_amd.utils.data import make_cifar_hard, stratified_kfold

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
ncand = int(sys.argv[2]) if len(sys.argv) > 2 else 6
epochs = int(sys.argv[3]) if len(sys.argv) > 3 else 1
dev = torch.device("cuda", 0)
x, y = make_cifar_hard(n=n, seed=0)
folds = stratified_kfold(np.argmax(y, 1), 5, seed=0)
grng.seed(1234)
genes = [GeneticCnnIndividual.generate_random_genes({"S_1": 3, "S_2": 10}) for _ in range(ncand)]
plans = [make_plan(g, (3, 5), (32, 32, 3), (20, 50), ((5, 5), (5, 5)), 500, 10) for g in genes]
cfg = E.TrainConfig(epochs=(epochs,), learning_rate=(1e-3,), batch_size=32, dtype="fp32", loss="bce_compat",
                    reset="all", seed=1234)


def run(split):
    out, i = [], 0
    for size in split:
        members = [(p, folds, list(range(5))) for p in plans[i:i + size]]
        out += E.make_population_job("hip", members, x, y, cfg, dev).launch().finish()
        i += size
    return out


splits = [[ncand], [ncand - 1, 1], [1] * ncand, [2, ncand - 2]]
res = {str(s): run(s) for s in splits}
base = res[str(splits[0])]
for s in splits[1:]:
    r = res[str(s)]
    same = [r[c] == base[c] for c in range(ncand)]
    diff = [max(abs(a - b) for a, b in zip(r[c]["val_loss"], base[c]["val_loss"])) for c in range(ncand)]
    print(json.dumps({"split": s, "bit_identical": same, "max_val_loss_diff": diff}), flush=True)
