"""Learning-curve probe: train one architecture fold-batched and print the
validation loss / binary / categorical accuracy after every epoch.

usage: python tools/probe_learning.py [--noise 1.2] [--epochs 20,4,1] [--genes S_1=101,S_2=0101110011]
                                      [--backend hip] [--loss bce_compat] [--samples 10000]
"""
import argparse
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--noise", type=float, default=1.0)
    ap.add_argument("--shift", type=int, default=5)
    ap.add_argument("--epochs", default="20,4,1")
    ap.add_argument("--lr", default="1e-3,1e-4,1e-5")
    ap.add_argument("--genes", default="S_1=101,S_2=0101110011")
    ap.add_argument("--backend", default="hip")
    ap.add_argument("--loss", default="bce_compat")
    ap.add_argument("--samples", type=int, default=10000)
    ap.add_argument("--nfold", type=int, default=5)
    a = ap.parse_args()
    genes = dict(kv.split("=") for kv in a.genes.split(","))
    dev = torch.device("cuda", 0)
    x, y = make_cifar_like(n=a.samples, seed=0, noise=a.noise, shift=a.shift)
    folds = stratified_kfold(np.argmax(y, 1), a.nfold, seed=0)
    plan = make_plan(genes, (3, 5), (32, 32, 3), (20, 50), ((5, 5), (5, 5)), 500, 10)
    epochs = [int(e) for e in a.epochs.split(",")]
    lrs = [float(v) for v in a.lr.split(",")]
    cfg = E.TrainConfig(epochs=(1,), learning_rate=(lrs[0],), batch_size=32, dtype="bf16", loss=a.loss)
    job = E.make_job(a.backend, plan, x, y, folds, cfg, dev)
    job.init_params()
    ep = 0
    t0 = time.perf_counter()
    for n, lr in zip(epochs, lrs):
        job.reset_optimizer(lr)
        for _ in range(n):
            job._new_epoch_order()
            for _ in range(job.steps_per_epoch):
                job.train_step()
            ep += 1
            job._eval = job.evaluate()
            job._done = None
            torch.cuda.synchronize()
            r = job.finish()
            print(json.dumps({"epoch": ep, "lr": lr, "noise": a.noise, "genes": genes,
                              "val_loss": float(np.mean(r["val_loss"])),
                              "bin_acc": float(np.mean(r["binary_accuracy"])),
                              "cat_acc": float(np.mean(r["categorical_accuracy"])),
                              "s": round(time.perf_counter() - t0, 2)}), flush=True)


if __name__ == "__main__":
    main()
