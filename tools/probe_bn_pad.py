"""Padded (32 x 32, BatchNorm statistics over the real 28 x 28 pixels) vs unpadded (generic kernels)
BatchNorm training at several learning rates / optimizers: val loss per fold and the largest relative
difference (tests/test_padded_geometry.py explains why Adam at lr 1e-3 is not a fair comparison)."""
import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np, torch
from gentun_amd.models import cnn_engine as E
from gentun_amd.models.genome import make_plan
from gentun_amd.utils.data import make_image_classification, stratified_kfold
x, y = make_image_classification(n=640, shape=(28, 28, 1), classes=10, seed=5, noise=0.35, shift=2)
folds = stratified_kfold(np.argmax(y, 1), 3, seed=0)
plan = make_plan({'S_1': '101', 'S_2': '0101110011'}, (3, 5), (28, 28, 1), (20, 50), ((5, 5), (5, 5)), 500, 10)
dev = torch.device("cuda", 0)
for lr in (1e-9, 1e-4, 1e-3):
    for opt in ("adam", "sgd"):
        res = {}
        for pad in (True, False):
            cfg = E.TrainConfig(epochs=(1,), learning_rate=(lr,), batch_size=32, dtype="fp32", loss="ce",
                                reset="all", pad_images=pad, batch_norm=True, optimizer=opt)
            job = E.make_job("hip", plan, x, y, folds, cfg, dev)
            job.launch()
            res[pad] = job.finish()
        a, b = np.array(res[True]["val_loss"]), np.array(res[False]["val_loss"])
        print(lr, opt, a, b, np.max(np.abs(a - b) / np.abs(b)), flush=True)
