"""Per-parameter gradient errors of the BN step vs fp64 (genome from argv)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np, torch
import test_hip_step_parity as T
from gentun_amd.models import cnn_engine as E
from gentun_amd.models.cnn_hip import HipPopJob
for gi in (1, 2):
    genes = T.GENES[gi]
    x, y, fold, plan = T._setup(genes)
    dev = torch.device("cuda", 0)
    cfg = E.TrainConfig(epochs=(1,), learning_rate=(1.0,), batch_size=32, dropout=0.0, loss="ce", dtype="fp32",
                        optimizer="sgd", momentum=0.9, use_graph=False, batch_norm=True)
    job = HipPopJob(plan, x, y, [fold], cfg, dev, fold_ids=[0])
    job.init_params()
    w0 = T._hip_weights(job)
    job.reset_optimizer(1.0)
    job._new_epoch_order()
    idx = job.epoch_idx[0, 0].cpu()
    job.train_step()
    torch.cuda.synchronize()
    got = T._hip_grads(job)
    xb = torch.from_numpy(np.asarray(x)[idx.numpy()]).permute(0, 3, 1, 2)
    yb = torch.from_numpy(np.asarray(y)[idx.numpy()]).double()
    ref = T._reference_grads(plan, w0, xb, yb, "ce", bn_eps=1e-3)
    print("genes", genes, [L.name + ":" + str(L.slots) + ":" + str(L.rows) + ":xin=" + str(L.xin) for L in job.layers])
    for L in job.layers:
        r = ref[L.name]
        g = got[L.name]
        print("  {:8s} w {:.2e} gamma {:.2e} beta {:.2e}   |g.w| {:.2e} |gamma| {:.2e}".format(
            L.name, T._rel(g[0], r[0]), T._rel(g[2], r[2]), T._rel(g[3], r[3]), r[0].abs().max().item(),
            r[2].abs().max().item()))
