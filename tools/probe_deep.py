"""HIP vs torch-oracle training of 3-stage S=(3,4,5) candidates (BASELINE cfg 4).

env: DTYPE (fp32), BN ("0,1": runs without / with BatchNorm), KERNELS ("20,50,100"),
BACKENDS ("hip,torch"), LRS ("1e-3,1e-4")."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from gentun_amd.models import cnn_engine as E
from gentun_amd.models.genome import make_plan
from gentun_amd.utils.data import make_cifar_like, stratified_kfold
dev = torch.device("cuda", 0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
ep = int(sys.argv[2]) if len(sys.argv) > 2 else 2
dtype = os.environ.get("DTYPE", "fp32")
bns = [bool(int(v)) for v in os.environ.get("BN", "0,1").split(",")]
kernels = tuple(int(v) for v in os.environ.get("KERNELS", "20,50,100").split(","))
backends = os.environ.get("BACKENDS", "hip,torch").split(",")
lrs = [float(v) for v in os.environ.get("LRS", "1e-3,1e-4").split(",")]
x, y = make_cifar_like(n=n, seed=0)
folds = stratified_kfold(np.argmax(y, 1), 3, seed=0)
for genes in ({'S_1': '000', 'S_2': '000000', 'S_3': '0000000000'}, {'S_1': '101', 'S_2': '010110', 'S_3': '0101110011'},
              {'S_1': '111', 'S_2': '111111', 'S_3': '1111111111'}):
    plan = make_plan(genes, (3, 4, 5), (32, 32, 3), kernels, ((5, 5),) * 3, 500, 10)
    for bn in bns:
        for lr in lrs:
            cfg = E.TrainConfig(epochs=(ep,), learning_rate=(lr,), batch_size=32, dtype=dtype, loss="ce",
                                batch_norm=bn, reset="all")
            out = {}
            for be in backends:
                r = E.make_job(be, plan, x, y, folds, cfg, dev).launch().finish()
                out[be] = [round(v, 3) for v in r["categorical_accuracy"]]
            print(json.dumps({"genes": "-".join(genes[k] for k in sorted(genes)), "kernels": kernels, "lr": lr,
                              "batch_norm": bn, "dtype": dtype, **out}), flush=True)
