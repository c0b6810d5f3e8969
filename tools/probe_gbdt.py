"""One GBDT cv call on the GPU path with fixed genes (for rocprofv3).
usage: python tools/probe_gbdt.py [rows] [features] [max_depth] [rounds] [subsample]
env OBJ=binary:logistic METRIC=auc: a binary target (regression target > its median) and that metric."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gentun_amd.models import gbdt, gbdt_hip  # noqa: E402
from gentun_amd.utils.data import make_regression  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
f = int(sys.argv[2]) if len(sys.argv) > 2 else 256
depth = int(sys.argv[3]) if len(sys.argv) > 3 else 10
rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 5
sub = float(sys.argv[5]) if len(sys.argv) > 5 else 1.0
x, y = make_regression(n=n, f=f, seed=0)
gbdt_hip.quantize_device(x)
obj = os.environ.get("OBJ", "reg:linear")
metric = os.environ.get("METRIC", "rmse")
if obj != "reg:linear":
    import numpy as np
    y = (y > np.median(y)).astype(np.float64)
p = {'objective': obj, 'eta': 0.3, 'max_depth': depth, 'subsample': sub, 'min_child_weight': 1, 'eval_metric': metric}
gbdt.cv(p, x, y, num_boost_round=1, nfold=5, seed=0, device="cuda:0")          # warm-up
t0 = time.perf_counter()
h = gbdt.cv(p, x, y, num_boost_round=rounds, nfold=5, seed=0, device="cuda:0")
dt = time.perf_counter() - t0
print(json.dumps({"rows": n, "features": f, "max_depth": depth, "trees": 5 * rounds, "s": round(dt, 3),
                  "ms_per_tree": round(1000 * dt / (5 * rounds), 3), "objective": obj,
                  "test_" + metric: h['test-%s-mean' % metric][-1]}))
