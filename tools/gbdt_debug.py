"""Reproduce test_gbdt_gpu's parameter sequence (CPU vs HIP GBDT)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from gentun_amd.models import gbdt
from gentun_amd.utils.data import make_regression
x, y = make_regression(n=20000, f=16, seed=4)
for p in ({'objective': 'reg:linear', 'eta': 0.3, 'max_depth': 4},
          {'objective': 'reg:linear', 'eta': 0.1, 'max_depth': 6, 'lambda': 3.0, 'alpha': 0.5, 'gamma': 0.1,
           'min_child_weight': 5, 'max_delta_step': 2},
          {'objective': 'reg:linear', 'eta': 0.2, 'max_depth': 5, 'subsample': 0.8, 'colsample_bytree': 0.7,
           'colsample_bylevel': 0.8}):
    a = gbdt.cv(p, x, y, num_boost_round=40, nfold=3, seed=0)['test-rmse-mean']
    b = gbdt.cv(p, x, y, num_boost_round=40, nfold=3, seed=0, device='cuda:0')['test-rmse-mean']
    c = gbdt.cv(p, x, y, num_boost_round=40, nfold=3, seed=0, device='cuda:0')['test-rmse-mean']
    print(np.round(a[:4], 4), np.round(b[:4], 4), np.round(c[:4], 4), flush=True)
