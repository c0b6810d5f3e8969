import sys, numpy as np
sys.path.insert(0, '/root/repo')
from gentun_amd.models import gbdt
from gentun_amd.utils.data import make_regression
x, y = make_regression(n=20000, f=16, seed=4)
for extra in ({'subsample': 0.8, 'colsample_bytree': 0.7}, {'subsample': 0.8, 'colsample_bylevel': 0.8},
              {'colsample_bytree': 0.7, 'colsample_bylevel': 0.8}):
    p = dict({'objective': 'reg:linear', 'eta': 0.2, 'max_depth': 5}, **extra)
    a = gbdt.cv(p, x, y, num_boost_round=5, nfold=3, seed=0)['test-rmse-mean']
    b = gbdt.cv(p, x, y, num_boost_round=5, nfold=3, seed=0, device='cuda:0')['test-rmse-mean']
    print(extra, np.round(a, 4), np.round(b, 4))
