"""Native GBDT engine (xgb.cv replacement; reference
gentun/models/xgboost_models.py:28-37)."""

import numpy as np
import pytest

from gentun_amd import GeneticAlgorithm, Population, XgboostIndividual, XgboostModel
from gentun_amd.models import gbdt
from gentun_amd.utils import rng
from gentun_amd.utils.data import load_iris_xy, make_regression


def test_quantize_exact_for_few_values():
    x = np.array([[0.5, 3], [0.1, 3], [0.5, 1], [0.9, 2]], np.float32)
    bins, nb = gbdt.quantize(x)
    assert list(nb) == [3, 3]
    assert bins[:, 0].tolist() == [1, 0, 1, 2] and bins[:, 1].tolist() == [2, 2, 0, 1]


def test_stump_fits_step_function():
    x = np.arange(40, dtype=np.float32).reshape(-1, 1)
    y = (x[:, 0] >= 20).astype(np.float32)
    p = {'objective': 'reg:linear', 'eta': 1.0, 'max_depth': 1, 'lambda': 0.0, 'min_child_weight': 0,
         'eval_metric': 'rmse'}
    h = gbdt.cv(p, x, y, num_boost_round=1, nfold=2, seed=0)
    assert h['train-rmse-mean'][0] < 1e-6 and h['test-rmse-mean'][0] < 0.25


def test_history_monotone_and_early_stopping():
    x, y = make_regression(n=3000, f=8, seed=1)
    h = gbdt.cv({'objective': 'reg:squarederror', 'eta': 0.3, 'max_depth': 4}, x, y, num_boost_round=400,
                nfold=3, early_stopping_rounds=10, seed=0)
    tr = h['train-rmse-mean']
    assert all(a >= b - 1e-9 for a, b in zip(tr, tr[1:]))
    te = h['test-rmse-mean']
    assert te[-1] == min(te)                # truncated at the best round
    assert len(te) < 400


def test_against_sklearn_hist_gbm():
    from sklearn.ensemble import HistGradientBoostingRegressor
    from sklearn.model_selection import KFold, cross_val_score
    x, y = make_regression(n=4000, f=8, seed=2)
    h = gbdt.cv({'objective': 'reg:linear', 'eta': 0.1, 'max_depth': 6}, x, y, num_boost_round=300, nfold=3,
                early_stopping_rounds=20, seed=0)
    ours = h['test-rmse-mean'][-1]
    sk = -cross_val_score(HistGradientBoostingRegressor(max_iter=300, learning_rate=0.1), x, y,
                          cv=KFold(3, shuffle=True, random_state=0), scoring='neg_root_mean_squared_error').mean()
    assert ours < 1.25 * sk


def test_objectives_and_metrics():
    x, y = load_iris_xy()
    h = gbdt.cv({'objective': 'multi:softprob', 'eval_metric': 'mlogloss', 'num_class': 3}, x, y,
                num_boost_round=30, nfold=5, seed=0)
    assert h['test-mlogloss-mean'][-1] < 0.4
    yb = (y == 2).astype(np.float64)
    h = gbdt.cv({'objective': 'binary:logistic', 'eval_metric': 'error'}, x, yb, num_boost_round=20, nfold=5)
    assert h['test-error-mean'][-1] < 0.1
    h = gbdt.cv({'objective': 'binary:logistic', 'eval_metric': 'auc', 'scale_pos_weight': 2.0}, x, yb,
                num_boost_round=20, nfold=5)
    assert h['test-auc-mean'][-1] > 0.95
    with pytest.raises(ValueError):
        gbdt.cv({'objective': 'rank:pairwise'}, x, y)


def test_regularisation_genes_take_effect():
    x, y = make_regression(n=2000, f=6, seed=3)
    base = {'objective': 'reg:linear', 'max_depth': 6}
    r0 = gbdt.cv(dict(base), x, y, num_boost_round=20, nfold=3)['train-rmse-mean'][-1]
    for k, v in (('gamma', 50.0), ('min_child_weight', 500), ('lambda', 1000.0), ('alpha', 200.0),
                 ('max_delta_step', 0.01)):
        r = gbdt.cv(dict(base, **{k: v}), x, y, num_boost_round=20, nfold=3)['train-rmse-mean'][-1]
        assert r > r0, k
    a = gbdt.cv(dict(base, subsample=0.5, colsample_bytree=0.5), x, y, num_boost_round=10, nfold=3, seed=1)
    b = gbdt.cv(dict(base, subsample=0.5, colsample_bytree=0.5), x, y, num_boost_round=10, nfold=3, seed=1)
    c = gbdt.cv(dict(base, subsample=0.5, colsample_bytree=0.5), x, y, num_boost_round=10, nfold=3, seed=2)
    assert a == b and a != c


def test_xgboost_model_api_with_pandas():
    import pandas as pd
    x, y = load_iris_xy()
    df = pd.DataFrame(x, columns=list("abcd"))
    m = XgboostModel(df, pd.Series(y), {'eta': 0.3, 'max_depth': 3}, nfold=3, num_boost_round=200,
                     early_stopping_rounds=10)
    v = m.cross_validate()
    assert 0.0 < v < 0.4


def test_iris_ga_baseline_cfg1():
    """BASELINE cfg 1: XGBoost-individual GA on Iris, population 10, CPU."""
    rng.seed(10)
    x, y = load_iris_xy()
    pop = Population(XgboostIndividual, x, y, size=10, additional_parameters={'nfold': 3, 'num_boost_round': 300,
                                                                             'early_stopping_rounds': 20},
                     maximize=False)
    ga = GeneticAlgorithm(pop, verbose=False)
    best = ga.run(2)
    assert best.get_fitness() < 0.35
    assert len(ga.history) == 2


def test_quantize_gpu_layout_matches_and_caches():
    """The GPU path's bins are the CPU engine's row-major bins padded to a
    4-byte row stride, computed once per dataset object (stable cache key);
    the feature-major layout of the engine is the transpose."""
    from gentun_amd.models import gbdt_hip
    from gentun_amd.ops import _lib
    rng = np.random.default_rng(5)
    x = rng.standard_normal((3000, 7)).astype(np.float32)
    x[:, 3] = np.round(x[:, 3])                      # few distinct values -> exact bins
    b, nb = gbdt.quantize(x)
    br, nb2, key = gbdt_hip.quantize_rm(x)
    assert br.shape == (3000, 8) and not br[:, 7].any()
    assert np.array_equal(b, br[:, :7]) and np.array_equal(nb, nb2)
    again = gbdt_hip.quantize_rm(x)
    assert again[0] is br and again[2] == key
    bt = np.zeros((7, 3000), np.uint8)
    nb3 = np.zeros(7, np.int32)
    xc = np.ascontiguousarray(x)
    _lib.gbdt().gbdt_quantize_fm(xc.ctypes.data, 3000, 7, bt.ctypes.data, nb3.ctypes.data)
    assert np.array_equal(b.T, bt)


def test_unsupported_booster_and_unknown_params_raise():
    """The reference forwards ``booster`` to xgb.cv; the engine only has
    gbtree, so gblinear / dart must raise rather than silently train trees."""
    import pytest
    from gentun_amd.models import gbdt
    x = np.random.default_rng(0).standard_normal((64, 3)).astype(np.float32)
    y = x[:, 0].copy()
    for booster in ("gblinear", "dart"):
        with pytest.raises(ValueError, match="booster"):
            gbdt.cv({"booster": booster}, x, y, num_boost_round=2, nfold=2)
    with pytest.raises(ValueError, match="unsupported GBDT parameter"):
        gbdt.cv({"max_leaves": 8}, x, y, num_boost_round=2, nfold=2)
    gbdt.cv({"booster": "gbtree", "silent": 1, "eval_metric": "rmse"}, x, y, num_boost_round=2, nfold=2)


def test_gpu_auc_falls_back_loudly():
    """GPU auc sorts 2 segments per fold (<= 32 folds). Beyond that device='cuda' must say (once)
    that the CV runs on the CPU engine instead of silently changing device.
    The check in gbdt_hip.cv happens before any device call, so it runs on CPU-only hosts too."""
    import warnings
    from gentun_amd.models import gbdt_hip
    x, y = load_iris_xy()
    yb = (y == 2).astype(np.float64)
    assert gbdt_hip.supported(1, [4], nfold=32) and not gbdt_hip.supported(1, [4], nfold=33)
    assert gbdt_hip.supported(1, [2], nfold=40)
    gbdt_hip._WARNED.clear()
    p = {'objective': 'binary:logistic', 'eval_metric': 'auc'}
    with pytest.warns(RuntimeWarning, match="auc with 33 folds"):
        h = gbdt.cv(dict(p), x, yb, num_boost_round=3, nfold=33, device='cuda')
    ref = gbdt.cv(dict(p), x, yb, num_boost_round=3, nfold=33)
    assert h['test-auc-mean'] == ref['test-auc-mean']          # the CPU engine's result
    with warnings.catch_warnings():
        warnings.simplefilter("error")                         # once per (objective, metrics, folds)
        gbdt.cv(dict(p), x, yb, num_boost_round=3, nfold=33, device='cuda')