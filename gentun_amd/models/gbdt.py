"""Python front-end of the native GBDT engine (``xgb.cv`` replacement).

``cv(params, x, y, num_boost_round, nfold, early_stopping_rounds, seed)``
returns a dict of per-round lists ``{'train-<m>-mean', 'train-<m>-std',
'test-<m>-mean', 'test-<m>-std'}`` truncated at the best round when early
stopping is on -- the shape ``xgb.cv`` returns as a DataFrame (reference
call site gentun/models/xgboost_models.py:32-37).

Folds: shuffled, non-stratified k-fold with the given seed (xgboost 0.72
``cv`` defaults: ``shuffle=True``, ``stratified=False``, ``seed=0``).
"""

import ctypes

import numpy as np

from ..ops import _lib
from ..utils.data import kfold

OBJECTIVES = {
    "reg:linear": 0, "reg:squarederror": 0, "reg:logistic": 1, "binary:logistic": 2, "binary:logitraw": 3,
    "multi:softmax": 4, "multi:softprob": 5,
}
METRICS = {"rmse": 0, "mae": 1, "logloss": 2, "error": 3, "auc": 4, "merror": 5, "mlogloss": 6}
DEFAULT_METRIC = {0: "rmse", 1: "rmse", 2: "logloss", 3: "logloss", 4: "merror", 5: "mlogloss"}
PARAM_ORDER = ("eta", "min_child_weight", "max_depth", "gamma", "max_delta_step", "subsample",
               "colsample_bytree", "colsample_bylevel", "lambda", "alpha", "scale_pos_weight", "base_score")
DEFAULTS = {"eta": 0.3, "min_child_weight": 1.0, "max_depth": 6, "gamma": 0.0, "max_delta_step": 0.0,
            "subsample": 1.0, "colsample_bytree": 1.0, "colsample_bylevel": 1.0, "lambda": 1.0, "alpha": 0.0,
            "scale_pos_weight": 1.0, "base_score": 0.5}
ALIASES = {"learning_rate": "eta", "reg_lambda": "lambda", "reg_alpha": "alpha", "min_split_loss": "gamma"}


def _as_arrays(x, y):
    x = np.ascontiguousarray(np.asarray(x, dtype=np.float32))
    y = np.ascontiguousarray(np.asarray(y, dtype=np.float32).reshape(-1))
    if x.ndim != 2 or x.shape[0] != y.shape[0]:
        raise ValueError("x must be 2-D with as many rows as y")
    return x, y


# keys the engine accepts without using: xgboost plumbing / verbosity knobs
IGNORED = {"silent", "verbosity", "nthread", "n_jobs", "seed", "random_state", "tree_method", "eval_metric",
           "objective", "booster", "num_class", "disable_default_eval_metric"}


def resolve_params(params):
    """Engine parameters from an xgboost-style dict. Only ``booster='gbtree'``
    exists here (the reference forwards ``booster`` to xgb.cv,
    gentun/models/xgboost_models.py:16-22): gblinear / dart raise instead of
    silently training trees, and unknown keys raise too."""
    booster = params.get("booster", "gbtree")
    if booster != "gbtree":
        raise ValueError("booster {!r} is not supported: the native engine implements gbtree only".format(booster))
    p = dict(DEFAULTS)
    for k, v in params.items():
        k = ALIASES.get(k, k)
        if k in p:
            p[k] = float(v)
        elif k not in IGNORED:
            raise ValueError("unsupported GBDT parameter {!r}".format(k))
    obj = params.get("objective", "reg:linear")
    if obj not in OBJECTIVES:
        raise ValueError("unsupported objective {!r}".format(obj))
    return p, OBJECTIVES[obj]


def cv(params, x, y, num_boost_round=10, nfold=3, early_stopping_rounds=None, seed=0, device=None,
       nthreads=0, folds=None):
    x_key = x                     # dataset identity: the GPU path caches its bins per dataset
    x, y = _as_arrays(x, y)
    p, obj = resolve_params(params)
    num_class = int(params.get("num_class", 0) or 0)
    if obj in (4, 5) and num_class < 2:
        num_class = int(y.max()) + 1
    metric = params.get("eval_metric") or DEFAULT_METRIC[obj]
    metrics = [metric] if isinstance(metric, str) else list(metric)
    for m in metrics:
        if m not in METRICS:
            raise ValueError("unsupported eval_metric {!r}".format(m))
    n = x.shape[0]
    if folds is None:
        folds = kfold(n, nfold, seed=seed)
    fold_of = np.full(n, -1, np.int32)
    for k, (_tr, va) in enumerate(folds):
        fold_of[va] = k
    nrounds = int(num_boost_round)
    hist = np.zeros((nrounds, len(metrics), 4), np.float64)
    parr = np.array([p[k] for k in PARAM_ORDER], np.float64)
    marr = np.array([METRICS[m] for m in metrics], np.int32)
    kept = None
    if device is not None and str(device).startswith("cuda"):
        from . import gbdt_hip
        kept = gbdt_hip.cv(x, y, fold_of, len(folds), parr, obj, num_class, marr, nrounds,
                           early_stopping_rounds or 0, seed, hist, x_key=x_key)
    if kept is None:
        lib = _lib.gbdt()
        kept = lib.gbdt_cv(x.ctypes.data, n, x.shape[1], y.ctypes.data, fold_of.ctypes.data, len(folds),
                           parr.ctypes.data, obj, num_class, marr.ctypes.data, len(metrics), nrounds,
                           int(early_stopping_rounds or 0), ctypes.c_ulonglong(seed & 0xFFFFFFFFFFFFFFFF),
                           int(nthreads), hist.ctypes.data)
    if kept < 0:
        raise RuntimeError("gbdt_cv failed ({})".format(kept))
    out = {}
    for j, m in enumerate(metrics):
        out["train-{}-mean".format(m)] = hist[:kept, j, 0].tolist()
        out["train-{}-std".format(m)] = hist[:kept, j, 1].tolist()
        out["test-{}-mean".format(m)] = hist[:kept, j, 2].tolist()
        out["test-{}-std".format(m)] = hist[:kept, j, 3].tolist()
    return out


def quantize(x):
    x, _ = _as_arrays(x, np.zeros(len(x)))
    n, f = x.shape
    bins = np.zeros((n, f), np.uint8)
    nb = np.zeros(f, np.int32)
    _lib.gbdt().gbdt_quantize(x.ctypes.data, n, f, bins.ctypes.data, nb.ctypes.data)
    return bins, nb
