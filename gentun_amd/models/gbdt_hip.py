"""MI355X GBDT path: host quantisation (C++), histogram / split / partition /
predict kernels on the GPU (csrc/hip/gbdt_hist.hip). Used by
:func:`gentun_amd.models.gbdt.cv` when ``device`` is a CUDA/HIP device;
objectives reg:linear/squarederror, reg:logistic, binary:logistic and the
rmse/mae/logloss/error metrics run on the GPU, anything else falls back to
the CPU engine."""

import ctypes

import numpy as np

from ..ops import _lib

GPU_OBJECTIVES = (0, 1, 2)
GPU_METRICS = (0, 1, 2, 3)


def supported(obj, metrics):
    return obj in GPU_OBJECTIVES and len(metrics) == 1 and int(metrics[0]) in GPU_METRICS


def _fn():
    L = _lib.hip()
    f = L.gbdt_cv_hip
    if not getattr(f, "_typed", False):
        c = ctypes
        f.argtypes = [c.c_void_p, c.c_void_p, c.c_int, c.c_int, c.c_void_p, c.c_void_p, c.c_int, c.c_void_p,
                      c.c_int, c.c_void_p, c.c_int, c.c_int, c.c_int, c.c_ulonglong, c.c_void_p]
        f.restype = c.c_int
        f._typed = True
    return f


_QCACHE = []      # (x object, shape, binsT, nbins): every GA candidate reuses its dataset's bins


def quantize_fm(x):
    """Feature-major uint8 bins [F][n] + bins per feature, cached per dataset
    object (quantisation is per-dataset work, not per-candidate)."""
    for ent in _QCACHE:
        if ent[0] is x and ent[1] == x.shape:
            return ent[2], ent[3]
    xc = np.ascontiguousarray(x, dtype=np.float32)
    n, f = xc.shape
    bins = np.zeros((f, n), np.uint8)
    nb = np.zeros(f, np.int32)
    _lib.gbdt().gbdt_quantize_fm(xc.ctypes.data, n, f, bins.ctypes.data, nb.ctypes.data)
    _QCACHE.append((x, x.shape, bins, nb))
    while len(_QCACHE) > 2:
        _QCACHE.pop(0)
    return bins, nb


def cv(x, y, fold_of, nfold, parr, obj, num_class, marr, nrounds, esr, seed, hist, x_key=None):
    if not supported(obj, marr):
        return None
    bins, nb = quantize_fm(x if x_key is None else x_key)
    fold_of = np.ascontiguousarray(fold_of.astype(np.int32))
    y = np.ascontiguousarray(y.astype(np.float32))
    marr = np.ascontiguousarray(marr.astype(np.int32))
    kept = _fn()(bins.ctypes.data, nb.ctypes.data, x.shape[0], x.shape[1], y.ctypes.data, fold_of.ctypes.data,
                 int(nfold), parr.ctypes.data, int(obj), marr.ctypes.data, len(marr), int(nrounds), int(esr),
                 ctypes.c_ulonglong(seed & 0xFFFFFFFFFFFFFFFF), hist.ctypes.data)
    return kept
