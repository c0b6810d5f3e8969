"""MI355X GBDT path: host quantisation (C++), histogram / split / partition /
predict kernels on the GPU (csrc/hip/gbdt_hist.hip: row-major bins, per-node
row segments, smaller-child histograms + subtraction). Used by
:func:`gentun_amd.models.gbdt.cv` when ``device`` is a CUDA/HIP device;
every objective (regression, logistic, binary, multi-class) and every metric
run on the GPU (auc: one radix sort of every fold's margins per round plus a
binary-search rank kernel). The one unsupported case, auc with more than 32
folds, falls back to the CPU engine with a one-time ``RuntimeWarning`` (never
silently)."""

import ctypes
import warnings

import numpy as np

from ..ops import _lib

GPU_OBJECTIVES = (0, 1, 2, 3, 4, 5)      # every objective of models/gbdt.py OBJECTIVES
GPU_METRICS = (0, 1, 2, 3, 4, 5, 6)      # every metric of models/gbdt.py METRICS
AUC, AUC_MAX_FOLDS = 4, 32                # auc sorts 2 segments per fold into a 6-bit segment id


def supported(obj, metrics, nfold=1):
    return (obj in GPU_OBJECTIVES and len(metrics) >= 1 and all(int(m) in GPU_METRICS for m in metrics)
            and not (nfold > AUC_MAX_FOLDS and any(int(m) == AUC for m in metrics)))


def _fn():
    L = _lib.hip()
    f = L.gbdt_cv_hip
    if not getattr(f, "_typed", False):
        c = ctypes
        f.argtypes = [c.c_void_p, c.c_int, c.c_void_p, c.c_int, c.c_int, c.c_void_p, c.c_void_p, c.c_int,
                      c.c_void_p, c.c_int, c.c_int, c.c_void_p, c.c_int, c.c_int, c.c_int, c.c_ulonglong,
                      c.c_longlong, c.c_void_p]
        f.restype = c.c_int
        f._typed = True
    return f


_QCACHE = []      # (x object, shape, bins, nbins, key): every GA candidate reuses its dataset's bins
_KEYS = [0]


def quantize_rm(x):
    """Row-major uint8 bins [n][Fs] (Fs = F rounded up to 4, zero padding) +
    bins per feature + a cache key, computed once per dataset object: the
    device keeps its copy of the bins for that key across candidates."""
    for ent in _QCACHE:
        if ent[0] is x and ent[1] == x.shape:
            return ent[2], ent[3], ent[4]
    xc = np.ascontiguousarray(x, dtype=np.float32)
    n, f = xc.shape
    b = np.zeros((n, f), np.uint8)
    nb = np.zeros(f, np.int32)
    _lib.gbdt().gbdt_quantize(xc.ctypes.data, n, f, b.ctypes.data, nb.ctypes.data)
    fs = (f + 3) // 4 * 4
    if fs != f:
        bp = np.zeros((n, fs), np.uint8)
        bp[:, :f] = b
        b = bp
    _KEYS[0] += 1
    _QCACHE.append((x, x.shape, b, nb, _KEYS[0]))
    while len(_QCACHE) > 2:
        _QCACHE.pop(0)
    return b, nb, _KEYS[0]


_DCACHE = []      # (x object, shape, nbins, key): datasets quantised on the device (G1 kernels)


def _qfn():
    L = _lib.hip()
    f = L.gbdt_quantize_hip
    if not getattr(f, "_typed", False):
        c = ctypes
        f.argtypes = [c.c_void_p, c.c_int, c.c_int, c.c_int, c.c_longlong, c.c_void_p]
        f.restype = c.c_int
        L.gbdt_bins_hip_copy.argtypes = [c.c_longlong, c.c_void_p, c.c_size_t]
        L.gbdt_bins_hip_copy.restype = c.c_int
        f._typed = True
    return f


def quantize_device(x, force=False, ident=None):
    """Quantise ``x`` on the GPU (gbdt_quant.hip: transpose, segmented radix
    sort, cuts, binary-search binning; bit-identical to the CPU engine) into
    the device bins cache. Returns ``(nbins, key, Fs)``; cached per dataset
    object (``ident``, default ``x``)."""
    ident = x if ident is None else ident
    if not force:
        for ent in _DCACHE:
            if ent[0] is ident and ent[1] == x.shape:
                return ent[2], ent[3], ent[4]
    xc = np.ascontiguousarray(x, dtype=np.float32)
    n, f = xc.shape
    fs = (f + 3) // 4 * 4
    nb = np.zeros(f, np.int32)
    _KEYS[0] += 1
    key = _KEYS[0]
    rc = _qfn()(xc.ctypes.data, n, f, fs, key, nb.ctypes.data)
    if rc != 0:
        raise RuntimeError("gbdt_quantize_hip failed ({})".format(rc))
    _DCACHE[:] = [e for e in _DCACHE if not (e[0] is ident)]
    _DCACHE.append((ident, x.shape, nb, key, fs))
    while len(_DCACHE) > 2:
        _DCACHE.pop(0)
    return nb, key, fs


def device_bins(x, key, fs):
    """Copy of the device-resident bins of ``key`` (tests / debugging)."""
    out = np.zeros((x.shape[0], fs), np.uint8)
    _qfn()
    rc = _lib.hip().gbdt_bins_hip_copy(key, out.ctypes.data, out.nbytes)
    if rc != 0:
        raise RuntimeError("bins of key {} not resident ({})".format(key, rc))
    return out


_WARNED = set()


def _warn_fallback(obj, marr, nfold):
    key = (int(obj), tuple(int(m) for m in marr), int(nfold))
    if key in _WARNED:
        return
    _WARNED.add(key)
    warnings.warn("gbdt.cv(device='cuda'): eval_metric auc with {} folds (GPU auc supports <= {}); this "
                  "cross-validation runs on the CPU engine (csrc/gbdt/engine.cpp)".format(nfold, AUC_MAX_FOLDS),
                  RuntimeWarning, stacklevel=3)


def cv(x, y, fold_of, nfold, parr, obj, num_class, marr, nrounds, esr, seed, hist, x_key=None):
    if not supported(obj, marr, nfold):
        _warn_fallback(obj, marr, nfold)
        return None
    xk = x if x_key is None else x_key
    fold_of = np.ascontiguousarray(fold_of.astype(np.int32))
    y = np.ascontiguousarray(y.astype(np.float32))
    marr = np.ascontiguousarray(marr.astype(np.int32))
    for attempt in (0, 1):
        nb, key, fs = quantize_device(x, force=attempt > 0, ident=xk)
        kept = _fn()(None, fs, nb.ctypes.data, x.shape[0], x.shape[1], y.ctypes.data,
                     fold_of.ctypes.data, int(nfold), parr.ctypes.data, int(obj), int(num_class), marr.ctypes.data,
                     len(marr), int(nrounds), int(esr), ctypes.c_ulonglong(seed & 0xFFFFFFFFFFFFFFFF), key,
                     hist.ctypes.data)
        if kept != -7:                       # -7: another dataset evicted the device bins
            return kept
    return kept
