"""Loader for the in-tree native libraries (built by ``tools/build_native.py``).

The libraries are plain shared objects with a C ABI, loaded with ctypes:
the HIP kernels take raw device pointers plus the ``hipStream_t`` of the
caller's current torch stream, so they are captured into HIP graphs exactly
like torch's own launches. If a library is missing it is built on first use
(hipcc cross-compiles without a GPU); on a GPU box a missing or unloadable
HIP library is a hard error -- there is no silent fallback.
"""

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
NATIVE_DIR = os.path.join(os.path.dirname(_HERE), "_native")
_LOCK = threading.Lock()
_LIBS = {}


def _path(name):
    return os.path.join(NATIVE_DIR, name)


def _ensure_built(name):
    import sys
    root = os.path.dirname(os.path.dirname(_HERE))
    if root not in sys.path:
        sys.path.insert(0, root)
    from tools import build_native
    return build_native.build_target(name)


def load(name):
    with _LOCK:
        lib = _LIBS.get(name)
        if lib is not None:
            return lib
        path = _path(name)
        if os.environ.get("GENTUN_NO_AUTOBUILD") != "1":
            try:
                _ensure_built(name)
            except Exception as exc:  # noqa: BLE001
                if not os.path.exists(path):
                    raise RuntimeError("native library {} missing and build failed: {}".format(name, exc))
        if not os.path.exists(path):
            raise RuntimeError("native library {} not found at {}".format(name, path))
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        _check_hash(name, lib)
        _LIBS[name] = lib
        return lib


def _check_hash(name, lib):
    """Refuse a library built from other sources than the tree's (a stale
    binary must never run silently). Skipped when the sources are absent
    (installed package)."""
    import sys
    root = os.path.dirname(os.path.dirname(_HERE))
    if not os.path.isdir(os.path.join(root, "csrc")):
        return
    if root not in sys.path:
        sys.path.insert(0, root)
    from tools import build_native
    if name not in build_native.TARGETS:
        return
    fn = lib.gt_build_hash
    fn.restype = ctypes.c_char_p
    have, want = fn().decode(), build_native.source_hash(name)
    if have != want:
        raise RuntimeError("native library {} is stale (built from sources {}, tree is {}): run "
                           "python tools/build_native.py".format(name, have, want))


def gbdt():
    """The C++ GBDT engine. ``GENTUN_GBDT_LIB`` names an alternative build of
    it (e.g. ``libgentun_gbdt_asan.so``, the host ASan/UBSan build)."""
    alt = os.environ.get("GENTUN_GBDT_LIB")
    lib = load(os.path.basename(alt) if alt else "libgentun_gbdt.so")
    if not getattr(lib, "_typed", False):
        c = ctypes
        lib.gbdt_cv.restype = c.c_int
        lib.gbdt_cv.argtypes = [c.c_void_p, c.c_int, c.c_int, c.c_void_p, c.c_void_p, c.c_int, c.c_void_p,
                                c.c_int, c.c_int, c.c_void_p, c.c_int, c.c_int, c.c_int, c.c_ulonglong, c.c_int,
                                c.c_void_p]
        lib.gbdt_quantize.restype = c.c_int
        lib.gbdt_quantize.argtypes = [c.c_void_p, c.c_int, c.c_int, c.c_void_p, c.c_void_p]
        lib.gbdt_quantize_fm.restype = c.c_int
        lib.gbdt_quantize_fm.argtypes = [c.c_void_p, c.c_int, c.c_int, c.c_void_p, c.c_void_p]
        lib._typed = True
    return lib


def hip():
    """The gfx950 kernel library (raises if it cannot be loaded).
    ``GENTUN_HIP_LIB`` points at an alternative build (kernel tuning runs)."""
    alt = os.environ.get("GENTUN_HIP_LIB")
    if alt:
        global _ALT
        if _ALT is None:
            _ALT = ctypes.CDLL(os.path.abspath(alt))
        return _ALT
    return load("libgentun_hip.so")


_ALT = None


def load_all(require_gpu=False):
    out = {"gbdt": gbdt()}
    try:
        out["hip"] = hip()
    except Exception:
        if require_gpu:
            raise
    return out
