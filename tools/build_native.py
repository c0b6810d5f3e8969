"""Build every native component in-tree (no JIT cache, no site-packages).

* ``gentun_amd/_native/libgentun_gbdt.so``  -- C++ GBDT engine (host)
* ``gentun_amd/_native/libgentun_hip.so``   -- HIP kernels for gfx950
  (Genetic-CNN conv/pool/dense/loss/Adam + GBDT histogram/split), compiled
  with ``hipcc --offload-arch=gfx950``; cross-compiles on a CPU-only host.

Rebuilds only when a source is newer than its library. Used by
``__graft_entry__.build()`` and lazily by :mod:`gentun_amd.ops._lib`.
"""

import glob
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gentun_amd", "_native")
ARCH = os.environ.get("GENTUN_HIP_ARCH", "gfx950")

TARGETS = {
    "libgentun_gbdt.so": {
        "sources": ["csrc/gbdt/engine.cpp"],
        "deps": [],
        "kind": "cxx",
    },
    # host sanitizer build of the GBDT engine: ASan + UBSan,
    # loaded through GENTUN_GBDT_LIB by tests/test_sanitizers.py
    "libgentun_gbdt_asan.so": {
        "sources": ["csrc/gbdt/engine.cpp"],
        "deps": [],
        "kind": "cxx_asan",
        "optional": True,
    },
    "libgentun_hip.so": {
        "sources": sorted(glob.glob(os.path.join(ROOT, "csrc", "hip", "*.hip"))),
        "deps": sorted(glob.glob(os.path.join(ROOT, "csrc", "hip", "*.h"))),
        "kind": "hip",
    },
}


def _abs(p):
    return p if os.path.isabs(p) else os.path.join(ROOT, p)


def _stale(lib, srcs):
    if not os.path.exists(lib):
        return True
    t = os.path.getmtime(lib)
    return any(os.path.getmtime(s) > t for s in srcs)


def hipcc():
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    return None


def build_target(name, verbose=False, force=False):
    spec = TARGETS[name]
    srcs = [_abs(s) for s in spec["sources"]]
    if not srcs:
        return None
    lib = os.path.join(OUT, name)
    if not force and not _stale(lib, srcs + [_abs(d) for d in spec["deps"]]):
        return lib
    os.makedirs(OUT, exist_ok=True)
    tmp = lib + ".tmp.{}".format(os.getpid())
    if spec["kind"] == "cxx":
        cmd = ["g++", "-O3", "-std=c++17", "-fPIC", "-shared", "-march=x86-64-v2", "-pthread", "-o", tmp] + srcs
    elif spec["kind"] == "cxx_asan":
        cmd = ["g++", "-O1", "-g", "-std=c++17", "-fPIC", "-shared", "-pthread", "-fno-omit-frame-pointer",
               "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-o", tmp] + srcs
    else:
        cc = hipcc()
        if cc is None:
            raise RuntimeError("hipcc not found; cannot build {}".format(name))
        cmd = [cc, "--offload-arch={}".format(ARCH), "-O3", "-std=c++17", "-fPIC", "-shared",
               "-munsafe-fp-atomics", "-I", os.path.join(ROOT, "csrc", "hip"), "-o", tmp] + srcs
    if verbose:
        print("[build]", " ".join(cmd), flush=True)
    subprocess.check_call(cmd, cwd=ROOT)
    os.replace(tmp, lib)
    return lib


def build_all(verbose=False, force=False):
    out = {}
    for name, spec in TARGETS.items():
        if spec.get("optional"):
            continue            # built on demand (sanitizer builds)
        out[name] = build_target(name, verbose=verbose, force=force)
    return out


if __name__ == "__main__":
    res = build_all(verbose=True, force="--force" in sys.argv)
    for k, v in res.items():
        print(k, "->", v)
