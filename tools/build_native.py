"""Build every native component in-tree (no JIT cache, no site-packages).

* ``gentun_amd/_native/libgentun_gbdt.so``  -- C++ GBDT engine (host)
* ``gentun_amd/_native/libgentun_hip.so``   -- HIP kernels for gfx950
  (Genetic-CNN conv/pool/dense/loss/Adam + GBDT histogram/split), compiled
  with ``hipcc --offload-arch=gfx950``; cross-compiles on a CPU-only host.

Staleness is decided by CONTENT, not mtimes: every library is compiled with
``-DGT_SRC_HASH=<sha256 of its sources, headers and compile command>`` and
exports ``gt_build_hash()``; a library whose embedded hash differs from the
current tree is rebuilt, and :mod:`gentun_amd.ops._lib` refuses to load one
(so a stale binary can never run against newer sources, e.g. after a
checkout). Used by ``__graft_entry__.build()`` and lazily by the loader.
"""

import ctypes
import glob
import hashlib
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


def source_hash(name):
    """sha256 over the target's sources + headers (repo-relative paths and
    bytes) and its compile flags: the value baked into the library."""
    spec = TARGETS[name]
    h = hashlib.sha256()
    h.update(spec["kind"].encode())
    h.update(" ".join(_flags(spec["kind"])).encode())
    for f in sorted(set(_abs(x) for x in spec["sources"] + spec["deps"])):
        h.update(os.path.relpath(f, ROOT).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:32]


def library_hash(lib):
    """The GT_SRC_HASH a built library carries (None if unreadable)."""
    try:
        handle = ctypes.CDLL(lib, mode=ctypes.RTLD_LOCAL)
        fn = handle.gt_build_hash
        fn.restype = ctypes.c_char_p
        return fn().decode()
    except (OSError, AttributeError):
        return None


def _stamp(lib):
    return lib + ".srchash"


def _stale(name, lib):
    if not os.path.exists(lib):
        return True
    want = source_hash(name)
    # the stamp file avoids dlopen()ing a multi-MB library just to compare
    try:
        with open(_stamp(lib)) as f:
            if f.read().strip() != want:
                return True
    except OSError:
        return True
    return library_hash(lib) != want


def _flags(kind):
    if kind == "cxx":
        return ["-O3", "-std=c++17", "-fPIC", "-shared", "-march=x86-64-v2", "-pthread"]
    if kind == "cxx_asan":
        return ["-O1", "-g", "-std=c++17", "-fPIC", "-shared", "-pthread", "-fno-omit-frame-pointer",
                "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"]
    return ["--offload-arch={}".format(ARCH), "-O3", "-std=c++17", "-fPIC", "-shared", "-munsafe-fp-atomics"]


def hipcc():
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    return None


class _BuildLock(object):
    """Exclusive ``fcntl.flock`` on ``<OUT>/.<name>.lock`` around one target's
    staleness check + build: under ``torchrun`` every rank loads the library
    at start-up, and on a cold or stale tree they would otherwise run hipcc
    concurrently into the same object files. The first rank builds, the others
    block, then find the library fresh and load it."""

    def __init__(self, name):
        os.makedirs(OUT, exist_ok=True)
        self.path = os.path.join(OUT, "." + name + ".lock")
        self.fd = None

    def __enter__(self):
        import fcntl
        self.fd = os.open(self.path, os.O_RDWR | os.O_CREAT, 0o666)
        fcntl.flock(self.fd, fcntl.LOCK_EX)
        return self

    def __exit__(self, *exc):
        import fcntl
        fcntl.flock(self.fd, fcntl.LOCK_UN)
        os.close(self.fd)
        return False


def build_target(name, verbose=False, force=False):
    spec = TARGETS[name]
    srcs = [_abs(s) for s in spec["sources"]]
    if not srcs:
        return None
    lib = os.path.join(OUT, name)
    if not force and not _stale(name, lib):
        return lib
    with _BuildLock(name):
        # re-checked under the lock: another process may have built it while this one waited
        if not force and not _stale(name, lib):
            return lib
        return _build_locked(name, spec, srcs, lib, verbose)


def _build_locked(name, spec, srcs, lib, verbose):
    tmp = lib + ".tmp.{}".format(os.getpid())
    want = source_hash(name)
    hflag = ['-DGT_SRC_HASH="{}"'.format(want)]
    if spec["kind"] in ("cxx", "cxx_asan"):
        cmd = ["g++"] + _flags(spec["kind"]) + hflag + ["-o", tmp] + srcs
    else:
        cc = hipcc()
        if cc is None:
            raise RuntimeError("hipcc not found; cannot build {}".format(name))
        # one object per translation unit, compiled in parallel, then linked (per-pid object
        # directory: nothing outside the lock ever sees a half-written object)
        objdir = os.path.join(ROOT, "build", "obj_{}_{}".format(name.split(".")[0], os.getpid()))
        os.makedirs(objdir, exist_ok=True)
        comp = [cc] + [f for f in _flags("hip") if f != "-shared"] + hflag + ["-I", os.path.join(ROOT, "csrc", "hip")]
        objs, cmds = [], []
        for src in srcs:
            obj = os.path.join(objdir, os.path.basename(src) + ".o")
            objs.append(obj)
            cmds.append(comp + ["-c", "-o", obj, src])
        from concurrent.futures import ThreadPoolExecutor
        jobs = max(1, min(len(cmds), int(os.environ.get("MAX_JOBS", "0")) or (os.cpu_count() or 4)))
        with ThreadPoolExecutor(jobs) as ex:
            for c in cmds:
                if verbose:
                    print("[build]", " ".join(c), flush=True)
            list(ex.map(lambda c: subprocess.check_call(c, cwd=ROOT), cmds))
        cmd = [cc, "--offload-arch={}".format(ARCH), "-shared", "-fPIC", "-o", tmp] + objs
    if verbose:
        print("[build]", " ".join(cmd), flush=True)
    subprocess.check_call(cmd, cwd=ROOT)
    if spec["kind"] == "hip":
        # the objects of the library now in place (tools/build_ab.sh ONLY= links against them)
        final = os.path.join(ROOT, "build", "obj_" + name.split(".")[0])
        shutil.rmtree(final, ignore_errors=True)
        os.replace(objdir, final)
    # the stamp goes first, atomically, then the library: a reader that sees the new library also
    # sees its stamp (a stamp newer than the library only triggers a rebuild check, which the
    # embedded hash then settles)
    stmp = _stamp(lib) + ".tmp.{}".format(os.getpid())
    with open(stmp, "w") as f:
        f.write(want + "\n")
    os.replace(stmp, _stamp(lib))
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
