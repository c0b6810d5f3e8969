"""Concurrent start-up build (tools/build_native.py): under torchrun every rank
loads the native libraries at start-up, so on a cold or stale tree several
processes call ``build_target`` at once. The file lock must make exactly one
of them compile and every one of them load the same, fresh library."""

import os
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = textwrap.dedent("""
    import sys, time
    sys.path.insert(0, {root!r})
    from tools import build_native as b
    b.OUT = {out!r}
    t_go = {t_go!r}
    while time.time() < t_go:
        time.sleep(0.005)
    lib = b.build_target("libgentun_gbdt.so", verbose=True)
    print("RESULT", lib, b.library_hash(lib), b.source_hash("libgentun_gbdt.so"), flush=True)
""")


def _run_concurrently(out, n):
    import time
    t_go = time.time() + 2.0
    procs = [subprocess.Popen([sys.executable, "-c", CHILD.format(root=ROOT, out=out, t_go=t_go)],
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for _ in range(n)]
    outs = [p.communicate(timeout=600)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs), outs
    return outs


def test_concurrent_builds_compile_once_and_agree(tmp_path):
    out = str(tmp_path / "native")
    os.makedirs(out)
    # a stale library in place: garbage bytes and a wrong stamp
    with open(os.path.join(out, "libgentun_gbdt.so"), "wb") as f:
        f.write(b"not a library")
    with open(os.path.join(out, "libgentun_gbdt.so.srchash"), "w") as f:
        f.write("0" * 32 + "\n")
    outs = _run_concurrently(out, 4)
    builds = sum(o.count("[build]") for o in outs)
    assert builds == 1, outs                       # one compile, the others waited and found it fresh
    results = [line.split()[1:] for o in outs for line in o.splitlines() if line.startswith("RESULT")]
    assert len(results) == 4
    libs = {r[0] for r in results}
    assert len(libs) == 1
    for _, have, want in results:
        assert have == want                        # every process loads the library of this tree
    with open(os.path.join(out, "libgentun_gbdt.so.srchash")) as f:
        assert f.read().strip() == results[0][2]
    # no temporaries left behind
    assert sorted(n for n in os.listdir(out) if ".tmp." in n) == []
    # a second round on the fresh library builds nothing
    outs = _run_concurrently(out, 3)
    assert sum(o.count("[build]") for o in outs) == 0, outs
