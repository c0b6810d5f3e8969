"""Host sanitizer runs of the native GBDT engine (SURVEY.md §5.2 -- the
reference has no race detection at all; its GBDT is xgboost's opaque
``xgb.cv``, gentun/models/xgboost_models.py:28-37).

``csrc/gbdt/engine_selftest.cpp`` drives the engine's C ABI over every
objective / metric / sampling path; it is compiled with engine.cpp under
ASan+UBSan and under TSan (the multi-threaded histograms and quantiser) and
run as a plain executable, so no Python or torch code shares the process.
CPU only."""

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRCS = [os.path.join(ROOT, "csrc", "gbdt", "engine.cpp"), os.path.join(ROOT, "csrc", "gbdt", "engine_selftest.cpp")]


@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_gbdt_engine_under_sanitizer(tmp_path, san):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    exe = str(tmp_path / "gbdt_selftest")
    cmd = ["g++", "-O1", "-g", "-std=c++17", "-pthread", "-fno-omit-frame-pointer", "-fsanitize=" + san,
           "-o", exe] + SRCS
    if "undefined" in san:
        cmd.insert(-len(SRCS) - 2, "-fno-sanitize-recover=undefined")
    build = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    if build.returncode != 0 and "cannot find" in build.stderr:
        pytest.skip("sanitizer runtime not installed: " + build.stderr[-200:])
    assert build.returncode == 0, build.stderr[-2000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1", TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0 and "selftest ok" in r.stdout, (r.stdout + r.stderr)[-4000:]
    assert "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
