"""Dead and hung ranks: a rank that exits or stops
answering mid-generation ends the attempt (gloo error or the per-rank
watchdog, exit 75), torchrun restarts the group in fresh processes
(``--max-restarts``) and the CLI resumes from the last generation checkpoint
(``--resume auto``): the GA trajectory equals an uninterrupted run's.
Real processes on gloo (CPU stand-in for RCCL); the reference's broker
redelivers a dead worker's job (gentun/worker.py:50-55)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _search(tmp, fault=None, restarts=0, watchdog="60:3:4"):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    env.pop("GENTUN_FAULT", None)
    if fault:
        env["GENTUN_FAULT"] = fault
        env["GENTUN_FAULT_ATTEMPT"] = "0"          # inject on the first attempt only
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--max-restarts={}".format(restarts), "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           "-m", "gentun_amd", "xgb", "--data", "iris", "--pop", "8", "--gens", "4", "--nfold", "3",
           "--rounds", "15", "--early-stopping", "5", "--seed", "5", "--backend", "gloo",
           "--checkpoint-dir", str(tmp), "--resume", "auto", "--watchdog", watchdog]
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=900, cwd=ROOT)
    out = None
    for line in r.stdout.splitlines():
        # (another rank's unflushed text can share the line under load: parse from the brace)
        if '{"' in line:
            try:
                out = json.loads(line[line.index('{"'):])
            except ValueError:
                pass
    return r, out


def _trajectory(out):
    assert out is not None, "no result JSON on stdout"
    return [(h["generation"], h["best_fitness"]) for h in out["history"]]


@pytest.fixture(scope="module")
def clean_run(tmp_path_factory):
    r, out = _search(tmp_path_factory.mktemp("clean"))
    assert r.returncode == 0, r.stderr[-3000:]
    return out


@pytest.mark.parametrize("kind", ["exit", "hang"])
def test_killed_or_hung_rank_run_completes_from_checkpoint(tmp_path, clean_run, kind):
    r, out = _search(tmp_path, fault="1:2:" + kind, restarts=1)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "injected {} on rank 1 generation 2".format(kind) in r.stderr
    if kind == "hang":
        assert "[watchdog]" in r.stderr                     # the stuck group was ended by the deadline
    assert _trajectory(out) == _trajectory(clean_run)
    assert out["best_genes"] == clean_run["best_genes"]
    assert os.path.exists(os.path.join(str(tmp_path), "gen_00004.json"))


def test_failed_share_is_retried_on_the_survivors(tmp_path, clean_run):
    """Every unit of rank 1 raises in one dispatch: the failed units are
    re-dispatched as a second round on the surviving rank (not retrained by
    rank 0 while the evaluators wait in a collective), so a TIGHT watchdog
    (factor 1.5 over the slowest dispatch) never fires, and the trajectory is
    the clean run's (serial rank-0 retries outlived the evaluators'
    deadlines)."""
    r, out = _search(tmp_path, fault="1:2:raise", restarts=0, watchdog="60:1.5:2")
    assert r.returncode == 0, r.stderr[-4000:]
    assert "injected fault on rank 1 generation 2" in r.stderr
    assert "[watchdog]" not in r.stderr
    assert _trajectory(out) == _trajectory(clean_run)


def test_blank_watchdog_spec_is_disabled_and_bad_spec_is_rejected():
    from gentun_amd.parallel.fault import parse_watchdog
    assert parse_watchdog(None) is None and parse_watchdog("") is None and parse_watchdog("  ") is None
    assert parse_watchdog("0") is None
    assert parse_watchdog("30:2:5") == {"first_s": 30.0, "factor": 2.0, "min_s": 5.0}
    with pytest.raises(ValueError, match="GENTUN_WATCHDOG"):
        parse_watchdog("soon")


def test_without_restarts_a_dead_rank_fails_fast(tmp_path):
    """No supervisor: the run ends with an error well before the 30-minute
    collective timeout (gloo connection error / watchdog), not a hang."""
    r, _ = _search(tmp_path, fault="1:2:hang", restarts=0, watchdog="30:3:4")
    assert r.returncode != 0


def test_supervisor_restarts_a_single_process_run(tmp_path):
    """python -m gentun_amd.parallel.fault -- CMD: fresh-process restarts for
    runs without torchrun (never an exec of a process that held the GPU)."""
    from gentun_amd.parallel import fault
    marker = tmp_path / "attempts"
    script = ("import os,sys; p={!r}; n=int(open(p).read()) if os.path.exists(p) else 0; "
              "open(p,'w').write(str(n+1)); sys.exit(0 if n >= 2 else 75)").format(str(marker))
    rc = fault.supervise([sys.executable, "-c", script], max_restarts=3)
    assert rc == 0 and marker.read_text() == "3"
    assert fault.supervise([sys.executable, "-c", "import sys; sys.exit(4)"], max_restarts=1) == 4
