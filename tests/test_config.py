"""RunConfig (gentun_amd/config.py): defaults, GENTUN_* overrides, validation,
and the CLI precedence flag > environment > default."""

import pytest

from gentun_amd.config import RunConfig


def test_defaults_match_reference_semantics():
    c = RunConfig()
    assert (c.loss, c.pairing, c.dtype, c.schedule) == ("bce_compat", "reference", "fp32", "auto")
    assert c.collective_timeout_s > 0 and c.backend is None


def test_env_overrides_and_types():
    env = {"GENTUN_SEED": "7", "GENTUN_LOSS": "ce", "GENTUN_POP_BATCH": "8", "GENTUN_PAIRING": "disjoint",
           "GENTUN_CHECKPOINT_DIR": "/tmp/ck", "GENTUN_DIST_BACKEND": "gloo", "GENTUN_STREAMS": ""}
    c = RunConfig.from_env(env)
    assert c.seed == 7 and isinstance(c.seed, int)
    assert (c.loss, c.pop_batch, c.pairing, c.checkpoint_dir, c.backend) == ("ce", 8, "disjoint", "/tmp/ck", "gloo")
    assert c.streams == 1                                   # empty variable = unset
    assert RunConfig.from_env(env, seed=3, loss=None).seed == 3     # explicit overrides win, None = keep


@pytest.mark.parametrize("bad", [{"loss": "mse"}, {"pairing": "x"}, {"dtype": "fp16"}, {"streams": 0},
                                 {"schedule": "round_robin"}, {"backend": "mpi"}])
def test_validation(bad):
    with pytest.raises(ValueError):
        RunConfig(**bad)


def test_roundtrip_json():
    import json
    c = RunConfig(seed=5, events="e.jsonl")
    assert RunConfig(**json.loads(c.to_json())) == c
    assert c.replace(seed=6).seed == 6 and c.seed == 5


def test_cli_precedence(monkeypatch):
    import argparse
    from gentun_amd import __main__ as cli
    monkeypatch.setenv("GENTUN_POP_BATCH", "4")
    monkeypatch.setenv("GENTUN_PAIRING", "disjoint")
    ap = argparse.ArgumentParser()
    cli._common(ap)
    args = ap.parse_args(["--pop-batch", "2"])
    cfg = cli._config(args)
    assert cfg.pop_batch == 2 and cfg.pairing == "disjoint" and cfg.streams == 1


@pytest.mark.parametrize("exc,expect", [("all_failed", "search_failed"), ("oserror", "propagates")])
def test_cli_maps_only_all_failed_to_the_final_exit(monkeypatch, tmp_path, exc, expect):
    """Only AllEvaluationsFailed becomes the non-restartable exit code 78; any
    other error (checkpoint OSError, HIP launch failure, dead peer) propagates,
    so the supervisor restarts the run from its checkpoint."""
    from gentun_amd import __main__ as cli
    from gentun_amd.algorithms import GeneticAlgorithm
    from gentun_amd.parallel.distributed import AllEvaluationsFailed
    from gentun_amd.parallel.fault import EXIT_SEARCH_FAILED
    monkeypatch.delenv("WORLD_SIZE", raising=False)

    def boom(self, n):
        raise AllEvaluationsFailed("x") if exc == "all_failed" else OSError("disk full")

    monkeypatch.setattr(GeneticAlgorithm, "run", boom)
    argv = ["xgb", "--data", "iris", "--pop", "2", "--gens", "1", "--algorithm", "tournament",
            "--checkpoint-dir", str(tmp_path)]
    if expect == "search_failed":
        with pytest.raises(SystemExit) as e:
            cli.main(argv)
        assert e.value.code == EXIT_SEARCH_FAILED
    else:
        # without a torchrun agent the evaluator ranks are released before the error propagates
        from gentun_amd.parallel.distributed import DistributedPopulation
        calls = []
        monkeypatch.delenv("TORCHELASTIC_USE_AGENT_STORE", raising=False)
        monkeypatch.setattr(DistributedPopulation, "shutdown", lambda self: calls.append(1))
        with pytest.raises(OSError):
            cli.main(argv)
        assert calls == [1]


def test_every_env_variable_is_registered():
    """The framework reads no GENTUN_* variable that config.ENV_VARS does not document (no hidden A/B
    switches in the hot path, verdict r4)."""
    import pathlib
    import re
    from gentun_amd.config import ENV_VARS, RunConfig
    root = pathlib.Path(__file__).resolve().parent.parent
    pat = re.compile(r"GENTUN_[A-Z0-9_]+")
    found = set()
    for sub in ("gentun_amd", "csrc", "examples"):          # (tools/ are development scripts)
        for f in (root / sub).rglob("*"):
            if f.suffix in (".py", ".hip", ".h", ".cpp") and "__pycache__" not in f.parts:
                found |= set(pat.findall(f.read_text(errors="ignore")))
    for f in ("bench.py", "__graft_entry__.py"):
        found |= set(pat.findall((root / f).read_text()))
    assert set(RunConfig.ENV) <= set(ENV_VARS)
    assert found <= set(ENV_VARS), sorted(found - set(ENV_VARS))


def test_graph_capture_refuses_fewer_hw_queues_than_streams():
    """GPU_MAX_HW_QUEUES below the captured step graph's stream count segfaults in HIP's graph
    launch (torch-only repro, tools/probe_hwq.py): the engine raises a clear error instead."""
    import pytest
    from gentun_amd.models import cnn_engine, cnn_hip
    n = 2 + cnn_hip.WGRAD_STREAMS
    with pytest.raises(RuntimeError, match="GPU_MAX_HW_QUEUES=3"):
        cnn_engine.check_hw_queues(n, env={"GPU_MAX_HW_QUEUES": "3"})
    cnn_engine.check_hw_queues(n, env={"GPU_MAX_HW_QUEUES": "4"})
    cnn_engine.check_hw_queues(n, env={})


def test_too_few_hw_queues_trains_eagerly_with_one_warning():
    """A job's launch() does not capture with too few hardware queues: it warns once and runs eager
    steps (a queue setting must not fail every candidate of a search)."""
    import warnings
    import pytest
    from gentun_amd.models import cnn_engine, cnn_hip
    n = 2 + cnn_hip.WGRAD_STREAMS
    del cnn_engine._HWQ_WARNED[:]
    assert cnn_engine.graph_or_eager(n, env={"GPU_MAX_HW_QUEUES": "8"})
    with pytest.warns(RuntimeWarning, match="eager steps"):
        assert not cnn_engine.graph_or_eager(n, env={"GPU_MAX_HW_QUEUES": "2"})
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        assert not cnn_engine.graph_or_eager(n, env={"GPU_MAX_HW_QUEUES": "2"})
