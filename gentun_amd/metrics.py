"""Observability: JSONL event log and wall-clock / device timers.

The reference only prints (gentun/algorithms.py:27,33-37).
We keep its human-readable lines and add a machine-readable event stream:
``evaluation`` events (rank, generation, genes, fold scores, fitness,
wall_s, FLOPs) and ``generation`` events (best, mean, evals, wall_s,
candidates/hour).
"""

import json
import os
import threading
import time


class EventLog(object):
    """Append-only JSONL writer (thread-safe, line-buffered)."""

    def __init__(self, path, rank=0):
        self.path = path
        self.rank = rank
        d = os.path.dirname(os.path.abspath(path))
        os.makedirs(d, exist_ok=True)
        self._f = open(path, "a", buffering=1)
        self._lock = threading.Lock()

    def write(self, kind, **fields):
        rec = {"ts": time.time(), "kind": kind, "rank": self.rank}
        rec.update(fields)
        line = json.dumps(rec, default=_default, sort_keys=True)
        with self._lock:
            self._f.write(line + "\n")

    def close(self):
        self._f.close()


def _default(o):
    if hasattr(o, "item"):
        return o.item()
    if isinstance(o, tuple):
        return list(o)
    return str(o)


def read_events(path, kind=None):
    out = []
    with open(path) as f:
        for line in f:
            line = line.strip()
            if not line:
                continue
            rec = json.loads(line)
            if kind is None or rec.get("kind") == kind:
                out.append(rec)
    return out


class Timer(object):
    """Accumulating named wall-clock timer (``with timer('train'): ...``)."""

    def __init__(self):
        self.totals = {}
        self.counts = {}

    def __call__(self, name):
        return _Span(self, name)

    def add(self, name, dt):
        self.totals[name] = self.totals.get(name, 0.0) + dt
        self.counts[name] = self.counts.get(name, 0) + 1

    def summary(self):
        return {k: {"total_s": v, "count": self.counts[k]} for k, v in self.totals.items()}


class _Span(object):
    def __init__(self, timer, name):
        self.timer, self.name = timer, name

    def __enter__(self):
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        self.timer.add(self.name, time.perf_counter() - self.t0)
        return False


def candidates_per_hour(n_candidates, seconds):
    return 3600.0 * n_candidates / seconds if seconds > 0 else float("nan")
