"""Failure detection and recovery for multi-rank searches.

The reference gets at-least-once execution from its broker: a job is acked
only after the reply, so RabbitMQ redelivers the job of a dead worker
(gentun/worker.py:50-55, prefetch 1 at :59). RCCL has no such semantics: a
rank that dies or hangs leaves every other rank blocked inside a collective
until the process group's timeout (30 min by default). Here:

* **fault injection** -- ``GENTUN_FAULT="rank:generation:kind"`` with kind
  ``raise`` (the evaluation raises: status code, local retry on rank 0),
  ``exit`` (the rank process dies mid-generation) or ``hang`` (the rank stops
  answering). ``GENTUN_FAULT_ATTEMPT`` limits the injection to one restart
  attempt (torchrun's ``TORCHELASTIC_RESTART_COUNT``), so the restarted
  group runs clean;
* **watchdog** -- a per-rank daemon thread with a deadline per generation,
  sized from the measured generation wall time (``factor`` x the slowest
  generation so far, never below ``min_s``; the first generation gets the
  configured collective timeout). A rank stuck past its deadline -- in a
  collective with a dead peer, or hung itself -- ends its process with exit
  code 75; ``os._exit`` from a thread, no exec of a process that holds the
  GPU;
* **restart** -- the launcher restarts the whole group in FRESH processes
  (``torchrun --max-restarts N`` is the supervisor for multi-rank runs;
  ``python -m gentun_amd.parallel.fault -- CMD`` for a single process), and
  the CLI's ``--resume auto`` continues from ``<checkpoint_dir>/latest.json``:
  the generation that was interrupted is re-evaluated, the GA stream is
  restored, so the trajectory is that of an uninterrupted run.
"""

import os
import subprocess
import sys
import threading
import time
import warnings

EXIT_WATCHDOG = 75
# a search that cannot continue (every evaluation failed): never restarted by supervise()
EXIT_SEARCH_FAILED = 78


def parse_fault(spec=None):
    """``(rank, generation, kind)`` of the injected fault, or None."""
    spec = os.environ.get("GENTUN_FAULT") if spec is None else spec
    if not spec:
        return None
    try:
        r, g, kind = spec.split(":")
        rank, gen = int(r), int(g)
    except ValueError:
        return None
    if kind not in ("raise", "exit", "hang"):
        return None
    attempt = os.environ.get("GENTUN_FAULT_ATTEMPT")
    if attempt is not None and os.environ.get("TORCHELASTIC_RESTART_COUNT", "0") != attempt:
        return None
    return rank, gen, kind


def inject(rank, generation):
    """Apply ``GENTUN_FAULT`` on the evaluating rank (called per generation)."""
    f = parse_fault()
    if f is None or f[0] != rank or f[1] != generation:
        return
    kind = f[2]
    if kind == "raise":
        raise RuntimeError("injected fault on rank {} generation {}".format(rank, generation))
    sys.stderr.write("[fault] injected {} on rank {} generation {}\n".format(kind, rank, generation))
    sys.stderr.flush()
    if kind == "exit":
        os._exit(3)
    # hang: stop answering (until the watchdog or the launcher ends the process)
    while True:
        time.sleep(3600)


class Watchdog(object):
    """Per-rank deadline on generations; expiry ends the process (exit 75).

    ``arm(generation)`` at the start of a generation, ``disarm()`` when its
    results are in; the budget adapts to the measured generation times."""

    def __init__(self, first_s=1800.0, factor=4.0, min_s=60.0, code=EXIT_WATCHDOG, on_expire=None):
        self.first_s = float(first_s)
        self.factor = float(factor)
        self.min_s = float(min_s)
        self.code = code
        self.on_expire = on_expire
        self.slowest = None
        self._deadline = None
        self._label = None
        self._t0 = None
        self._lock = threading.Lock()
        self._thread = threading.Thread(target=self._run, name="gentun-watchdog", daemon=True)
        self._thread.start()

    def budget(self):
        if self.slowest is None:
            return self.first_s
        return max(self.min_s, self.factor * self.slowest)

    def arm(self, label):
        with self._lock:
            self._label = label
            self._t0 = time.monotonic()
            self._deadline = self._t0 + self.budget()

    def disarm(self):
        with self._lock:
            if self._t0 is not None:
                wall = time.monotonic() - self._t0
                self.slowest = wall if self.slowest is None else max(self.slowest, wall)
            self._deadline = None
            self._t0 = None

    def _run(self):
        while True:
            time.sleep(0.2)
            with self._lock:
                expired = self._deadline is not None and time.monotonic() > self._deadline
                label = self._label
            if expired:
                msg = "[watchdog] {} exceeded its {:.0f} s budget: ending rank process (exit {})".format(
                    label, self.budget(), self.code)
                sys.stderr.write(msg + "\n")
                sys.stderr.flush()
                if self.on_expire is not None:
                    self.on_expire()
                os._exit(self.code)


_WATCHDOG = None


def watchdog():
    """The process-wide watchdog, created on first use from
    ``GENTUN_WATCHDOG`` = ``first_s[:factor[:min_s]]`` ("0" disables)."""
    global _WATCHDOG
    kw = parse_watchdog(os.environ.get("GENTUN_WATCHDOG"))
    if kw is None:
        return None
    if _WATCHDOG is None:
        _WATCHDOG = Watchdog(**kw)
    return _WATCHDOG


def parse_watchdog(spec):
    """``first_s[:factor[:min_s]]`` -> Watchdog kwargs; None when unset,
    empty / blank (e.g. ``GENTUN_WATCHDOG= torchrun ...``) or "0". A malformed
    spec raises ValueError naming the variable (the CLI validates it once at
    startup, so every rank fails at once with that message)."""
    if spec is None or not spec.strip() or spec.strip() == "0":
        return None
    try:
        parts = [float(v) for v in spec.strip().split(":")]
    except ValueError:
        raise ValueError("GENTUN_WATCHDOG={!r}: expected first_s[:factor[:min_s]] (numbers) or 0".format(spec))
    if not 1 <= len(parts) <= 3 or any(p <= 0 for p in parts):
        raise ValueError("GENTUN_WATCHDOG={!r}: expected 1-3 positive numbers first_s[:factor[:min_s]]".format(spec))
    return dict(zip(("first_s", "factor", "min_s"), parts))


def supervise(cmd, max_restarts=3, env=None, restart_codes=None):
    """Run ``cmd`` as a child process, re-running it (fresh process, never an
    exec of one that held the GPU) while it fails, at most ``max_restarts``
    times. The child is expected to resume from its own checkpoint
    (``--resume auto``). Returns the last exit code."""
    attempt = 0
    while True:
        e = dict(os.environ if env is None else env)
        e["TORCHELASTIC_RESTART_COUNT"] = str(attempt)
        rc = subprocess.call(cmd, env=e)
        if rc == 0:
            return 0
        if rc == EXIT_SEARCH_FAILED:
            return rc
        if attempt >= max_restarts or (restart_codes is not None and rc not in restart_codes):
            return rc
        warnings.warn("child exited with {}; restart {} of {}".format(rc, attempt + 1, max_restarts))
        attempt += 1


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    max_restarts = 3
    if argv and argv[0].startswith("--max-restarts"):
        max_restarts = int(argv[0].split("=", 1)[1]) if "=" in argv[0] else int(argv.pop(1))
        argv.pop(0)
    if argv and argv[0] == "--":
        argv.pop(0)
    if not argv:
        sys.stderr.write("usage: python -m gentun_amd.parallel.fault [--max-restarts=N] -- CMD ...\n")
        return 2
    return supervise(argv, max_restarts=max_restarts)


if __name__ == "__main__":
    sys.exit(main())
