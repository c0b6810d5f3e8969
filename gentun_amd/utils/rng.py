"""Process-wide host RNG for the GA layer.

The reference draws every GA decision from the global ``random`` module and
never seeds it (gentun/individuals.py:10, gentun/algorithms.py:6; SURVEY.md
Q12). We keep one ``random.Random`` instance that starts OS-seeded (same
default behaviour) but can be seeded, snapshotted into a checkpoint and
restored, so a resumed or multi-GPU run replays the identical GA trajectory.

Device-side randomness (weight init, dropout, shuffles) never uses this
stream: it is keyed by (run seed, genes, fold, step) so fitness does not
depend on how candidates are spread over GPUs (SURVEY.md §7.3 hard part 4).
"""

import hashlib
import random

_RNG = random.Random()


def get():
    return _RNG


def seed(value):
    """Seed the GA stream (``None`` -> OS entropy, like the reference)."""
    _RNG.seed(value)


def get_state():
    """Serialisable snapshot of the GA stream (text, for JSON checkpoints)."""
    version, internal, gauss = _RNG.getstate()
    return {"version": version, "internal": list(internal), "gauss": gauss}


def set_state(state):
    _RNG.setstate((state["version"], tuple(state["internal"]), state["gauss"]))


def stable_hash(*parts):
    """64-bit hash that is identical on every rank / process / Python run
    (Python's ``hash`` of str is salted per process)."""
    h = hashlib.blake2b(digest_size=8)
    for p in parts:
        h.update(repr(p).encode())
        h.update(b"\x1f")
    return int.from_bytes(h.digest(), "little")

