"""Per-generation checkpoint / resume: a resumed run replays
the uninterrupted run exactly."""

import json
import os

from fake_species import BitIndividual
from gentun_amd import GeneticAlgorithm, Population, RussianRouletteGA
from gentun_amd.checkpoint import FORMAT, load
from gentun_amd.metrics import EventLog, read_events
from gentun_amd.utils import rng


def _hist(ga):
    return [(h["generation"], h["best_fitness"], h["evals"], tuple(sorted(h["best_genes"].items())))
            for h in ga.history]


def _run(cls, gens, seed, ckdir=None, **kw):
    rng.seed(seed)
    pop = Population(BitIndividual, None, None, size=10)
    ga = cls(pop, seed=seed, checkpoint_dir=ckdir, verbose=False, **kw)
    ga.run(gens)
    return ga


def test_checkpoint_format(tmp_path):
    ga = _run(RussianRouletteGA, 2, 5, ckdir=str(tmp_path))
    st = load(str(tmp_path))
    assert st["format"] == FORMAT and st["generation"] == 2
    assert st["species"] == "BitIndividual"
    assert st["algorithm"]["class"] == "RussianRouletteGA"
    assert len(st["individuals"]) == 10 and all("genes" in r and "fitness" in r for r in st["individuals"])
    assert os.path.exists(tmp_path / "gen_00001.json")
    json.dumps(st)   # plain JSON


def test_resume_replays_uninterrupted_run(tmp_path):
    for cls in (RussianRouletteGA, GeneticAlgorithm):
        full = _run(cls, 5, 42)
        d = tmp_path / cls.__name__
        _run(cls, 3, 42, ckdir=str(d))                 # "crashes" after generation 3
        resumed = cls.resume(str(d / "gen_00003.json"), BitIndividual, verbose=False)
        assert resumed.generation == 4
        resumed.run(5)
        assert _hist(resumed) == _hist(full)
        assert resumed.best_individual.get_fitness() == full.best_individual.get_fitness()


def test_event_log(tmp_path):
    path = str(tmp_path / "events.jsonl")
    log = EventLog(path)
    rng.seed(1)
    GeneticAlgorithm(Population(BitIndividual, None, None, size=6), event_log=log, verbose=False).run(3)
    log.close()
    ev = read_events(path, "generation")
    assert [e["generation"] for e in ev] == [1, 2, 3]
    assert ev[0]["evals"] == 6 and "candidates_per_hour" in ev[0]
