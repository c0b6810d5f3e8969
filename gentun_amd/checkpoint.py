"""Per-generation checkpoints ("handler checkpoint format", gentun-ckpt/1).

The reference has no checkpointing at all; its only
serialisation is the JSON wire format ``[i, genes, additional_parameters]`` /
``[i, fitness]`` (gentun/master.py:118, gentun/worker.py:38,50). This format
is a superset of that wire format, written atomically (tmp + fsync +
rename) once per evaluated generation, and is plain JSON -- nothing in it is
ever unpickled.
"""

import json
import os
import tempfile

from .utils import rng as _rng

FORMAT = "gentun-ckpt/1"


def _jsonable(value):
    if isinstance(value, tuple):
        return [_jsonable(v) for v in value]
    if isinstance(value, list):
        return [_jsonable(v) for v in value]
    if isinstance(value, dict):
        return {str(k): _jsonable(v) for k, v in value.items()}
    if hasattr(value, "item") and not isinstance(value, (str, bytes)):
        try:
            return value.item()
        except Exception:
            pass
    return value


def lists_to_tuples(value):
    """JSON turns tuples into lists; the species constructors expect tuples
    (cf. gentun/worker.py:39-42, applied recursively here)."""
    if isinstance(value, list):
        return tuple(lists_to_tuples(v) for v in value)
    if isinstance(value, dict):
        return {k: lists_to_tuples(v) for k, v in value.items()}
    return value


def atomic_write_json(path, obj):
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    fd, tmp = tempfile.mkstemp(prefix=".ckpt-", dir=d)
    try:
        with os.fdopen(fd, "w") as f:
            json.dump(obj, f, indent=1, sort_keys=True)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, path)
    except BaseException:
        if os.path.exists(tmp):
            os.unlink(tmp)
        raise


def _individual_record(i, ind):
    return {"i": i, "genes": _jsonable(ind.get_genes()), "fitness": ind.fitness,
            "fold_scores": _jsonable(getattr(ind, "fold_scores", None)),
            "fold_metrics": _jsonable(getattr(ind, "fold_metrics", None))}


def generation_state(ga):
    pop = ga.population
    algo = {"class": type(ga).__name__, "tournament_size": ga.tournament_size, "elitism": ga.elitism,
            "seed": ga.seed}
    for key in ("crossover_probability", "mutation_probability", "pairing"):
        if hasattr(ga, key):
            algo[key] = getattr(ga, key)
    best = ga.best_individual
    return {
        "format": FORMAT,
        "generation": ga.generation,
        "species": pop.get_species().__name__,
        "algorithm": algo,
        "population": {"class": type(pop).__name__, "maximize": pop.get_fitness_criteria(),
                       "crossover_rate": getattr(pop, "crossover_rate", None),
                       "mutation_rate": getattr(pop, "mutation_rate", None)},
        "additional_parameters": _jsonable(pop[0].get_additional_parameters()) if pop.get_size() else {},
        "individuals": [_individual_record(i, ind) for i, ind in enumerate(pop)],
        "best": None if best is None else _individual_record(-1, best),
        "rng": {"python_random_state": _rng.get_state(), "run_seed": ga.seed},
        "history": _jsonable(ga.history),
    }


def save_generation(directory, ga):
    state = generation_state(ga)
    path = os.path.join(directory, "gen_{:05d}.json".format(ga.generation))
    atomic_write_json(path, state)
    atomic_write_json(os.path.join(directory, "latest.json"), state)
    return path


def load(path):
    if os.path.isdir(path):
        path = os.path.join(path, "latest.json")
    with open(path) as f:
        state = json.load(f)
    if state.get("format") != FORMAT:
        raise ValueError("{} is not a {} checkpoint".format(path, FORMAT))
    return state


def _rebuild(species, x_train, y_train, rec, extra):
    ind = species(x_train, y_train, genes=dict(rec["genes"]), **extra)
    ind.set_fitness(rec["fitness"])
    ind.fold_scores = rec.get("fold_scores")
    if rec.get("fold_metrics"):
        ind.fold_metrics = rec["fold_metrics"]
    return ind


def resume(cls, path, species, x_train, y_train, evaluator=None, population_factory=None, **ga_kwargs):
    """Rebuild (population, GA, RNG, history) from ``path`` and breed the
    next generation so ``run(N)`` continues exactly where it stopped."""
    from .populations import Population
    state = load(path)
    if state["species"] != species.__name__:
        raise ValueError("checkpoint species {} != {}".format(state["species"], species.__name__))
    extra = lists_to_tuples(state["additional_parameters"])
    pstate = state["population"]
    individuals = [_rebuild(species, x_train, y_train, rec, extra) for rec in state["individuals"]]
    for ind in individuals:
        if pstate.get("crossover_rate") is not None:
            ind.crossover_rate = pstate["crossover_rate"]
        if pstate.get("mutation_rate") is not None:
            ind.mutation_rate = pstate["mutation_rate"]
    if population_factory is not None:
        pop = population_factory(individuals)
    else:
        pop = Population(species, x_train, y_train, individual_list=individuals,
                         crossover_rate=pstate.get("crossover_rate") or 0.5,
                         mutation_rate=pstate.get("mutation_rate") or 0.015,
                         maximize=pstate["maximize"], additional_parameters=extra, evaluator=evaluator)
    algo = dict(state["algorithm"])
    kwargs = {}
    if cls.__name__ == "RussianRouletteGA" or "crossover_probability" in algo:
        for key in ("crossover_probability", "mutation_probability", "pairing"):
            if key in algo:
                kwargs[key] = algo[key]
    else:
        kwargs["tournament_size"] = algo.get("tournament_size", 5)
        kwargs["elitism"] = algo.get("elitism", True)
    kwargs.update(ga_kwargs)
    ga = cls(pop, **kwargs)
    ga.seed = algo.get("seed")
    ga.history = list(state.get("history", []))
    if state.get("best") is not None:
        ga.best_individual = _rebuild(species, x_train, y_train, state["best"], extra)
    _rng.set_state(state["rng"]["python_random_state"])
    ga.generation = state["generation"]
    ga.breed()
    ga.generation += 1
    return ga
