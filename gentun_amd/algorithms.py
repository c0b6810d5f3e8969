"""Search algorithms: tournament GA with elitism and the Genetic-CNN paper's
Russian-roulette GA.

Reference parity: gentun/algorithms.py:9-56 (``GeneticAlgorithm``) and
:59-99 (``RussianRouletteGA``), including the quirks documented in SURVEY.md
§2.2 / §9: the elite is inserted as the *same object* (Q-elitism identity),
roulette pairs overlap ``(i, i+1)`` for ``i < size//2`` (Q4, default
``pairing="reference"``), and the population left after ``run(N)`` is never
evaluated (Q13).

Extensions (backward compatible): ``seed=`` (Q12), ``run()`` returns the
best individual, per-generation ``history`` with candidates/hour, JSONL event
log and atomic per-generation checkpoints (``checkpoint_dir=``) that
``resume()`` continues from.
"""

import math
import time

from .utils import rng as _rng
from . import checkpoint as _ckpt


class GeneticAlgorithm(object):

    def __init__(self, population, tournament_size=5, elitism=True, seed=None,
                 checkpoint_dir=None, event_log=None, verbose=True):
        if seed is not None:
            # the breeding stream is derived from the run seed, not the seed
            # itself: a caller that seeded the stream with the same value to
            # draw the initial population must not see those draws replayed
            # by selection / crossover / mutation
            _rng.seed(_rng.stable_hash(seed, "ga-breeding"))
        self.population = population
        self.x_train, self.y_train = population.get_data()
        self.tournament_size = tournament_size
        self.elitism = elitism
        self.generation = 1
        self.seed = seed
        self.checkpoint_dir = checkpoint_dir
        self.event_log = event_log
        if event_log is not None and getattr(population, "event_log", False) is None:
            # a distributed population writes its per-unit evaluation events into the GA's log
            population.event_log = event_log
        self.verbose = verbose
        self.history = []
        self.best_individual = None

    # ------------------------------------------------------------ utilities
    def get_population_type(self):
        return self.population.__class__

    def _new_population(self, individual_list):
        return self.population.empty_like(individual_list)

    def _say(self, *lines):
        if self.verbose:
            for line in lines:
                print(line)

    def _evaluate_and_report(self):
        """Evaluate the current generation, print the reference's lines and
        record history. Returns the fittest individual."""
        self._say("Evaluating generation #{}...".format(self.generation))
        pending = len(self.population.pending())
        self.population.ga_generation = self.generation       # tags distributed evaluation events
        t0 = time.perf_counter()
        fittest = self.population.get_fittest()
        wall = time.perf_counter() - t0
        self._say("Fittest individual is:", str(fittest),
                  "Fitness value is: {}\n".format(round(fittest.get_fitness(), 4)))
        fits = [ind.get_fitness() for ind in self.population]
        rec = {
            "generation": self.generation,
            "best_fitness": fittest.get_fitness(),
            "best_genes": dict(fittest.get_genes()),
            "mean_fitness": sum(fits) / len(fits),
            "evals": pending,
            "wall_s": wall,
            "candidates_per_hour": (3600.0 * pending / wall) if wall > 0 and pending else None,
        }
        cat = (getattr(fittest, "fold_metrics", None) or {}).get("categorical_accuracy")
        if cat:
            # Genetic-CNN: the fitness is the reference's binary accuracy; record categorical too
            rec["best_cat_acc"] = float(sum(cat) / len(cat))
        # population means over the members that evaluated (a failed one carries +-inf)
        finite = [f for f in fits if math.isfinite(f)]
        rec["mean_fitness_finite"] = sum(finite) / len(finite) if finite else None
        cats = [(getattr(ind, "fold_metrics", None) or {}).get("categorical_accuracy") for ind in self.population]
        cats = [float(sum(c) / len(c)) for c in cats if c]
        if cats:
            rec["mean_cat_acc"] = sum(cats) / len(cats)
        self.history.append(rec)
        if self.best_individual is None or self._better(fittest.get_fitness(), self.best_individual.get_fitness()):
            self.best_individual = fittest
        if self.event_log is not None:
            self.event_log.write("generation", **rec)
        return fittest

    def _better(self, a, b):
        return a > b if self.population.get_fitness_criteria() else a < b

    def _checkpoint(self):
        """Persist the (already evaluated) current generation."""
        if self.checkpoint_dir is not None:
            _ckpt.save_generation(self.checkpoint_dir, self)

    # ----------------------------------------------------------------- loop
    @classmethod
    def resume(cls, checkpoint_path, species, x_train=None, y_train=None, evaluator=None, **kwargs):
        """Rebuild a GA from a generation checkpoint and advance it past the
        checkpointed generation, so ``run(N)`` continues at ``generation+1``."""
        return _ckpt.resume(cls, checkpoint_path, species, x_train, y_train, evaluator, **kwargs)

    def run(self, max_generations):
        self._say("Starting genetic algorithm...\n")
        while self.generation <= max_generations:
            self.evolve_population()
            self.generation += 1
        return self.best_individual

    def evolve_population(self):
        self._evaluate_and_report()
        self._checkpoint()
        self.breed()

    def breed(self):
        """Build the next generation from the (evaluated) current one."""
        nxt = self._new_population([])
        if self.elitism:
            nxt.add_individual(self.population.get_fittest())   # same object, as in the reference
        while nxt.get_size() < self.population.get_size():
            child = self.tournament_select().reproduce(self.tournament_select())
            child.mutate()
            nxt.add_individual(child)
        self.population = nxt

    def tournament_select(self):
        """Fittest of ``tournament_size`` distinct random members."""
        idx = _rng.get().sample(range(self.population.get_size()), self.tournament_size)
        contenders = [self.population[i] for i in idx]
        pick = max if self.population.get_fitness_criteria() else min
        return pick(contenders, key=lambda ind: ind.get_fitness())


class RussianRouletteGA(GeneticAlgorithm):
    """Fitness-proportional resampling, then pairwise crossover / mutation
    (reference: gentun/algorithms.py:59-99).

    ``pairing="reference"`` keeps the reference's overlapping pairs
    (0,1),(1,2),...; ``"disjoint"`` uses (0,1),(2,3),... so every member can
    vary.
    """

    def __init__(self, population, crossover_probability=0.2, mutation_probability=0.8, seed=None,
                 pairing="reference", checkpoint_dir=None, event_log=None, verbose=True):
        super(RussianRouletteGA, self).__init__(population, seed=seed, checkpoint_dir=checkpoint_dir,
                                                event_log=event_log, verbose=verbose)
        if pairing not in ("reference", "disjoint"):
            raise ValueError("pairing must be 'reference' or 'disjoint'")
        self.crossover_probability = crossover_probability
        self.mutation_probability = mutation_probability
        self.pairing = pairing

    def roulette_weights(self, eps=1e-15):
        pop = self.population
        fits = [pop[i].get_fitness() for i in range(pop.get_size())]
        if pop.get_fitness_criteria():
            w = list(fits)
        else:
            w = [1.0 / (f + eps) for f in fits]
        # a candidate whose evaluation failed twice carries the worst possible
        # fitness (-inf when maximizing, +inf -> weight 0 when minimizing):
        # it gets weight 0, and the floor is taken over the finite weights
        finite = [x for x in w if math.isfinite(x)]
        floor = min(finite) if finite else 0.0
        w = [x - floor if math.isfinite(x) else 0.0 for x in w]
        if sum(w) == 0.0:
            w = [1.0] * len(w)
        return w

    def evolve_population(self, eps=1e-15):
        self._evaluate_and_report()
        self._checkpoint()
        self.breed(eps)

    def breed(self, eps=1e-15):
        r = _rng.get()
        size = self.population.get_size()
        weights = self.roulette_weights(eps)
        chosen = r.choices(range(size), weights=weights, k=size)
        nxt = self._new_population([self.population[i].copy() for i in chosen])
        pairs = range(size // 2) if self.pairing == "reference" else range(0, size - 1, 2)
        for i in pairs:
            if r.random() < self.crossover_probability:
                nxt[i].crossover(nxt[i + 1])
            else:
                if r.random() < self.mutation_probability:
                    nxt[i].mutate()
                if r.random() < self.mutation_probability:
                    nxt[i + 1].mutate()
        self.population = nxt
