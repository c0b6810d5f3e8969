"""GA semantics (reference gentun/algorithms.py, gentun/populations.py;
SURVEY.md §2.2 and Appendix A.2 probe facts)."""

import pytest

from fake_species import EVALS, BitIndividual, NumIndividual
from gentun_amd import GeneticAlgorithm, GridPopulation, Population, RussianRouletteGA, XgboostIndividual
from gentun_amd.utils import rng


def _count(fn):
    EVALS["n"] = 0
    fn()
    return EVALS["n"]


def test_tournament_eval_count_identity():
    for pop_size, gens in ((20, 5), (10, 3)):
        rng.seed(7)
        pop = Population(BitIndividual, None, None, size=pop_size)
        ga = GeneticAlgorithm(pop, verbose=False)
        n = _count(lambda: ga.run(gens))
        assert n == pop_size + (pop_size - 1) * (gens - 1)      # 96 for 20 x 5 (App. A.2)


def test_elitism_keeps_same_object_and_history():
    rng.seed(3)
    pop = Population(BitIndividual, None, None, size=8)
    ga = GeneticAlgorithm(pop, verbose=False)
    ga.evolve_population()
    fittest = pop.get_fittest()          # all cached now
    assert ga.population[0] is fittest
    assert ga.history[0]["evals"] == 8
    assert ga.history[0]["best_fitness"] == fittest.get_fitness()


def test_run_returns_best_and_improves():
    rng.seed(11)
    ga = GeneticAlgorithm(Population(BitIndividual, None, None, size=12), verbose=False)
    best = ga.run(6)
    assert best.get_fitness() == max(h["best_fitness"] for h in ga.history)
    assert ga.history[-1]["best_fitness"] >= ga.history[0]["best_fitness"]


def test_tournament_needs_five_members():
    rng.seed(1)
    ga = GeneticAlgorithm(Population(BitIndividual, None, None, size=4), verbose=False)
    with pytest.raises(ValueError):
        ga.run(1)


def test_minimize():
    rng.seed(5)
    pop = Population(NumIndividual, None, None, size=10, maximize=False)
    ga = GeneticAlgorithm(pop, verbose=False)
    best = ga.run(5)
    assert best.get_fitness() == min(h["best_fitness"] for h in ga.history)
    assert ga.history[0]["best_fitness"] == min(ind.get_fitness() for ind in pop)


def test_seed_determinism():
    def trajectory():
        rng.seed(99)
        ga = RussianRouletteGA(Population(BitIndividual, None, None, size=10), verbose=False)
        ga.run(4)
        return [(h["best_fitness"], h["evals"], tuple(sorted(h["best_genes"].items()))) for h in ga.history]
    assert trajectory() == trajectory()


class _Recorder(BitIndividual):
    log = []

    def crossover(self, partner):
        _Recorder.log.append((id(self), id(partner)))

    def mutate(self):
        pass


@pytest.mark.parametrize("pairing,expected", [("reference", [(0, 1), (1, 2), (2, 3)]),
                                              ("disjoint", [(0, 1), (2, 3), (4, 5)])])
def test_roulette_pairs(pairing, expected):
    rng.seed(0)
    pop = Population(_Recorder, None, None, size=6)
    for ind in pop:
        ind.set_fitness(1.0)
    ga = RussianRouletteGA(pop, crossover_probability=1.0, mutation_probability=0.0, pairing=pairing,
                           verbose=False)
    _Recorder.log = []
    ga.breed()
    pos = {id(ind): i for i, ind in enumerate(ga.population)}
    assert [(pos[a], pos[b]) for a, b in _Recorder.log] == expected     # App. A.2


def test_roulette_weights_and_no_elitism():
    rng.seed(2)
    pop = Population(BitIndividual, None, None, size=5)
    fits = [1.0, 2.0, 3.0, 4.0, 5.0]
    for ind, f in zip(pop, fits):
        ind.set_fitness(f)
    ga = RussianRouletteGA(pop, verbose=False)
    assert ga.roulette_weights() == [0.0, 1.0, 2.0, 3.0, 4.0]     # worst gets weight 0
    for ind in pop:
        ind.set_fitness(2.0)
    assert ga.roulette_weights() == [1.0] * 5                      # all equal -> uniform
    pop2 = Population(NumIndividual, None, None, size=3, maximize=False)
    for ind, f in zip(pop2, (1.0, 0.5, 0.25)):
        ind.set_fitness(f)
    w = RussianRouletteGA(pop2, verbose=False).roulette_weights()
    assert w[0] == 0.0 and w[2] > w[1] > 0
    # offspring are copies: fitness memo preserved when not varied
    ga = RussianRouletteGA(pop, crossover_probability=0.0, mutation_probability=0.0, verbose=False)
    ga.breed()
    assert all(ind.get_fitness_status() for ind in ga.population)
    assert all(new is not old for new in ga.population for old in pop)


def test_roulette_upper_half_never_varied_in_reference_pairing():
    rng.seed(4)
    pop = Population(BitIndividual, None, None, size=8, mutation_rate=1.0)
    for ind in pop:
        ind.set_fitness(1.0)
    ga = RussianRouletteGA(pop, crossover_probability=0.0, mutation_probability=1.0, verbose=False)
    ga.breed()
    status = [ind.get_fitness_status() for ind in ga.population]
    assert status[:5] == [False] * 5          # indices 0..size/2 mutated
    assert status[5:] == [True] * 3           # size/2+1 .. size-1 untouched (Q4)


def test_population_checks_and_fittest_ties():
    rng.seed(6)
    pop = Population(BitIndividual, None, None, size=4)
    with pytest.raises(AssertionError):
        pop.add_individual(NumIndividual(None, None))
    with pytest.raises(AssertionError):
        Population(BitIndividual, None, None, individual_list=[NumIndividual(None, None)])
    with pytest.raises(ValueError):
        Population(BitIndividual, None, None)
    for ind in pop:
        ind.set_fitness(1.0)
    assert pop.get_fittest() is pop[0]
    pop2 = Population(BitIndividual, None, None, size=3, maximize=False)
    for ind, f in zip(pop2, (3.0, 1.0, 1.0)):
        ind.set_fitness(f)
    assert pop2.get_fittest() is pop2[1]


def test_grid_population():
    grid = {'eta': [0.001, 0.005, 0.01, 0.015, 0.2], 'max_depth': range(3, 11),
            'colsample_bytree': [0.80, 0.85, 0.90, 0.95, 1.0]}
    pop = GridPopulation(XgboostIndividual, genes_grid=grid, additional_parameters={'nfold': 3}, maximize=False)
    assert pop.get_size() == 200                                   # App. A.2
    assert all(ind.get_genes()['lambda'] == 1.0 for ind in pop)   # default filled in
    assert all(ind.nfold == 3 for ind in pop)
    pop = GridPopulation(XgboostIndividual, None, None, genes_grid={'eta': [0.1, 0.2]})   # Q8: None params
    assert pop.get_size() == 2
    with pytest.raises(ValueError):
        GridPopulation(XgboostIndividual, genes_grid={'nope': [1]})
    from gentun_amd import GeneticCnnIndividual
    with pytest.raises(ValueError):
        GridPopulation(GeneticCnnIndividual, genes_grid={'S_1': ['101']})


class _BatchEval(object):
    def __init__(self):
        self.calls = []

    def evaluate(self, inds):
        self.calls.append(len(inds))
        for ind in inds:
            ind.evaluate_fitness()
        return len(inds)


def test_evaluator_batches_pending_and_travels_with_generations():
    rng.seed(8)
    ev = _BatchEval()
    pop = Population(BitIndividual, None, None, size=10, evaluator=ev)
    ga = GeneticAlgorithm(pop, verbose=False)
    ga.run(3)
    assert ev.calls == [10, 9, 9]       # one batch per generation; the elite is cached
    assert ga.population.evaluator is ev
