"""Failure paths of the GA layer: a candidate whose evaluation fails on its
rank AND in the rank-0 retry gets the worst fitness, and the Russian-roulette
GA keeps running (its weights ignore non-finite fitness)."""
import math
import warnings

from fake_species import FlakyBitIndividual

from gentun_amd import Population, RussianRouletteGA
from gentun_amd.parallel import ThreadComm
from gentun_amd.parallel.distributed import DistributedPopulation, GentunWorker
from gentun_amd.utils import rng


def test_roulette_weights_ignore_minus_inf():
    rng.seed(3)
    pop = Population(FlakyBitIndividual, None, None, size=6)
    for i, f in enumerate([2.0, float("-inf"), 5.0, 3.0, float("nan"), 2.0]):
        pop[i].set_fitness(f)
    ga = RussianRouletteGA(pop, verbose=False)
    w = ga.roulette_weights()
    assert w == [0.0, 0.0, 3.0, 1.0, 0.0, 0.0]
    ga.breed()                          # random.choices accepts the weights


def test_double_failure_gets_worst_fitness_and_rr_ga_survives():
    import threading
    comms = ThreadComm.group(2)
    worker = threading.Thread(target=lambda: GentunWorker(FlakyBitIndividual, None, None, comm=comms[1]).work())
    worker.start()
    try:
        FlakyBitIndividual.FAILS[0] = 0
        rng.seed(11)
        pop = DistributedPopulation(FlakyBitIndividual, None, None, size=12, comm=comms[0])
        ga = RussianRouletteGA(pop, seed=11, verbose=False)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            best = ga.run(4)
        fits = [h["best_fitness"] for h in ga.history]
        assert all(math.isfinite(f) for f in fits)
        assert math.isfinite(best.get_fitness())
        assert FlakyBitIndividual.FAILS[0] >= 2          # rank evaluation + rank-0 retry both failed
        failed = [ind for ind in ga.population.individuals if ind.fitness is not None and ind.fitness == float("-inf")]
        for ind in failed:
            assert ind.genes['A'].startswith('11')
    finally:
        ga.population.shutdown()
        worker.join(timeout=30)
