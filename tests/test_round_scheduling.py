"""Generation-size robustness of the distributed evaluator: with a
population-batched evaluator the work unit is one (candidate, fold), so a
Russian-roulette generation that re-evaluates only ~14 of 32 candidates
still spreads evenly over 8 ranks (master.py:108-129 sends
whole candidates); evaluation *rounds* (``evaluate_in_parallel(limit=)``)
evaluate a generation in bounded slices, as the headline bench does."""
import threading

import numpy as np

from gentun_amd import GeneticCnnIndividual, LocalBatchEvaluator, RussianRouletteGA
from gentun_amd.parallel import ThreadComm, lpt_assign, make_units
from gentun_amd.parallel.distributed import DistributedPopulation, GentunWorker
from gentun_amd.utils import rng
from gentun_amd.utils.data import make_image_classification

TINY = dict(nodes=(3, 3), input_shape=(8, 8, 1), kernels_per_layer=(2, 3), kernel_sizes=((3, 3), (3, 3)),
            dense_units=8, dropout_probability=0.5, classes=3, nfold=5, epochs=(1,), learning_rate=(1e-3,),
            batch_size=16, backend="torch", device="cpu", seed=3, reset="all")


def _rr_generation_sizes(pop=32, gens=30, seed=0):
    """Pending counts of successive RR-GA generations (bit-string species)."""
    from fake_species import BitIndividual
    from gentun_amd import Population
    rng.seed(seed)
    p = Population(BitIndividual, None, None, size=pop, crossover_rate=0.3, mutation_rate=0.1)
    ga = RussianRouletteGA(p, seed=seed, verbose=False)
    sizes = []
    for _ in range(gens):
        sizes.append(len(ga.population.pending()))
        ga.population.get_fittest()
        ga.breed()
    return sizes


def test_per_fold_units_balance_a_14_of_32_generation_on_8_ranks():
    sizes = _rr_generation_sizes()
    assert sizes[0] == 32 and 8 <= np.mean(sizes[1:]) <= 20        # ~43 % re-evaluated per generation
    rng_costs = np.random.default_rng(0).uniform(13.0, 88.0, 14)  # MFLOP/sample range of the S=(3,5) space
    units, ucost = make_units(list(rng_costs), 5, 8, True, per_fold=True)
    assert len(units) == 70 and all(len(f) == 1 for _, f in units)
    owner = lpt_assign(ucost, 8)
    groups = np.bincount(owner, minlength=8)
    loads = np.bincount(owner, weights=ucost, minlength=8)
    assert groups.max() - groups.min() <= 2                         # 8-9 groups per rank
    assert loads.max() / loads.mean() < 1.15                        # cost-balanced
    # whole-candidate units (the previous policy) put 1-2 candidates = 5-10 groups per rank
    whole, wcost = make_units(list(rng_costs), 5, 8, True, per_fold=False)
    wl = np.bincount(lpt_assign(wcost, 8), weights=wcost, minlength=8)
    assert wl.max() / wl.mean() > loads.max() / loads.mean()


def test_rounds_with_per_fold_units_match_a_single_process_run():
    x, y = make_image_classification(n=60, shape=(8, 8, 1), classes=3, seed=1)
    world = 4
    comms = ThreadComm.group(world)
    evs = [LocalBatchEvaluator(device="cpu", streams=1, pop_batch=4) for _ in range(world)]
    threads = [threading.Thread(target=lambda r=r: GentunWorker(GeneticCnnIndividual, x, y, comm=comms[r],
                                                              evaluator=evs[r]).work(), daemon=True)
               for r in range(1, world)]
    for t in threads:
        t.start()
    rng.seed(5)
    pop = DistributedPopulation(GeneticCnnIndividual, x, y, size=6, crossover_rate=0.3, mutation_rate=0.1,
                                additional_parameters=TINY, comm=comms[0], evaluator=evs[0])
    n1 = pop.evaluate_in_parallel(limit=4)
    d = pop.last_dispatch
    assert n1 == 4 and len(pop.pending()) == 2
    assert d["units"] == 20 and sum(d["per_rank_units"]) == 20 and min(d["per_rank_units"]) >= 3   # cost-LPT
    n2 = pop.evaluate_in_parallel(limit=4)
    assert n2 == 2 and not pop.pending()
    dist = [(ind.get_fitness(), ind.fold_metrics["categorical_accuracy"]) for ind in pop]
    pop.shutdown()
    for t in threads:
        t.join(timeout=60)
    # the same candidates evaluated whole, in one process
    local = []
    for ind in pop:
        twin = GeneticCnnIndividual(x, y, genes=dict(ind.get_genes()), **TINY)
        twin.evaluate_fitness()
        local.append((twin.get_fitness(), twin.fold_metrics["categorical_accuracy"]))
    for (fd, cd), (fl, cl) in zip(dist, local):
        assert abs(fd - fl) < 1e-6 and np.allclose(cd, cl)


def test_sequential_fold_candidates_are_never_split():
    """reset="kernels" (the reference's fold protocol) chains the folds of a
    candidate, so the distributed evaluator keeps each candidate one unit."""
    x, y = make_image_classification(n=60, shape=(8, 8, 1), classes=3, seed=1)
    comms = ThreadComm.group(2)
    evs = [LocalBatchEvaluator(device="cpu", streams=1, pop_batch=4) for _ in range(2)]
    t = threading.Thread(target=lambda: GentunWorker(GeneticCnnIndividual, x, y, comm=comms[1],
                                                     evaluator=evs[1]).work(), daemon=True)
    t.start()
    rng.seed(6)
    params = dict(TINY, reset="kernels", nfold=3)
    pop = DistributedPopulation(GeneticCnnIndividual, x, y, size=2, additional_parameters=params, comm=comms[0],
                                evaluator=evs[0])
    pop.evaluate_in_parallel()
    assert pop.last_dispatch["units"] == 2
    assert all(len(ind.fold_scores) == 3 for ind in pop)
    pop.shutdown()
    t.join(timeout=60)


def test_balanced_round_slack_saves_a_round():
    """cap 5 per round: without slack 11 pending -> 4, 4, 3; with one extra
    candidate allowed per round -> 6, 5 (larger launches, no round below
    cap - 1 whenever the pending set allows it)."""
    from gentun_amd.parallel.scheduler import balanced_round

    def rounds(n, slack):
        out = []
        while n:
            r = balanced_round(n, 5, slack)
            out.append(r)
            n -= r
        return out
    assert rounds(11, 0) == [4, 4, 3]
    assert rounds(11, 1) == [6, 5]
    assert rounds(14, 1) == [5, 5, 4]
    assert rounds(32, 1) == [6, 6, 5, 5, 5, 5]
    for n in range(4, 40):
        rs = rounds(n, 1)
        assert sum(rs) == n and max(rs) <= 6 and (min(rs) >= 4 or n == 7)      # 7 = 4 + 3
