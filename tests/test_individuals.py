"""Individual / operator semantics (reference gentun/individuals.py)."""

import pytest

from gentun_amd import GeneticCnnIndividual, XgboostIndividual, random_log_uniform
from gentun_amd.individuals import Individual, default_xgboost_genome
from gentun_amd.utils import rng


def setup_function(_):
    rng.seed(1234)


def test_random_log_uniform_ranges():
    for _ in range(2000):
        assert 0.001 <= random_log_uniform(0.001, 1.0, 10) <= 1.0
        assert 0.0 <= random_log_uniform(0.0, 10.0, 0) <= 10.0
        assert 0.0 <= random_log_uniform(0.0, 1.0, -10) <= 1.0
    vals = sorted(random_log_uniform(0.0, 1.0, -10) for _ in range(4001))
    assert vals[2000] > 0.9          # reverse-log concentrates next to the maximum
    vals = sorted(random_log_uniform(0.001, 1.0, 10) for _ in range(4001))
    assert 0.01 < vals[2000] < 0.1   # log-uniform median ~ 0.032


def test_xgboost_genes_follow_priors():
    genome = default_xgboost_genome()
    for _ in range(200):
        ind = XgboostIndividual(None, None)
        assert set(ind.get_genes()) == set(genome)
        for name, (default, lo, hi, _base) in genome.items():
            v = ind.get_genes()[name]
            assert lo <= v <= hi
            if isinstance(default, int):
                assert isinstance(v, int)
            else:
                assert round(v, 4) == v
    assert ind.get_additional_parameters()['objective'] == 'reg:linear'
    assert ind.crossover_rate == 0.5 and ind.mutation_rate == 0.015


def test_cnn_genome_and_genes():
    ind = GeneticCnnIndividual(None, None)
    assert ind.get_genome() == {'S_1': 3, 'S_2': 10}
    assert all(set(v) <= {'0', '1'} and len(v) == ind.get_genome()[k] for k, v in ind.get_genes().items())
    deep = GeneticCnnIndividual(None, None, nodes=(3, 4, 5), kernels_per_layer=(8, 16, 32),
                                kernel_sizes=((3, 3),) * 3)
    assert deep.get_genome() == {'S_1': 3, 'S_2': 6, 'S_3': 10}
    assert ind.crossover_rate == 0.3 and ind.mutation_rate == 0.1
    with pytest.raises(AssertionError):
        GeneticCnnIndividual(None, None, genes={'S_1': '1', 'S_2': '0000000000'})


def test_validation_errors():
    with pytest.raises(TypeError):
        XgboostIndividual(None, None, genome=[1, 2], genes={})
    with pytest.raises(ValueError):
        XgboostIndividual(None, None, genes={'eta': 0.1})
    with pytest.raises(AssertionError):
        Individual(None, None, {'a': 1}, {'a': 1}, 0.5, 0.5, additional_parameters={'x': 1})


def test_reproduce_crossover_mutate_copy():
    a = XgboostIndividual(None, None, crossover_rate=0.0)
    b = XgboostIndividual(None, None)
    a.set_fitness(1.0)
    b.set_fitness(2.0)
    child = a.reproduce(b)
    assert child.get_genes() == a.get_genes() and child.fitness is None
    assert child.crossover_rate == a.crossover_rate
    a.crossover_rate = 1.0
    child = a.reproduce(b)
    assert child.get_genes() == b.get_genes()
    ga, gb = dict(a.get_genes()), dict(b.get_genes())
    a.crossover(b)                     # rate 1: swap every gene, in place
    assert a.get_genes() == gb and b.get_genes() == ga
    assert a.fitness is None and b.fitness is None
    c = a.copy()
    c.set_fitness(3.0)
    assert a.fitness is None
    a.set_fitness(5.0)
    d = a.copy()
    assert d.fitness == 5.0 and d.get_genes() == a.get_genes() and d.get_genes() is not a.get_genes()
    a.mutation_rate = 0.0
    a.mutate()
    assert a.fitness == 5.0
    a.mutation_rate = 1.0
    a.mutate()
    assert a.fitness is None


def test_cnn_mutate_flips_every_bit_at_rate_one():
    ind = GeneticCnnIndividual(None, None, genes={'S_1': '101', 'S_2': '0000011111'}, mutation_rate=1.0)
    ind.set_fitness(0.5)
    ind.mutate()
    assert ind.get_genes() == {'S_1': '010', 'S_2': '1111100000'}
    assert ind.fitness is None
    ind.set_fitness(0.7)
    ind.mutation_rate = 0.0
    ind.mutate()
    assert ind.fitness == 0.7


def test_str_is_pformat_of_genes():
    ind = GeneticCnnIndividual(None, None, genes={'S_1': '101', 'S_2': '0000011111'})
    assert str(ind) == "{'S_1': '101', 'S_2': '0000011111'}"


def test_species_mismatch_asserts():
    a = XgboostIndividual(None, None)
    b = GeneticCnnIndividual(None, None)
    with pytest.raises(AssertionError):
        a.reproduce(b)
    with pytest.raises(AssertionError):
        a.crossover(b)
