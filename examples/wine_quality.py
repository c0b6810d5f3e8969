#!/usr/bin/env python
"""GBDT hyper-parameter search: population 100, tournament GA x 10
(reference tests/test_wine-quality.py:15-25)."""
import _common

if __name__ == "__main__":
    from gentun import GeneticAlgorithm, Population, XgboostIndividual

    x_train, y_train = _common.wine()
    size, gens = (6, 2) if _common.SMALL else (100, 10)
    extra = {'nfold': 3, 'num_boost_round': 30} if _common.SMALL else {'nfold': 3}
    pop = Population(
        XgboostIndividual, x_train, y_train, size=size, additional_parameters=extra, maximize=False
    )
    ga = GeneticAlgorithm(pop)
    ga.run(gens)
