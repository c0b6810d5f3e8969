#!/usr/bin/env python
"""GBDT hyper-parameter search: population 100, tournament GA x 10
(reference tests/test_wine-quality.py:15-25)."""
import _common

if __name__ == "__main__":
    from gentun import GeneticAlgorithm, Population, XgboostIndividual

    x_train, y_train = _common.wine()
    pop = Population(
        XgboostIndividual, x_train, y_train, size=100, additional_parameters={'nfold': 3}, maximize=False
    )
    ga = GeneticAlgorithm(pop)
    ga.run(10)
