#!/usr/bin/env python
"""Grid-initialised GBDT search: 5 x 8 x 5 = 200 individuals, GA x 10
(reference tests/test_grid_wine-quality.py:15-30)."""
import _common

if __name__ == "__main__":
    from gentun import GeneticAlgorithm, GridPopulation, XgboostIndividual

    x_train, y_train = _common.wine()
    grid = {
        'eta': [0.001, 0.005, 0.01, 0.015, 0.2],
        'max_depth': range(3, 11),
        'colsample_bytree': [0.80, 0.85, 0.90, 0.95, 1.0],
    }
    if _common.SMALL:
        grid = {'eta': [0.1, 0.3], 'max_depth': [3, 4, 5]}
    extra = {'nfold': 3, 'num_boost_round': 30} if _common.SMALL else {'nfold': 3}
    pop = GridPopulation(
        XgboostIndividual, x_train, y_train, genes_grid=grid,
        additional_parameters=extra, maximize=False
    )
    ga = GeneticAlgorithm(pop)
    ga.run(2 if _common.SMALL else 10)
