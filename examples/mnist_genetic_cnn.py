#!/usr/bin/env python
"""Genetic CNN paper replica (section 4.1.1): population 20, Russian-roulette
GA x 50 (reference tests/test_mnist.py:17-34). Candidates are fold-batched on
the GPU, 4 in flight on separate HIP streams; the run is checkpointed per
generation under ./ckpt_mnist (resume with ``GeneticAlgorithm.resume``)."""
import _common

if __name__ == "__main__":
    from gentun import GeneticCnnIndividual, Population, RussianRouletteGA
    from gentun_amd import LocalBatchEvaluator

    x_train, y_train = _common.mnist_like()
    size, gens = (4, 2) if _common.SMALL else (20, 50)
    params = dict(_common.cnn_schedule(), batch_size=32)
    pop = Population(
        GeneticCnnIndividual, x_train, y_train, size=size, crossover_rate=0.3, mutation_rate=0.1,
        additional_parameters=params, maximize=True, evaluator=LocalBatchEvaluator(streams=4)
    )
    ga = RussianRouletteGA(pop, crossover_probability=0.2, mutation_probability=0.8, seed=0,
                           checkpoint_dir=None if _common.SMALL else "ckpt_mnist")
    ga.run(gens)
