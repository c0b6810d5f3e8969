#!/usr/bin/env python
"""Distributed Genetic CNN (reference tests/mnist_master.py + mnist_worker.py),
one evaluator rank per MI355X:

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/distributed_cnn.py
"""
import _common

if __name__ == "__main__":
    import torch

    from gentun import DistributedPopulation, GeneticCnnIndividual, GentunWorker, RussianRouletteGA
    from gentun_amd import LocalBatchEvaluator
    from gentun_amd.parallel import from_env

    x_train, y_train = _common.mnist_like()
    device = None
    if torch.cuda.is_available():
        import os
        device = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
        torch.cuda.set_device(device)
    comm = from_env(device=device)
    evaluator = LocalBatchEvaluator(device=device, streams=4)
    if comm.rank == 0:
        size, gens = (4, 2) if _common.SMALL else (20, 50)
        pop = DistributedPopulation(
            GeneticCnnIndividual, x_train, y_train, size=size, crossover_rate=0.3, mutation_rate=0.1,
            additional_parameters=dict(_common.cnn_schedule(), batch_size=32), maximize=True, comm=comm,
            evaluator=evaluator
        )
        ga = RussianRouletteGA(pop, crossover_probability=0.2, mutation_probability=0.8)
        ga.run(gens)
        pop.shutdown()
    else:
        GentunWorker(GeneticCnnIndividual, x_train, y_train, comm=comm, evaluator=evaluator).work()
    comm.finish()
