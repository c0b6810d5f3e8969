#!/usr/bin/env python
"""Distributed GBDT search (reference tests/sample_master.py + sample_worker.py).

The broker is replaced by a torch.distributed process group: launch ONE
command, rank 0 is the master, every other rank a worker:

    torchrun --nproc-per-node 4 --master-addr 127.0.0.1 examples/distributed_xgb.py

(CPU-only hosts get the gloo backend, GPU hosts RCCL.)"""
import _common

if __name__ == "__main__":
    from gentun import DistributedPopulation, GeneticAlgorithm, GentunWorker, XgboostIndividual
    from gentun_amd.parallel import from_env

    small = _common.SMALL                                      # CI-sized run
    size, gens = (10, 2) if small else (100, 10)
    extra = {'nfold': 3, 'num_boost_round': 40} if small else {'nfold': 3}
    x_train, y_train = _common.wine()
    comm = from_env()
    if comm.rank == 0:
        pop = DistributedPopulation(
            XgboostIndividual, x_train, y_train, size=size, additional_parameters=extra, maximize=False,
            host='localhost', user='guest', password='guest', comm=comm
        )
        ga = GeneticAlgorithm(pop)
        ga.run(gens)
        pop.shutdown()
    else:
        gw = GentunWorker(XgboostIndividual, x_train, y_train, host='localhost', user='guest', password='guest',
                          comm=comm)
        gw.work()
    comm.finish()
