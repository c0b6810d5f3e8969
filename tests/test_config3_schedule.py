"""Config-3 shape on 8 processes (gloo): a population of 32 candidates in
total over 8 evaluator ranks (bench.py ``--population 32``), both fold
protocols. Per-fold units (reset="all") give every rank exactly 20
(candidate, fold) groups of a 32-candidate round and 8-9 groups of a
14-candidate Russian-roulette generation; the reference's sequential folds
(reset="kernels", gentun/models/keras_models.py carries biases from fold to
fold) keep candidates whole: 4 per rank. SURVEY.md §2.2 / master.py:108-129
dispatches whole candidates to a RabbitMQ pull queue instead."""
import multiprocessing as mp
import os
import socket

import pytest

WORLD = 8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _proc(rank, port, reset, q):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(WORLD), "LOCAL_RANK": str(rank), "OMP_NUM_THREADS": "1"})
    import torch
    torch.set_num_threads(1)
    from gentun_amd import GeneticCnnIndividual, LocalBatchEvaluator
    from gentun_amd.parallel import DistComm
    from gentun_amd.parallel.distributed import DistributedPopulation, GentunWorker
    from gentun_amd.utils import rng
    from gentun_amd.utils.data import make_image_classification
    x, y = make_image_classification(n=40, shape=(8, 8, 1), classes=3, seed=1)
    ev = LocalBatchEvaluator(device="cpu", streams=1, pop_batch=4)
    comm = DistComm(backend="gloo", timeout_s=120)
    if rank == 0:
        params = dict(nodes=(3, 3), input_shape=(8, 8, 1), kernels_per_layer=(2, 3),
                      kernel_sizes=((3, 3), (3, 3)), dense_units=8, dropout_probability=0.5, classes=3, nfold=5,
                      epochs=(1,), learning_rate=(1e-3,), batch_size=16, backend="torch", device="cpu", seed=3,
                      reset=reset)
        rng.seed(9)
        pop = DistributedPopulation(GeneticCnnIndividual, x, y, size=32, crossover_rate=0.3, mutation_rate=0.1,
                                    additional_parameters=params, comm=comm, evaluator=ev)
        out = []
        n = pop.evaluate_round(per_rank=4)                 # cap 4 x 8 = 32: one round of 32
        out.append((n, dict(pop.last_dispatch)))
        # a Russian-roulette-sized generation: 14 of 32 pending
        for ind in list(pop)[:14]:
            ind.set_fitness(None)
        n = pop.evaluate_round(per_rank=4)
        out.append((n, dict(pop.last_dispatch)))
        ok = all(ind.get_fitness() is not None and ind.get_fitness() > float("-inf") for ind in pop)
        pop.shutdown()
        q.put((out, ok))
    else:
        GentunWorker(GeneticCnnIndividual, x, y, comm=comm, evaluator=ev).work()
    comm.destroy()


def _run(reset):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_proc, args=(r, port, reset, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    try:
        res = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    return res


@pytest.mark.timeout(300)
def test_config3_per_fold_groups_on_8_ranks():
    (full, part), ok = _run("all")
    assert ok
    n, d = full
    assert n == 32 and d["units"] == 160 and d["per_rank_units"] == [20] * WORLD
    n, d = part
    assert n == 14 and d["units"] == 70 and sum(d["per_rank_units"]) == 70
    assert max(d["per_rank_units"]) - min(d["per_rank_units"]) <= 2      # cost-LPT: 8-9 groups, +-1


@pytest.mark.timeout(300)
def test_config3_sequential_folds_keep_candidates_whole_on_8_ranks():
    (full, part), ok = _run("kernels")
    assert ok
    n, d = full
    assert n == 32 and d["units"] == 32 and d["per_rank_units"] == [4] * WORLD
    n, d = part
    assert n == 14 and d["units"] == 14 and max(d["per_rank_units"]) - min(d["per_rank_units"]) <= 1
