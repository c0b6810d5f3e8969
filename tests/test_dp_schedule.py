"""X5 on the HIP executor's launch schedule: with the batch
split over 2 data-parallel ranks (real processes, gloo), each rank runs the
population schedule (gentun_amd/models/pop_schedule.py, the float64
interpreter of tests/test_pop_schedule.py that mirrors the HIP step launch by
launch) on its rows, the gradients are summed by ONE all-reduce of a flat
buffer -- cnn_hip.HipPopJob._dp_allreduce's placement: after every weight
gradient, before the optimizer -- and every group's weight gradients equal
the single-process full-batch ones. The HIP kernels themselves run the same
split on a GPU in tests/test_hip_dp.py."""
import os
import random
import socket

import pytest
import torch
import torch.multiprocessing as mp

from test_pop_schedule import _params, _plans, _random_genes, _run_schedule
from gentun_amd.models.pop_schedule import PopulationSchedule

NODES, HW, CIN, KERNELS, KS, G, BFULL = (3, 5), 8, 3, (4, 6), ((5, 5), (5, 5)), 6, 4


def _problem():
    rng = random.Random(5)
    genes = [_random_genes(rng, NODES) for _ in range(G)]
    sched = PopulationSchedule(_plans(NODES, HW, CIN, KERNELS, KS, genes))
    gen = torch.Generator().manual_seed(5)
    P = _params(sched, gen)
    x = torch.randn(BFULL, CIN, HW, HW, generator=gen, dtype=torch.float64)
    hs = HW >> len(NODES)
    R = torch.randn(G, BFULL, KERNELS[-1], hs, hs, generator=gen, dtype=torch.float64)
    return sched, P, x, R


def _flat(grads):
    keys = sorted(grads)
    return keys, torch.cat([torch.cat([grads[k][0].reshape(-1), grads[k][1].reshape(-1)]) for k in keys])


def _rank(rank, world, port, out):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:{}".format(port), rank=rank, world_size=world)
    sched, P, x, R = _problem()
    r0, r1 = rank * BFULL // world, (rank + 1) * BFULL // world
    keys, flat = _flat(_run_schedule(sched, x[r0:r1], P, R[:, r0:r1]))
    dist.all_reduce(flat)                   # the one flat all-reduce of a data-parallel step
    if rank == 0:
        out.put((keys, flat.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_rank_schedule_gradients_equal_full_batch():
    sched, P, x, R = _problem()
    keys, ref = _flat(_run_schedule(sched, x, P, R))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got_keys, got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got_keys == keys and len(keys) >= G * len(NODES)
    torch.testing.assert_close(torch.from_numpy(got), ref, rtol=1e-12, atol=1e-12)
