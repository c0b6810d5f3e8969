"""Distributed evaluation: master + evaluator ranks
over collectives. Ranks are threads on a ThreadComm test double and real
processes on the ``gloo`` backend (CPU stand-in for RCCL)."""

import os
import socket
import threading

import numpy as np
import pytest
import torch.multiprocessing as mp

from fake_species import BitIndividual, NumIndividual
from gentun_amd import GeneticAlgorithm, Population, RussianRouletteGA, XgboostIndividual
from gentun_amd.parallel import GenomeCodec, ThreadComm, lpt_assign, make_units
from gentun_amd.parallel.distributed import DistributedGridPopulation, DistributedPopulation, GentunWorker
from gentun_amd.parallel.evaluators import SequentialEvaluator
from gentun_amd.utils import rng


def test_codec_roundtrip():
    ind = XgboostIndividual(None, None)
    c = GenomeCodec(ind.get_genome())
    genes = ind.get_genes()
    back = c.decode(c.encode(genes))
    assert back == genes and all(type(back[k]) is type(genes[k]) for k in genes)
    from gentun_amd import GeneticCnnIndividual
    cnn = GeneticCnnIndividual(None, None, genes={'S_1': '101', 'S_2': '0110011001'})
    c = GenomeCodec(cnn.get_genome())
    assert c.width == 13 and c.decode(c.encode(cnn.get_genes())) == cnn.get_genes()


def test_scheduler():
    owner = lpt_assign([5, 4, 3, 3, 3], 2)
    loads = [sum(c for c, o in zip([5, 4, 3, 3, 3], owner) if o == r) for r in range(2)]
    assert sorted(loads) == [8, 10]
    assert lpt_assign([1, 1, 1], 2) == lpt_assign([1, 1, 1], 2)    # deterministic
    units, costs = make_units([10.0, 20.0], 5, 8)
    assert len(units) == 2 * 4 and sorted(len(f) for _, f in units) == [1, 1, 1, 1, 1, 1, 2, 2]
    assert sorted(f for _, fids in units if _ == 0 for f in fids) == [0, 1, 2, 3, 4]
    units, _ = make_units([1.0] * 10, 5, 8)
    assert all(len(f) == 5 for _, f in units)                        # enough candidates: no split


def _ga_run(pop, cls, gens):
    ga = cls(pop, verbose=False) if cls is RussianRouletteGA else cls(pop, verbose=False)
    ga.run(gens)
    return [(h["best_fitness"], h["evals"], tuple(sorted(h["best_genes"].items()))) for h in ga.history]


def _threaded(world, species, cls, gens, seed, size=12, fault=None, maximize=True, schedule="dynamic"):
    comms = ThreadComm.group(world)
    out = {}

    def worker(r):
        GentunWorker(species, None, None, comm=comms[r], evaluator=SequentialEvaluator()).work()

    threads = [threading.Thread(target=worker, args=(r,), daemon=True) for r in range(1, world)]
    for t in threads:
        t.start()
    old = os.environ.get("GENTUN_FAULT")
    if fault:
        os.environ["GENTUN_FAULT"] = fault
    try:
        rng.seed(seed)
        pop = DistributedPopulation(species, None, None, size=size, comm=comms[0],
                                    evaluator=SequentialEvaluator(), maximize=maximize, schedule=schedule)
        out["hist"] = _ga_run(pop, cls, gens)
        out["pop"] = pop
        pop.shutdown()
    finally:
        if fault:
            if old is None:
                os.environ.pop("GENTUN_FAULT", None)
            else:
                os.environ["GENTUN_FAULT"] = old
    for t in threads:
        t.join(timeout=30)
        assert not t.is_alive()
    return out


def _local(species, cls, gens, seed, size=12, maximize=True):
    rng.seed(seed)
    pop = Population(species, None, None, size=size, maximize=maximize)
    return _ga_run(pop, cls, gens)


@pytest.mark.parametrize("cls", [GeneticAlgorithm, RussianRouletteGA])
def test_threaded_ranks_match_local_run(cls):
    for world in (2, 3):
        assert _threaded(world, BitIndividual, cls, 4, seed=21)["hist"] == _local(BitIndividual, cls, 4, seed=21)
    got = _threaded(3, NumIndividual, GeneticAlgorithm, 3, seed=5, maximize=False)["hist"]
    assert got == _local(NumIndividual, GeneticAlgorithm, 3, seed=5, maximize=False)


def test_fault_injection_is_recovered():
    res = _threaded(3, BitIndividual, GeneticAlgorithm, 3, seed=8, fault="1:2:raise")
    assert res["hist"] == _local(BitIndividual, GeneticAlgorithm, 3, seed=8)


def test_next_generation_keeps_communicator():
    comms = ThreadComm.group(1)
    rng.seed(2)
    pop = DistributedPopulation(BitIndividual, None, None, size=6, comm=comms[0], evaluator=SequentialEvaluator())
    ga = GeneticAlgorithm(pop, verbose=False)
    ga.run(2)
    assert isinstance(ga.population, DistributedPopulation) and ga.population.comm is comms[0]   # Q1 fixed


def test_distributed_grid_population():
    comms = ThreadComm.group(1)
    pop = DistributedGridPopulation(XgboostIndividual, None, None, genes_grid={'eta': [0.1, 0.2, 0.3]},
                                    comm=comms[0])
    assert pop.get_size() == 3 and isinstance(pop, DistributedPopulation)


# ---------------------------------------------------------------------------
# real processes over torch.distributed (gloo)
# ---------------------------------------------------------------------------

def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _proc(rank, world, port, q):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank)})
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from fake_species import BitIndividual as Bit
    from gentun_amd.parallel import DistComm
    from gentun_amd.parallel.distributed import DistributedPopulation as DP, GentunWorker as GW
    from gentun_amd.parallel.evaluators import SequentialEvaluator as SE
    from gentun_amd import RussianRouletteGA as RR
    from gentun_amd.utils import rng as r
    comm = DistComm(backend="gloo", timeout_s=60)
    if rank == 0:
        r.seed(77)
        pop = DP(Bit, None, None, size=10, comm=comm, evaluator=SE())
        ga = RR(pop, verbose=False)
        ga.run(4)
        pop = ga.population
        pop.sync_ranks()
        pop.shutdown()
        q.put([(h["best_fitness"], h["evals"], tuple(sorted(h["best_genes"].items()))) for h in ga.history])
    else:
        GW(Bit, None, None, comm=comm, evaluator=SE()).work()
    comm.destroy()


def test_gloo_processes_match_local_run():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 2
    procs = [ctx.Process(target=_proc, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    hist = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert hist == _local(BitIndividual, RussianRouletteGA, 4, seed=77, size=10)


def _msg_proc(rank, world, port, q):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank)})
    os.environ.pop("TORCHELASTIC_USE_AGENT_STORE", None)
    from gentun_amd.parallel import DistComm
    comm = DistComm(backend="gloo", timeout_s=60)
    big = np.arange(20000, dtype=np.float64).reshape(100, 200)            # 160 KB: beyond one message tensor
    sent = [np.array([3, 1, 4], np.int64), np.frombuffer(b"blob", np.uint8).copy(), big,
            np.zeros((0, 3), np.float32)]
    got = comm.broadcast_arrays(sent if rank == 0 else None)
    ok = len(got) == len(sent) and all(a.dtype == b.dtype and a.shape == b.shape and np.array_equal(a, b)
                                       for a, b in zip(sent, got))
    one = comm.broadcast_array(np.array([7.5], np.float32) if rank == 0 else None)
    ok = ok and one.dtype == np.float32 and float(one[0]) == 7.5 and comm.messages == 2
    # X6 tickets on the communicator's own rendezvous store: every value taken exactly once
    tickets = [comm.ticket("t") for _ in range(5)]
    allt = comm.all_gather_array(np.array(tickets, np.int64))
    ok = ok and sorted(np.concatenate(allt).tolist()) == list(range(5 * world))
    comm.barrier()
    q.put((rank, ok))
    comm.destroy()


def test_gloo_one_message_broadcast_and_own_store_tickets():
    """A dispatch message (several arrays, also beyond the fixed 32 KB tensor)
    arrives intact on every rank as one message; tickets count on the store
    DistComm created itself (no private torch.distributed state)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_msg_proc, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == {0: True, 1: True, 2: True}


def test_dispatch_is_one_message_per_round():
    """Rank 0 sends one broadcast message per evaluation round (header, config
    blob and genome table together), not one per array."""
    comms = ThreadComm.group(2)
    counts = {"n": 0}
    orig = ThreadComm.broadcast_arrays

    def counting(self, arrays, src=0):
        if self.rank == 0:
            counts["n"] += 1
        return orig(self, arrays, src)

    ThreadComm.broadcast_arrays = counting
    try:
        t = threading.Thread(target=lambda: GentunWorker(BitIndividual, None, None, comm=comms[1],
                                                         evaluator=SequentialEvaluator()).work(), daemon=True)
        t.start()
        rng.seed(5)
        pop = DistributedPopulation(BitIndividual, None, None, size=6, comm=comms[0], evaluator=SequentialEvaluator())
        pop.evaluate_in_parallel()
        assert counts["n"] == 1
        pop.shutdown()
        t.join(timeout=30)
        assert counts["n"] == 2
    finally:
        ThreadComm.broadcast_arrays = orig


def test_comm_uses_no_private_torch_symbols():
    import inspect
    from gentun_amd.parallel import comm
    src = inspect.getsource(comm)
    assert "_get_default_store" not in src and "distributed_c10d" not in src


def test_dynamic_and_static_schedules_agree():
    """Work stealing (ticket counter) and static LPT give the same GA run;
    every unit is evaluated exactly once."""
    a = _threaded(3, BitIndividual, GeneticAlgorithm, 3, seed=11, schedule="dynamic")
    b = _threaded(3, BitIndividual, GeneticAlgorithm, 3, seed=11, schedule="lpt")
    assert a["hist"] == b["hist"]
    da, db = a["pop"].last_dispatch, b["pop"].last_dispatch
    assert da["schedule"] == "dynamic" and db["schedule"] == "lpt"
    assert sum(da["per_rank_units"]) == da["units"] and sum(db["per_rank_units"]) == db["units"]


class _SlowOnRank1(BitIndividual):
    """Evaluation takes 50 ms on the thread named 'rank1', 1 ms elsewhere."""

    def evaluate_fitness(self):
        import time
        time.sleep(0.05 if threading.current_thread().name == "rank1" else 0.001)
        return super(_SlowOnRank1, self).evaluate_fitness()


def test_dynamic_schedule_balances_a_slow_rank():
    comms = ThreadComm.group(3)

    def worker(r):
        GentunWorker(_SlowOnRank1, None, None, comm=comms[r], evaluator=SequentialEvaluator()).work()

    threads = [threading.Thread(target=worker, args=(r,), name="rank{}".format(r), daemon=True) for r in (1, 2)]
    for t in threads:
        t.start()
    rng.seed(3)
    pop = DistributedPopulation(_SlowOnRank1, None, None, size=30, comm=comms[0], evaluator=SequentialEvaluator(),
                                schedule="dynamic")
    pop.evaluate_in_parallel()
    per = pop.last_dispatch["per_rank_units"]
    pop.shutdown()
    for t in threads:
        t.join(timeout=30)
    assert sum(per) == 30
    assert per[1] < per[2] and per[1] < per[0]        # the slow rank took fewer units
    assert all(ind.get_fitness() is not None for ind in pop)


def test_ticket_counters():
    from gentun_amd.parallel.comm import LocalComm
    c = LocalComm()
    assert [c.ticket("a"), c.ticket("a"), c.ticket("b")] == [0, 1, 0]
    comms = ThreadComm.group(4)
    got = []
    lock = threading.Lock()

    def take(cm):
        for _ in range(25):
            v = cm.ticket("k")
            with lock:
                got.append(v)

    ts = [threading.Thread(target=take, args=(cm,)) for cm in comms]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert sorted(got) == list(range(100))


def test_auto_schedule_follows_the_evaluator():
    """Population-batched evaluators get static LPT (balanced per-rank cost
    sums); one-at-a-time evaluators keep dynamic pull-queue claiming."""
    from gentun_amd.parallel import LocalComm
    from gentun_amd.parallel.distributed import DistributedPopulation
    from gentun_amd.parallel.evaluators import LocalBatchEvaluator, SequentialEvaluator
    import torch
    mk = lambda ev: DistributedPopulation(BitIndividual, None, None, size=6, comm=LocalComm(), evaluator=ev)
    assert mk(LocalBatchEvaluator(device=torch.device("cpu"), pop_batch=16)).schedule == "lpt"
    assert mk(SequentialEvaluator()).schedule == "dynamic"


def test_gpu_individual_runs_on_evaluating_rank_device():
    """Additional parameters come from rank 0's broadcast, so an XGB
    individual asking for 'cuda:0' must be moved to the evaluating rank's GPU."""
    from types import SimpleNamespace
    from gentun_amd.parallel.distributed import _localize_device
    ev = SimpleNamespace(device="cuda:3")
    ind = SimpleNamespace(device="cuda:0")
    _localize_device(ind, ev)
    assert ind.device == "cuda:3"
    cpu_ind = SimpleNamespace(device=None)
    _localize_device(cpu_ind, ev)
    assert cpu_ind.device is None
    ind2 = SimpleNamespace(device="cuda:0")
    _localize_device(ind2, SimpleNamespace(device="cpu"))
    assert ind2.device == "cuda:0"


def _rccl_proc(port, q):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": "0",
                       "WORLD_SIZE": "1", "LOCAL_RANK": "0"})
    import sys
    import numpy as np
    import torch
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from fake_species import BitIndividual as Bit
    from gentun_amd.parallel import DistComm
    from gentun_amd.parallel.distributed import DistributedPopulation as DP
    from gentun_amd.parallel.evaluators import SequentialEvaluator as SE
    from gentun_amd import RussianRouletteGA as RR
    from gentun_amd.utils import rng as r
    torch.cuda.set_device(0)
    comm = DistComm(backend="nccl", timeout_s=60, device=torch.device("cuda", 0))
    assert comm.backend == "nccl" and comm.device.type == "cuda"
    arrays = [np.arange(12, dtype=np.float32).reshape(3, 4), np.array([1, -2, 3], np.int64),
              np.frombuffer(b"genome", np.uint8).copy(), np.zeros((0,), np.float64)]
    for a in arrays:
        b = comm.broadcast_array(a)
        assert b.dtype == a.dtype and b.shape == a.shape and np.array_equal(a, b)
    g = comm.all_gather_array(np.array([0.5, np.nan], np.float32))
    assert len(g) == 1 and g[0][0] == 0.5 and np.isnan(g[0][1])
    comm.barrier()
    r.seed(77)
    pop = DP(Bit, None, None, size=10, comm=comm, evaluator=SE())
    ga = RR(pop, verbose=False)
    ga.run(4)
    pop = ga.population
    pop.sync_ranks()
    pop.shutdown()
    q.put([(h["best_fitness"], h["evals"], tuple(sorted(h["best_genes"].items()))) for h in ga.history])
    comm.destroy()


@pytest.mark.gpu
def test_rccl_single_rank_matches_local_run():
    """The RCCL (backend "nccl") communicator on one GPU: typed broadcast /
    all_gather round trips and a distributed GA identical to the local run."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_proc, args=(_free_port(), q))
    p.start()
    hist = q.get(timeout=100)
    p.join(timeout=30)
    assert p.exitcode == 0
    assert hist == _local(BitIndividual, RussianRouletteGA, 4, seed=77, size=10)
