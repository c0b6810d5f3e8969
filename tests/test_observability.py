"""Observability parity: the reference's progress lines and
a complete per-evaluation JSONL log in distributed runs.

* rank 0 prints " [*] Got fitness for individual i" once the gather returned
  it (gentun/master.py:72); the evaluating rank prints " [.] Evaluating
  individual i" (gentun/worker.py:43) -- ``i`` = population index;
* rank 0's event log holds one ``evaluation`` row per work unit of EVERY rank
  (rank, GA generation, dispatch, genes, folds, fold scores, fitness, wall_s);
* the Genetic-CNN engine prints "KFold i/n" and "Training N epochs with
  learning rate lr" (keras_models.py:134,137) when ``verbose``.

Two real processes on the gloo backend (CPU stand-in for RCCL)."""

import contextlib
import io
import os
import socket
import sys

import numpy as np
import torch.multiprocessing as mp

from gentun_amd.metrics import read_events


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _proc(rank, world, port, outdir, schedule):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank)})
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from fake_species import SlowBitIndividual as Bit
    from gentun_amd import GeneticAlgorithm
    from gentun_amd.metrics import EventLog
    from gentun_amd.parallel import DistComm
    from gentun_amd.parallel.distributed import DistributedPopulation, GentunWorker
    from gentun_amd.parallel.evaluators import SequentialEvaluator
    from gentun_amd.utils import rng
    buf = io.StringIO()
    comm = DistComm(backend="gloo", timeout_s=60)
    with contextlib.redirect_stdout(buf):
        if rank == 0:
            rng.seed(5)
            log = EventLog(os.path.join(outdir, "events.jsonl"))
            pop = DistributedPopulation(Bit, None, None, size=8, comm=comm, evaluator=SequentialEvaluator(),
                                        schedule=schedule)
            ga = GeneticAlgorithm(pop, verbose=False, event_log=log)
            ga.run(2)
            ga.population.shutdown()
            log.close()
        else:
            GentunWorker(Bit, None, None, comm=comm, evaluator=SequentialEvaluator()).work()
    comm.destroy()
    with open(os.path.join(outdir, "stdout{}.txt".format(rank)), "w") as f:
        f.write(buf.getvalue())


def _run(tmp_path, schedule):
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_proc, args=(r, 2, port, str(tmp_path), schedule)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    out = [open(os.path.join(str(tmp_path), "stdout{}.txt".format(r))).read() for r in range(2)]
    return out, read_events(os.path.join(str(tmp_path), "events.jsonl"))


def _check(out, events):
    evals = [e for e in events if e["kind"] == "evaluation"]
    gens = [e for e in events if e["kind"] == "generation"]
    assert [g["generation"] for g in gens] == [1, 2]
    # one row per unit; every unit came back from some rank, and both ranks evaluated
    assert len(evals) == sum(g["evals"] for g in gens)
    assert {e["rank"] for e in evals} == {0, 1}
    assert all(e["status"] == "ok" and e["fitness"] is not None and e["wall_s"] >= 0 for e in evals)
    assert sorted({e["generation"] for e in evals}) == [1, 2]
    for e in evals:                                 # BitIndividual: fitness = popcount of the genes
        assert e["fitness"] == sum(v.count("1") for v in e["genes"].values())
        assert e["fold_scores"] == [e["fitness"]] and e["folds"] == [0]
    # the reference's lines: every evaluated individual is announced by the rank that took it ...
    took = {r: {int(l.split()[-1]) for l in out[r].splitlines() if "[.] Evaluating individual" in l} for r in (0, 1)}
    for e in evals:
        assert e["i"] in took[e["rank"]]
    # ... and its fitness is reported on rank 0 after the gather
    got = [int(l.split()[-1]) for l in out[0].splitlines() if "[*] Got fitness for individual" in l]
    assert len(got) == len(evals)
    assert "[*] Got fitness" not in out[1]


def test_distributed_progress_lines_and_event_log_static(tmp_path):
    _check(*_run(tmp_path, "lpt"))


def test_distributed_progress_lines_and_event_log_dynamic(tmp_path):
    _check(*_run(tmp_path, "dynamic"))


def test_cnn_engine_prints_reference_fold_lines(capsys):
    """"KFold i/n" per fold and "Training N epochs with learning rate lr" per
    stage (keras_models.py:134,137), on the torch executor (CPU)."""
    import torch
    from gentun_amd.models.cnn import GeneticCnnModel
    from gentun_amd.utils.data import make_cifar_like
    x, y = make_cifar_like(n=40, seed=0)
    m = GeneticCnnModel(x, y, {'S_1': '1', 'S_2': '1'}, (2, 2), x.shape[1:], (4, 4), ((3, 3), (3, 3)), 8, 0.5, 10,
                        nfold=2, epochs=(1, 1), learning_rate=(1e-3, 1e-4), batch_size=16, backend="torch",
                        device=torch.device("cpu"), reset="kernels", verbose=True)
    fit = m.cross_validate()
    assert np.isfinite(fit)
    lines = [l for l in capsys.readouterr().out.splitlines() if l.startswith(("KFold", "Training"))]
    assert lines == ["KFold 1/2", "Training 1 epochs with learning rate 0.001",
                     "Training 1 epochs with learning rate 0.0001",
                     "KFold 2/2", "Training 1 epochs with learning rate 0.001",
                     "Training 1 epochs with learning rate 0.0001"]
