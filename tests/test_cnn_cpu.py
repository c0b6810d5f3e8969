"""Genetic-CNN fitness on the CPU (torch oracle path): fold-batched training,
Keras-compatible loss/metric semantics and the fitness plumbing."""

import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from gentun_amd import GeneticCnnIndividual, Population, RussianRouletteGA
from gentun_amd.models import cnn_engine as E
from gentun_amd.models.genome import make_plan
from gentun_amd.utils import rng
from gentun_amd.utils.data import make_image_classification, stratified_kfold

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _data(n=300):
    return make_image_classification(n=n, shape=(16, 16, 1), classes=4, seed=0, noise=0.3)


def test_loss_semantics_match_keras_definitions():
    logits = torch.tensor([[[2.0, 0.0, -1.0, 0.5]]])
    y = torch.tensor([[[1.0, 0.0, 0.0, 0.0]]])
    p = torch.softmax(logits, -1)
    per, binc, catc = E.loss_and_metrics(logits, y, "bce_compat")
    ref = -(y * torch.log(p) + (1 - y) * torch.log(1 - p)).mean(-1)
    assert torch.allclose(per, ref)
    assert binc.item() == 4.0 and catc.item() == 1.0     # binary_accuracy counts all 4 outputs
    per, _, _ = E.loss_and_metrics(logits, y, "ce")
    assert torch.allclose(per, -torch.log(p[..., 0]))
    # chance-level binary accuracy is 1 - 1/C, not 1/C
    per, binc, catc = E.loss_and_metrics(torch.zeros(1, 1, 10), torch.eye(10)[None, :1], "bce_compat")
    assert binc.item() == 9.0 and catc.item() == 1.0


@pytest.mark.parametrize("optimizer,lr", [("adam", 1e-3), ("sgd", 3e-3)])
def test_fold_batched_torch_training_learns(optimizer, lr):
    x, y = _data(900)
    folds = stratified_kfold(np.argmax(y, 1), 3, seed=0)
    plan = make_plan({'S_1': '000', 'S_2': '0000000000'}, (3, 5), (16, 16, 1), (8, 16), ((3, 3), (3, 3)), 64, 4)
    cfg = E.TrainConfig(epochs=(8,), learning_rate=(lr,), batch_size=16, dtype="fp32", loss="ce",
                        optimizer=optimizer, momentum=0.9)
    res = E.make_job("torch", plan, x, y, folds, cfg, "cpu").launch().finish()
    if optimizer == "sgd":           # plain SGD on a Glorot-init ReLU net is slow: require progress only
        assert np.mean(res["val_loss"]) < np.log(4) - 0.005
        return
    assert np.mean(res["categorical_accuracy"]) > 0.4 and max(res["categorical_accuracy"]) > 0.5  # chance 0.25
    assert len(res["binary_accuracy"]) == 3


def test_fold_results_independent_of_grouping():
    x, y = _data(200)
    folds = stratified_kfold(np.argmax(y, 1), 2, seed=0)
    plan = make_plan({'S_1': '100', 'S_2': '0000000000'}, (3, 5), (16, 16, 1), (8, 16), ((3, 3), (3, 3)), 32, 4)
    # dropout off: the torch oracle draws dropout masks from torch's global RNG
    # (the HIP path keys them by fold id; tests/test_hip_train.py checks that)
    cfg = E.TrainConfig(epochs=(1,), learning_rate=(1e-3,), batch_size=16, dtype="fp32", loss="ce", dropout=0.0,
                        reset="all")
    together = E.make_job("torch", plan, x, y, folds, cfg, "cpu", fold_ids=[0, 1]).launch().finish()
    alone = E.make_job("torch", plan, x, y, [folds[1]], cfg, "cpu", fold_ids=[1]).launch().finish()
    assert abs(together["val_loss"][1] - alone["val_loss"][0]) < 1e-4


def test_individual_fitness_and_small_search():
    x, y = _data(160)
    rng.seed(3)
    extra = dict(nodes=(3, 3), input_shape=(16, 16, 1), kernels_per_layer=(4, 8), kernel_sizes=((3, 3), (3, 3)),
                 dense_units=16, classes=4, nfold=2, epochs=(1,), learning_rate=(1e-3,), batch_size=16,
                 backend="torch", device="cpu", dtype="fp32")
    ind = GeneticCnnIndividual(x, y, **extra)
    f = ind.get_fitness()
    assert 0.0 <= f <= 1.0 and len(ind.fold_scores) == 2
    pop = Population(GeneticCnnIndividual, x, y, size=4, crossover_rate=0.3, mutation_rate=0.1,
                     additional_parameters=extra)
    ga = RussianRouletteGA(pop, verbose=False)
    best = ga.run(2)
    assert best.get_fitness() == max(h["best_fitness"] for h in ga.history)


def test_bench_contract_cpu():
    """bench.py prints exactly one JSON line with the driver's keys."""
    env = dict(os.environ, PYTHONPATH=ROOT)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1", "--warmup", "0",
                          "--per-gpu", "1", "--epochs", "1", "--lr", "1e-3", "--samples", "120", "--nfold", "2",
                          "--backend", "torch"], capture_output=True, text=True, env=env, timeout=600, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.strip()]
    assert len(lines) == 1
    rec = json.loads(lines[0])
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
                "vs_baseline", "dtype", "data", "config"):
        assert key in rec
    assert rec["n_gpus"] == 1 and rec["value"] > 0 and rec["higher_is_better"] is True


def test_sgd_momentum_update_rule():
    """One Keras-SGD step: v = mu v - lr g ; p += v (velocity reset per lr stage)."""
    x, y = _data(64)
    folds = stratified_kfold(np.argmax(y, 1), 2, seed=0)
    plan = make_plan({'S_1': '000', 'S_2': '0000000000'}, (3, 5), (16, 16, 1), (4, 4), ((3, 3), (3, 3)), 8, 4)
    cfg = E.TrainConfig(epochs=(1,), learning_rate=(0.1,), batch_size=8, dtype="fp32", loss="ce", dropout=0.0,
                        optimizer="sgd", momentum=0.5, reset="all")
    job = E.make_job("torch", plan, x, y, folds, cfg, "cpu")
    job.init_params()
    job.reset_optimizer(0.1)
    job._new_epoch_order()
    p0 = job.flat.detach().clone()
    job.train_step()
    g1 = job.flat.grad.clone()
    p1 = job.flat.detach().clone()
    assert torch.allclose(p1, p0 - 0.1 * g1, atol=1e-6)
    job.train_step()
    g2 = job.flat.grad.clone()
    assert torch.allclose(job.flat.detach(), p1 + 0.5 * (-0.1 * g1) - 0.1 * g2, atol=1e-6)
    with pytest.raises(ValueError):
        E.TrainConfig(optimizer="rmsprop")


def test_bench_contract_two_ranks_gloo():
    """The driver's multi-GPU launch (torch.distributed.run, one process per
    rank) rehearsed on CPU with gloo: one JSON line from rank 0, n_gpus = 2,
    whole-job candidates counted once."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1",
           "--warmup", "0", "--per-gpu", "1", "--epochs", "1", "--lr", "1e-3", "--samples", "120", "--nfold", "2",
           "--backend", "torch"]
    out = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=600, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.strip().startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["timed_candidates"] == 2 and rec["value"] > 0
    assert rec["config"]["parallelism"].startswith("population-dp2")
    assert rec["metric"].startswith("candidates/hour + best val-acc@genN") and rec["dtype"] == "fp32"


def test_reference_sequential_folds_carry_biases():
    """reset="kernels" (default, keras_models.py:120-125,135): folds run in
    sequence; fold k+1 re-draws the kernels and starts from the biases fold k
    trained."""
    x, y = _data(200)
    folds = stratified_kfold(np.argmax(y, 1), 3, seed=0)
    plan = make_plan({'S_1': '101', 'S_2': '0000000000'}, (3, 5), (16, 16, 1), (8, 16), ((3, 3), (3, 3)), 32, 4)
    cfg = E.TrainConfig(epochs=(1,), learning_rate=(1e-2,), batch_size=16, dtype="fp32", loss="ce", dropout=0.0)
    assert cfg.reset == "kernels" and cfg.batching == "keras"
    job = E.make_job("torch", plan, x, y, folds, cfg, "cpu")
    assert isinstance(job, E.SequentialFoldJob)
    seen = []

    def spy(orig):
        def hook(j):
            orig(j)
            seen.append({n: t.detach().clone() for n, t in j._views().items()})
        return hook

    made = job.make

    def make(f):
        j = made(f)
        j.after_init = None
        return j
    job.make = make
    # run the folds by hand to look at the weights between them
    prev = None
    finals = []
    for f in range(3):
        j = job.make(f)
        if prev is not None:
            j.after_init = spy(E._carry_biases(prev))
        j.launch()
        j.finish()
        finals.append({n: t.detach().clone() for n, t in j._views().items()})
        prev = j
    for f in (1, 2):
        start = seen[f - 1]
        for n in start:
            if n.endswith(".b"):
                assert torch.equal(start[n], finals[f - 1][n]), n          # biases carried over
                assert not torch.equal(start[n], torch.zeros_like(start[n])) or n == "dense2.b"
            else:
                assert not torch.equal(start[n], finals[f - 1][n]), n      # kernels re-drawn
    res = E.make_job("torch", plan, x, y, folds, cfg, "cpu").launch().finish()
    assert len(res["val_loss"]) == 3


def test_keras_short_last_batch_weights():
    """batching="keras": 10 steps of 16 for 150 training rows, the last with
    6 real rows; the torch oracle's loss is the mean over those rows only."""
    x, y = _data(190)
    fold = (np.arange(150), np.arange(150, 190))
    plan = make_plan({'S_1': '000', 'S_2': '0000000000'}, (3, 5), (16, 16, 1), (4, 8), ((3, 3), (3, 3)), 16, 4)
    k = E.TrainConfig(epochs=(1,), learning_rate=(1e-3,), batch_size=16, dtype="fp32", loss="ce", dropout=0.0)
    w = E.TrainConfig(epochs=(1,), learning_rate=(1e-3,), batch_size=16, dtype="fp32", loss="ce", dropout=0.0,
                      batching="wrap")
    jk = E.make_job("torch", plan, x, y, [fold], k, "cpu")
    jw = E.make_job("torch", plan, x, y, [fold], w, "cpu")
    assert jk.steps_per_epoch == 10
    assert jk.epoch_valid[:, 0].tolist() == [16] * 9 + [6]
    assert jw.epoch_valid[:, 0].tolist() == [16] * 10
    rk = jk.launch().finish()
    rw = jw.launch().finish()
    assert rk["val_loss"][0] != rw["val_loss"][0]
