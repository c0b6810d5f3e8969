"""Optional BatchNorm (TrainConfig.batch_norm; off by default, the reference
network has none): the torch oracle's per-group BatchNorm against
torch.nn.BatchNorm2d, the Keras short batch, the sequential-fold carry-over
and the plumbing from the individual down to the executors (CPU)."""

import numpy as np
import pytest
import torch

from gentun_amd import GeneticCnnIndividual
from gentun_amd.models import cnn_engine as E
from gentun_amd.models.genome import make_plan
from gentun_amd.utils.data import make_image_classification, stratified_kfold


def _job(G=2, B=8, bn=True, reset="all", n=120):
    x, y = make_image_classification(n=n, shape=(8, 8, 1), classes=4, seed=0, noise=0.3)
    folds = stratified_kfold(np.argmax(y, 1), max(2, G), seed=0)
    plan = make_plan({'S_1': '101', 'S_2': '0000000000'}, (3, 5), (8, 8, 1), (4, 8), ((3, 3), (3, 3)), 16, 4)
    cfg = E.TrainConfig(epochs=(1,), learning_rate=(1e-2,), batch_size=B, dtype="fp32", loss="ce", dropout=0.0,
                        batch_norm=bn, reset=reset)
    return E.make_job("torch", plan, x, y, folds[:G], cfg, "cpu"), x, y, folds, plan, cfg


def _reference_bn(z, gamma, beta, rm, rv, train, momentum=0.01, eps=1e-3):
    m = torch.nn.BatchNorm2d(z.shape[1], eps=eps, momentum=momentum).double()
    with torch.no_grad():
        m.weight.copy_(gamma)
        m.bias.copy_(beta)
        m.running_mean.copy_(rm)
        m.running_var.copy_(rv)
    m.train(train)
    out = m(z.double())
    return out, m.running_mean.detach(), m.running_var.detach()


@pytest.mark.parametrize("train", [True, False])
def test_oracle_bn_matches_batchnorm2d(train):
    job, *_ = _job(G=2, B=8)
    torch.manual_seed(0)
    G, C, H, W, B = 2, 5, 6, 6, 8
    z = torch.randn(B, G * C, H, W) * 3 + 2
    job.bn_run = {"t": torch.stack([torch.randn(G, C), torch.rand(G, C) + 0.5])}
    run0 = job.bn_run["t"].clone()
    P = {"t.gamma": torch.rand(G, C) + 0.5, "t.beta": torch.randn(G, C)}
    out = job._bn(z, "t", P, train, torch.full((G,), B))
    for g in range(G):
        sl = slice(g * C, (g + 1) * C)
        ref, rm, rv = _reference_bn(z[:, sl], P["t.gamma"][g], P["t.beta"][g], run0[0, g], run0[1, g], train)
        assert torch.allclose(out[:, sl].double(), ref, atol=2e-5, rtol=1e-5)
        assert torch.allclose(job.bn_run["t"][0, g].double(), rm, atol=1e-6)
        assert torch.allclose(job.bn_run["t"][1, g].double(), rv, atol=1e-5)


def test_oracle_bn_short_batch_uses_real_rows_only():
    """Keras short last batch: the statistics of group g come from its first
    nval[g] rows only, exactly BatchNorm2d on those rows."""
    job, *_ = _job(G=2, B=8)
    torch.manual_seed(1)
    G, C, H, W, B = 2, 3, 4, 4, 8
    z = torch.randn(B, G * C, H, W)
    job.bn_run = {"t": torch.stack([torch.zeros(G, C), torch.ones(G, C)])}
    P = {"t.gamma": torch.ones(G, C), "t.beta": torch.zeros(G, C)}
    nval = torch.tensor([8, 5])
    out = job._bn(z, "t", P, True, nval)
    ref, rm, rv = _reference_bn(z[:5, C:], torch.ones(C), torch.zeros(C), torch.zeros(C), torch.ones(C), True)
    assert torch.allclose(out[:5, C:].double(), ref, atol=2e-5)
    assert torch.allclose(job.bn_run["t"][1, 1].double(), rv, atol=1e-5)


def test_bn_training_learns_and_differs_from_plain():
    res = {}
    for bn in (False, True):
        job, *_ = _job(G=2, B=16, bn=bn, n=300)
        res[bn] = job.launch().finish()
    assert res[True]["val_loss"] != res[False]["val_loss"]
    assert np.all(np.isfinite(res[True]["val_loss"]))
    assert np.mean(res[True]["val_loss"]) < np.log(4) + 0.5


def test_bn_parameters_and_carry_over():
    """gamma starts at 1, beta at 0; sequential folds keep gamma / beta /
    running statistics (reset_weights re-draws kernels only,
    keras_models.py:120-125)."""
    job, x, y, folds, plan, cfg = _job(G=1, B=8, bn=True, reset="kernels")
    job.init_params()
    names = [n for n, _, _, _ in job.shapes]
    assert sum(n.endswith(".gamma") for n in names) == len(plan.convs())
    v = job._views()
    assert all(torch.all(v[n] == 1) for n in names if n.endswith(".gamma"))
    other = E.make_job("torch", plan, x, y, [folds[1]], cfg, "cpu", fold_ids=[1])
    other.init_params()
    with torch.no_grad():
        for n in names:
            if n.endswith(".gamma") or n.endswith(".beta"):
                other._views()[n].add_(0.25)
        for r in other.bn_run.values():
            r.add_(0.5)
    job.copy_biases_from(other)
    va, vb = job._views(), other._views()
    for n in names:
        if n.endswith((".gamma", ".beta", ".b")):
            assert torch.equal(va[n], vb[n]), n
        else:
            assert not torch.equal(va[n], vb[n]), n
    for k in job.bn_run:
        assert torch.equal(job.bn_run[k], other.bn_run[k])


def test_batch_norm_flows_from_the_individual():
    x, y = make_image_classification(n=60, shape=(8, 8, 1), classes=4, seed=0)
    ind = GeneticCnnIndividual(x, y, nodes=(3, 3), input_shape=(8, 8, 1), kernels_per_layer=(4, 4),
                               kernel_sizes=((3, 3), (3, 3)), dense_units=8, classes=4, nfold=2, epochs=(1,),
                               learning_rate=(1e-3,), batch_size=8, backend="torch", device="cpu", batch_norm=True)
    assert ind.get_additional_parameters()["batch_norm"] is True
    assert ind.build_fitness_model().cfg.batch_norm is True
    assert ind.copy().batch_norm is True
    assert E.TrainConfig().batch_norm is False
