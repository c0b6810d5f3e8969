"""Population-batched torch executor (TorchPopJob, comparator (a)): several
architectures of one search space in one set of grouped convolutions must
train like the one-architecture oracle (TorchFoldJob), in both fold
protocols. Different group counts change the CPU conv kernels' blocking, so
agreement is to fp32 rounding noise, not bitwise."""

import numpy as np
import pytest
import torch

from gentun_amd.models import cnn_engine as E
from gentun_amd.models.genome import make_plan
from gentun_amd.utils.data import make_cifar_like, stratified_kfold

GENES = [{'S_1': '101', 'S_2': '0101110011'},
         {'S_1': '000', 'S_2': '1000000001'},      # stage 1 without a DAG
         {'S_1': '010', 'S_2': '0000000000'}]      # isolated nodes / stage 2 without a DAG


@pytest.mark.parametrize("reset", ["all", "kernels"])
def test_torch_pop_matches_single_jobs(reset):
    x, y = make_cifar_like(n=160, seed=0)
    folds = stratified_kfold(np.argmax(y, 1), 2, seed=0)
    plans = [make_plan(g, (3, 5), (32, 32, 3), (8, 12), ((5, 5), (5, 5)), 32, 10) for g in GENES]
    cfg = E.TrainConfig(epochs=(1,), learning_rate=(1e-3,), batch_size=32, use_graph=False, reset=reset)
    singles = []
    for p in plans:
        job = E.make_job("torch", p, x, y, folds, cfg, torch.device("cpu"))
        job.launch()
        singles.append(job.finish())
    pop = E.make_population_job("torch", [(p, folds, [0, 1]) for p in plans], x, y, cfg, torch.device("cpu"))
    pop.launch()
    res = pop.finish()
    assert len(res) == len(plans)
    for k, (a, b) in enumerate(zip(singles, res)):
        for key in ("val_loss", "binary_accuracy", "categorical_accuracy"):
            np.testing.assert_allclose(a[key], b[key], rtol=0, atol=1e-4, err_msg="member {} {}".format(k, key))


def test_torch_pop_rejects_mixed_spaces():
    x, y = make_cifar_like(n=64, seed=0)
    folds = stratified_kfold(np.argmax(y, 1), 2, seed=0)
    a = make_plan(GENES[0], (3, 5), (32, 32, 3), (8, 12), ((5, 5), (5, 5)), 32, 10)
    b = make_plan(GENES[0], (3, 5), (32, 32, 3), (8, 16), ((5, 5), (5, 5)), 32, 10)
    cfg = E.TrainConfig(epochs=(1,), learning_rate=(1e-3,), batch_size=32, use_graph=False, reset="all")
    with pytest.raises(ValueError):
        E.make_population_job("torch", [(a, folds, [0, 1]), (b, folds, [0, 1])], x, y, cfg, torch.device("cpu"))
