"""Intra-candidate data parallelism (optional): two gloo
ranks each train on half of every batch and all-reduce the gradients; the
trajectory equals the single-process run of the same job (dropout masks and
the Keras short last batch included)."""

import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _job(dp_group=None):
    from gentun_amd.models import cnn_engine as E
    from gentun_amd.models.genome import make_plan
    from gentun_amd.utils.data import make_image_classification
    x, y = make_image_classification(n=60, shape=(8, 8, 1), classes=4, seed=0, noise=0.3)
    fold = (np.arange(40), np.arange(40, 60))          # 40 training rows: batches of 16, 16 and 8
    plan = make_plan({'S_1': '101', 'S_2': '0000000000'}, (3, 5), (8, 8, 1), (4, 8), ((3, 3), (3, 3)), 16, 4)
    cfg = E.TrainConfig(epochs=(1,), learning_rate=(1e-2,), batch_size=16, dtype="fp32", loss="bce_compat",
                        dropout=0.5, dp_group=dp_group)
    return E.TorchFoldJob(plan, x, y, [fold, (fold[0][::-1].copy(), fold[1])], cfg, "cpu", fold_ids=[0, 1])


def _train(job):
    job.init_params()
    job.reset_optimizer(1e-2)
    job._new_epoch_order()
    for _ in range(job.steps_per_epoch):
        job.train_step()
    return job.flat.detach().clone()


def _worker(rank, port, out):
    import torch.distributed as dist
    torch.set_num_threads(1)
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:{}".format(port), rank=rank, world_size=2)
    try:
        flat = _train(_job(dp_group=dist.group.WORLD))
        torch.save(flat, os.path.join(out, "rank{}.pt".format(rank)))
    finally:
        dist.destroy_process_group()


def test_two_rank_data_parallel_matches_single_process():
    single = _train(_job())
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(port, d), nprocs=2, join=True)
        r0 = torch.load(os.path.join(d, "rank0.pt"), weights_only=True)
        r1 = torch.load(os.path.join(d, "rank1.pt"), weights_only=True)
    assert torch.equal(r0, r1)                          # identical optimizer steps on every rank
    assert torch.allclose(r0, single, atol=2e-6, rtol=1e-5), (r0 - single).abs().max()


def test_data_parallel_rejects_batchnorm():
    from gentun_amd.models import cnn_engine as E

    class FakeGroup(object):
        pass
    job = _job()
    job.cfg.batch_norm = True
    job.cfg.dp_group = FakeGroup()
    with pytest.raises(ValueError, match="BatchNorm"):
        job.train_step()
