"""X5 on the HIP executor (optional): two ranks (gloo, both on
GPU 0 -- the multi-GPU path is RCCL with the same code) each train rows
[r0, r1) of every batch of a population job with the HIP kernels, the
gradients (conv weight gradients after their split-K reduce, dW1 from the
dense weight-gradient kernel in gradient-only mode, dW2 / db2 / db1) are
summed by one all-reduce, and the identical optimizer step follows. The
trajectory equals the single-process run of the same job up to the gradient
summation order (dropout keyed by the full-batch row, Keras short last batch
normalised by the full batch; SGD-momentum -- see _job).

The bound is derived, not ad hoc: data parallelism changes only the ORDER in
which every gradient is summed (two half-batch sums, then the all-reduce).
The reference scale for that is the same single-process job with its conv
weight gradients summed in a different split-K order (``K.WGRAD_FAST_SPLITS``:
another split count = another fp32 summation order of the same terms, nothing
else changes). The data-parallel trajectory must stay within a small multiple
of that reordering drift (ReLU decisions near zero turn rounding-level
differences into larger parameter differences over the steps; both drifts see
the same amplification) AND under an absolute ceiling, so a growing reorder
drift cannot widen the bound unnoticed. Measured values are
appended to ``$GENTUN_DP_RECORD`` when set (profiles/r5/dp_drift_r5.txt)."""

import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

# data-parallel drift allowed, in units of the single-process reordering drift (see module docstring)
DP_ORDER_FACTOR = 8.0
# and in absolute terms (relative to the largest parameter)
DP_MAX_DRIFT = 5e-4


def _job(dp_group=None, hw=32):
    # hw 28: MNIST-sized images, stored zero-padded to 32 x 32 (the padded fast path)
    from gentun_amd.models import cnn_engine as E
    from gentun_amd.models.genome import make_plan
    from gentun_amd.utils.data import make_image_classification, stratified_kfold
    x, y = make_image_classification(n=520, shape=(hw, hw, 3), classes=10, seed=3, noise=0.35, shift=3)
    folds = stratified_kfold(np.argmax(y, 1), 2, seed=0)     # 260 training rows: a short last batch
    plans = [make_plan(g, (3, 5), (hw, hw, 3), (20, 50), ((5, 5), (5, 5)), 500, 10)
             for g in ({'S_1': '101', 'S_2': '0101110011'}, {'S_1': '000', 'S_2': '1000000001'})]
    # SGD: Adam turns the summation-order noise of near-zero gradients into +-lr steps (sign flips), which
    # would hide a real mismatch; with SGD-momentum the two trajectories must agree to fp32 rounding
    cfg = E.TrainConfig(epochs=(1,), learning_rate=(1e-2,), batch_size=32, dtype="fp32", loss="bce_compat",
                        reset="all", optimizer="sgd", momentum=0.9, dp_group=dp_group)
    return E.make_population_job("hip", [(p, folds, [0, 1]) for p in plans], x, y, cfg, torch.device("cuda", 0))


def _reordered_single(hw):
    """The single-process run with every specialised conv wgrad summed in another split order."""
    from gentun_amd.ops import cnn_kernels as K
    old = K.WGRAD_FAST_SPLITS
    K.WGRAD_FAST_SPLITS = 4
    try:
        return _train(_job(hw=hw))
    finally:
        K.WGRAD_FAST_SPLITS = old


def _train(job):
    job.launch()
    res = job.finish()
    torch.cuda.synchronize()
    return job.flat.detach().cpu().clone(), res


def _worker(rank, port, out, ct1, hw):
    import torch.distributed as dist
    from gentun_amd.ops import cnn_kernels as K
    torch.cuda.set_device(0)
    K.lib().gt_conv_set_s2in_ct1(int(ct1))
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:{}".format(port), rank=rank, world_size=2)
    try:
        flat, res = _train(_job(dp_group=dist.group.WORLD, hw=hw))
        torch.save({"flat": flat, "cat": [r["categorical_accuracy"] for r in res]},
                   os.path.join(out, "rank{}.pt".format(rank)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("ct1,hw", [("1", 32), ("0", 32), ("1", 28)])
def test_two_rank_hip_data_parallel_matches_single_process(ct1, hw):
    # ct1: the stage-2 input-conv dgrad with one co tile per wave (the default) or the packed tile;
    # hw 28: the zero-padded MNIST geometry on two ranks
    from gentun_amd.ops import cnn_kernels as K
    old = K.lib().gt_conv_set_s2in_ct1(int(ct1))
    try:
        _compare(ct1, hw)
    finally:
        K.lib().gt_conv_set_s2in_ct1(old)


def _compare(ct1, hw):
    single, sres = _train(_job(hw=hw))
    again, _ = _train(_job(hw=hw))
    assert torch.equal(single, again)                       # the executor itself is deterministic
    reorder, _ = _reordered_single(hw)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(port, d, ct1, hw), nprocs=2, join=True)
        r0 = torch.load(os.path.join(d, "rank0.pt"), weights_only=True)
        r1 = torch.load(os.path.join(d, "rank1.pt"), weights_only=True)
    assert torch.equal(r0["flat"], r1["flat"])              # identical optimizer steps on every rank
    scale = single.abs().max().item()
    d_dp = (r0["flat"] - single).abs().max().item() / scale
    d_order = (reorder - single).abs().max().item() / scale
    line = "[dp] ct1={} hw={} relative drift: data-parallel {:.3e}, single-process split reorder {:.3e}, ratio {:.2f}".format(
        ct1, hw, d_dp, d_order, d_dp / max(d_order, 1e-30))
    print(line)
    if os.environ.get("GENTUN_DP_RECORD"):
        with open(os.environ["GENTUN_DP_RECORD"], "a") as f:
            f.write(line + "\n")
    assert d_order > 0                                      # the reorder really changed the summation
    assert d_dp <= DP_ORDER_FACTOR * max(d_order, 2.0 ** -23), (d_dp, d_order)
    assert d_dp <= DP_MAX_DRIFT, (d_dp, d_order)
    for a, b in zip(r0["cat"], [r["categorical_accuracy"] for r in sres]):
        assert np.allclose(a, b, atol=0.02)
