"""MNIST's 28 x 28 on the shape-specialised kernels: the HIP executor stores
the image zero-padded to 32 x 32 (bottom / right) and every forward epilogue
writes exact zeros outside the real rows / columns (ops/cnn_kernels.padded_hw,
ConvArgs::Hr / Wr). The padded network must BE the unpadded one: same
Glorot draws (keyed by the real index), zero W1 rows for padded pixels, and
training results equal to the unpadded run (generic kernels) up to
summation-order rounding. Reference default shape: gentun/individuals.py:221-223."""

import numpy as np
import pytest
import torch

from gentun_amd.ops import cnn_kernels as K


def test_padded_hw_rule():
    assert K.padded_hw(28, 28, 2) == (32, 32)          # MNIST S=(3,5): 32 / 16 / 8-wide stages
    assert K.padded_hw(32, 32, 2) == (32, 32)          # already a power of two
    assert K.padded_hw(28, 28, 3) == (28, 28)          # 28 / 8 is odd: floor pooling inside the padding
    assert K.padded_hw(28, 28, 2, batch_norm=True) == (32, 32)   # BN counts the real pixels only (BnArgs::Hr)
    assert K.padded_hw(20, 20, 2) == (20, 20)          # > 25 % wider
    assert K.padded_hw(28, 30, 2) == (28, 30)          # not square


def test_device_data_and_schedule_padding():
    from gentun_amd.models.cnn_engine import DeviceData
    from gentun_amd.models.genome import make_plan
    from gentun_amd.models.pop_schedule import PopulationSchedule
    x = np.random.RandomState(0).rand(4, 28, 28, 1).astype(np.float32)
    y = np.eye(10, dtype=np.float32)[[0, 1, 2, 3]]
    dd = DeviceData(x, y, torch.device("cpu"), "nhwc8f", pad_hw=(32, 32))
    assert tuple(dd.x.shape) == (4, 32, 32, 8)
    assert torch.equal(dd.x[:, :28, :28, :1], torch.from_numpy(x))
    assert float(dd.x[:, 28:].abs().sum()) == 0.0 and float(dd.x[:, :, 28:].abs().sum()) == 0.0
    plan = make_plan({'S_1': '101', 'S_2': '0101110011'}, (3, 5), (28, 28, 1), (20, 50), ((5, 5), (5, 5)), 500, 10)
    sched = PopulationSchedule([plan], hw=(32, 32))
    assert [(st.H, st.W, st.Hr, st.Wr) for st in sched.stages] == [(32, 32, 28, 28), (16, 16, 14, 14)]
    assert all((L.Hr, L.Wr) == (L.H * 28 // 32, L.W * 28 // 32) for L in sched.layers)


def _mnist_like(n=640):
    from gentun_amd.utils.data import make_image_classification, stratified_kfold
    x, y = make_image_classification(n=n, shape=(28, 28, 1), classes=10, seed=5, noise=0.35, shift=2)
    return x, y, stratified_kfold(np.argmax(y, 1), 3, seed=0)


# (dtype, max relative val-loss difference, max categorical-accuracy difference): bf16 rounds every
# activation to 8 bits, so padded (fast kernels) and unpadded (generic kernels) differ at bf16 level
PADDED_TOL = {"fp32": (2e-4, 0.05), "bf16": (2e-2, 0.1), "fp32+bn": (5e-4, 0.05)}


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,bn", [("fp32", False), ("bf16", False), ("fp32", True)])
@pytest.mark.parametrize("genes", [{'S_1': '101', 'S_2': '0101110011'}, {'S_1': '000', 'S_2': '0000000000'}])
def test_padded_mnist_matches_unpadded(genes, dtype, bn):
    """Reference default shape (28 x 28 x 1, kernels (20, 50), 5 x 5 stage convs): padded (fast
    kernels) and unpadded (generic kernels) training agree to summation-order rounding (fp32) or
    bf16 rounding (bf16), and the padded job really ran at 32 x 32.

    With BatchNorm (statistics over the real pixels only, zeros outside them: cnn_bn.hip BnArgs::Hr) the
    comparison runs SGD: the conv bias in front of BN has an analytically zero gradient, so both runs see
    pure rounding noise there, and Adam turns noise into +-lr steps (tools/probe_bn_pad.py on MI355X:
    identical at lr 1e-9, 1.3e-5 at Adam lr 1e-4, 1.5e-4 with SGD at 1e-3, but 2.7 % with Adam at 1e-3)."""
    from gentun_amd.models import cnn_engine as E
    from gentun_amd.models.genome import make_plan
    x, y, folds = _mnist_like()
    plan = make_plan(genes, (3, 5), (28, 28, 1), (20, 50), ((5, 5), (5, 5)), 500, 10)
    dev = torch.device("cuda", 0)
    res = {}
    for pad in (True, False):
        cfg = E.TrainConfig(epochs=(1,), learning_rate=(1e-3,), batch_size=32, dtype=dtype, loss="ce",
                            reset="all", pad_images=pad, batch_norm=bn, optimizer="sgd" if bn else "adam")
        job = E.make_job("hip", plan, x, y, folds, cfg, dev)
        assert (job.pad_hw == (32, 32)) == pad and tuple(job.data.x.shape[1:3]) == ((32, 32) if pad else (28, 28))
        job.launch()
        res[pad] = job.finish()
        if pad:
            # W1 rows of padded pixels (final 8 x 8 with 7 x 7 real) stay exactly zero through training
            W1 = job.views["W1"][0].view(job.Q, 8, 8, job.final_cp, job.Up)
            assert float(W1[:, 7:].abs().max()) == 0.0 and float(W1[:, :, 7:].abs().max()) == 0.0
    a, b = np.array(res[True]["val_loss"]), np.array(res[False]["val_loss"])
    tol_loss, tol_acc = PADDED_TOL[dtype + ("+bn" if bn else "")]
    assert np.all(np.isfinite(a)) and np.max(np.abs(a - b) / np.abs(b)) < tol_loss, (a, b)
    # near chance after one short epoch a rounding-level logit difference flips a few argmaxes (a fold
    # is ~214 samples): the loss is the tight check, the accuracy may move by a handful of samples
    ca, cb = np.array(res[True]["categorical_accuracy"]), np.array(res[False]["categorical_accuracy"])
    assert np.max(np.abs(ca - cb)) <= tol_acc, (ca, cb)
