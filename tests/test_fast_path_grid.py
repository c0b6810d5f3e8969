"""The fast path covers user-chosen architectures (VERDICT r5 missing #1): the
reference lets the user pick input_shape, kernels_per_layer and kernel_sizes
(gentun/individuals.py:221-223) and builds any of them at cuDNN speed
(keras_models.py:97-118). The HIP executor pads each stage's channels up to a
count the shape-specialised kernels are instantiated for
(cnn_kernels.stage_channel_pads) and stores slightly-smaller images
zero-padded (padded_hw, BatchNorm included), so every conv launch -- forward,
data gradient, weight gradient -- of every configuration of this grid runs a
shape-specialised kernel. The CPU test probes the dispatch tables (no launch);
the GPU test builds the real jobs and probes their launch arguments."""

import itertools

import numpy as np
import pytest

GRID = list(itertools.product([(32, 32, 3), (28, 28, 1)], [(16, 32), (20, 50), (32, 64), (64, 128)], [5, 3],
                              [False, True]))


def _lib_or_skip():
    try:
        from gentun_amd.ops import cnn_kernels as K
        K.lib()
        return K
    except Exception as exc:  # noqa: BLE001
        pytest.skip("HIP kernel library not loadable here: {}".format(exc))


def _plan(shape, kernels, k, genes=None):
    from gentun_amd.models.genome import make_plan
    genes = genes or {'S_1': '111', 'S_2': '1111111111'}
    return make_plan(genes, (3, 5), shape, kernels, ((k, k), (k, k)), 500, 10)


@pytest.mark.parametrize("shape,kernels,k,bn", GRID)
def test_every_launch_of_the_grid_is_fast(shape, kernels, k, bn):
    _lib_or_skip()
    from gentun_amd.models.cnn_hip import fast_path_report
    for ngroups in (2, 25, 80):
        r = fast_path_report(_plan(shape, kernels, k), ngroups=ngroups, batch_norm=bn)
        assert r["generic_launches"] == 0, r
        assert r["stored_hw"] == [32, 32]
        assert all(p >= c for p, c in zip(r["stage_channels_padded"], kernels))


def test_stage_pads_prefer_the_cheapest_fast_combination():
    K = _lib_or_skip()
    assert K.stage_channel_pads(3, [20, 50], [(5, 5)] * 2, 32, 32, 1) == [24, 56]
    assert K.stage_channel_pads(3, [16, 32], [(5, 5)] * 2, 32, 32, 1) == [24, 56]
    assert K.stage_channel_pads(3, [64, 128, 256], [(5, 5)] * 3, 32, 32, 1) == [64, 128, 256]
    # no fast combination within 2x of the channel counts: plain 8-padding (generic kernels)
    assert K.stage_channel_pads(3, [300, 600], [(5, 5)] * 2, 32, 32, 1) == [304, 600]


@pytest.mark.gpu
@pytest.mark.parametrize("shape,kernels,k,bn", GRID[::3] + [GRID[-1]])
def test_real_jobs_launch_only_fast_kernels(shape, kernels, k, bn):
    """The executor's own launch arguments (every forward conv, data gradient and weight gradient of a
    2-candidate population job) hit the shape-specialised kernels."""
    import torch
    from gentun_amd.models import cnn_engine as E
    from gentun_amd.ops import cnn_kernels as K
    from gentun_amd.utils.data import make_image_classification, stratified_kfold
    x, y = make_image_classification(n=96, shape=shape, classes=10, seed=1)
    folds = stratified_kfold(np.argmax(y, 1), 3, seed=0)
    plans = [_plan(shape, kernels, k, g) for g in ({'S_1': '111', 'S_2': '1111111111'},
                                                   {'S_1': '101', 'S_2': '0101110011'})]
    cfg = E.TrainConfig(epochs=(1,), learning_rate=(1e-3,), batch_size=32, dtype="fp32", reset="all", batch_norm=bn)
    job = E.make_population_job("hip", [(p, folds, [0, 1, 2]) for p in plans], x, y, cfg, torch.device("cuda", 0))
    L = K.lib()
    nconv = nw = 0
    for kind, a, Lr in job.fwd_ops + job.bwd_ops:
        if kind == "conv":
            assert L.gt_conv_fast_probe_any(a) == 1, (Lr.name, a.KH, a.Cinp, a.Coutp, a.W)
            nconv += 1
        elif kind == "wgrad":
            assert L.gt_wgrad_fast_band(a.KH, a.KW, a.Cinp, a.Coutp, a.H, a.W, a.prec) > 0, Lr.name
            nw += 1
    assert nconv > 0 and nw > 0
    assert job.pad_hw in (None, (32, 32)) and tuple(job.data.x.shape[1:3]) == (32, 32)
