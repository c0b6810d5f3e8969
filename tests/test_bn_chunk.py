"""BatchNorm chunk geometry (CPU): pixels per workgroup are a function of the layer shape only (the
sums of a group never depend on the launch's other groups), whole row pairs where the 2x2 pool is fused
into the BN-apply launch, and small enough that wide stages fill the GPU."""

import pytest

from gentun_amd.ops import cnn_kernels as K


@pytest.mark.parametrize("H,W,Cp", [(32, 32, 24), (16, 16, 56), (8, 8, 104), (32, 32, 64), (16, 16, 128),
                                    (8, 8, 256), (28, 28, 24), (14, 14, 56), (7, 7, 104), (4, 4, 8)])
def test_bn_chunk_px(H, W, Cp):
    c = K.bn_chunk_px(H, W, Cp)
    assert c <= K.BN_CHUNK_PX and K.BN_CHUNK_PX % c == 0
    pooled = K.BN_CHUNK_PX % (2 * W) == 0
    if pooled:
        assert c % (2 * W) == 0                    # the fused pool needs whole row pairs per chunk
    # halved as far as allowed: either within the value budget or at the floor of the rule
    floor = 2 * W if pooled else 64
    assert c * Cp <= K.BN_CHUNK_VALUES or c // 2 < floor or (pooled and (c // 2) % (2 * W))
    assert K.bn_chunk_px(H, W, Cp) == c            # deterministic


def test_wide_stage_fills_the_gpu():
    # 256 channels at 8x8, batch 32: 4 chunks per group at 512 pixels, 32 now (800 workgroups at 25 groups)
    c = K.bn_chunk_px(8, 8, 256)
    assert -(-(32 * 64) // c) * 25 >= 512
