"""Streaming dense forward / data-gradient kernels (cnn_dense.hip:
dense_fwd_stream_kernel, dense_dgrad_stream_kernel -- the defaults) against
the round-2 kernels they replace (gt_dense_set_stream(0)): same k-step order
and reduction order, so the outputs must be BIT-identical, in both
precisions, with the fused partial logits, dropout and a padded batch."""

import ctypes

import pytest
import torch

from gentun_amd.ops import cnn_kernels as Km

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _lib():
    L = Km.lib()
    L.gt_dense_set_stream.argtypes = [ctypes.c_int]
    L.gt_dense_set_stream.restype = ctypes.c_int
    L.gt_dense_set_dgrad2.argtypes = [ctypes.c_int]
    L.gt_dense_set_dgrad2.restype = ctypes.c_int
    L.gt_dense_set_f32mma.argtypes = [ctypes.c_int]
    L.gt_dense_set_f32mma.restype = ctypes.c_int
    return L


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


@pytest.mark.parametrize("prec", [1, 0])
@pytest.mark.parametrize("G,B,Fp,Up", [(5, 32, 3584, 512), (3, 20, 392, 128)])
def test_dense_stream_bit_identical(prec, G, B, Fp, Up):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    L = _lib()
    torch.manual_seed(0)
    adt = torch.float32 if prec else torch.bfloat16
    C = 10
    w1 = torch.randn(G, Fp, Up, device=DEV) * 0.05                 # fp32 master [G][Fp][Up]
    wt = w1.transpose(1, 2).contiguous().to(adt)                   # the copy dense_fwd reads [G][Up][Fp]
    x = torch.randn(G, B, Fp, device=DEV).to(adt)
    b1 = torch.randn(G, Up, device=DEV) * 0.1
    w2 = torch.randn(G, Up, C, device=DEV) * 0.05
    st = torch.zeros(8, dtype=torch.int32, device=DEV)
    fids = torch.arange(G, dtype=torch.int32, device=DEV)
    dH = torch.randn(G, B, Up, device=DEV)
    from gentun_amd.models.cnn_hip import split_planes
    dHp = split_planes(dH, 3 if prec else 1).view(torch.int16).contiguous()     # head_bwd's planes
    outs = []
    old_f32 = L.gt_dense_set_f32mma(0)       # the bf16x6 kernels among themselves (fp32: f32-MFMA test below)
    for mode in (0, 1, 2):                   # round-2 kernels, streaming v1, streaming v2 (dH planes)
        old = L.gt_dense_set_stream(1 if mode else 0)
        try:
            out = torch.zeros(G, B, Up, dtype=adt, device=DEV)
            plog = torch.zeros(G, Up // 16, B, C, device=DEV)
            a = Km.DenseFwdArgs()
            a.x, a.wt, a.bias, a.out, a.st, a.fold_ids = x.data_ptr(), wt.data_ptr(), b1.data_ptr(), \
                out.data_ptr(), st.data_ptr(), fids.data_ptr()
            a.G, a.B, a.Fp, a.Up, a.drop_p, a.train, a.seed = G, B, Fp, Up, 0.5, 1, 7
            a.w2, a.plog, a.C, a.prec = w2.data_ptr(), plog.data_ptr(), C, prec
            Km.check(L.gt_dense_fwd(a, _stream()), "dense_fwd")
            dx = torch.zeros(G, B, Fp, dtype=adt, device=DEV)
            d = Km.DenseDgradArgs()
            d.dH, d.wt, d.dx, d.G, d.B, d.Fp, d.Up, d.prec = dH.data_ptr(), wt.data_ptr(), dx.data_ptr(), \
                G, B, Fp, Up, prec
            d.w1 = w1.data_ptr() if mode else 0
            d.dHp = dHp.data_ptr() if mode == 2 else 0
            Km.check(L.gt_dense_dgrad(d, _stream()), "dense_dgrad")
            torch.cuda.synchronize()
            outs.append((out.clone(), plog.clone(), dx.clone()))
        finally:
            L.gt_dense_set_stream(old)
    L.gt_dense_set_f32mma(old_f32)
    for k in (1, 2):
        for name, r0, r1 in zip(("h", "plog", "dx"), outs[0], outs[k]):
            assert torch.equal(r0, r1), "{} {} differs: max {}".format(k, name, (r0.float() - r1.float()).abs().max().item())
    # and against the math (fp32: split-MFMA level; bf16: bf16 level)
    ref = torch.bmm(dH.double(), w1.double().transpose(1, 2))
    err = (outs[1][2].double() - ref).abs().max().item() / ref.abs().max().item()
    assert err < (1e-5 if prec else 2e-2)


@pytest.mark.parametrize("prec", [1, 0])
@pytest.mark.parametrize("G,B,Fp,Up,ks", [(5, 32, 3584, 512, None), (3, 20, 392, 128, 3), (2, 64, 392, 128, 1)])
def test_dense_fwd_split_k(prec, G, B, Fp, Up, ks):
    """Split-K forward from the fp32 W1 master (dense_fwd_sk_kernel, the
    default): same dropout mask as the streaming kernel, values at the
    split-MFMA level of an fp64 reference, bitwise deterministic across
    launches and independent of how many groups share the launch."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    L = _lib()
    torch.manual_seed(1)
    adt = torch.float32 if prec else torch.bfloat16
    C = 10
    w1 = torch.randn(G, Fp, Up, device=DEV) * 0.05
    if not prec:
        w1 = w1.to(torch.bfloat16).float()                         # the bf16 path multiplies RNE roundings
    wt = w1.transpose(1, 2).contiguous().to(adt)
    x = torch.randn(G, B, Fp, device=DEV).to(adt)
    b1 = torch.randn(G, Up, device=DEV) * 0.1
    w2 = torch.randn(G, Up, C, device=DEV) * 0.05
    st = torch.zeros(8, dtype=torch.int32, device=DEV)
    fids = torch.arange(G, dtype=torch.int32, device=DEV)
    ks = ks or L.gt_dense_fwd_splits(Fp)

    def run(g, sk):
        out = torch.zeros(g, B, Up, dtype=adt, device=DEV)
        plog = torch.zeros(g, Up // 16, B, C, device=DEV)
        a = Km.DenseFwdArgs()
        a.x, a.wt, a.bias, a.out, a.st, a.fold_ids = x.data_ptr(), wt.data_ptr(), b1.data_ptr(), \
            out.data_ptr(), st.data_ptr(), fids.data_ptr()
        a.G, a.B, a.Fp, a.Up, a.drop_p, a.train, a.seed = g, B, Fp, Up, 0.5, 1, 7
        a.w2, a.plog, a.C, a.prec = w2.data_ptr(), plog.data_ptr(), C, prec
        keep = []
        if sk:
            nby, nut = -(-B // 32), Up // 64
            part = torch.empty(g * nby * nut * ks * 4 * 2 * 64 * 4, device=DEV)
            cnt = torch.zeros(g * nby * nut, dtype=torch.int32, device=DEV)
            keep = [part, cnt]
            a.w1, a.part, a.cnt, a.ks = w1.data_ptr(), part.data_ptr(), cnt.data_ptr(), ks
        Km.check(L.gt_dense_fwd(a, _stream()), "dense_fwd")
        torch.cuda.synchronize()
        return out.clone(), plog.clone()

    ref_h, ref_p = run(G, False)
    h1, p1 = run(G, True)
    h2, p2 = run(G, True)
    assert torch.equal(h1, h2) and torch.equal(p1, p2)
    hs, ps = run(2, True)                                          # groups 0-1 alone
    assert torch.equal(hs, h1[:2]) and torch.equal(ps, p1[:2])
    assert ((h1 == 0) != (ref_h == 0)).float().mean().item() < 1e-4   # same dropout mask (ReLU ties aside)
    z = torch.relu(torch.bmm(x.double(), w1.double()) + b1.double()[:, None, :])
    keep_mask = (ref_h != 0)
    dense = (z * 2.0 * keep_mask).float()                          # inverted dropout, p = 0.5
    err = ((h1.float() - dense).abs().max() / dense.abs().max()).item()
    assert err < (1e-5 if prec else 2e-2), err


@pytest.mark.parametrize("G,B,Fp,Up", [(5, 32, 3584, 512), (3, 20, 392, 128), (2, 64, 392, 96)])
def test_dense_f32_mfma_dgrad(G, B, Fp, Up):
    """fp32 data gradient on the f32-input MFMA (dense_dgrad_f32_kernel, the fp32 default): exact f32
    products, so dx sits at fp32-accumulation level of an fp64 reference (tighter than the bf16x6 kernel it
    replaces, which it matches to that level); bitwise deterministic and independent of the groups sharing
    the launch; feature / batch tails (Fp 392 is not a multiple of the 128-feature tile, B 20 not of 32)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    L = _lib()
    torch.manual_seed(3)
    w1 = torch.randn(G, Fp, Up, device=DEV) * 0.05
    wt = w1.transpose(1, 2).contiguous()
    dH = torch.randn(G, B, Up, device=DEV)

    def run(g, f32):
        old = L.gt_dense_set_f32mma(f32)
        try:
            dx = torch.zeros(g, B, Fp, device=DEV)
            d = Km.DenseDgradArgs()
            d.dH, d.wt, d.dx, d.G, d.B, d.Fp, d.Up, d.prec = dH.data_ptr(), wt.data_ptr(), dx.data_ptr(), g, B, Fp, Up, 1
            d.w1 = w1.data_ptr()
            Km.check(L.gt_dense_dgrad(d, _stream()), "dense_dgrad")
            torch.cuda.synchronize()
            return dx
        finally:
            L.gt_dense_set_f32mma(old)

    dx1, dx2, dxs, dx0 = run(G, 1), run(G, 1), run(2, 1), run(G, 0)
    assert torch.equal(dx1, dx2) and torch.equal(dxs, dx1[:2])
    ref = torch.bmm(dH.double(), w1.double().transpose(1, 2))
    err = ((dx1.double() - ref).abs().max() / ref.abs().max()).item()
    assert err < 2e-6, err
    assert ((dx1 - dx0).abs().max() / dx1.abs().max()).item() < 1e-5


def test_dense_copy_kernels_refuse_a_missing_copy():
    """A job on the split-K path does not maintain the transposed W1 copy and passes none; turning the
    split-K switch off afterwards must fail the launch (-3), not train on a stale copy."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    L = _lib()
    L.gt_dense_set_sk.argtypes = [ctypes.c_int]
    L.gt_dense_set_sk.restype = ctypes.c_int
    G, B, Fp, Up, C = 1, 32, 64, 64, 10
    w1 = torch.zeros(G, Fp, Up, device=DEV)
    x = torch.zeros(G, B, Fp, device=DEV)
    out = torch.zeros(G, B, Up, device=DEV)
    b1 = torch.zeros(G, Up, device=DEV)
    a = Km.DenseFwdArgs()
    a.x, a.wt, a.bias, a.out = x.data_ptr(), 0, b1.data_ptr(), out.data_ptr()
    a.G, a.B, a.Fp, a.Up, a.C, a.prec, a.w1, a.ks = G, B, Fp, Up, C, 1, w1.data_ptr(), 1
    old = L.gt_dense_set_sk(0)
    try:
        assert L.gt_dense_fwd(a, _stream()) == -3
    finally:
        L.gt_dense_set_sk(old)
