"""Dense head kernels (csrc/hip/cnn_dense.hip) straight from the fp32 W1 master: the split-K forward
(dense_fwd_sk_kernel + the in-order range reduce and epilogue) in both precisions, the data gradient (fp32:
the f32-input MFMA; bf16 mode: the bf16 MFMA on head_bwd's bf16 dH), against fp64 references; bitwise
deterministic, independent of how many groups share a launch, dropout semantics, and launchers that refuse
to run without the master (there is no transposed W1 copy any more)."""

import ctypes

import pytest
import torch

from gentun_amd.ops import cnn_kernels as Km

pytestmark = pytest.mark.gpu
DEV = "cuda"
SHAPES = [(5, 32, 3584, 512), (3, 20, 392, 128), (2, 64, 392, 128)]


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _fwd(L, x, w1, b1, w2, g, B, Fp, Up, prec, drop_p, train, ks):
    C = w2.shape[-1]
    adt = torch.float32 if prec else torch.bfloat16
    out = torch.zeros(g, B, Up, dtype=adt, device=DEV)
    plog = torch.zeros(g, Up // 16, B, C, device=DEV)
    st = torch.zeros(8, dtype=torch.int32, device=DEV)
    fids = torch.arange(g, dtype=torch.int32, device=DEV)
    nby, nut = -(-B // 32), Up // 64
    part = torch.empty(g * nby * nut * ks * 4 * 2 * 64 * 4, device=DEV)
    a = Km.DenseFwdArgs()
    a.x, a.wt, a.bias, a.out, a.st, a.fold_ids = x.data_ptr(), 0, b1.data_ptr(), out.data_ptr(), st.data_ptr(), \
        fids.data_ptr()
    a.G, a.B, a.Fp, a.Up, a.drop_p, a.train, a.seed = g, B, Fp, Up, drop_p, train, 7
    a.w2, a.plog, a.C, a.prec = w2.data_ptr(), plog.data_ptr(), C, prec
    a.w1, a.part, a.ks = w1.data_ptr(), part.data_ptr(), ks
    Km.check(L.gt_dense_fwd(a, _stream()), "dense_fwd")
    torch.cuda.synchronize()
    return out.clone(), plog.clone()


@pytest.mark.parametrize("prec", [1, 0])
@pytest.mark.parametrize("G,B,Fp,Up", SHAPES)
def test_dense_fwd_split_k(prec, G, B, Fp, Up):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    L = Km.lib()
    torch.manual_seed(1)
    adt = torch.float32 if prec else torch.bfloat16
    w1 = torch.randn(G, Fp, Up, device=DEV) * 0.05
    x = torch.randn(G, B, Fp, device=DEV).to(adt)
    b1 = torch.randn(G, Up, device=DEV) * 0.1
    w2 = torch.randn(G, Up, 10, device=DEV) * 0.05
    for ks in sorted({1, 3, L.gt_dense_fwd_splits(Fp)}):
        h0, p0 = _fwd(L, x, w1, b1, w2, G, B, Fp, Up, prec, 0.0, 0, ks)        # no dropout
        h1, p1 = _fwd(L, x, w1, b1, w2, G, B, Fp, Up, prec, 0.5, 1, ks)
        h2, p2 = _fwd(L, x, w1, b1, w2, G, B, Fp, Up, prec, 0.5, 1, ks)
        assert torch.equal(h1, h2) and torch.equal(p1, p2)
        hs, ps = _fwd(L, x, w1, b1, w2, 2, B, Fp, Up, prec, 0.5, 1, ks)        # groups 0-1 alone
        assert torch.equal(hs, h1[:2]) and torch.equal(ps, p1[:2])
        wr = w1.double() if prec else w1.to(torch.bfloat16).double()          # bf16 mode: RNE-rounded master
        z = torch.relu(torch.bmm(x.double(), wr) + b1.double()[:, None, :])
        err = ((h0.double() - z).abs().max() / z.abs().max()).item()
        assert err < (1e-5 if prec else 2e-2), (ks, err)
        # inverted dropout p = 0.5: about half of the positive units kept, each at twice its value
        pos, kept = h0.float() > 0, h1.float() != 0
        frac = (kept & pos).sum().item() / max(1, pos.sum().item())
        assert 0.45 < frac < 0.55, frac
        assert not (kept & ~pos).any()
        assert torch.allclose(h1.float()[kept], 2 * h0.float()[kept], rtol=1e-6 if prec else 1e-2)
        # fused partial logits = the stored activations times W2
        ref = torch.einsum("gbu,guc->gbc", h1.double(), w2.double())
        assert ((p1.sum(1).double() - ref).abs().max() / ref.abs().max()).item() < 1e-5


@pytest.mark.parametrize("prec", [1, 0])
@pytest.mark.parametrize("G,B,Fp,Up", SHAPES)
def test_dense_dgrad(prec, G, B, Fp, Up):
    """fp32: exact f32 products (fp32-accumulation level of fp64); bf16 mode: the bf16 MFMA on the
    RNE-rounded master and head_bwd's bf16 dH. Tails: Fp 392 is not a multiple of the 128-feature tile,
    B 20 not of 32."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    L = Km.lib()
    torch.manual_seed(3)
    adt = torch.float32 if prec else torch.bfloat16
    w1 = torch.randn(G, Fp, Up, device=DEV) * 0.05
    dH = torch.randn(G, B, Up, device=DEV)
    dHp = dH.to(torch.bfloat16).contiguous()

    def run(g):
        dx = torch.zeros(g, B, Fp, dtype=adt, device=DEV)
        d = Km.DenseDgradArgs()
        d.dH, d.wt, d.dx, d.G, d.B, d.Fp, d.Up, d.prec = dH.data_ptr(), 0, dx.data_ptr(), g, B, Fp, Up, prec
        d.w1, d.dHp = w1.data_ptr(), dHp.data_ptr()
        Km.check(L.gt_dense_dgrad(d, _stream()), "dense_dgrad")
        torch.cuda.synchronize()
        return dx

    dx1, dx2, dxs = run(G), run(G), run(2)
    assert torch.equal(dx1, dx2) and torch.equal(dxs, dx1[:2])
    if prec:
        ref = torch.bmm(dH.double(), w1.double().transpose(1, 2))
    else:
        ref = torch.bmm(dHp.double(), w1.to(torch.bfloat16).double().transpose(1, 2))
    err = ((dx1.double() - ref).abs().max() / ref.abs().max()).item()
    assert err < (2e-6 if prec else 2e-2), err


def test_dense_launchers_refuse_a_missing_master():
    """There is no transposed W1 copy to fall back on: without the master (or the bf16 dH plane of the
    bf16-mode data gradient) the launchers fail (-3) instead of reading stale or absent weights."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    L = Km.lib()
    G, B, Fp, Up = 1, 32, 64, 64
    x, out, b1 = (torch.zeros(G, B, Fp, device=DEV), torch.zeros(G, B, Up, device=DEV),
                  torch.zeros(G, Up, device=DEV))
    a = Km.DenseFwdArgs()
    a.x, a.bias, a.out, a.G, a.B, a.Fp, a.Up, a.C, a.prec, a.ks = x.data_ptr(), b1.data_ptr(), out.data_ptr(), \
        G, B, Fp, Up, 10, 1, 1
    assert L.gt_dense_fwd(a, _stream()) == -3
    d = Km.DenseDgradArgs()
    d.dH, d.dx, d.G, d.B, d.Fp, d.Up, d.prec = out.data_ptr(), x.data_ptr(), G, B, Fp, Up, 1
    assert L.gt_dense_dgrad(d, _stream()) == -3
    w1 = torch.zeros(G, Fp, Up, device=DEV)
    d.w1, d.prec = w1.data_ptr(), 0
    assert L.gt_dense_dgrad(d, _stream()) == -3
