"""Numerics of every Genetic-CNN HIP kernel against a plain PyTorch fp32
reference of the same op (inputs rounded to bf16 first, so only the
kernel's accumulation/rounding differs)."""

import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0) if torch.cuda.is_available() else None


def K():
    from gentun_amd.ops import cnn_kernels
    cnn_kernels.lib()
    return cnn_kernels


def stream():
    return torch.cuda.current_stream().cuda_stream


def bf(x):
    return x.to(torch.bfloat16)


def nhwc_pad(x_nchw, cp):
    n, c, h, w = x_nchw.shape
    out = torch.zeros((n, h, w, cp), dtype=x_nchw.dtype, device=x_nchw.device)
    out[..., :c] = x_nchw.permute(0, 2, 3, 1)
    return out


def conv_ref(xs_nchw, w_oihw, bias, relu):
    x = sum(xs_nchw)
    y = F.conv2d(x, w_oihw, bias, padding=(w_oihw.shape[2] // 2, w_oihw.shape[3] // 2))
    return F.relu(y) if relu else y


def pack_w(w_oihw, coutp, cinp):
    co, ci, kh, kw = w_oihw.shape
    out = torch.zeros((coutp, kh, kw, cinp), dtype=w_oihw.dtype, device=w_oihw.device)
    out[:co, :, :, :ci] = w_oihw.permute(0, 2, 3, 1)
    return out


@pytest.mark.parametrize("H,W,cin,cout,k,nin", [(32, 32, 3, 20, 5, 1), (32, 32, 20, 20, 3, 3), (16, 16, 20, 50, 5, 1),
                                               (16, 16, 50, 50, 3, 2), (8, 8, 64, 128, 3, 1), (7, 7, 50, 50, 3, 4),
                                               (28, 28, 1, 20, 5, 1), (16, 16, 50, 200, 5, 1)])
def test_conv_fwd(H, W, cin, cout, k, nin):
    """Dense (legacy) group mode: every group, inputs 0..nin-1 summed."""
    Km = K()
    torch.manual_seed(0)
    G, B = 2, 3
    cinp, coutp = (cin + 7) // 8 * 8, (cout + 7) // 8 * 8
    xs = [bf(torch.randn(G, B, cin, H, W, device=DEV)).float() for _ in range(nin)]
    w = bf(torch.randn(G, cout, cin, k, k, device=DEV) * 0.2).float()
    b = torch.randn(G, cout, device=DEV) * 0.1
    x_in = [torch.stack([nhwc_pad(x[g], cinp) for g in range(G)]).to(torch.bfloat16).contiguous() for x in xs]
    wp = torch.stack([pack_w(w[g], coutp, cinp) for g in range(G)]).to(torch.bfloat16).contiguous()
    bp = torch.zeros(G, coutp, device=DEV)
    bp[:, :cout] = b
    out = torch.zeros(G, B, H, W, coutp, dtype=torch.bfloat16, device=DEV)
    a = Km.ConvArgs()
    for i, t in enumerate(x_in):
        a.inp[i] = t.data_ptr()
    a.out[0] = out.data_ptr()
    a.n_in, a.n_out, a.acc_flags, a.relu = nin, 1, 0, 1
    a.w, a.bias = wp.data_ptr(), bp.data_ptr()
    a.G, a.B, a.H, a.W, a.Cinp, a.Coutp, a.KH, a.KW = G, B, H, W, cinp, coutp, k, k
    a.TH = Km.conv_tile_rows(H, W)
    a.ngroups = G
    Km.check(Km.lib().gt_conv_fwd(a, stream()), "conv")
    torch.cuda.synchronize()
    for g in range(G):
        # the fused Add is rounded to bf16 before the MFMA: mirror that
        xsum = bf(sum(x[g] for x in xs)).float()
        ref = conv_ref([xsum], w[g], b[g], True)
        got = out[g, ..., :cout].float().permute(0, 3, 1, 2)
        tol = 2e-2 * ref.abs().max().item() + 1e-2
        assert (got - ref).abs().max().item() < tol
        if coutp > cout:
            assert out[g, ..., cout:].abs().max().item() == 0


@pytest.mark.parametrize("staged_mask,k", [(True, 3), (False, 3), (False, 5)])
def test_conv_dgrad_mask_and_accumulate(staged_mask, k):
    """dgrad = conv of (dy * (y>0)) with flipped/transposed weights, fanned out
    into two outputs, one accumulating. ``staged_mask``: the ReLU mask is
    applied while staging (register kernel); else dy arrives pre-masked (the
    LDS-DMA kernel's single-input path)."""
    Km = K()
    torch.manual_seed(1)
    G, B, H, W, cin, cout = 2, 2, 16, 16, 20, 50
    cinp, coutp = 24, 56
    x = bf(torch.randn(G, B, cin, H, W, device=DEV)).float()
    w = bf(torch.randn(G, cout, cin, k, k, device=DEV) * 0.2).float()
    y = torch.stack([F.relu(F.conv2d(x[g], w[g], padding=k // 2)) for g in range(G)])
    dy = bf(torch.randn_like(y)).float()
    y = bf(y).float()
    ref = torch.stack([torch.nn.grad.conv2d_input(x[g].shape, w[g], dy[g] * (y[g] > 0), padding=k // 2)
                       for g in range(G)])
    wp = torch.stack([pack_w(w[g], coutp, cinp) for g in range(G)]).float()
    wT = wp.flip(2, 3).permute(0, 4, 2, 3, 1).contiguous().to(torch.bfloat16)
    dy_p = torch.stack([nhwc_pad(dy[g], coutp) for g in range(G)]).to(torch.bfloat16).contiguous()
    y_p = torch.stack([nhwc_pad(y[g], coutp) for g in range(G)]).to(torch.bfloat16).contiguous()
    out0 = torch.zeros(G, B, H, W, cinp, dtype=torch.bfloat16, device=DEV)
    prev = bf(torch.randn(G, B, H, W, cinp, device=DEV))
    prev[..., cin:] = 0
    out1 = prev.clone()
    if not staged_mask:
        dy_p = (dy_p.float() * (y_p.float() > 0)).to(torch.bfloat16).contiguous()
    a = Km.ConvArgs()
    a.inp[0] = dy_p.data_ptr()
    a.mask = y_p.data_ptr() if staged_mask else 0
    a.out[0], a.out[1] = out0.data_ptr(), out1.data_ptr()
    pmask = bf(torch.randn(G, B, H, W, cinp, device=DEV))
    a.out_mask[1] = pmask.data_ptr()        # final writer of out1 applies its ReLU mask
    a.n_in, a.n_out, a.acc_flags, a.relu = 1, 2, 2, 0
    a.w, a.bias = wT.data_ptr(), 0
    a.G, a.B, a.H, a.W, a.Cinp, a.Coutp, a.KH, a.KW, a.TH = G, B, H, W, coutp, cinp, k, k, 4
    a.ngroups = G
    Km.check(Km.lib().gt_conv_fwd(a, stream()), "dgrad")
    torch.cuda.synchronize()
    got0 = out0[..., :cin].float().permute(0, 1, 4, 2, 3)
    tol = 2e-2 * ref.abs().max().item()
    assert (got0 - ref).abs().max().item() < tol
    got1 = out1[..., :cin].float().permute(0, 1, 4, 2, 3)
    ref1 = (ref + prev[..., :cin].float().permute(0, 1, 4, 2, 3)) * (pmask[..., :cin] > 0).permute(0, 1, 4, 2, 3)
    assert (got1 - ref1).abs().max().item() < tol + 2e-2 * ref1.abs().max().item()


@pytest.mark.parametrize("H", [16, 32])
def test_conv_group_table_slots_accumulate_mask(H):
    """Population mode: a launch over a SUBSET of groups, each summing its own
    input slots and writing / accumulating / ReLU-masking its own outputs;
    groups outside the table are untouched (H=32: shape-specialised kernel,
    H=16: generic kernel)."""
    Km = K()
    torch.manual_seed(7)
    Q, B, W, cin, cout, k = 4, 2, H, 20, 20, 3
    cp = 24
    slots = [bf(torch.randn(Q, B, H, W, cp, device=DEV)) for _ in range(3)]
    for s in slots:
        s[..., cin:] = 0
    w = bf(torch.randn(Q, cout, cin, k, k, device=DEV) * 0.2).float()
    wp = torch.stack([pack_w(w[g], cp, cp) for g in range(Q)]).to(torch.bfloat16).contiguous()
    bias = torch.zeros(Q, cp, device=DEV)
    bias[:, :cout] = torch.randn(Q, cout, device=DEV) * 0.1
    out0 = torch.full((Q, B, H, W, cp), 3.0, dtype=torch.bfloat16, device=DEV)
    out1 = bf(torch.randn(Q, B, H, W, cp, device=DEV))
    out1[..., cout:] = 0
    prev1 = out1.clone()
    mask1 = bf(torch.randn(Q, B, H, W, cp, device=DEV))
    # group 3: slots {0, 2} -> write out0; group 1: slot {1} -> accumulate into out1, then ReLU-mask
    rows = torch.tensor([[3, 0b101, 0b1, 0], [1, 0b010, 0b10 | (0b10 << 8) | (0b10 << 16), 0]],
                        dtype=torch.int32, device=DEV)
    a = Km.ConvArgs()
    for i, s in enumerate(slots):
        a.inp[i] = s.data_ptr()
    a.out[0], a.out[1] = out0.data_ptr(), out1.data_ptr()
    a.out_mask[1] = mask1.data_ptr()
    a.gtab, a.ngroups = rows.data_ptr(), 2
    a.relu = 1
    a.w, a.bias = wp.data_ptr(), bias.data_ptr()
    a.G, a.B, a.H, a.W, a.Cinp, a.Coutp, a.KH, a.KW = Q, B, H, W, cp, cp, k, k
    a.TH = Km.conv_tile_rows(H, W)
    Km.check(Km.lib().gt_conv_fwd(a, stream()), "conv(gtab)")
    torch.cuda.synchronize()

    def ref(g, ins):
        x = bf(sum(slots[i][g].float() for i in ins))[..., :cin].permute(0, 3, 1, 2).float()
        return conv_ref([x], w[g], bias[g, :cout], True).permute(0, 2, 3, 1)

    r3 = ref(3, [0, 2])
    tol = 2e-2 * r3.abs().max().item() + 1e-2
    assert (out0[3, ..., :cout].float() - r3).abs().max().item() < tol
    r1 = (ref(1, [1]) + prev1[1, ..., :cout].float()) * (mask1[1, ..., :cout].float() > 0)
    assert (out1[1, ..., :cout].float() - r1).abs().max().item() < tol + 2e-2 * r1.abs().max().item()
    for g in (0, 2):
        assert torch.all(out0[g] == 3.0)
        assert torch.equal(out1[g], prev1[g])
    assert torch.all(out0[1] == 3.0) and torch.equal(out1[3], prev1[3])


def test_pool_group_select():
    """Per-group pool source (x0 or x1) and gradient target."""
    Km = K()
    torch.manual_seed(8)
    Q, B, H, W, cp = 3, 2, 8, 8, 8
    x0 = bf(torch.randn(Q, B, H, W, cp, device=DEV))
    x1 = bf(torch.randn(Q, B, H, W, cp, device=DEV))
    sel = torch.tensor([0, 1, 0], dtype=torch.int32, device=DEV)
    y = torch.zeros(Q, B, H // 2, W // 2, cp, dtype=torch.bfloat16, device=DEV)
    Km.check(Km.lib().gt_pool_fwd(x0.data_ptr(), x1.data_ptr(), sel.data_ptr(), y.data_ptr(), Q * B, B, H, W, cp, 0,
                                  stream()), "pool")
    dy = bf(torch.randn_like(y.float()))
    dx0 = torch.full_like(x0, 5.0)
    dx1 = torch.full_like(x1, 5.0)
    Km.check(Km.lib().gt_pool_bwd(x0.data_ptr(), x1.data_ptr(), sel.data_ptr(), dy.data_ptr(), dx0.data_ptr(),
                                  dx1.data_ptr(), Q * B, B, H, W, cp, 1, 0, stream()), "poolb")
    torch.cuda.synchronize()
    for g in range(Q):
        src = (x1 if sel[g] else x0)[g].float().permute(0, 3, 1, 2).clone().requires_grad_(True)
        yr = F.max_pool2d(src, 2, 2)
        assert torch.equal(y[g].float().permute(0, 3, 1, 2), yr.detach())
        yr.backward(dy[g].float().permute(0, 3, 1, 2))
        got = (dx1 if sel[g] else dx0)[g].float().permute(0, 3, 1, 2)
        assert torch.allclose(got, src.grad * (src > 0), atol=1e-6)
        assert torch.all((dx0 if sel[g] else dx1)[g] == 5.0)


@pytest.mark.parametrize("H,W,relu", [(8, 8, 1), (7, 7, 1), (14, 14, 0), (16, 16, 1)])
def test_pool_argmax_mask(H, W, relu):
    """Training-forward argmax mask + mask backward: bit-identical to the
    recomputing pool_bwd (ties, zeros, negative maxima, odd sizes included)."""
    Km = K()
    torch.manual_seed(9)
    Q, B, cp = 3, 2, 16
    # coarse values: many ties and exact zeros inside the 2x2 cells
    x0 = bf(torch.randint(-2, 3, (Q, B, H, W, cp), device=DEV).float())
    x1 = bf(torch.randint(-2, 3, (Q, B, H, W, cp), device=DEV).float())
    sel = torch.tensor([1, 0, 1], dtype=torch.int32, device=DEV)
    args = (x0.data_ptr(), x1.data_ptr(), sel.data_ptr())
    y_ref = torch.zeros(Q, B, H // 2, W // 2, cp, dtype=torch.bfloat16, device=DEV)
    y = torch.zeros_like(y_ref)
    mask = torch.full((Q * B, H // 2, W // 2, cp), 255, dtype=torch.uint8, device=DEV)
    Km.check(Km.lib().gt_pool_fwd(*args, y_ref.data_ptr(), Q * B, B, H, W, cp, 0, stream()), "pool")
    Km.check(Km.lib().gt_pool_fwd_mask(*args, y.data_ptr(), Q * B, B, H, W, cp, mask.data_ptr(), 0, stream()),
             "poolm")
    dy = bf(torch.randn_like(y.float()))
    dx_ref = [torch.full_like(x0, 5.0), torch.full_like(x1, 5.0)]
    dx = [torch.full_like(x0, 5.0), torch.full_like(x1, 5.0)]
    Km.check(Km.lib().gt_pool_bwd(*args, dy.data_ptr(), dx_ref[0].data_ptr(), dx_ref[1].data_ptr(), Q * B, B, H, W,
                                  cp, relu, 0, stream()), "poolb")
    Km.check(Km.lib().gt_pool_bwd_mask(mask.data_ptr(), sel.data_ptr(), dy.data_ptr(), dx[0].data_ptr(),
                                       dx[1].data_ptr(), Q * B, B, H, W, cp, relu, 0, stream()), "poolbm")
    torch.cuda.synchronize()
    assert torch.equal(y.float(), y_ref.float())
    assert int(mask.max()) <= 7
    assert torch.equal(dx[0], dx_ref[0]) and torch.equal(dx[1], dx_ref[1])


@pytest.mark.parametrize("H,W,cin,cout,k,nin,first", [(32, 32, 3, 20, 5, 1, True), (16, 16, 50, 50, 3, 2, False),
                                                      (32, 32, 20, 20, 3, 1, False), (8, 8, 64, 128, 3, 1, False)])
def test_conv_wgrad(H, W, cin, cout, k, nin, first):
    Km = K()
    torch.manual_seed(2)
    G, B = 2, 4
    cinp, coutp = (cin + 7) // 8 * 8, (cout + 7) // 8 * 8
    xs = [bf(torch.randn(G, B, cin, H, W, device=DEV)).float() for _ in range(nin)]
    y = bf(torch.randn(G, B, cout, H, W, device=DEV)).float()
    dy = bf(torch.randn(G, B, cout, H, W, device=DEV)).float()
    xsum = bf(sum(xs)).float()
    dz = dy * (y > 0)
    ref = torch.stack([torch.nn.grad.conv2d_weight(xsum[g], (cout, cin, k, k), dz[g], padding=k // 2)
                       for g in range(G)])
    refb = dz.sum((1, 3, 4))
    x_in = [torch.stack([nhwc_pad(x[g], cinp) for g in range(G)]).to(torch.bfloat16).contiguous() for x in xs]
    gather = None
    if first:
        # dataset of 3*G*B images, gathered through a [1][G][B] table
        data = torch.zeros(3 * G * B, H, W, cinp, dtype=torch.bfloat16, device=DEV)
        perm = torch.randperm(3 * G * B, device=DEV)[:G * B]
        data[perm] = x_in[0].view(G * B, H, W, cinp)
        gather = perm.view(1, G, B).to(torch.int64).contiguous()
        x_in = [data]
    dz_p = torch.stack([nhwc_pad(dz[g], coutp) for g in range(G)]).to(torch.bfloat16).contiguous()
    Kdim = k * k * cinp
    npix = B * H * W
    pps, S = Km.wgrad_split(npix, Kdim, coutp, target_blocks=16)
    pw = torch.zeros(S, G, coutp, Kdim, device=DEV)
    pb = torch.zeros(S, G, coutp, device=DEV)
    st = torch.zeros(8, dtype=torch.int32, device=DEV)
    a = Km.WgradArgs()
    for i, t in enumerate(x_in):
        a.inp[i] = t.data_ptr()
    a.n_in = len(x_in)
    a.gather = gather.data_ptr() if gather is not None else 0
    a.st = st.data_ptr()
    a.dz, a.part_w, a.part_b = dz_p.data_ptr(), pw.data_ptr(), pb.data_ptr()
    a.G, a.B, a.H, a.W, a.Cinp, a.Coutp, a.KH, a.KW, a.S, a.pps = G, B, H, W, cinp, coutp, k, k, S, pps
    a.ngroups = G
    Km.check(Km.lib().gt_conv_wgrad(a, stream()), "wgrad")
    torch.cuda.synchronize()
    got = pw.sum(0).view(G, coutp, k, k, cinp)[:, :cout, :, :, :cin].permute(0, 1, 4, 2, 3)
    tol = 1e-2 * ref.abs().max().item() + 1e-3
    assert (got - ref).abs().max().item() < tol
    gotb = pb.sum(0)[:, :cout]
    assert (gotb - refb).abs().max().item() < 1e-2 * refb.abs().max().item() + 1e-3


@pytest.mark.parametrize("H,W", [(32, 32), (7, 7), (14, 14)])
def test_pool_fwd_bwd(H, W):
    Km = K()
    torch.manual_seed(3)
    N, C, cp = 6, 20, 24
    x = bf(torch.randn(N, C, H, W, device=DEV)).float()
    xr = x.clone().requires_grad_(True)
    y = F.max_pool2d(xr, 2, 2)
    dy = bf(torch.randn_like(y)).float()
    y.backward(dy)
    xp = nhwc_pad(x, cp).to(torch.bfloat16).contiguous()
    yp = torch.zeros(N, H // 2, W // 2, cp, dtype=torch.bfloat16, device=DEV)
    Km.check(Km.lib().gt_pool_fwd(xp.data_ptr(), 0, 0, yp.data_ptr(), N, 1, H, W, cp, 0, stream()), "pool")
    dyp = nhwc_pad(dy, cp).to(torch.bfloat16).contiguous()
    dxp = torch.full((N, H, W, cp), 7.0, dtype=torch.bfloat16, device=DEV)
    Km.check(Km.lib().gt_pool_bwd(xp.data_ptr(), 0, 0, dyp.data_ptr(), dxp.data_ptr(), 0, N, 1, H, W, cp, 0, 0,
                                  stream()), "poolb")
    dxm = torch.full((N, H, W, cp), 7.0, dtype=torch.bfloat16, device=DEV)
    Km.check(Km.lib().gt_pool_bwd(xp.data_ptr(), 0, 0, dyp.data_ptr(), dxm.data_ptr(), 0, N, 1, H, W, cp, 1, 0,
                                  stream()), "poolm")
    torch.cuda.synchronize()
    assert torch.equal(yp[..., :C].float().permute(0, 3, 1, 2), y.detach())
    assert torch.allclose(dxp[..., :C].float().permute(0, 3, 1, 2), xr.grad, atol=1e-6)
    assert torch.allclose(dxm[..., :C].float().permute(0, 3, 1, 2), xr.grad * (x > 0), atol=1e-6)


def test_dense_fwd_dgrad():
    Km = K()
    torch.manual_seed(4)
    G, B, Fp, Up = 3, 32, 3584, 512
    x = bf(torch.randn(G, B, Fp, device=DEV)).float()
    w1 = (torch.randn(G, Fp, Up, device=DEV) * 0.02)
    b1 = torch.randn(G, Up, device=DEV) * 0.1
    w1b = bf(w1).float()
    ref = F.relu(torch.baddbmm(b1[:, None], x, w1b))
    xb = x.to(torch.bfloat16).contiguous()
    out = torch.zeros(G, B, Up, dtype=torch.bfloat16, device=DEV)
    st = torch.zeros(8, dtype=torch.int32, device=DEV)
    a = Km.DenseFwdArgs()
    a.x, a.wt, a.bias, a.out, a.st, a.fold_ids = xb.data_ptr(), 0, b1.data_ptr(), out.data_ptr(), st.data_ptr(), 0
    a.G, a.B, a.Fp, a.Up, a.drop_p, a.train, a.seed = G, B, Fp, Up, 0.5, 0, 1
    # W1 from the fp32 master (rounded to bf16 on staging), split-K partial ranges
    ks = Km.lib().gt_dense_fwd_splits(Fp)
    part = torch.empty(G * (Up // 64) * ks * 4 * 2 * 64 * 4, device=DEV)
    a.w1, a.part, a.ks = w1.data_ptr(), part.data_ptr(), ks
    Cc = 10
    w2 = torch.randn(G, Up, Cc, device=DEV) * 0.05
    plog = torch.zeros(G, Up // 16, B, Cc, device=DEV)
    a.w2, a.plog, a.C = w2.data_ptr(), plog.data_ptr(), Cc
    Km.check(Km.lib().gt_dense_fwd(a, stream()), "dense")
    torch.cuda.synchronize()
    reflog = torch.einsum("gbu,guc->gbc", out.float(), w2)
    assert torch.allclose(plog.sum(1), reflog, rtol=1e-4, atol=1e-4)
    # dropout statistics in train mode
    out2 = torch.zeros_like(out)
    a.out, a.train = out2.data_ptr(), 1
    Km.check(Km.lib().gt_dense_fwd(a, stream()), "dense-train")
    dH = torch.randn(G, B, Up, device=DEV)
    dx = torch.zeros(G, B, Fp, dtype=torch.bfloat16, device=DEV)
    dHp = dH.to(torch.bfloat16).contiguous()                    # head_bwd's bf16 dH plane
    d = Km.DenseDgradArgs()
    d.dH, d.wt, d.dx, d.G, d.B, d.Fp, d.Up = dH.data_ptr(), 0, dx.data_ptr(), G, B, Fp, Up
    d.w1, d.dHp = w1.data_ptr(), dHp.data_ptr()
    Km.check(Km.lib().gt_dense_dgrad(d, stream()), "dgrad")
    torch.cuda.synchronize()
    assert (out.float() - ref).abs().max().item() < 2e-2 * ref.abs().max().item()
    kept = (out2.float() != 0)
    pos = (ref > 0)
    frac = (kept & pos).sum().item() / max(1, pos.sum().item())
    assert 0.4 < frac < 0.6
    both = kept & pos
    assert torch.allclose(out2.float()[both], 2 * out.float()[both], rtol=2e-2, atol=1e-2)
    refdx = torch.bmm(bf(dH).float(), bf(w1).float().transpose(1, 2))
    assert (dx.float() - refdx).abs().max().item() < 2e-2 * refdx.abs().max().item()


def _adam_ref(p, m, v, g, lr, t):
    m = 0.9 * m + 0.1 * g
    v = 0.999 * v + 0.001 * g * g
    lr_t = lr * math.sqrt(1 - 0.999 ** t) / (1 - 0.9 ** t)
    return p - lr_t * m / (v.sqrt() + 1e-7), m, v


@pytest.mark.parametrize("Fp,Cp,Cr,Ur", [(400, 0, 0, 0), (392, 56, 50, 500)])
def test_dense_wgrad_adam_and_step_begin(Fp, Cp, Cr, Ur):
    """Fused dW1 + Adam on the fp32 master; second case: a feature count
    that is not a multiple of the 16-row tile plus padded channels / units
    (skipped by the kernel, zero in the reference)."""
    Km = K()
    torch.manual_seed(5)
    G, B, Up = 2, 32, 512
    x = bf(torch.randn(G, B, Fp, device=DEV)).float()
    dH = torch.randn(G, B, Up, device=DEV)
    p = torch.randn(G, Fp, Up, device=DEV)
    m = torch.randn(G, Fp, Up, device=DEV) * 0.01
    v = torch.rand(G, Fp, Up, device=DEV) * 0.01
    if Cp:
        pad_f = (torch.arange(Fp, device=DEV) % Cp) >= Cr
        pad_u = torch.arange(Up, device=DEV) >= Ur
        x[:, :, pad_f] = 0
        dH[:, :, pad_u] = 0
        for t in (p, m, v):
            t[:, pad_f, :] = 0
            t[:, :, pad_u] = 0
    st = torch.zeros(8, dtype=torch.int32, device=DEV)
    stf = st.view(torch.float32)
    stf[2] = 4.0   # t before this step
    stf[3] = 1e-3
    Km.check(Km.lib().gt_step_begin(st.data_ptr(), stream()), "step_begin")
    g = torch.bmm(x.transpose(1, 2), dH)
    rp, rm, rv = _adam_ref(p.clone(), m.clone(), v.clone(), g, 1e-3, 5)
    a = Km.DenseWgradAdamArgs()
    xb = x.to(torch.bfloat16).contiguous()
    a.x, a.dH, a.p, a.m, a.v, a.wt, a.st = xb.data_ptr(), dH.data_ptr(), p.data_ptr(), m.data_ptr(), v.data_ptr(), \
        0, st.data_ptr()
    a.G, a.B, a.Fp, a.Up = G, B, Fp, Up
    a.Cp, a.Cr, a.Ur = Cp, Cr, Ur
    Km.check(Km.lib().gt_dense_wgrad_adam(a, stream()), "wgrad_adam")
    torch.cuda.synchronize()
    assert st[1].item() == 0 and st[0].item() == 1 and abs(stf[2].item() - 5.0) < 1e-6
    assert torch.allclose(m, rm, rtol=1e-4, atol=1e-5)
    assert torch.allclose(v, rv, rtol=1e-4, atol=1e-6)
    assert torch.allclose(p, rp, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("loss", ["bce_compat", "ce"])
def test_head(loss):
    Km = K()
    from gentun_amd.models.cnn_engine import loss_and_metrics
    torch.manual_seed(6)
    G, B, Up, C, N = 2, 32, 512, 10, 100
    h = bf(F.relu(torch.randn(G, B, Up, device=DEV))).float()
    w2 = torch.randn(G, Up, C, device=DEV) * 0.05
    b2 = torch.randn(G, C, device=DEV) * 0.1
    labels = torch.randint(0, C, (N,), device=DEV)
    gather = torch.randint(0, N, (1, G, B), device=DEV)
    y = F.one_hot(labels[gather[0]], C).float()
    hr = h.clone().requires_grad_(True)
    w2r = w2.clone().requires_grad_(True)
    b2r = b2.clone().requires_grad_(True)
    logits = torch.baddbmm(b2r[:, None], hr, w2r)
    per, binc, catc = loss_and_metrics(logits, y, loss)
    per.mean(-1).sum().backward()
    dH = torch.zeros(G, B, Up, device=DEV)
    gw2, gb2, gb1 = torch.zeros_like(w2), torch.zeros_like(b2), torch.zeros(G, Up, device=DEV)
    st = torch.zeros(8, dtype=torch.int32, device=DEV)
    hb = h.to(torch.bfloat16).contiguous()
    a = Km.HeadArgs()
    a.h, a.w2, a.b2, a.labels, a.gather, a.st = hb.data_ptr(), w2.data_ptr(), b2.data_ptr(), labels.data_ptr(), \
        gather.data_ptr(), st.data_ptr()
    dzw = torch.zeros(G, B, C, device=DEV)
    a.dH, a.gw2, a.gb2, a.gb1, a.eval_out = dH.data_ptr(), gw2.data_ptr(), gb2.data_ptr(), gb1.data_ptr(), 0
    a.dz = dzw.data_ptr()
    plog = torch.einsum("gbu,guc->gbc", h, w2).unsqueeze(1).contiguous()   # one "tile" holding the full sum
    plog = torch.cat([plog, torch.zeros(G, Up // 16 - 1, B, C, device=DEV)], 1).contiguous()
    a.plog = plog.data_ptr()
    a.G, a.B, a.Up, a.C, a.loss_ce, a.drop_scale, a.eval = G, B, Up, C, int(loss == "ce"), 2.0, 0
    Km.check(Km.lib().gt_head(a, stream()), "head")
    ev = torch.zeros(G, B, 3, device=DEV)
    a.eval, a.eval_out = 1, ev.data_ptr()
    Km.check(Km.lib().gt_head(a, stream()), "head-eval")
    torch.cuda.synchronize()
    refdH = hr.grad * 2.0 * (h > 0)
    assert torch.allclose(dH, refdH, rtol=1e-3, atol=1e-6)
    assert torch.allclose(gw2, w2r.grad, rtol=1e-3, atol=1e-6)
    assert torch.allclose(gb2, b2r.grad, rtol=1e-3, atol=1e-6)
    assert torch.allclose(gb1, refdH.sum(1), rtol=1e-3, atol=1e-5)
    assert torch.allclose(ev[..., 0], per.detach(), rtol=1e-4, atol=1e-6)
    assert torch.equal(ev[..., 1], binc)
    assert torch.equal(ev[..., 2], catc)


@pytest.mark.parametrize("tiled,dims", [(False, (2, 16, 3, 3, 8)), (True, (2, 16, 3, 3, 8)),
                                        (True, (1, 104, 3, 3, 104)), (True, (2, 56, 5, 5, 24)),
                                        (False, (1, 256, 3, 3, 24)), (True, (2, 256, 3, 3, 40)),
                                        (True, (1, 200, 3, 3, 16))])
def test_adam_segments_with_partials_and_transpose(tiled, dims):
    """Multi-tensor Adam over split-K partials, bf16 copy and the flipped /
    transposed dgrad copy; ``tiled``: (group, 128-row co band, 64-column) tile
    blocks with the transposed copy staged through LDS (Co > 128: several
    bands, the last one partial)."""
    Km = K()
    import ctypes
    torch.manual_seed(7)
    G, co, kh, kw, ci = dims
    S = 3
    n = G * co * kh * kw * ci
    p = torch.randn(n, device=DEV)
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    parts = torch.randn(S, n, device=DEV)
    bfc = torch.zeros(n, dtype=torch.bfloat16, device=DEV)
    bfT = torch.zeros(n, dtype=torch.bfloat16, device=DEV)
    sg = Km.AdamSeg()
    sg.p, sg.m, sg.v, sg.g, sg.bf, sg.bfT = p.data_ptr(), m.data_ptr(), v.data_ptr(), parts.data_ptr(), \
        bfc.data_ptr(), bfT.data_ptr()
    sg.n, sg.gstride, sg.S = n, n, S
    sg.tG, sg.tCo, sg.tKH, sg.tKW, sg.tCi = G, co, kh, kw, ci
    ntiles = Km.adam_tiles(G, co, kh, kw, ci) if tiled else 0
    assert bool(ntiles) == tiled
    sg.tiled = 1 if ntiles else 0
    raw = bytes(memoryview((Km.AdamSeg * 1)(sg)).cast("B"))
    segs = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(DEV)
    blk = [[0, t] for t in range(ntiles)] if ntiles else [[0, o] for o in Km.adam_blocks(n)]
    blocks = torch.tensor(blk, dtype=torch.int32, device=DEV)
    st = torch.zeros(8, dtype=torch.int32, device=DEV)
    st.view(torch.float32)[3] = 1e-2
    Km.check(Km.lib().gt_step_begin(st.data_ptr(), stream()), "sb")
    a = Km.AdamArgs()
    a.segs, a.blocks, a.st = segs.data_ptr(), blocks.data_ptr(), st.data_ptr()
    rp, rm, rv = _adam_ref(p.clone(), m.clone(), v.clone(), parts.sum(0), 1e-2, 1)
    Km.check(Km.lib().gt_adam_segments(ctypes.byref(a), blocks.shape[0], stream()), "adam")
    torch.cuda.synchronize()
    assert torch.allclose(p, rp, rtol=1e-5, atol=1e-6)
    # the copies are the kernel's own fp32 result rounded (p may differ from
    # the reference in the last bits, which can flip a bf16 rounding)
    assert torch.equal(bfc, p.to(torch.bfloat16))
    W = p.view(G, co, kh, kw, ci)
    WT = W.flip(2, 3).permute(0, 4, 2, 3, 1).contiguous().to(torch.bfloat16).view(-1)
    assert torch.equal(bfT, WT)


@pytest.mark.parametrize("n,S", [(5000, 2), (4096, 1), (1000, 3)])
def test_adam_segments_vector_path_bit_identical(n, S):
    """Element-wise segments run 4 elements per thread with 16-byte loads / stores when every pointer is
    16-byte aligned, else one element per thread: the same arithmetic and partial-sum order, so a
    misaligned copy of the same state (pointers one float in) must give bitwise the same p / m / v."""
    Km = K()
    import ctypes
    torch.manual_seed(3)
    base = [torch.randn(n, device=DEV) for _ in range(3)]
    base[2] = base[2].abs()
    parts = torch.randn(S, n + 4, device=DEV)
    out = []
    for off in (0, 1):
        bufs = [torch.zeros(n + off, device=DEV) for _ in range(3)]
        for b, t in zip(bufs, base):
            b[off:] = t
        p, m, v = (b[off:] for b in bufs)
        gsrc = torch.zeros(S, n + 4, device=DEV)
        gsrc[:, off:off + n] = parts[:, :n]
        sg = Km.AdamSeg()
        sg.p, sg.m, sg.v, sg.g = p.data_ptr(), m.data_ptr(), v.data_ptr(), gsrc.data_ptr() + 4 * off
        sg.bf = sg.bfT = 0
        sg.n, sg.gstride, sg.S, sg.npl, sg.tiled = n, n + 4, S, 1, 0
        raw = bytes(memoryview((Km.AdamSeg * 1)(sg)).cast("B"))
        segs = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(DEV)
        blocks = torch.tensor([[0, o] for o in Km.adam_blocks(n)], dtype=torch.int32, device=DEV)
        st = torch.zeros(8, dtype=torch.int32, device=DEV)
        st.view(torch.float32)[3] = 1e-2
        Km.check(Km.lib().gt_step_begin(st.data_ptr(), stream()), "sb")
        a = Km.AdamArgs()
        a.segs, a.blocks, a.st = segs.data_ptr(), blocks.data_ptr(), st.data_ptr()
        Km.check(Km.lib().gt_adam_segments(ctypes.byref(a), blocks.shape[0], stream()), "adam")
        torch.cuda.synchronize()
        out.append((p.clone(), m.clone(), v.clone()))
    for x, y in zip(*out):
        assert torch.equal(x, y)
    g = parts[:, :n].sum(0)
    rp, rm, rv = _adam_ref(base[0].clone(), base[1].clone(), base[2].clone(), g, 1e-2, 1)
    assert torch.allclose(out[0][0], rp, rtol=1e-5, atol=1e-6)
    assert torch.allclose(out[0][1], rm, rtol=1e-5, atol=1e-6)


def test_glorot_init_kernel():
    """One-launch Philox Glorot init: real region matches the host reference
    draw element by element, padding is zero, values span (-limit, limit)."""
    import ctypes as C
    Km = K()
    L = Km.lib()
    G, d, r = 2, (8, 3, 3, 24), (5, 3, 3, 20)
    t = torch.full((G,) + d, 7.0, device=DEV)
    seeds = torch.tensor([1234567, 987654321012], dtype=torch.int64, device=DEV)
    sg = Km.InitSeg()
    sg.p, sg.seeds = t.data_ptr(), seeds.data_ptr()
    for i in range(4):
        sg.d[i], sg.r[i] = d[i], r[i]
    sg.G, sg.tag, sg.limit = G, 5, 0.3
    arr = (Km.InitSeg * 1)(sg)
    segs = torch.frombuffer(bytearray(bytes(memoryview(arr).cast("B"))), dtype=torch.uint8).to(DEV)
    nblk = -(-t.numel() // 256)
    blocks = torch.tensor([[0, o * 256] for o in range(nblk)], dtype=torch.int32, device=DEV)
    ia = Km.InitArgs()
    ia.segs, ia.blocks = segs.data_ptr(), blocks.data_ptr()
    Km.check(L.gt_glorot_init(ia, nblk, stream()), "init")
    torch.cuda.synchronize()
    h = t.cpu()
    assert (h[:, r[0]:] == 0).all() and (h[..., r[3]:] == 0).all()
    real = h[:, :r[0], :, :, :r[3]]
    assert real.abs().max().item() < 0.3 and real.abs().min().item() >= 0.0
    assert abs(real.mean().item()) < 0.03 and real.std().item() > 0.15      # U(-.3,.3): std .173
    for g, key in enumerate([1234567, 987654321012]):
        for (i0, i1, i2, i3) in [(0, 0, 0, 0), (4, 2, 2, 19), (2, 1, 0, 7)]:
            lin = ((i0 * r[1] + i1) * r[2] + i2) * r[3] + i3
            ref = L.gt_glorot_ref(C.c_uint64(key), C.c_uint64(lin), 5, C.c_float(0.3))
            assert abs(h[g, i0, i1, i2, i3].item() - ref) < 1e-7


@pytest.mark.parametrize("H,cin,cout,k,nin,dgrad", [(32, 3, 20, 5, 1, False), (32, 20, 20, 3, 2, False),
                                                    (16, 20, 50, 5, 1, False), (16, 50, 50, 3, 3, False),
                                                    (32, 20, 20, 3, 1, True), (16, 50, 50, 3, 1, True),
                                                    (16, 50, 20, 5, 1, True),
                                                    # deep S=(3,4,5) stage 3 (8x8, 100 channels: 7 co tiles)
                                                    (8, 50, 100, 5, 1, False), (8, 100, 100, 3, 3, False),
                                                    (8, 100, 100, 3, 1, True), (8, 100, 50, 5, 1, True)])
def test_conv_fast_equals_generic(H, cin, cout, k, nin, dgrad):
    """The shape-specialised kernels (cnn_conv_fast.hip) walk the reduction in
    the generic kernel's chunk order: outputs are bit-identical, in group-table
    mode with accumulation and ReLU masks."""
    Km = K()
    torch.manual_seed(11)
    Q, B, W = 5, 4, H
    cinp, coutp = (cin + 7) // 8 * 8, (cout + 7) // 8 * 8
    ins = [bf(torch.randn(Q, B, H, W, cinp, device=DEV)) for _ in range(nin)]
    w = bf(torch.randn(Q, coutp, k, k, cinp, device=DEV) * 0.2)
    bias = torch.randn(Q, coutp, device=DEV) * 0.1
    prev = bf(torch.randn(Q, B, H, W, coutp, device=DEV))
    mask = bf(torch.randn(Q, B, H, W, coutp, device=DEV))
    rows = torch.tensor([[4, (1 << nin) - 1, 0b11 | (0b10 << 8) | (0b10 << 16), 0],
                         [1, (1 << nin) - 1, 0b01, 0], [2, 1, 0b10 | (0b10 << 16), 0]], dtype=torch.int32, device=DEV)
    outs = []
    for fast in (0, 1):
        o0 = torch.zeros(Q, B, H, W, coutp, dtype=torch.bfloat16, device=DEV)
        o1 = prev.clone()
        a = Km.ConvArgs()
        for i, s in enumerate(ins):
            a.inp[i] = s.data_ptr()
        a.out[0], a.out[1], a.out_mask[1] = o0.data_ptr(), o1.data_ptr(), mask.data_ptr()
        a.gtab, a.ngroups, a.relu = rows.data_ptr(), 3, 0 if dgrad else 1
        a.w, a.bias = w.data_ptr(), 0 if dgrad else bias.data_ptr()
        a.G, a.B, a.H, a.W, a.Cinp, a.Coutp, a.KH, a.KW = Q, B, H, W, cinp, coutp, k, k
        a.TH = Km.conv_tile_rows(H, W)
        old = Km.lib().gt_conv_set_fast(fast)
        Km.check(Km.lib().gt_conv_fwd(a, stream()), "conv")
        Km.lib().gt_conv_set_fast(old)
        torch.cuda.synchronize()
        outs.append((o0, o1))
    assert outs[0][0].abs().max().item() > 0
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("H,cin,cout,k,nin,first", [(32, 3, 20, 5, 1, True), (32, 20, 20, 3, 2, False),
                                                    (16, 20, 50, 5, 1, False), (16, 50, 50, 3, 3, False),
                                                    (16, 50, 50, 3, 1, False)])
@pytest.mark.parametrize("splits,nb", [(None, 0), (2, 1), (2, 2)])
def test_conv_wgrad_fast(H, cin, cout, k, nin, first, splits, nb):
    """Shape-specialised wgrad (whole-dW workgroups over image bands, LDS-DMA
    double buffering, transposed LDS reads) vs a PyTorch fp32 reference, in
    group-table mode over a subset of groups (DAG input sums, batch gather)."""
    Km = K()
    torch.manual_seed(12)
    Q, B, W = 3, 4, H
    cinp, coutp = (cin + 7) // 8 * 8, (cout + 7) // 8 * 8
    band = Km.wgrad_band(k, k, cinp, coutp, H, W)
    assert band[0] > 0
    if splits:
        band = (band[0], splits)          # several bands per workgroup
    old_nb = Km.lib().gt_wgrad_set_nb(nb)
    xs = [bf(torch.randn(Q, B, cin, H, W, device=DEV)).float() for _ in range(nin)]
    dz = bf(torch.randn(Q, B, cout, H, W, device=DEV)).float()
    x_in = [torch.stack([nhwc_pad(x[g], cinp) for g in range(Q)]).to(torch.bfloat16).contiguous() for x in xs]
    gather = None
    if first:
        data = torch.zeros(3 * Q * B, H, W, cinp, dtype=torch.bfloat16, device=DEV)
        perm = torch.randperm(3 * Q * B, device=DEV)[:Q * B]
        data[perm] = x_in[0].view(Q * B, H, W, cinp)
        gather = perm.view(1, Q, B).to(torch.int64).contiguous()
        x_in = [data]
    dz_p = torch.stack([nhwc_pad(dz[g], coutp) for g in range(Q)]).to(torch.bfloat16).contiguous()
    Kdim = k * k * cinp
    pps, S = Km.wgrad_split(B * H * W, Kdim, coutp, band=band)
    pw = torch.full((S, Q, coutp, Kdim), 9.0, device=DEV)
    pb = torch.full((S, Q, coutp), 9.0, device=DEV)
    st = torch.zeros(8, dtype=torch.int32, device=DEV)
    rows = torch.tensor([[2, (1 << nin) - 1, 0, 0], [0, (1 << nin) - 1, 0, 0]], dtype=torch.int32, device=DEV)
    a = Km.WgradArgs()
    for i, t in enumerate(x_in):
        a.inp[i] = t.data_ptr()
    a.gather = gather.data_ptr() if gather is not None else 0
    a.st, a.gtab, a.ngroups = st.data_ptr(), rows.data_ptr(), 2
    a.dz, a.part_w, a.part_b = dz_p.data_ptr(), pw.data_ptr(), pb.data_ptr()
    a.G, a.B, a.H, a.W, a.Cinp, a.Coutp, a.KH, a.KW, a.S, a.pps = Q, B, H, W, cinp, coutp, k, k, S, pps
    Km.check(Km.lib().gt_conv_wgrad(a, stream()), "wgrad_fast")
    torch.cuda.synchronize()
    Km.lib().gt_wgrad_set_nb(old_nb)
    xsum = bf(sum(xs)).float()
    for g in (0, 2):
        ref = torch.nn.grad.conv2d_weight(xsum[g], (cout, cin, k, k), dz[g], padding=k // 2)
        got = pw[:, g].sum(0).view(coutp, k, k, cinp)[:cout, :, :, :cin].permute(0, 3, 1, 2)
        assert (got - ref).abs().max().item() < 1e-2 * ref.abs().max().item() + 1e-3
        refb = dz[g].sum((0, 2, 3))
        assert (pb[:, g].sum(0)[:cout] - refb).abs().max().item() < 1e-2 * refb.abs().max().item() + 1e-3
    assert torch.all(pw[:, 1] == 9.0)          # group 1 is not in the table: untouched


@pytest.mark.parametrize("H,cin,cout,k", [(32, 20, 20, 3), (16, 50, 50, 3), (16, 20, 50, 5), (32, 3, 20, 5)])
def test_conv_fast_bf16_tile_forward(H, cin, cout, k):
    """Forward launches stage the output tile in bf16 (epi_bf16): same bits as
    the fp32-tile epilogue when nothing accumulates."""
    Km = K()
    torch.manual_seed(13)
    Q, B, W = 3, 4, H
    cinp, coutp = (cin + 7) // 8 * 8, (cout + 7) // 8 * 8
    x = bf(torch.randn(Q, B, H, W, cinp, device=DEV))
    w = bf(torch.randn(Q, coutp, k, k, cinp, device=DEV) * 0.2)
    bias = torch.randn(Q, coutp, device=DEV) * 0.1
    rows = torch.tensor([[2, 1, 1, 0], [0, 1, 1, 0]], dtype=torch.int32, device=DEV)
    outs = []
    for e in (0, 1):
        o = torch.full((Q, B, H, W, coutp), 7.0, dtype=torch.bfloat16, device=DEV)
        a = Km.ConvArgs()
        a.inp[0], a.out[0] = x.data_ptr(), o.data_ptr()
        a.gtab, a.ngroups, a.relu, a.epi_bf16 = rows.data_ptr(), 2, 1, e
        a.w, a.bias = w.data_ptr(), bias.data_ptr()
        a.G, a.B, a.H, a.W, a.Cinp, a.Coutp, a.KH, a.KW = Q, B, H, W, cinp, coutp, k, k
        a.TH = Km.conv_tile_rows(H, W)
        Km.check(Km.lib().gt_conv_fwd(a, stream()), "conv")
        torch.cuda.synchronize()
        outs.append(o)
    assert torch.equal(outs[0], outs[1])
    assert torch.all(outs[1][1] == 7.0)


@pytest.mark.parametrize("H,cin,cout,k,first", [(8, 104, 104, 3, False), (8, 56, 104, 5, False),
                                                (8, 104, 56, 5, False), (7, 50, 50, 3, False),
                                                (8, 3, 24, 5, True)])
def test_conv_small_images_multi_tile(H, cin, cout, k, first):
    """Generic conv with several whole small images per workgroup (8x8 stages
    of the deep S=(3,4,5) space): bit-identical to one image per workgroup
    (same per-pixel reduction order), correct against PyTorch, in group-table
    mode with N-ary input sums (+ the input-sum copy for the wgrad), batch
    gather, a batch that is not a multiple of the images per tile, and groups
    outside the table left untouched."""
    Km = K()
    L = Km.lib()
    torch.manual_seed(21)
    Q, B, W = 3, 6, H
    cinp, coutp = (cin + 7) // 8 * 8, (cout + 7) // 8 * 8
    nin = 1 if first else 3
    slots = [bf(torch.randn(Q, B, H, W, cinp, device=DEV)) for _ in range(nin)]
    for s in slots:
        s[..., cin:] = 0
    gather = None
    if first:
        data = torch.zeros(2 * Q * B, H, W, cinp, dtype=torch.bfloat16, device=DEV)
        perm = torch.randperm(2 * Q * B, device=DEV)[:Q * B]
        data[perm] = slots[0].view(Q * B, H, W, cinp)
        gather = perm.view(1, Q, B).to(torch.int64).contiguous()
    w = bf(torch.randn(Q, cout, cin, k, k, device=DEV) * 0.1).float()
    wp = torch.stack([pack_w(w[g], coutp, cinp) for g in range(Q)]).to(torch.bfloat16).contiguous()
    bias = torch.zeros(Q, coutp, device=DEV)
    bias[:, :cout] = torch.randn(Q, cout, device=DEV) * 0.1
    st = torch.zeros(8, dtype=torch.int32, device=DEV)
    in_mask = 1 if first else 0b111
    rows = torch.tensor([[2, in_mask, 1, 0], [0, 1 if first else 0b101, 1, 0]], dtype=torch.int32, device=DEV)
    outs, xsums = [], []
    for imgs in (1, 4):
        out = torch.full((Q, B, H, W, coutp), 5.0, dtype=torch.bfloat16, device=DEV)
        xs = torch.zeros(Q, B, H, W, cinp, dtype=torch.bfloat16, device=DEV)
        a = Km.ConvArgs()
        if first:
            a.inp[0], a.gather, a.st = data.data_ptr(), gather.data_ptr(), st.data_ptr()
        else:
            for i, s in enumerate(slots):
                a.inp[i] = s.data_ptr()
            a.xsum = xs.data_ptr()
        a.out[0] = out.data_ptr()
        a.gtab, a.ngroups, a.relu = rows.data_ptr(), 2, 1
        a.w, a.bias = wp.data_ptr(), bias.data_ptr()
        a.G, a.B, a.H, a.W, a.Cinp, a.Coutp, a.KH, a.KW = Q, B, H, W, cinp, coutp, k, k
        a.TH = Km.conv_tile_rows(H, W)
        old = L.gt_conv_set_imgs(imgs)
        Km.check(L.gt_conv_fwd(a, stream()), "conv(imgs={})".format(imgs))
        L.gt_conv_set_imgs(old)
        torch.cuda.synchronize()
        outs.append(out)
        xsums.append(xs)
    assert torch.equal(outs[0], outs[1])
    assert torch.equal(xsums[0], xsums[1])
    assert torch.all(outs[1][1] == 5.0)
    for g, ins in ((2, [0, 1, 2][:nin]), (0, [0] if first else [0, 2])):
        xsum = bf(sum(slots[i][g].float() for i in ins))
        if len(ins) > 1:
            assert torch.equal(xsums[1][g], xsum)
        x = xsum[..., :cin].permute(0, 3, 1, 2).float()
        r = conv_ref([x], w[g], bias[g, :cout], True).permute(0, 2, 3, 1)
        tol = 2e-2 * r.abs().max().item() + 1e-2
        assert (outs[1][g, ..., :cout].float() - r).abs().max().item() < tol
