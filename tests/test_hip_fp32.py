"""fp32 precision of the HIP kernels (``dtype='fp32'``, the reference's
Keras/TF float32): fp32 tensors, every matrix product on the bf16 matrix
cores as the exact 3-way split of its fp32 operands (csrc/hip/common.h).

Each kernel is checked against a float64 CPU oracle of the same op on the
same fp32 inputs; the error must be fp32-level (<= 1e-5 of the output range,
the verdict's bar was 1e-4) and is reported next to the error of torch's own
fp32 CPU op on the same inputs."""

import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

DEV = torch.device("cuda", 0) if torch.cuda.is_available() else None
TOL = 1e-5


def _split(w, npl=3):
    from gentun_amd.models.cnn_hip import split_planes
    return split_planes(w, npl)


def test_split_planes_exact_cpu():
    """The 3-plane split is exact: plane sum == fp32 value, bit for bit, over
    a wide exponent range (plane 0 = RNE bf16 rounding)."""
    g = torch.Generator().manual_seed(0)
    w = torch.randn(100000, generator=g) * torch.exp(torch.randn(100000, generator=g) * 8)
    pl = _split(w)
    back = pl[0].float() + pl[1].float() + pl[2].float()
    assert torch.equal(back, w)
    assert torch.equal(pl[0], w.to(torch.bfloat16))
    # the worst product error of the six kept terms stays within 2^-22 relative
    a, b = w[:50000].double(), w[50000:].double()
    pa, pb = _split(w[:50000]).double(), _split(w[50000:]).double()
    kept = sum(pa[i] * pb[j] for i in range(3) for j in range(3) if i + j <= 2)
    rel = ((kept - a * b).abs() / (a * b).abs().clamp_min(1e-300)).max().item()
    assert rel <= 2.0 ** -22, rel


def K():
    from gentun_amd.ops import cnn_kernels
    cnn_kernels.lib()
    return cnn_kernels


def stream():
    return torch.cuda.current_stream().cuda_stream


def nhwc_pad(x_nchw, cp):
    n, c, h, w = x_nchw.shape
    out = torch.zeros((n, h, w, cp), dtype=x_nchw.dtype, device=x_nchw.device)
    out[..., :c] = x_nchw.permute(0, 2, 3, 1)
    return out


def pack_w(w_oihw, coutp, cinp):
    co, ci, kh, kw = w_oihw.shape
    out = torch.zeros((coutp, kh, kw, cinp), dtype=w_oihw.dtype, device=w_oihw.device)
    out[:co, :, :, :ci] = w_oihw.permute(0, 2, 3, 1)
    return out


def rel(got, ref):
    return ((got.double().cpu() - ref.double().cpu()).abs().max() / ref.double().abs().max().clamp_min(1e-30)).item()


def report(name, ours, torch32):
    print("[fp32] {:<40s} rel.err HIP {:.2e}  torch-fp32 {:.2e}".format(name, ours, torch32))


CONV_SHAPES = [(32, 32, 3, 20, 5, 1), (32, 32, 20, 20, 3, 3), (16, 16, 20, 50, 5, 1), (16, 16, 50, 50, 3, 2),
               (16, 16, 50, 20, 5, 1), (8, 8, 64, 128, 3, 1), (7, 7, 50, 50, 3, 4), (14, 14, 20, 50, 5, 2),
               # stage 3 of the deep (20,50,100) space: shape-specialised 8x8 kernels
               (8, 8, 50, 100, 5, 1), (8, 8, 100, 100, 3, 2), (8, 8, 100, 50, 5, 1),
               # wide layers of the deep (64,128,256) space: channel-blocked patch staging
               (8, 8, 256, 256, 5, 1), (8, 8, 256, 100, 5, 2), (16, 16, 128, 128, 5, 3), (32, 32, 64, 64, 5, 2),
               # ... and their shape-specialised tile kernels (round 3): every conv / dgrad shape of the space
               (32, 32, 3, 64, 5, 1), (32, 32, 64, 64, 3, 2), (16, 16, 64, 128, 5, 1), (16, 16, 128, 128, 3, 2),
               (16, 16, 128, 64, 5, 1), (8, 8, 128, 256, 5, 1), (8, 8, 256, 256, 3, 3), (8, 8, 256, 128, 5, 1),
               # round 6, user-chosen architectures (cnn_conv_fast_ext.hip): 32 / 64-channel stages ...
               (32, 32, 3, 32, 5, 1), (32, 32, 32, 32, 3, 2), (16, 16, 32, 64, 5, 1), (16, 16, 64, 64, 3, 2),
               (16, 16, 64, 32, 5, 1),
               # ... and 3x3 stage-input convs (forward and, as the transposed shape, data gradient)
               (32, 32, 3, 20, 3, 1), (16, 16, 20, 50, 3, 1), (16, 16, 50, 20, 3, 1), (8, 8, 50, 100, 3, 1),
               (8, 8, 100, 50, 3, 1), (32, 32, 3, 64, 3, 1), (16, 16, 64, 128, 3, 1), (16, 16, 128, 64, 3, 1),
               (8, 8, 128, 256, 3, 1), (8, 8, 256, 128, 3, 1), (32, 32, 3, 32, 3, 1), (16, 16, 32, 64, 3, 1),
               (16, 16, 64, 32, 3, 1)]


@pytest.mark.gpu
@pytest.mark.parametrize("H,W,cin,cout,k,nin", CONV_SHAPES)
@pytest.mark.parametrize("pk,wfrag", [(0, 0), (1, 0), (1, 1)])
def test_conv_fwd_fp32(H, W, cin, cout, k, nin, pk, wfrag):
    """Forward conv (shape-specialised and generic kernels): fused N-ary Add
    in fp32, split MFMA, bias + ReLU; the input sum written for the wgrad
    (``xsum``) is the exact fp32 sum. ``pk``: the real output channel count
    is passed, so shapes with <= 4 real channels in the last 16-channel tile
    run the packed-tile kernel (plane rows, 3 MFMAs per k-step)."""
    Km = K()
    torch.manual_seed(10)
    G, B = 2, 3
    cinp, coutp = (cin + 7) // 8 * 8, (cout + 7) // 8 * 8
    xs = [torch.randn(G, B, cin, H, W) for _ in range(nin)]
    w = torch.randn(G, cout, cin, k, k) * (1.0 / math.sqrt(cin * k * k))
    b = torch.randn(G, cout) * 0.1
    x_in = [torch.stack([nhwc_pad(x[g], cinp) for g in range(G)]).to(DEV).contiguous() for x in xs]
    wp = torch.stack([pack_w(w[g], coutp, cinp) for g in range(G)]).to(DEV)
    # wfrag: the fragment-major planes (ConvArgs::wfrag) of the shape-specialised kernels
    wpl = Km.frag_planes(wp.contiguous(), W) if wfrag else _split(wp).contiguous()
    bp = torch.zeros(G, coutp, device=DEV)
    bp[:, :cout] = b.to(DEV)
    out = torch.full((G, B, H, W, coutp), 7.0, device=DEV)
    xsum = torch.zeros(G, B, H, W, cinp, device=DEV)
    rows = torch.tensor([[g, (1 << nin) - 1, 1, 0] for g in range(G)], dtype=torch.int32, device=DEV)
    a = Km.ConvArgs()
    for i, t in enumerate(x_in):
        a.inp[i] = t.data_ptr()
    a.out[0] = out.data_ptr()
    a.gtab, a.ngroups = rows.data_ptr(), G
    a.relu, a.epi_bf16 = 1, 1
    a.w, a.bias, a.wps = wpl.data_ptr(), bp.data_ptr(), wpl[0].numel()
    a.xsum = xsum.data_ptr() if nin > 1 else 0
    a.G, a.B, a.H, a.W, a.Cinp, a.Coutp, a.KH, a.KW = G, B, H, W, cinp, coutp, k, k
    a.TH = Km.conv_tile_rows(H, W)
    a.prec = 1
    a.cout_real = cout if pk else 0
    a.wfrag = wfrag
    if wfrag and not Km.lib().gt_conv_fast_probe_any(a):
        assert Km.lib().gt_conv_fwd(a, stream()) == -102           # generic kernels refuse fragment planes
        pytest.skip("generic-kernel shape: no fragment-major planes")
    Km.check(Km.lib().gt_conv_fwd(a, stream()), "conv")
    torch.cuda.synchronize()
    worst = worst32 = 0.0
    for g in range(G):
        x32 = sum(x[g] for x in xs)
        ref = F.relu(F.conv2d(x32.double(), w[g].double(), b[g].double(), padding=k // 2))
        r32 = F.relu(F.conv2d(x32, w[g], b[g], padding=k // 2))
        got = out[g, ..., :cout].permute(0, 3, 1, 2)
        worst, worst32 = max(worst, rel(got, ref)), max(worst32, rel(r32, ref))
        assert torch.all(out[g, ..., cout:] == 0)
        if nin > 1:
            assert torch.equal(xsum[g, ..., :cin].permute(0, 3, 1, 2).cpu(), x32)
    report("conv_fwd {}x{} {}->{} k{} n{}{}".format(H, W, cin, cout, k, nin, " wfrag" if wfrag else ""), worst, worst32)
    assert worst < TOL


@pytest.mark.gpu
@pytest.mark.parametrize("k,H", [(3, 16), (5, 16), (3, 32), (3, 8), (3, -16)])
@pytest.mark.parametrize("wfrag", [0, 1])
def test_conv_dgrad_fanout_fp32(k, H, wfrag):
    """Data gradient = conv of dz with the flipped / transposed weight planes;
    DAG fan-out into two slots, one accumulating, one ReLU-masked."""
    Km = K()
    torch.manual_seed(11)
    wide = H < 0                           # H = -16: 50 -> 50 at 16x16 (4 output tiles, packed last)
    H = abs(H)
    G, B, W = 2, 2, H
    cin, cout = (50, 50) if wide else (20, 50) if H == 16 else (20, 20) if H == 32 else (64, 128)
    cinp, coutp = (cin + 7) // 8 * 8, (cout + 7) // 8 * 8
    w = torch.randn(G, cout, cin, k, k) / math.sqrt(cout * k * k)
    dz = torch.randn(G, B, cout, H, W)
    ref = torch.stack([torch.nn.grad.conv2d_input((B, cin, H, W), w[g].double(), dz[g].double(), padding=k // 2)
                       for g in range(G)])
    r32 = torch.stack([torch.nn.grad.conv2d_input((B, cin, H, W), w[g], dz[g], padding=k // 2) for g in range(G)])
    wp = torch.stack([pack_w(w[g], coutp, cinp) for g in range(G)]).to(DEV)
    wT = Km.frag_planes(wp.contiguous(), W, dgrad=True) if wfrag else \
        _split(wp.flip(2, 3).permute(0, 4, 2, 3, 1).contiguous()).contiguous()
    dz_p = torch.stack([nhwc_pad(dz[g], coutp) for g in range(G)]).to(DEV).contiguous()
    out0 = torch.zeros(G, B, H, W, cinp, device=DEV)
    prev = torch.randn(G, B, H, W, cinp, device=DEV)
    prev[..., cin:] = 0
    out1 = prev.clone()
    pmask = torch.randn(G, B, H, W, cinp, device=DEV)
    rows = torch.tensor([[g, 1, 0b11 | (0b10 << 8) | (0b10 << 16), 0] for g in range(G)], dtype=torch.int32,
                        device=DEV)
    a = Km.ConvArgs()
    a.inp[0] = dz_p.data_ptr()
    a.out[0], a.out[1] = out0.data_ptr(), out1.data_ptr()
    a.out_mask[1] = pmask.data_ptr()
    a.gtab, a.ngroups, a.relu = rows.data_ptr(), G, 0
    a.w, a.bias, a.wps = wT.data_ptr(), 0, wT[0].numel()
    a.G, a.B, a.H, a.W, a.Cinp, a.Coutp, a.KH, a.KW = G, B, H, W, coutp, cinp, k, k
    a.TH = Km.conv_tile_rows(H, W)
    a.prec = 1
    a.cout_real = cin                      # packed last tile where the shape allows (20 = 16 + 4)
    a.wfrag = wfrag
    if wfrag and not Km.lib().gt_conv_fast_probe_any(a):
        assert Km.lib().gt_conv_fwd(a, stream()) == -102           # generic kernels refuse fragment planes
        pytest.skip("generic-kernel shape: no fragment-major planes")
    Km.check(Km.lib().gt_conv_fwd(a, stream()), "dgrad")
    torch.cuda.synchronize()
    got0 = out0[..., :cin].permute(0, 1, 4, 2, 3)
    e0, e32 = rel(got0, ref), rel(r32, ref)
    ref1 = (ref + prev[..., :cin].permute(0, 1, 4, 2, 3).double().cpu()) * \
        (pmask[..., :cin] > 0).permute(0, 1, 4, 2, 3).cpu()
    e1 = rel(out1[..., :cin].permute(0, 1, 4, 2, 3), ref1)
    report("conv_dgrad k{} H{} (write / acc+mask)".format(k, H), max(e0, e1), e32)
    assert e0 < TOL and e1 < TOL


@pytest.mark.gpu
@pytest.mark.parametrize("H,W,cin,cout,k,nin,first", [(32, 32, 3, 20, 5, 1, True), (32, 32, 20, 20, 3, 1, False),
                                                      (16, 16, 20, 50, 5, 1, False), (16, 16, 50, 50, 3, 2, False),
                                                      (8, 8, 64, 128, 3, 1, False), (14, 14, 50, 50, 3, 3, False),
                                                      (8, 8, 256, 256, 5, 1, False), (16, 16, 128, 128, 5, 2, False),
                                                      (8, 8, 50, 100, 5, 1, False), (8, 8, 100, 100, 3, 2, False),
                                                      # wide deep space, shape-specialised (round 3)
                                                      (32, 32, 3, 64, 5, 1, True), (32, 32, 64, 64, 3, 2, False),
                                                      (16, 16, 64, 128, 5, 1, False), (16, 16, 128, 128, 3, 1, False),
                                                      (8, 8, 128, 256, 5, 1, False), (8, 8, 256, 256, 3, 2, False),
                                                      # round 6: 32 / 64-channel stages, 3x3 stage-input convs
                                                      (32, 32, 3, 32, 5, 1, True), (32, 32, 32, 32, 3, 2, False),
                                                      (16, 16, 32, 64, 5, 1, False), (16, 16, 64, 64, 3, 1, False),
                                                      (32, 32, 3, 20, 3, 1, True), (16, 16, 20, 50, 3, 1, False),
                                                      (32, 32, 3, 64, 3, 1, True), (16, 16, 64, 128, 3, 1, False),
                                                      (8, 8, 50, 100, 3, 1, False), (8, 8, 128, 256, 3, 1, False),
                                                      (32, 32, 3, 32, 3, 1, True), (16, 16, 32, 64, 3, 1, False)])
@pytest.mark.parametrize("pk", [0, 1])
def test_conv_wgrad_fp32(H, W, cin, cout, k, nin, first, pk):
    """Weight + bias gradient (specialised register-staged kernel and the
    generic one), deterministic split-K partials summed in fixed order.
    ``pk``: real output channels passed -> packed last co tile where <= 4 real
    channels fall in it (20, 50); the padded rows' partials stay exactly 0."""
    Km = K()
    torch.manual_seed(12)
    G, B = 2, 4
    cinp, coutp = (cin + 7) // 8 * 8, (cout + 7) // 8 * 8
    xs = [torch.randn(G, B, cin, H, W) for _ in range(nin)]
    dz = torch.randn(G, B, cout, H, W) * (torch.rand(G, B, cout, H, W) > 0.4)
    x32 = sum(xs)
    ref = torch.stack([torch.nn.grad.conv2d_weight(x32[g].double(), (cout, cin, k, k), dz[g].double(),
                                                   padding=k // 2) for g in range(G)])
    r32 = torch.stack([torch.nn.grad.conv2d_weight(x32[g], (cout, cin, k, k), dz[g], padding=k // 2)
                       for g in range(G)])
    refb = dz.double().sum((1, 3, 4))
    x_in = [torch.stack([nhwc_pad(x[g], cinp) for g in range(G)]).to(DEV).contiguous() for x in xs]
    gather = None
    if first:
        data = torch.zeros(3 * G * B, H, W, cinp, device=DEV)
        perm = torch.randperm(3 * G * B, device=DEV)[:G * B]
        data[perm] = x_in[0].view(G * B, H, W, cinp)
        gather = perm.view(1, G, B).to(torch.int64).contiguous()
        x_in = [data]
    dz_p = torch.stack([nhwc_pad(dz[g], coutp) for g in range(G)]).to(DEV).contiguous()
    Kdim = k * k * cinp
    npix = B * H * W
    pps, S = Km.wgrad_split(npix, Kdim, coutp, target_blocks=16,
                            band=Km.wgrad_band(k, k, cinp, coutp, H, W, 1))
    pw = torch.zeros(S, G, coutp, Kdim, device=DEV)
    pb = torch.zeros(S, G, coutp, device=DEV)
    st = torch.zeros(8, dtype=torch.int32, device=DEV)
    rows = torch.tensor([[g, (1 << len(x_in)) - 1, 0, 0] for g in range(G)], dtype=torch.int32, device=DEV)
    a = Km.WgradArgs()
    for i, t in enumerate(x_in):
        a.inp[i] = t.data_ptr()
    a.gtab, a.ngroups = rows.data_ptr(), G
    a.gather = gather.data_ptr() if gather is not None else 0
    a.st = st.data_ptr()
    a.dz, a.part_w, a.part_b = dz_p.data_ptr(), pw.data_ptr(), pb.data_ptr()
    a.G, a.B, a.H, a.W, a.Cinp, a.Coutp, a.KH, a.KW, a.S, a.pps = G, B, H, W, cinp, coutp, k, k, S, pps
    a.prec = 1
    a.cout_real = cout if pk else 0
    Km.check(Km.lib().gt_conv_wgrad(a, stream()), "wgrad")
    torch.cuda.synchronize()
    assert torch.all(pw[:, :, cout:] == 0) and torch.all(pb[:, :, cout:] == 0)
    got = pw.sum(0).view(G, coutp, k, k, cinp)[:, :cout, :, :, :cin].permute(0, 1, 4, 2, 3)
    ew, e32 = rel(got, ref), rel(r32, ref)
    eb = rel(pb.sum(0)[:, :cout], refb)
    report("conv_wgrad {}x{} {}->{} k{} n{}{}".format(H, W, cin, cout, k, nin, " gather" if first else ""),
           max(ew, eb), e32)
    assert ew < TOL and eb < TOL


@pytest.mark.gpu
def test_pool_fp32_exact():
    Km = K()
    torch.manual_seed(13)
    N, C, cp, H, W = 6, 20, 24, 16, 16
    x = torch.randn(N, C, H, W, device=DEV)
    xr = x.clone().requires_grad_(True)
    y = F.max_pool2d(xr, 2, 2)
    dy = torch.randn_like(y)
    y.backward(dy)
    xp = nhwc_pad(x, cp).contiguous()
    yp = torch.zeros(N, H // 2, W // 2, cp, device=DEV)
    mask = torch.zeros(N, H // 2, W // 2, cp, dtype=torch.uint8, device=DEV)
    Km.check(Km.lib().gt_pool_fwd_mask(xp.data_ptr(), 0, 0, yp.data_ptr(), N, 1, H, W, cp, mask.data_ptr(), 1,
                                       stream()), "pool")
    dyp = nhwc_pad(dy, cp).contiguous()
    dxp = torch.full((N, H, W, cp), 7.0, device=DEV)
    Km.check(Km.lib().gt_pool_bwd_mask(mask.data_ptr(), 0, dyp.data_ptr(), dxp.data_ptr(), 0, N, 1, H, W, cp, 0, 1,
                                       stream()), "poolb")
    torch.cuda.synchronize()
    assert torch.equal(yp[..., :C].permute(0, 3, 1, 2), y.detach())
    assert torch.equal(dxp[..., :C].permute(0, 3, 1, 2), xr.grad)


@pytest.mark.gpu
def test_dense_fwd_dgrad_fp32():
    Km = K()
    torch.manual_seed(14)
    G, B, Fp, Up, C = 2, 32, 3584, 512, 10
    x = torch.relu(torch.randn(G, B, Fp))
    w1 = torch.randn(G, Fp, Up) / math.sqrt(Fp)
    b1 = torch.randn(G, Up) * 0.1
    ref = F.relu(torch.baddbmm(b1[:, None].double(), x.double(), w1.double()))
    r32 = F.relu(torch.baddbmm(b1[:, None], x, w1))
    w1d = w1.to(DEV).contiguous()                         # the fp32 master [G][Fp][Up]
    xd, b1d = x.to(DEV).contiguous(), b1.to(DEV).contiguous()
    out = torch.zeros(G, B, Up, device=DEV)
    st = torch.zeros(8, dtype=torch.int32, device=DEV)
    w2 = (torch.randn(G, Up, C) * 0.05).to(DEV)
    plog = torch.zeros(G, Up // 16, B, C, device=DEV)
    a = Km.DenseFwdArgs()
    a.x, a.wt, a.bias, a.out, a.st, a.fold_ids = xd.data_ptr(), 0, b1d.data_ptr(), out.data_ptr(), st.data_ptr(), 0
    a.G, a.B, a.Fp, a.Up, a.drop_p, a.train, a.seed = G, B, Fp, Up, 0.0, 0, 1
    a.w2, a.plog, a.C = w2.data_ptr(), plog.data_ptr(), C
    a.prec = 1
    ks = Km.lib().gt_dense_fwd_splits(Fp)
    part = torch.empty(G * (Up // 64) * ks * 4 * 2 * 64 * 4, device=DEV)
    a.w1, a.part, a.ks = w1d.data_ptr(), part.data_ptr(), ks
    Km.check(Km.lib().gt_dense_fwd(a, stream()), "dense")
    dH = torch.randn(G, B, Up)
    dHd = dH.to(DEV).contiguous()
    dx = torch.zeros(G, B, Fp, device=DEV)
    d = Km.DenseDgradArgs()
    d.dH, d.wt, d.dx, d.G, d.B, d.Fp, d.Up = dHd.data_ptr(), 0, dx.data_ptr(), G, B, Fp, Up
    d.prec, d.w1 = 1, w1d.data_ptr()
    Km.check(Km.lib().gt_dense_dgrad(d, stream()), "dgrad")
    torch.cuda.synchronize()
    ef, ef32 = rel(out, ref), rel(r32, ref)
    refdx = torch.bmm(dH.double(), w1.double().transpose(1, 2))
    ed, ed32 = rel(dx, refdx), rel(torch.bmm(dH, w1.transpose(1, 2)), refdx)
    reflog = torch.einsum("gbu,guc->gbc", out.double().cpu(), w2.double().cpu())
    el = rel(plog.sum(1), reflog)
    report("dense_fwd", ef, ef32)
    report("dense_dgrad", ed, ed32)
    assert ef < TOL and ed < TOL and el < TOL


@pytest.mark.gpu
def test_dense_wgrad_adam_fp32_planes():
    """Fused dW1 (fp32 VALU) + Adam on the fp32 master (nothing else is written: every W1 reader takes
    the master)."""
    Km = K()
    torch.manual_seed(15)
    G, B, Fp, Up = 2, 32, 400, 512
    x = torch.randn(G, B, Fp, device=DEV)
    dH = torch.randn(G, B, Up, device=DEV)
    p = torch.randn(G, Fp, Up, device=DEV)
    m = torch.randn(G, Fp, Up, device=DEV) * 0.01
    v = torch.rand(G, Fp, Up, device=DEV) * 0.01
    st = torch.zeros(8, dtype=torch.int32, device=DEV)
    stf = st.view(torch.float32)
    stf[2], stf[3] = 4.0, 1e-3
    Km.check(Km.lib().gt_step_begin(st.data_ptr(), stream()), "step_begin")
    g = torch.bmm(x.double().transpose(1, 2), dH.double())
    mm = 0.9 * m.double() + 0.1 * g
    vv = 0.999 * v.double() + 0.001 * g * g
    lr_t = 1e-3 * math.sqrt(1 - 0.999 ** 5) / (1 - 0.9 ** 5)
    rp = p.double() - lr_t * mm / (vv.sqrt() + 1e-7)
    a = Km.DenseWgradAdamArgs()
    a.x, a.dH, a.p, a.m, a.v, a.wt, a.st = x.data_ptr(), dH.data_ptr(), p.data_ptr(), m.data_ptr(), v.data_ptr(), \
        0, st.data_ptr()
    a.G, a.B, a.Fp, a.Up = G, B, Fp, Up
    a.prec = 1
    Km.check(Km.lib().gt_dense_wgrad_adam(a, stream()), "wgrad_adam")
    torch.cuda.synchronize()
    assert rel(m, mm) < TOL
    assert (p.double() - rp).abs().max().item() < 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("loss", ["bce_compat", "ce"])
def test_head_fp32(loss):
    Km = K()
    torch.manual_seed(16)
    G, B, Up, C, N = 2, 32, 512, 10, 100
    h = F.relu(torch.randn(G, B, Up, device=DEV))
    w2 = torch.randn(G, Up, C, device=DEV) * 0.05
    b2 = torch.randn(G, C, device=DEV) * 0.1
    labels = torch.randint(0, C, (N,), device=DEV)
    gather = torch.randint(0, N, (1, G, B), device=DEV)
    y = F.one_hot(labels[gather[0]], C).double()
    hr, w2r, b2r = (t.double().clone().requires_grad_(True) for t in (h, w2, b2))
    logits = torch.baddbmm(b2r[:, None], hr, w2r)
    p = torch.softmax(logits, -1)
    pc = p.clamp(1e-7, 1 - 1e-7)
    per = -(y * torch.log(pc) + (1 - y) * torch.log(1 - pc)).mean(-1) if loss == "bce_compat" else \
        -(y * torch.log(p)).sum(-1)
    per.mean(-1).sum().backward()
    dH = torch.zeros(G, B, Up, device=DEV)
    gw2, gb2, gb1 = torch.zeros_like(w2), torch.zeros_like(b2), torch.zeros(G, Up, device=DEV)
    st = torch.zeros(8, dtype=torch.int32, device=DEV)
    a = Km.HeadArgs()
    a.h, a.w2, a.b2, a.labels, a.gather, a.st = h.data_ptr(), w2.data_ptr(), b2.data_ptr(), labels.data_ptr(), \
        gather.data_ptr(), st.data_ptr()
    dzw = torch.zeros(G, B, C, device=DEV)
    a.dH, a.gw2, a.gb2, a.gb1, a.eval_out, a.dz = dH.data_ptr(), gw2.data_ptr(), gb2.data_ptr(), gb1.data_ptr(), \
        0, dzw.data_ptr()
    plog = torch.einsum("gbu,guc->gbc", h, w2).unsqueeze(1).contiguous()
    plog = torch.cat([plog, torch.zeros(G, Up // 16 - 1, B, C, device=DEV)], 1).contiguous()
    a.plog = plog.data_ptr()
    a.G, a.B, a.Up, a.C, a.loss_ce, a.drop_scale, a.eval, a.prec = G, B, Up, C, int(loss == "ce"), 1.0, 0, 1
    Km.check(Km.lib().gt_head(a, stream()), "head")
    torch.cuda.synchronize()
    refdH = hr.grad * (h.double() > 0)
    assert rel(dH, refdH) < 1e-5
    assert rel(gw2, w2r.grad) < 1e-5
    assert rel(gb1, refdH.sum(1)) < 1e-5
    assert rel(gb2, b2r.grad) < 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("tiled", [False, True])
def test_adam_segments_fp32_planes(tiled):
    """Conv-weight Adam over split-K partials writing the 3 planes of the
    bf16 copy and of the flipped / transposed dgrad copy."""
    Km = K()
    import ctypes
    torch.manual_seed(17)
    G, co, kh, kw, ci = 2, 24, 3, 3, 24
    S = 3
    n = G * co * kh * kw * ci
    p = torch.randn(n, device=DEV)
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    parts = torch.randn(S, n, device=DEV)
    bfp = torch.zeros(3, n, dtype=torch.bfloat16, device=DEV)
    bfT = torch.zeros(3, G, ci, kh, kw, co, dtype=torch.bfloat16, device=DEV)
    st = torch.zeros(8, dtype=torch.int32, device=DEV)
    stf = st.view(torch.float32)
    stf[2], stf[3] = 0.0, 1e-3
    Km.check(Km.lib().gt_step_begin(st.data_ptr(), stream()), "step_begin")
    sg = Km.AdamSeg()
    sg.p, sg.m, sg.v, sg.g = p.data_ptr(), m.data_ptr(), v.data_ptr(), parts.data_ptr()
    sg.bf, sg.bfT = bfp.data_ptr(), bfT.data_ptr()
    sg.n, sg.gstride, sg.S = n, n, S
    sg.tG, sg.tCo, sg.tKH, sg.tKW, sg.tCi = G, co, kh, kw, ci
    sg.npl, sg.pstride_bf, sg.pstride_bfT = 3, n, bfT[0].numel()
    nt = Km.adam_tiles(G, co, kh, kw, ci) if tiled else 0
    sg.tiled = 1 if nt else 0
    blocks = [(0, t) for t in range(nt)] if nt else [(0, o) for o in Km.adam_blocks(n)]
    segs = (Km.AdamSeg * 1)(sg)
    segs_t = torch.frombuffer(bytearray(bytes(memoryview(segs).cast("B"))), dtype=torch.uint8).to(DEV)
    blocks_t = torch.tensor(np.asarray(blocks, np.int32).reshape(-1, 2), device=DEV)
    aa = Km.AdamArgs()
    aa.segs, aa.blocks, aa.st = segs_t.data_ptr(), blocks_t.data_ptr(), st.data_ptr()
    p0 = p.clone()
    Km.check(Km.lib().gt_adam_segments(aa, len(blocks), stream()), "adam")
    torch.cuda.synchronize()
    g = parts.sum(0)
    lr_t = 1e-3 * math.sqrt(1 - 0.999) / (1 - 0.9)
    mm, vv = 0.1 * g, 0.001 * g * g
    rp = p0 - lr_t * mm / (vv.sqrt() + 1e-7)
    assert torch.allclose(p, rp, rtol=1e-6, atol=1e-6)
    assert torch.equal(bfp, _split(p))
    w = p.view(G, co, kh, kw, ci)
    assert torch.equal(bfT, _split(w.flip(2, 3).permute(0, 4, 2, 3, 1).contiguous()))
    del ctypes


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["write_acc_mask", "unpool"])
def test_s2in_dgrad_variants(mode):
    """The S=(3,5) stage-2 input-conv data gradient (5x5, 50 -> 20, 16x16) at
    the bench launch (25 groups x batch 32) in both kernel variants: the
    packed last co tile (default: channels 16-19 as 9-term plane rows) and one
    co tile per wave (GENTUN_S2IN_CT1: six-term products everywhere).

    * both are fp32-level against the fp64 oracle (<= TOL of the output range,
      reported next to torch fp32's own error);
    * channels 0-15 run the SAME k order and MFMA sequence in both -> bitwise
      equal (an indexing fault or race at a tile edge would break this);
    * every variant is deterministic launch to launch (bitwise)."""
    Km = K()
    L = Km.lib()
    torch.manual_seed(21)
    G, B, H, W, k = 25, 32, 16, 16, 5
    cin, cout = 20, 50                       # forward conv: 20 -> 50; its dgrad maps dz (50) to dx (20)
    cinp, coutp = 24, 56
    w = torch.randn(G, cout, cin, k, k) / math.sqrt(cout * k * k)
    dz = torch.randn(G, B, cout, H, W)
    ref = torch.stack([torch.nn.grad.conv2d_input((B, cin, H, W), w[g].double(), dz[g].double(), padding=2)
                       for g in range(G)])                                    # [G, B, cin, H, W]
    r32 = torch.stack([torch.nn.grad.conv2d_input((B, cin, H, W), w[g], dz[g], padding=2) for g in range(G)])
    wp = torch.stack([pack_w(w[g], coutp, cinp) for g in range(G)]).to(DEV)
    wT = _split(wp.flip(2, 3).permute(0, 4, 2, 3, 1).contiguous()).contiguous()
    dz_p = torch.stack([nhwc_pad(dz[g], coutp) for g in range(G)]).to(DEV).contiguous()
    prev = torch.randn(G, B, H, W, cinp, device=DEV)
    prev[..., cin:] = 0
    pmask = torch.randn(G, B, H, W, cinp, device=DEV)
    pm = torch.randint(0, 8, (G * B, H, W, cinp), dtype=torch.uint8, device=DEV)
    sel = (torch.arange(G, dtype=torch.int32, device=DEV) % 2).contiguous()
    outs = {}
    for variant in (0, 1, 0, 1):
        o0 = torch.zeros(G, B, H, W, cinp, device=DEV)
        o1 = prev.clone()
        x0 = torch.full((G, B, 2 * H, 2 * W, cinp), 4.0, device=DEV)
        x1 = torch.full((G, B, 2 * H, 2 * W, cinp), 6.0, device=DEV)
        a = Km.ConvArgs()
        a.inp[0] = dz_p.data_ptr()
        if mode == "unpool":
            rows = torch.tensor([[g, 1, 1 | (1 << 25), 0] for g in range(G)], dtype=torch.int32, device=DEV)
            a.out[0] = o0.data_ptr()
            a.pool_y, a.pool_mask, a.unpool_x1, a.unpool_sel = x0.data_ptr(), pm.data_ptr(), x1.data_ptr(), \
                sel.data_ptr()
        else:
            rows = torch.tensor([[g, 1, 0b11 | (0b10 << 8) | (0b10 << 16), 0] for g in range(G)], dtype=torch.int32,
                                device=DEV)
            a.out[0], a.out[1] = o0.data_ptr(), o1.data_ptr()
            a.out_mask[1] = pmask.data_ptr()
        a.gtab, a.ngroups, a.relu, a.epi_bf16 = rows.data_ptr(), G, 0, 0
        a.w, a.bias, a.wps = wT.data_ptr(), 0, wT[0].numel()
        a.G, a.B, a.H, a.W, a.Cinp, a.Coutp, a.KH, a.KW = G, B, H, W, coutp, cinp, k, k
        a.TH, a.prec, a.cout_real = Km.conv_tile_rows(H, W), 1, cin
        old = L.gt_conv_set_s2in_ct1(variant)
        try:
            Km.check(L.gt_conv_fwd(a, stream()), "dgrad")
            torch.cuda.synchronize()
        finally:
            L.gt_conv_set_s2in_ct1(old)
        got = (x0, x1) if mode == "unpool" else (o0, o1)
        if variant in outs:                                  # second launch of the same variant: bitwise
            for t0, t1 in zip(outs[variant], got):
                assert torch.equal(t0, t1), ("nondeterministic", variant)
        outs[variant] = got
    e32 = rel(r32, ref)
    if mode == "unpool":
        # un-pooled gradient: value at the argmax cell of each 2x2 cell when bit 2 (max > 0) is set
        mk = pm.view(G, B, H, W, cinp)[..., :cin].long().cpu()
        refn = ref.permute(0, 1, 3, 4, 2)                                       # [G, B, H, W, cin]
        for variant in (0, 1):
            x0, x1 = outs[variant]
            for g in range(G):
                dst = (x1 if sel[g].item() else x0)[g].cpu().double()[..., :cin]        # [B, 2H, 2W, cin]
                cell = dst.view(B, H, 2, W, 2, cin).permute(0, 1, 3, 2, 4, 5).reshape(B, H, W, 4, cin)
                want = torch.zeros(B, H, W, 4, cin, dtype=torch.float64)
                hit = (mk[g] & 4) > 0
                idx = (mk[g] & 3)
                want.scatter_(3, idx.unsqueeze(3), torch.where(hit, refn[g], torch.zeros_like(refn[g])).unsqueeze(3))
                e = ((cell - want).abs().max() / refn.abs().max()).item()
                assert e < TOL, (variant, g, e)
            report("s2in dgrad unpool variant {}".format(variant), e, e32)
        other = (outs[0][0] != 4.0) | (outs[0][1] != 6.0)
        assert other.any()
        c0 = [t.view(G, B, 2 * H, 2 * W, cinp)[..., :16] for t in outs[0]]
        c1 = [t.view(G, B, 2 * H, 2 * W, cinp)[..., :16] for t in outs[1]]
        assert all(torch.equal(a0, a1) for a0, a1 in zip(c0, c1))
        return
    refm = (ref + prev[..., :cin].permute(0, 1, 4, 2, 3).double().cpu()) * \
        (pmask[..., :cin] > 0).permute(0, 1, 4, 2, 3).cpu()
    for variant in (0, 1):
        o0, o1 = outs[variant]
        e0 = rel(o0[..., :cin].permute(0, 1, 4, 2, 3), ref)
        e1 = rel(o1[..., :cin].permute(0, 1, 4, 2, 3), refm)
        report("s2in dgrad variant {} (write / acc+mask)".format(variant), max(e0, e1), e32)
        assert e0 < TOL and e1 < TOL, (variant, e0, e1)
        assert (o0[..., cin:] == 0).all()                                # padding channels stay zero
    for i in range(2):
        assert torch.equal(outs[0][i][..., :16], outs[1][i][..., :16])   # same k order: bitwise
        d = (outs[0][i][..., 16:cin] - outs[1][i][..., 16:cin]).abs().max().item()
        assert d <= 4 * e32 * ref.abs().max().item() + 1e-30, d         # 9- vs 6-term: rounding only

