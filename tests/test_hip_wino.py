"""Winograd F(2x2, 3x3) fp32 convolutions (csrc/hip/cnn_conv_wino.hip): the
3x3 node / output convs of the S=(3,5) space and their data gradients.

Every launch is checked against a float64 oracle of the same op (error must
stay fp32-level, <= 1e-5 of the output range, and is reported next to
torch's own fp32 error), the weight transform against an fp64 G g G^T, the
fused epilogues (pool + argmax mask, un-pool, DAG fan-out, zero-padded
image) against the direct shape-specialised kernels or exact references,
and the small-launch tile height for bit-identity (batch invariance)."""

import math

import pytest
import torch
import torch.nn.functional as F

from test_hip_fp32 import K, _split, nhwc_pad, pack_w, rel, report, stream

DEV = torch.device("cuda", 0) if torch.cuda.is_available() else None
TOL = 1e-5
pytestmark = pytest.mark.gpu

G_MAT = [[1.0, 0.0, 0.0], [0.5, 0.5, 0.5], [0.5, -0.5, 0.5], [0.0, 0.0, 1.0]]


def _u_ref(master, dgrad):
    """fp64 U [Q][16][R][K] of fp32 master weights [Q][Cop][3][3][Cip]."""
    Km = K()
    Q, cop, _, _, cip = master.shape
    w = master.double().cpu()
    if dgrad:
        w = w.flip(2, 3).permute(0, 4, 2, 3, 1)          # [Q][Cip][3][3][Cop]
    Gm = torch.tensor(G_MAT, dtype=torch.float64)
    u = torch.einsum("ia,qrabc,jb->qijrc", Gm, w, Gm)    # [Q][4][4][rows][cols]
    R, Kc = Km.wino_dims(cop, cip) if dgrad else Km.wino_dims(cip, cop)
    out = torch.zeros(Q, 16, R, Kc, dtype=torch.float64)
    out[:, :, :u.shape[3], :u.shape[4]] = u.reshape(Q, 16, u.shape[3], u.shape[4])
    return out


def _master(G, cout, cin, seed, scale=None):
    g = torch.Generator().manual_seed(seed)
    w = torch.randn(G, cout, cin, 3, 3, generator=g) * (scale or 1.0 / math.sqrt(cin * 9))
    cinp, coutp = (cin + 7) // 8 * 8, (cout + 7) // 8 * 8
    wp = torch.stack([pack_w(w[q], coutp, cinp) for q in range(G)]).to(DEV).contiguous()
    return w, wp


@pytest.mark.parametrize("cin,cout", [(50, 50), (20, 20), (20, 50)])
@pytest.mark.parametrize("dgrad", [False, True])
def test_wino_weight_transform(cin, cout, dgrad):
    Km = K()
    _, wp = _master(3, cout, cin, 1)
    planes = Km.wino_unpack(Km.wino_weights(wp, dgrad=dgrad))
    torch.cuda.synchronize()
    got = (planes[0].double() + planes[1].double() + planes[2].double()).cpu()
    ref = _u_ref(wp, dgrad)
    assert got.shape == ref.shape
    err = ((got - ref).abs().max() / ref.abs().max()).item()
    print("[wino] U transform {}->{} dgrad={} rel.err {:.2e}".format(cin, cout, dgrad, err))
    assert err < 1e-6
    # padding rows / columns are exactly zero (the kernel reads them)
    rows, cols = (cin, cout) if dgrad else (cout, cin)
    assert float(got[:, :, rows:].abs().max() if got.shape[2] > rows else 0.0) == 0.0
    assert float(got[:, :, :, cols:].abs().max() if got.shape[3] > cols else 0.0) == 0.0
    # plane 0 is the RNE bf16 rounding of the fp32 value (the split is exact)
    assert torch.equal(planes[0].cpu(), (got.float()).to(torch.bfloat16))


def _fwd_args(Km, x_in, out, U, bp, G, B, H, W, cinp, coutp, nin, pool=None, xsum=None, hr=0):
    rows = torch.tensor([[g, (1 << nin) - 1, 1 | ((1 << 24) if pool is not None else 0), 0] for g in range(G)],
                        dtype=torch.int32, device=DEV)
    a = Km.ConvArgs()
    for i, t in enumerate(x_in):
        a.inp[i] = t.data_ptr()
    a.out[0] = out.data_ptr()
    a.gtab, a.ngroups = rows.data_ptr(), G
    a.relu, a.epi_bf16 = 1, 1
    a.w, a.bias, a.wps = U.data_ptr(), bp.data_ptr(), U[0].numel()
    a.xsum = xsum.data_ptr() if xsum is not None else 0
    a.G, a.B, a.H, a.W, a.Cinp, a.Coutp, a.KH, a.KW = G, B, H, W, cinp, coutp, 3, 3
    a.TH = Km.conv_tile_rows(H, W)
    a.prec, a.wino = 1, 1
    if pool is not None:
        a.pool_y, a.pool_mask = pool[0].data_ptr(), pool[1].data_ptr()
    if hr:
        a.Hr, a.Wr = hr, hr
    a._keep = rows
    return a


@pytest.mark.parametrize("H,cin,cout,nin,B", [(16, 50, 50, 1, 3), (16, 50, 50, 3, 3), (16, 50, 50, 2, 32),
                                              (16, 53, 50, 1, 3), (16, 50, 56, 2, 2)])
@pytest.mark.parametrize("pool", [False, True])
def test_wino_conv_fwd(H, cin, cout, nin, B, pool):
    """Forward: fused N-ary Add (exact fp32 sum also written to xsum), Winograd product, bias +
    ReLU; with ``pool`` the lane-local fused 2x2 max-pool and its argmax mask."""
    Km = K()
    torch.manual_seed(20)
    G, W = 2, H
    cinp, coutp = (cin + 7) // 8 * 8, (cout + 7) // 8 * 8
    xs = [torch.randn(G, B, cin, H, W) for _ in range(nin)]
    w, wp = _master(G, cout, cin, 2)
    b = torch.randn(G, cout) * 0.1
    x_in = [torch.stack([nhwc_pad(x[g], cinp) for g in range(G)]).to(DEV).contiguous() for x in xs]
    U = Km.wino_weights(wp)
    bp = torch.zeros(G, coutp, device=DEV)
    bp[:, :cout] = b.to(DEV)
    out = torch.full((G, B, H, W, coutp), 7.0, device=DEV)
    xsum = torch.zeros(G, B, H, W, cinp, device=DEV) if nin > 1 else None
    pl = None
    if pool:
        pl = (torch.full((G, B, H // 2, W // 2, coutp), 9.0, device=DEV),
              torch.zeros((G * B, H // 2, W // 2, coutp), dtype=torch.uint8, device=DEV))
    a = _fwd_args(Km, x_in, out, U, bp, G, B, H, W, cinp, coutp, nin, pool=pl, xsum=xsum)
    Km.check(Km.lib().gt_conv_fwd(a, stream()), "wino conv")
    torch.cuda.synchronize()
    worst = worst32 = 0.0
    for g in range(G):
        x32 = sum(x[g] for x in xs)
        ref = F.relu(F.conv2d(x32.double(), w[g].double(), b[g].double(), padding=1))
        r32 = F.relu(F.conv2d(x32, w[g], b[g], padding=1))
        got = out[g, ..., :cout].permute(0, 3, 1, 2)
        worst, worst32 = max(worst, rel(got, ref)), max(worst32, rel(r32, ref))
        assert torch.all(out[g, ..., cout:] == 0)
        if nin > 1:
            assert torch.equal(xsum[g, ..., :cin].permute(0, 3, 1, 2).cpu(), x32)
    report("wino conv_fwd {}x{} {}->{} n{} B{}{}".format(H, W, cin, cout, nin, B, " pool" if pool else ""),
           worst, worst32)
    assert worst < TOL
    if pool:
        y = out.view(G * B, H, W, coutp).permute(0, 3, 1, 2)
        ref_p = F.max_pool2d(y, 2, 2).permute(0, 2, 3, 1).reshape(G, B, H // 2, W // 2, coutp)
        assert torch.equal(pl[0], ref_p)
        # argmax rule: first strict maximum over (0,0), (0,1), (1,0), (1,1); bit 2 = maximum > 0
        q = torch.stack([y[:, :, 0::2, 0::2], y[:, :, 0::2, 1::2], y[:, :, 1::2, 0::2], y[:, :, 1::2, 1::2]], 0)
        arg = torch.zeros_like(q[0], dtype=torch.int64)
        m = q[0].clone()
        for k in (1, 2, 3):
            better = q[k] > m
            arg[better], m[better] = k, q[k][better]
        want = (arg | torch.where(m > 0, 4, 0)).to(torch.uint8).permute(0, 2, 3, 1)
        assert torch.equal(pl[1], want)


def test_wino_padded_image_zeros():
    """Zero-padded image (MNIST 14 x 14 stored as 16 x 16): exact zeros outside the real extent,
    the conv of the real image inside."""
    Km = K()
    torch.manual_seed(21)
    G, B, H, hr, cin, cout = 2, 2, 16, 14, 50, 50
    cinp = coutp = 56
    x = torch.zeros(G, B, cin, H, H)
    x[..., :hr, :hr] = torch.randn(G, B, cin, hr, hr)
    w, wp = _master(G, cout, cin, 3)
    b = torch.randn(G, cout) * 0.1
    x_in = [torch.stack([nhwc_pad(x[g], cinp) for g in range(G)]).to(DEV).contiguous()]
    U = Km.wino_weights(wp)
    bp = torch.zeros(G, coutp, device=DEV)
    bp[:, :cout] = b.to(DEV)
    out = torch.full((G, B, H, H, coutp), 7.0, device=DEV)
    a = _fwd_args(Km, x_in, out, U, bp, G, B, H, H, cinp, coutp, 1, hr=hr)
    Km.check(Km.lib().gt_conv_fwd(a, stream()), "wino conv")
    torch.cuda.synchronize()
    assert float(out[:, :, hr:].abs().max()) == 0.0 and float(out[:, :, :, hr:].abs().max()) == 0.0
    for g in range(G):
        ref = F.relu(F.conv2d(x[g, ..., :hr, :hr].double(), w[g].double(), b[g].double(), padding=1))
        assert rel(out[g, :, :hr, :hr, :cout].permute(0, 3, 1, 2), ref) < TOL


def _dgrad_args(Km, dz_p, outs, masks, wts, G, B, H, W, cinp, coutp, flags, wino):
    rows = torch.tensor([[g, 1, f, 0] for g, f in zip(range(G), flags)], dtype=torch.int32, device=DEV)
    a = Km.ConvArgs()
    a.inp[0] = dz_p.data_ptr()
    for k, t in enumerate(outs):
        a.out[k] = t.data_ptr()
    for k, t in enumerate(masks):
        a.out_mask[k] = t.data_ptr() if t is not None else 0
    a.gtab, a.ngroups, a.relu = rows.data_ptr(), G, 0
    a.w, a.bias, a.wps = wts.data_ptr(), 0, wts[0].numel()
    a.G, a.B, a.H, a.W, a.Cinp, a.Coutp, a.KH, a.KW = G, B, H, W, coutp, cinp, 3, 3
    a.TH = Km.conv_tile_rows(H, W)
    a.prec, a.wino = 1, 1 if wino else 0
    a._keep = rows
    return a


@pytest.mark.parametrize("H,cin,cout", [(16, 50, 50), (16, 56, 49)])
def test_wino_dgrad_fanout(H, cin, cout):
    """Data gradient = Winograd conv of dz with U of the flipped, transposed kernel; DAG fan-out into
    two slots, one accumulating, one ReLU-masked."""
    Km = K()
    torch.manual_seed(22)
    G, B, W = 2, 2, H
    cinp, coutp = (cin + 7) // 8 * 8, (cout + 7) // 8 * 8
    w, wp = _master(G, cout, cin, 4, scale=1.0 / math.sqrt(cout * 9))
    dz = torch.randn(G, B, cout, H, W)
    ref = torch.stack([torch.nn.grad.conv2d_input((B, cin, H, W), w[g].double(), dz[g].double(), padding=1)
                       for g in range(G)])
    r32 = torch.stack([torch.nn.grad.conv2d_input((B, cin, H, W), w[g], dz[g], padding=1) for g in range(G)])
    UT = Km.wino_weights(wp, dgrad=True)
    dz_p = torch.stack([nhwc_pad(dz[g], coutp) for g in range(G)]).to(DEV).contiguous()
    out0 = torch.zeros(G, B, H, W, cinp, device=DEV)
    prev = torch.randn(G, B, H, W, cinp, device=DEV)
    prev[..., cin:] = 0
    out1 = prev.clone()
    pmask = torch.randn(G, B, H, W, cinp, device=DEV)
    a = _dgrad_args(Km, dz_p, [out0, out1], [None, pmask], UT, G, B, H, W, cinp, coutp,
                    [0b11 | (0b10 << 8) | (0b10 << 16)] * G, True)
    Km.check(Km.lib().gt_conv_fwd(a, stream()), "wino dgrad")
    torch.cuda.synchronize()
    got0 = out0[..., :cin].permute(0, 1, 4, 2, 3)
    e0, e32 = rel(got0, ref), rel(r32, ref)
    ref1 = (ref + prev[..., :cin].permute(0, 1, 4, 2, 3).double().cpu()) * \
        (pmask[..., :cin] > 0).permute(0, 1, 4, 2, 3).cpu()
    e1 = rel(out1[..., :cin].permute(0, 1, 4, 2, 3), ref1)
    report("wino conv_dgrad H{} (write / acc+mask)".format(H), max(e0, e1), e32)
    assert e0 < TOL and e1 < TOL


def test_wino_dgrad_unpool_matches_direct():
    """A 3x3 data gradient whose output is a pool's gradient (a 3x3 stage-input kernel) un-pools it
    in the epilogue: same scatter as the direct shape-specialised kernel, values to fp32 rounding."""
    Km = K()
    torch.manual_seed(23)
    G, B, H, cin, cout = 2, 2, 16, 50, 50
    cinp = coutp = 56
    _, wp = _master(G, cout, cin, 5, scale=1.0 / math.sqrt(cout * 9))
    dz_p = torch.randn(G, B, H, H, coutp, device=DEV)
    dz_p[..., cout:] = 0
    # argmax mask of a forward pool whose output had this (H x W) shape: random cells, ~70 % positive
    arg = torch.randint(0, 4, (G * B, H, H, cinp), device=DEV)
    pos = (torch.rand(G * B, H, H, cinp, device=DEV) < 0.7).to(torch.int64) * 4
    mask = (arg | pos).to(torch.uint8).contiguous()
    sel = torch.tensor([0, 1], dtype=torch.int32, device=DEV)
    res = {}
    for wino in (False, True):
        x0 = torch.full((G, B, 2 * H, 2 * H, cinp), 5.0, device=DEV)
        x1 = torch.full((G, B, 2 * H, 2 * H, cinp), 5.0, device=DEV)
        wts = Km.wino_weights(wp, dgrad=True) if wino else \
            _split(wp.flip(2, 3).permute(0, 4, 2, 3, 1).contiguous()).contiguous()
        a = _dgrad_args(Km, dz_p, [x0], [None], wts, G, B, H, H, cinp, coutp, [1 | (1 << 25)] * G, wino)
        a.pool_y, a.pool_mask, a.unpool_x1, a.unpool_sel = x0.data_ptr(), mask.data_ptr(), x1.data_ptr(), \
            sel.data_ptr()
        a.cout_real = cin
        Km.check(Km.lib().gt_conv_fwd(a, stream()), "dgrad unpool")
        torch.cuda.synchronize()
        res[wino] = (x0.clone(), x1.clone())
    for k in (0, 1):
        d, w_ = res[False][k], res[True][k]
        assert torch.equal(d == 0, w_ == 0) and torch.equal(d == 5.0, w_ == 5.0)
        assert rel(w_, d) < TOL


def test_wino_small_launch_tiles_bit_identical():
    """Below ~300 workgroups the half-height tile runs; a group's output must be bit-identical to the
    same group inside a large launch (batch invariance of candidate results)."""
    Km = K()
    torch.manual_seed(24)
    Gbig, B, H, cin, cout = 10, 32, 16, 50, 50
    cinp = coutp = 56
    x = torch.randn(Gbig, B, H, H, cinp, device=DEV)
    x[..., cin:] = 0
    _, wp = _master(Gbig, cout, cin, 6)
    U = Km.wino_weights(wp)
    bp = torch.randn(Gbig, coutp, device=DEV) * 0.1
    bp[:, cout:] = 0
    outs = {}
    for ng in (Gbig, 1):                                  # 10 x 32 x 2 = 640 workgroups vs 64
        out = torch.zeros(Gbig, B, H, H, coutp, device=DEV)
        a = _fwd_args(Km, [x], out, U, bp, Gbig, B, H, H, cinp, coutp, 1)
        a.ngroups = ng
        assert Km.lib().gt_conv_fast_probe(a) == (8 if ng == Gbig else 4)
        Km.check(Km.lib().gt_conv_fwd(a, stream()), "wino conv")
        torch.cuda.synchronize()
        outs[ng] = out[0].clone()
    assert torch.equal(outs[Gbig], outs[1])


def test_wino_refuses_unsupported_shapes():
    """wino = 1 on a shape without an instantiation is an error (the weights are U planes: falling
    back onto the direct kernels would silently compute garbage)."""
    Km = K()
    a = Km.ConvArgs()
    a.G, a.B, a.H, a.W, a.Cinp, a.Coutp, a.KH, a.KW, a.ngroups = 1, 1, 8, 8, 104, 104, 3, 3, 1
    a.prec, a.wino = 1, 1
    assert Km.lib().gt_conv_fwd(a, stream()) == -101
    assert Km.lib().gt_conv_wino_supported(104, 104, 8, 8) == 0
    assert Km.lib().gt_conv_wino_supported(56, 56, 16, 16) == 1
    assert Km.lib().gt_conv_wino_supported(24, 24, 32, 32) == 0      # stage 1: the direct kernel is faster


def test_winograd_executor_matches_direct():
    """cnn_hip.WINOGRAD = True (off by default: slower in the step, profiles/r6/wino_bench_r6.txt) trains
    the same network: the stage-2 3x3 layers on the Winograd kernels with weights re-transformed after every
    optimizer step give the direct kernels' validation losses to fp32 summation-order rounding."""
    import numpy as np
    from gentun_amd.models import cnn_engine as E
    from gentun_amd.models import cnn_hip
    from gentun_amd.models.genome import make_plan
    from gentun_amd.utils.data import make_image_classification, stratified_kfold
    x, y = make_image_classification(n=640, shape=(32, 32, 3), classes=10, seed=5, noise=0.35, shift=2)
    folds = stratified_kfold(np.argmax(y, 1), 3, seed=0)
    plan = make_plan({'S_1': '101', 'S_2': '0101110011'}, (3, 5), (32, 32, 3), (20, 50), ((5, 5), (5, 5)), 500, 10)
    res, old = {}, cnn_hip.WINOGRAD
    try:
        for wino in (False, True):
            cnn_hip.WINOGRAD = wino
            cfg = E.TrainConfig(epochs=(1,), learning_rate=(1e-2,), batch_size=32, dtype="fp32", loss="ce",
                                reset="all", optimizer="sgd")
            job = E.make_job("hip", plan, x, y, folds, cfg, DEV)
            assert any(L.wino for L in job.layers) == wino
            job.launch()
            res[wino] = job.finish()
    finally:
        cnn_hip.WINOGRAD = old
    a, b = np.array(res[True]["val_loss"]), np.array(res[False]["val_loss"])
    assert np.all(np.isfinite(a)) and np.max(np.abs(a - b) / np.abs(b)) < 2e-4, (a, b)
