"""Variants of the shape-specialised fp32 conv against each other: the tile
kernel's LDS-tile epilogue vs its register-direct epilogue (the default for
16 / 32-wide images) must be BIT-identical for every output -- forward with
bias / ReLU / N-ary input sum / ``xsum`` / fused 2x2 pool + argmax mask, data
gradient with the DAG fan-out (accumulate, ReLU mask, several output slots)
and the fused un-pool -- for every shape-specialised fp32 layer of the S=(3,5)
space incl. the packed last co tile; and the fp32 wgrad's column slices vs
one workgroup. (Round 3-5 persistent variants of this file -- two-team "duo",
fixed-role "pipe" -- were measured slower and deleted:
profiles/r5/conv_f32_sched_pipe_ab_r5.txt.)"""

import pytest
import torch

DEV = torch.device("cuda", 0) if torch.cuda.is_available() else None

# (H, W, cin, cout, k): the fp32 shape-specialised layers (gt_conv_fast)
SHAPES = [(32, 32, 3, 20, 5), (32, 32, 20, 20, 3), (16, 16, 20, 50, 5), (16, 16, 50, 50, 3), (16, 16, 50, 20, 5)]


def K():
    from gentun_amd.ops import cnn_kernels
    cnn_kernels.lib()
    return cnn_kernels


def pad8(c):
    return (c + 7) // 8 * 8


def _run(Km, a, mode, wgs):
    """mode 0: tile kernel, LDS-tile epilogue; 3: tile kernel, register-direct epilogue
    (gt_conv_set_regepi). ``wgs`` is unused (kept so the parametrisations stay comparable)."""
    import ctypes
    L = Km.lib()
    L.gt_conv_set_regepi.argtypes = [ctypes.c_int]
    L.gt_conv_set_regepi.restype = ctypes.c_int
    old_re = L.gt_conv_set_regepi(1 if mode == 3 else 0)
    try:
        Km.check(L.gt_conv_fwd(a, torch.cuda.current_stream().cuda_stream), "conv")
        torch.cuda.synchronize()
    finally:
        L.gt_conv_set_regepi(old_re)


def _split(w):
    from gentun_amd.models.cnn_hip import split_planes
    return split_planes(w, 3).contiguous()


@pytest.mark.gpu
@pytest.mark.parametrize("H,W,cin,cout,k", SHAPES)
@pytest.mark.parametrize("nin", [1, 3])
def test_epilogue_variants_forward_bit_identical(H, W, cin, cout, k, nin, wgs=0):
    Km = K()
    torch.manual_seed(H + cin + k + nin)
    G, B = 3, 8
    cinp, coutp = pad8(cin), pad8(cout)
    xs = []
    for _ in range(nin):
        x = torch.zeros(G, B, H, W, cinp, device=DEV)
        x[..., :cin] = torch.randn(G, B, H, W, cin, device=DEV)
        xs.append(x)
    w = torch.zeros(G, coutp, k, k, cinp, device=DEV)
    w[:, :cout, :, :, :cin] = torch.randn(G, cout, k, k, cin, device=DEV) * 0.1
    wpl = _split(w)
    bias = torch.zeros(G, coutp, device=DEV)
    bias[:, :cout] = torch.randn(G, cout, device=DEV) * 0.1
    # group 0 sums every input and pools, group 1 reads input 0 only, group 2 sums and pools
    full = (1 << nin) - 1
    rows = torch.tensor([[0, full, 1 | (1 << 24), 0], [1, 1, 1, 0], [2, full, 1 | (1 << 24), 0]],
                        dtype=torch.int32, device=DEV)
    outs = {}
    for mode in (0, 3):
        out = torch.full((G, B, H, W, coutp), 7.0, device=DEV)
        xsum = torch.full((G, B, H, W, cinp), 3.0, device=DEV)
        py = torch.full((G, B, H // 2, W // 2, coutp), 5.0, device=DEV)
        pm = torch.full((G * B, H // 2, W // 2, coutp), 9, dtype=torch.uint8, device=DEV)
        a = Km.ConvArgs()
        for i, t in enumerate(xs):
            a.inp[i] = t.data_ptr()
        a.out[0] = out.data_ptr()
        a.gtab, a.ngroups, a.relu, a.epi_bf16 = rows.data_ptr(), G, 1, 1
        a.w, a.bias, a.wps = wpl.data_ptr(), bias.data_ptr(), wpl[0].numel()
        a.xsum = xsum.data_ptr() if nin > 1 else 0
        a.pool_y, a.pool_mask = py.data_ptr(), pm.data_ptr()
        a.G, a.B, a.H, a.W, a.Cinp, a.Coutp, a.KH, a.KW = G, B, H, W, cinp, coutp, k, k
        a.TH, a.prec, a.cout_real = Km.conv_tile_rows(H, W), 1, cout
        _run(Km, a, mode, wgs)
        outs[mode] = (out, xsum, py, pm)
    for m in (3,):
        for name, t0, t2 in zip(("out", "xsum", "pool_y", "pool_mask"), outs[0], outs[m]):
            assert torch.equal(t0, t2), (m, name)
    # the reference kernel really pooled groups 0 and 2 (sanity of the comparison itself)
    assert not torch.equal(outs[0][2][0], torch.full_like(outs[0][2][0], 5.0))


@pytest.mark.gpu
@pytest.mark.parametrize("H,W,cin,cout,k", SHAPES)
def test_epilogue_variants_data_gradient_bit_identical(H, W, cin, cout, k, wgs=0):
    """Data-gradient launches (conv with flipped weights, no bias / ReLU):
    per group write / accumulate / ReLU-mask into up to two output slots."""
    Km = K()
    torch.manual_seed(100 + H + cin)
    G, B = 3, 8
    cinp, coutp = pad8(cin), pad8(cout)
    dz = torch.zeros(G, B, H, W, cinp, device=DEV)
    dz[..., :cin] = torch.randn(G, B, H, W, cin, device=DEV)
    w = torch.zeros(G, coutp, k, k, cinp, device=DEV)
    w[:, :cout, :, :, :cin] = torch.randn(G, cout, k, k, cin, device=DEV) * 0.1
    wpl = _split(w)
    masks = [torch.randn(G, B, H, W, coutp, device=DEV) for _ in range(2)]
    init = [torch.randn(G, B, H, W, coutp, device=DEV) for _ in range(2)]
    # bits 0-7 write, 8-15 accumulate, 16-23 ReLU mask
    rows = torch.tensor([[0, 1, 1 | (1 << 8) | (1 << 16), 0], [1, 1, 3 | (1 << 9) | (1 << 17), 0],
                         [2, 1, 2 | (1 << 16 + 1), 0]], dtype=torch.int32, device=DEV)
    outs = {}
    for mode in (0, 3):
        o = [t.clone() for t in init]
        a = Km.ConvArgs()
        a.inp[0] = dz.data_ptr()
        a.out[0], a.out[1] = o[0].data_ptr(), o[1].data_ptr()
        a.out_mask[0], a.out_mask[1] = masks[0].data_ptr(), masks[1].data_ptr()
        a.gtab, a.ngroups, a.relu, a.epi_bf16 = rows.data_ptr(), G, 0, 0
        a.w, a.bias, a.wps = wpl.data_ptr(), 0, wpl[0].numel()
        a.G, a.B, a.H, a.W, a.Cinp, a.Coutp, a.KH, a.KW = G, B, H, W, cinp, coutp, k, k
        a.TH, a.prec, a.cout_real = Km.conv_tile_rows(H, W), 1, cout
        _run(Km, a, mode, wgs)
        outs[mode] = o
    for m in (3,):
        for i in range(2):
            assert torch.equal(outs[0][i], outs[m][i]), (m, i)
    assert not torch.equal(outs[0][0], init[0])


@pytest.mark.gpu
@pytest.mark.parametrize("H,W,cin,cout,k", [(16, 16, 50, 20, 5), (16, 16, 50, 50, 3)])
def test_epilogue_variants_unpool_bit_identical(H, W, cin, cout, k):
    """A data gradient whose output is a pool's gradient scatters it to the
    forward's argmax cells of the pool source (slot chosen per group)."""
    Km = K()
    torch.manual_seed(7)
    G, B = 3, 8
    cinp, coutp = pad8(cin), pad8(cout)
    dz = torch.zeros(G, B, H, W, cinp, device=DEV)
    dz[..., :cin] = torch.randn(G, B, H, W, cin, device=DEV)
    w = torch.zeros(G, coutp, k, k, cinp, device=DEV)
    w[:, :cout, :, :, :cin] = torch.randn(G, cout, k, k, cin, device=DEV) * 0.1
    wpl = _split(w)
    pm = torch.randint(0, 8, (G * B, H, W, coutp), dtype=torch.uint8, device=DEV)
    sel = torch.tensor([0, 1, 0], dtype=torch.int32, device=DEV)
    rows = torch.tensor([[g, 1, 1 | (1 << 25), 0] for g in range(G)], dtype=torch.int32, device=DEV)
    outs = {}
    for mode in (0, 3):
        x0 = torch.full((G, B, 2 * H, 2 * W, coutp), 4.0, device=DEV)
        x1 = torch.full((G, B, 2 * H, 2 * W, coutp), 6.0, device=DEV)
        dummy = torch.zeros(G, B, H, W, coutp, device=DEV)
        a = Km.ConvArgs()
        a.inp[0], a.out[0] = dz.data_ptr(), dummy.data_ptr()
        a.gtab, a.ngroups, a.relu, a.epi_bf16 = rows.data_ptr(), G, 0, 0
        a.w, a.bias, a.wps = wpl.data_ptr(), 0, wpl[0].numel()
        a.pool_y, a.pool_mask, a.unpool_x1, a.unpool_sel = x0.data_ptr(), pm.data_ptr(), x1.data_ptr(), sel.data_ptr()
        a.G, a.B, a.H, a.W, a.Cinp, a.Coutp, a.KH, a.KW = G, B, H, W, cinp, coutp, k, k
        a.TH, a.prec, a.cout_real = Km.conv_tile_rows(H, W), 1, cout
        _run(Km, a, mode, 6)
        outs[mode] = (x0, x1, dummy)
    for m in (3,):
        for i in range(3):
            assert torch.equal(outs[0][i], outs[m][i]), (m, i)


@pytest.mark.gpu
@pytest.mark.parametrize("H,W,cin,cout,k", SHAPES[:4])
@pytest.mark.parametrize("nin", [1, 2])
def test_wgrad_column_slices_bit_identical(H, W, cin, cout, k, nin):
    """Small launches slice the fp32 wgrad's k-column tiles over NZ = 2 / 4 / 8
    workgroups per (split, group) (8: 4-wave workgroups): every weight
    gradient (and the bias column) is bit-identical to the one-workgroup
    kernel, for single and summed (DAG) inputs and the packed last co tile."""
    import ctypes
    Km = K()
    L = Km.lib()
    L.gt_wgrad_set_nz.argtypes = [ctypes.c_int]
    L.gt_wgrad_set_nz.restype = ctypes.c_int
    torch.manual_seed(3 + k + nin)
    G, B = 2, 8
    cinp, coutp = pad8(cin), pad8(cout)
    xs = []
    for _ in range(nin):
        x = torch.zeros(G, B, H, W, cinp, device=DEV)
        x[..., :cin] = torch.randn(G, B, H, W, cin, device=DEV)
        xs.append(x)
    dz = torch.zeros(G, B, H, W, coutp, device=DEV)
    dz[..., :cout] = torch.randn(G, B, H, W, cout, device=DEV)
    kd = k * k * cinp
    pps, S = Km.wgrad_split(B * H * W, kd, coutp, G, band=Km.wgrad_band(k, k, cinp, coutp, H, W, 1))
    rows = torch.tensor([[g, (1 << nin) - 1, 0, 0] for g in range(G)], dtype=torch.int32, device=DEV)
    st = torch.zeros(8, dtype=torch.int32, device=DEV)
    res = {}
    for nz in (1, 2, 4, 8):
        pw = torch.full((S, G, coutp, kd), 9.0, device=DEV)
        pb = torch.full((S, G, coutp), 9.0, device=DEV)
        a = Km.WgradArgs()
        for i, t in enumerate(xs):
            a.inp[i] = t.data_ptr()
        a.gtab, a.ngroups, a.gather, a.st = rows.data_ptr(), G, 0, st.data_ptr()
        a.dz, a.part_w, a.part_b = dz.data_ptr(), pw.data_ptr(), pb.data_ptr()
        a.G, a.B, a.H, a.W, a.Cinp, a.Coutp, a.KH, a.KW, a.S, a.pps = G, B, H, W, cinp, coutp, k, k, S, pps
        a.prec, a.cout_real = 1, cout
        old = L.gt_wgrad_set_nz(nz)
        try:
            Km.check(L.gt_conv_wgrad(a, torch.cuda.current_stream().cuda_stream), "wgrad")
            torch.cuda.synchronize()
        finally:
            L.gt_wgrad_set_nz(old)
        res[nz] = (pw, pb)
    for nz in (2, 4, 8):
        assert torch.equal(res[1][0], res[nz][0]), nz
        assert torch.equal(res[1][1], res[nz][1]), nz
    assert not torch.equal(res[1][0], torch.full_like(res[1][0], 9.0))
