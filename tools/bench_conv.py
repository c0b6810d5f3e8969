"""Per-kernel timing of the conv kernels on the S=(3,5) layer shapes at a
population launch size (G groups x batch 32), both precisions, with the
diagnostic ``dbg`` switches (bit 0 skip MFMA, 1 skip stores, 2 skip loads)
to split a kernel's time into its phases. HIP-graph replay, events.

usage: DTYPE=fp32 G=80 python tools/bench_conv.py [reps]
Prints one JSON line per (kernel, shape, dbg): us per call, useful TFLOP/s,
ideal MFMA-bound us (2.5 PF bf16 / number of MFMA terms per product).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from gentun_amd.models.cnn_hip import split_planes
from gentun_amd.ops import cnn_kernels as K

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
DT = os.environ.get("DTYPE", "fp32")
prec, npl = K.PREC[DT], K.NPL[DT]
adt = torch.float32 if prec else torch.bfloat16
G, B = int(os.environ.get("G", "80")), 32
DBGS = [int(d) for d in os.environ.get("DBGS", "0,1,2,4,7").split(",")]
dev = torch.device("cuda", 0)
L = K.lib()
L.gt_conv_set_regepi.argtypes = [__import__("ctypes").c_int]
L.gt_conv_set_regepi(int(os.environ.get("REGEPI", "1")))


def pad8(c):
    return (c + 7) // 8 * 8


def timeit(fn):
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        for _ in range(2):
            fn(side.cuda_stream)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(side):
        graph.capture_begin(capture_error_mode="thread_local")
        for _ in range(reps):
            fn(side.cuda_stream)
        graph.capture_end()
    torch.cuda.synchronize()
    graph.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(3):
        graph.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000.0 / (3 * reps)


shapes = [("s1_in 5x5 3->20", 32, 3, 20, 5, 1), ("s1_n 3x3 20->20", 32, 20, 20, 3, 1),
          ("s1_n sum3", 32, 20, 20, 3, 3), ("s2_in 5x5 20->50", 16, 20, 50, 5, 1),
          ("s2_n 3x3 50->50", 16, 50, 50, 3, 1), ("s2_n sum2", 16, 50, 50, 3, 2)]
only = os.environ.get("ONLY")
for name, H, cin, cout, k, nin in shapes:
    if only and only not in name:
        continue
    W = H
    cinp, coutp = pad8(cin), pad8(cout)
    xs = [torch.randn(G, B, H, W, cinp, device=dev).to(adt) for _ in range(nin)]
    w = split_planes(torch.randn(G, coutp, k, k, cinp, device=dev) * 0.1, npl).contiguous()
    wT = split_planes(torch.randn(G, cinp, k, k, coutp, device=dev) * 0.1, npl).contiguous()
    bias = torch.zeros(G, coutp, device=dev)
    y = torch.randn(G, B, H, W, coutp, device=dev).to(adt)
    dy = torch.randn(G, B, H, W, coutp, device=dev).to(adt)
    dx = torch.zeros(G, B, H, W, cinp, device=dev).to(adt)
    xsum = torch.zeros(G, B, H, W, cinp, device=dev).to(adt)
    st = torch.zeros(8, dtype=torch.int32, device=dev)
    rows = torch.tensor([[g, (1 << nin) - 1, 1, 0] for g in range(G)], dtype=torch.int32, device=dev)
    drows = torch.tensor([[g, 1, 1 | (1 << 8), 0] for g in range(G)], dtype=torch.int32, device=dev)
    flops = 2.0 * G * B * H * W * cout * cin * k * k
    mfma_terms = 6 if prec else 1
    # padded MACs / MFMA rate: the MFMA-bound floor of the padded GEMM
    mac = G * B * H * W * ((coutp + 15) // 16 * 16) * (-(-(k * k * cinp) // 32) * 32)
    floor_us = mac * mfma_terms / 1.25e15 * 1e6
    for kind in ("conv_fwd", "conv_dgrad", "conv_wgrad"):
        for dbg in DBGS if kind != "conv_wgrad" else [0]:
            if kind == "conv_fwd":
                a = K.ConvArgs()
                for i, t in enumerate(xs):
                    a.inp[i] = t.data_ptr()
                a.out[0] = y.data_ptr()
                a.gtab, a.ngroups, a.relu, a.epi_bf16 = rows.data_ptr(), G, 1, 1
                a.w, a.bias, a.st, a.wps = w.data_ptr(), bias.data_ptr(), st.data_ptr(), w[0].numel()
                a.xsum = xsum.data_ptr() if nin > 1 else 0
                a.G, a.B, a.H, a.W, a.Cinp, a.Coutp, a.KH, a.KW = G, B, H, W, cinp, coutp, k, k
                a.TH, a.prec, a.dbg = K.conv_tile_rows(H, W), prec, dbg
                a.cout_real = cout
                fn = lambda s: K.check(L.gt_conv_fwd(a, s), kind)      # noqa: E731
            elif kind == "conv_dgrad":
                a = K.ConvArgs()
                a.inp[0], a.out[0] = dy.data_ptr(), dx.data_ptr()
                a.gtab, a.ngroups, a.relu, a.epi_bf16 = drows.data_ptr(), G, 0, 0
                a.w, a.bias, a.st, a.wps = wT.data_ptr(), 0, st.data_ptr(), wT[0].numel()
                a.G, a.B, a.H, a.W, a.Cinp, a.Coutp, a.KH, a.KW = G, B, H, W, coutp, cinp, k, k
                a.TH, a.prec, a.dbg = K.conv_tile_rows(H, W), prec, dbg
                a.cout_real = cin
                fn = lambda s: K.check(L.gt_conv_fwd(a, s), kind)      # noqa: E731
            else:
                npix = B * H * W
                Kdim = k * k * cinp
                pps, S = K.wgrad_split(npix, Kdim, coutp, G, band=K.wgrad_band(k, k, cinp, coutp, H, W, prec))
                pw = torch.zeros(S, G, coutp, Kdim, device=dev)
                pb = torch.zeros(S, G, coutp, device=dev)
                a = K.WgradArgs()
                for i, t in enumerate(xs):
                    a.inp[i] = t.data_ptr()
                a.gtab, a.ngroups = rows.data_ptr(), G
                a.gather, a.st = 0, st.data_ptr()
                a.dz, a.part_w, a.part_b = dy.data_ptr(), pw.data_ptr(), pb.data_ptr()
                a.G, a.B, a.H, a.W, a.Cinp, a.Coutp, a.KH, a.KW, a.S, a.pps = G, B, H, W, cinp, coutp, k, k, S, pps
                a.prec = prec
                a.cout_real = cout
                fn = lambda s: K.check(L.gt_conv_wgrad(a, s), kind)    # noqa: E731
            us = timeit(fn)
            print(json.dumps({"regepi": os.environ.get("REGEPI", "1"), "dtype": DT, "G": G, "kernel": kind, "shape": name, "dbg": dbg, "us": round(us, 1),
                              "tflops_useful": round(flops / us / 1e6, 1),
                              "mfma_floor_us": round(floor_us, 1), "mfma_eff": round(floor_us / us, 3)}), flush=True)
