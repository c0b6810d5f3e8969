"""Per-kernel timing of the Genetic-CNN HIP kernels on the real layer shapes
(fold-batched G=5, batch 32), with HIP events, N reps after warm-up.

usage: python tools/bench_kernels.py [reps]
Prints one JSON line per (kernel, shape): us per call, TFLOP/s, GB/s (ideal bytes).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from gentun_amd.ops import cnn_kernels as K

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
TILES = tuple(int(t) for t in os.environ.get("GENTUN_TILES", "128").split(","))
dev = torch.device("cuda", 0)
L = K.lib()
L.gt_conv_set_fast(int(os.environ.get("GENTUN_CONV_FAST", "1")))
L.gt_wgrad_set_nb(int(os.environ.get("GENTUN_WGRAD_NB", "0")))
G, B = int(os.environ.get("GENTUN_BENCH_G", "5")), 32


def pad8(c):
    return (c + 7) // 8 * 8


def timeit(fn):
    """Per-launch GPU time of ``fn(stream)``: ``reps`` launches captured in one
    HIP graph and replayed, so host launch overhead (ctypes + hipLaunchKernel,
    ~10 us) does not hide kernels shorter than it."""
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        for _ in range(3):
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
          ("s2_n 3x3 50->50", 16, 50, 50, 3, 1), ("deep 3x3 128->128 @8", 8, 128, 128, 3, 1)]
stream = torch.cuda.current_stream().cuda_stream
only = os.environ.get("GENTUN_BENCH_ONLY")          # "kernel:shape_index" (PMC runs)
if only:
    only_k, only_i = only.split(":")
    shapes = [shapes[int(only_i)]]
else:
    only_k = None
for name, H, cin, cout, k, nin in shapes:
    W = H
    cinp, coutp = pad8(cin), pad8(cout)
    xs = [torch.randn(G, B, H, W, cinp, device=dev).to(torch.bfloat16) for _ in range(nin)]
    w = (torch.randn(G, coutp, k, k, cinp, device=dev) * 0.1).to(torch.bfloat16)
    wT = (torch.randn(G, cinp, k, k, coutp, device=dev) * 0.1).to(torch.bfloat16)
    bias = torch.zeros(G, coutp, device=dev)
    y = torch.randn(G, B, H, W, coutp, device=dev).to(torch.bfloat16)
    dy = torch.randn(G, B, H, W, coutp, device=dev).to(torch.bfloat16)
    dx = torch.zeros(G, B, H, W, cinp, device=dev).to(torch.bfloat16)
    st = torch.zeros(8, dtype=torch.int32, device=dev)
    TH = K.conv_tile_rows(H, W)
    flops = 2.0 * G * B * H * W * cout * cin * k * k
    # fwd
    a = K.ConvArgs()
    for i, t in enumerate(xs):
        a.inp[i] = t.data_ptr()
    a.out[0] = y.data_ptr()
    a.n_in, a.n_out, a.acc_flags, a.relu = nin, 1, 0, 1
    a.w, a.bias, a.st = w.data_ptr(), bias.data_ptr(), st.data_ptr()
    a.G, a.B, a.H, a.W, a.Cinp, a.Coutp, a.KH, a.KW, a.TH = G, B, H, W, cinp, coutp, k, k, TH
    a.ngroups = G
    a.dbg = int(os.environ.get("GENTUN_CONV_DBG", "0"))
    a.epi_bf16 = int(os.environ.get("GENTUN_EPI_BF16", "0"))
    for tp in TILES:
        a.TH = K.conv_tile_rows(H, W, tp)
        us = timeit(lambda st: K.check(L.gt_conv_fwd(a, st), "fwd")) if only_k in (None, "conv_fwd") else 0.0
        byt = (nin * G * B * H * W * cinp + G * B * H * W * coutp) * 2
        print(json.dumps({"kernel": "conv_fwd", "tile": tp, "shape": name, "us": round(us, 2),
                          "tflops": round(flops / max(us, 1e-9) / 1e6, 2),
                          "gbs": round(byt / max(us, 1e-9) / 1e3, 1)}), flush=True)
    # dgrad
    d = K.ConvArgs()
    d.inp[0], d.mask, d.out[0] = dy.data_ptr(), 0, dx.data_ptr()
    d.n_in, d.n_out, d.acc_flags, d.relu = 1, 1, 0, 0
    d.w, d.bias, d.st = wT.data_ptr(), 0, st.data_ptr()
    d.G, d.B, d.H, d.W, d.Cinp, d.Coutp, d.KH, d.KW, d.TH = G, B, H, W, coutp, cinp, k, k, TH
    d.ngroups = G
    for tp in TILES:
        d.TH = K.conv_tile_rows(H, W, tp)
        us = timeit(lambda st: K.check(L.gt_conv_fwd(d, st), "dgrad")) if only_k in (None, "conv_dgrad") else 0.0
        byt = (2 * G * B * H * W * coutp + G * B * H * W * cinp) * 2
        print(json.dumps({"kernel": "conv_dgrad", "tile": tp, "shape": name, "us": round(us, 2),
                          "tflops": round(flops / max(us, 1e-9) / 1e6, 2),
                          "gbs": round(byt / max(us, 1e-9) / 1e3, 1)}), flush=True)
    # wgrad
    npix = B * H * W
    Kdim = k * k * cinp
    pps, S = K.wgrad_split(npix, Kdim, coutp, G, band=K.wgrad_band(k, k, cinp, coutp, H, W))
    pw = torch.zeros(S, G, coutp, Kdim, device=dev)
    pb = torch.zeros(S, G, coutp, device=dev)
    wa = K.WgradArgs()
    for i, t in enumerate(xs):
        wa.inp[i] = t.data_ptr()
    wa.n_in, wa.gather, wa.st = nin, 0, st.data_ptr()
    wa.dz, wa.part_w, wa.part_b = dy.data_ptr(), pw.data_ptr(), pb.data_ptr()
    wa.G, wa.B, wa.H, wa.W, wa.Cinp, wa.Coutp, wa.KH, wa.KW, wa.S, wa.pps = G, B, H, W, cinp, coutp, k, k, S, pps
    wa.ngroups = G
    us = timeit(lambda st: K.check(L.gt_conv_wgrad(wa, st), "wgrad")) if only_k in (None, "conv_wgrad") else 0.0
    byt = (nin * G * B * H * W * cinp + 2 * G * B * H * W * coutp) * 2 + S * G * coutp * Kdim * 4
    print(json.dumps({"kernel": "conv_wgrad", "shape": name, "us": round(us, 2), "tflops": round(flops / max(us, 1e-9) / 1e6, 2),
                      "gbs": round(byt / max(us, 1e-9) / 1e3, 1), "S": S}), flush=True)
