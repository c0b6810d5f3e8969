"""Winograd F(2x2, 3x3) vs the direct shape-specialised fp32 conv on the S=(3,5)
3x3 layer shapes at a population launch (G groups x batch 32): forward (two
summed DAG inputs, bias + ReLU) and data gradient (one accumulate + ReLU-mask
slot), plus the weight transform of one layer. HIP-graph replay, events.

usage: G=25 python tools/bench_wino.py [reps]     -> one JSON line per (shape, kernel, op)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from gentun_amd.models.cnn_hip import split_planes
from gentun_amd.ops import cnn_kernels as K

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
G, B = int(os.environ.get("G", "25")), 32
dev = torch.device("cuda", 0)
L = K.lib()


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


SHAPES = (("s2 3x3 50->50", 16, 50, 50), ("s1 3x3 20->20", 32, 20, 20))
ONLY = os.environ.get("ONLY")           # e.g. ONLY=s2: one shape; OPS=fwd: one op (PMC passes)
OPS = os.environ.get("OPS", "fwd,dgrad").split(",")
for name, H, cin, cout in SHAPES:
    if ONLY and not name.startswith(ONLY):
        continue
    cinp, coutp = (cin + 7) // 8 * 8, (cout + 7) // 8 * 8
    torch.manual_seed(0)
    x = [torch.randn(G, B, H, H, cinp, device=dev) for _ in range(2)]
    for t in x:
        t[..., cin:] = 0
    master = torch.zeros(G, coutp, 3, 3, cinp, device=dev)
    master[:, :cout, :, :, :cin] = torch.randn(G, cout, 3, 3, cin, device=dev) * 0.05
    wdir = split_planes(master, 3).contiguous()
    wdirT = split_planes(master.flip(2, 3).permute(0, 4, 2, 3, 1).contiguous(), 3).contiguous()
    U = K.wino_weights(master)
    UT = K.wino_weights(master, dgrad=True)
    bias = torch.zeros(G, coutp, device=dev)
    out = torch.zeros(G, B, H, H, coutp, device=dev)
    xsum = torch.zeros(G, B, H, H, cinp, device=dev)
    dz = torch.randn(G, B, H, H, coutp, device=dev)
    dx = torch.zeros(G, B, H, H, cinp, device=dev)
    nin = int(os.environ.get("NIN", "2"))     # summed DAG inputs of the forward (NIN > 1 also writes xsum)
    rows_f = torch.tensor([[g, (1 << nin) - 1, 1, 0] for g in range(G)], dtype=torch.int32, device=dev)
    rows_d = torch.tensor([[g, 1, 1 | (1 << 8) | (1 << 16), 0] for g in range(G)], dtype=torch.int32, device=dev)
    res = {}
    for wino in (0, 1):
        a = K.ConvArgs()
        a.inp[0], a.inp[1] = x[0].data_ptr(), x[1].data_ptr()
        a.out[0] = out.data_ptr()
        a.gtab, a.ngroups, a.relu, a.epi_bf16 = rows_f.data_ptr(), G, 1, 1
        wt = U if wino else wdir
        a.w, a.wps, a.bias, a.xsum = wt.data_ptr(), wt[0].numel(), bias.data_ptr(), xsum.data_ptr() if nin > 1 else 0
        a.G, a.B, a.H, a.W, a.Cinp, a.Coutp, a.KH, a.KW = G, B, H, H, cinp, coutp, 3, 3
        a.TH, a.prec, a.wino, a.cout_real = K.conv_tile_rows(H, H), 1, wino, cout
        d = K.ConvArgs()
        d.inp[0] = dz.data_ptr()
        d.out[0], d.out_mask[0] = dx.data_ptr(), x[0].data_ptr()
        d.gtab, d.ngroups, d.relu = rows_d.data_ptr(), G, 0
        wt = UT if wino else wdirT
        d.w, d.wps = wt.data_ptr(), wt[0].numel()
        d.G, d.B, d.H, d.W, d.Cinp, d.Coutp, d.KH, d.KW = G, B, H, H, coutp, cinp, 3, 3
        d.TH, d.prec, d.wino, d.cout_real = K.conv_tile_rows(H, H), 1, wino, cin
        kind = "wino" if wino else "direct"
        for op, args in (("fwd", a), ("dgrad", d)):
            if op not in OPS:
                continue
            for dbg in [int(v) for v in os.environ.get("DBGS" if wino else "DBGS_DIRECT", "0").split(",")]:
                if dbg:       # diagnostics: the Winograd kernel without some of its phases (wrong results)
                    args.dbg = dbg
                    us = timeit(lambda s, args=args: K.check(L.gt_conv_fwd(args, s), "conv"))
                    args.dbg = 0
                    print(json.dumps({"G": G, "shape": name, "kernel": kind, "op": op, "dbg": dbg,
                                      "us": round(us, 1)}), flush=True)
            us = timeit(lambda s, args=args: K.check(L.gt_conv_fwd(args, s), "conv"))
            torch.cuda.synchronize()
            o = (out if op == "fwd" else dx).clone()
            res[(op, wino)] = o
            flops = 2.0 * G * B * H * H * cin * cout * 9
            print(json.dumps({"G": G, "shape": name, "kernel": kind, "op": op, "us": round(us, 1),
                              "useful_tflops": round(flops / us * 1e-6, 1)}), flush=True)
    for op in OPS:
        d, w_ = res[(op, 0)].double(), res[(op, 1)].double()
        print(json.dumps({"shape": name, "op": op, "wino_vs_direct_rel": (w_ - d).abs().max().item() /
                          d.abs().max().item()}), flush=True)
    tr = K.WinoTransform([K.wino_segment(master, U, False), K.wino_segment(master, UT, True)], dev)
    us = timeit(lambda s: tr.run(s))
    print(json.dumps({"G": G, "shape": name, "kernel": "wino_wtrans (fwd + dgrad)", "us": round(us, 1)}), flush=True)
