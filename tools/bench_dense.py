"""Dense head kernel timing (dense_fwd, dense_dgrad; fp32) at the bench's
population-launch size: G groups x batch 32, Fp = 3584 (8x8x56 pooled
features of S=(3,5) kernels (20,50)), Up = 512. HIP-graph replay of `reps`
launches; GB/s counts the fp32 W1 bytes (the roofline term).

usage: python tools/bench_dense.py [G] [reps]
"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from gentun_amd.ops import cnn_kernels as Km

G = int(sys.argv[1]) if len(sys.argv) > 1 else 25
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
B, Fp, Up, C = 32, 3584, 512, 10
dev = "cuda"
L = Km.lib()
torch.manual_seed(0)
w1 = torch.randn(G, Fp, Up, device=dev) * 0.05
wt = w1.transpose(1, 2).contiguous()
x = torch.randn(G, B, Fp, device=dev)
b1 = torch.zeros(G, Up, device=dev)
w2 = torch.randn(G, Up, C, device=dev)
st = torch.zeros(8, dtype=torch.int32, device=dev)
out = torch.zeros(G, B, Up, device=dev)
plog = torch.zeros(G, Up // 16, B, C, device=dev)
dH = torch.randn(G, B, Up, device=dev)
dx = torch.zeros(G, B, Fp, device=dev)
a = Km.DenseFwdArgs()
a.x, a.wt, a.bias, a.out, a.st = x.data_ptr(), wt.data_ptr(), b1.data_ptr(), out.data_ptr(), st.data_ptr()
a.G, a.B, a.Fp, a.Up, a.drop_p, a.train, a.seed = G, B, Fp, Up, 0.5, 1, 1
a.w2, a.plog, a.C, a.prec = w2.data_ptr(), plog.data_ptr(), C, 1
ks = L.gt_dense_fwd_splits(Fp)
part = torch.empty(G * (Up // 64) * ks * 4 * 2 * 64 * 4, device=dev)
a.w1, a.part, a.ks = w1.data_ptr(), part.data_ptr(), ks
d = Km.DenseDgradArgs()
d.dH, d.wt, d.dx, d.G, d.B, d.Fp, d.Up, d.prec = dH.data_ptr(), wt.data_ptr(), dx.data_ptr(), G, B, Fp, Up, 1
d.w1 = w1.data_ptr()
# fused dW1 + Adam on the fp32 master / m / v (padded channels 50 of 56, units 500 of 512: the bench shapes)
pm, vm = torch.zeros_like(w1), torch.ones_like(w1) * 1e-3
st[:] = 0
st.view(torch.float32)[3] = 1e-3
L.gt_step_begin(st.data_ptr(), None)
wa = Km.DenseWgradAdamArgs()
wa.x, wa.dH, wa.p, wa.m, wa.v, wa.wt, wa.st = x.data_ptr(), dH.data_ptr(), w1.data_ptr(), pm.data_ptr(), \
    vm.data_ptr(), 0, st.data_ptr()
wa.G, wa.B, wa.Fp, wa.Up, wa.Cp, wa.Cr, wa.Ur, wa.prec = G, B, Fp, Up, 56, 50, 500, 1
flush = torch.empty(512 * 1024 * 1024 // 4, device=dev)     # 512 MB: evicts the Infinity Cache


def timeit(fn, cold):
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        for _ in range(3):
            fn(side.cuda_stream)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        if cold:
            flush.add_(1.0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(side):
            e0.record()
            fn(side.cuda_stream)
            e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1000.0)
    ts.sort()
    return ts[len(ts) // 2]


wbytes = G * Fp * Up * 4
for name, fn in (("dense_fwd", lambda s: Km.check(L.gt_dense_fwd(a, ctypes.c_void_p(s)), "fwd")),
                 ("dense_dgrad", lambda s: Km.check(L.gt_dense_dgrad(d, ctypes.c_void_p(s)), "dgrad")),
                 ("dense_wgrad_adam", lambda s: Km.check(L.gt_dense_wgrad_adam(wa, ctypes.c_void_p(s)), "wadam"))):
    for cold in (True, False):
        us = timeit(fn, cold)
        print(json.dumps({"kernel": name, "G": G, "cold": cold, "us": round(us, 1),
                          "w1_GBps": round(wbytes / us / 1e3, 1),
                          # p/m/v read + written over the real rows / units (the kernel's HBM floor)
                          "pmv_GBps": round(6 * G * 3200 * 500 * 4 / us / 1e3, 1) if name == "dense_wgrad_adam" else None,
                          }), flush=True)
