"""Torch-only repro for the GPU_MAX_HW_QUEUES=3 start-up crash (verdict r4 item 6a): capture a HIP graph
that forks onto K side streams and joins back (the population step's shape: main chain + wgrad streams
+ W1 stream), replay it. usage: GPU_MAX_HW_QUEUES=3 python tools/probe_hwq.py K"""
import sys

import torch

k = int(sys.argv[1]) if len(sys.argv) > 1 else 3
x = torch.randn(1 << 20, device="cuda")
side = [torch.cuda.Stream() for _ in range(k)]
cap = torch.cuda.Stream()


def body():
    cur = torch.cuda.current_stream()
    outs = []
    for s in side:
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            outs.append(x * 2 + 1)
    y = x.sin()
    for s in side:
        cur.wait_stream(s)
    return y + sum(outs)


with torch.cuda.stream(cap):
    body()
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=cap):
    z = body()
for _ in range(20):
    g.replay()
torch.cuda.synchronize()
print("hw queues probe: %d side streams, graph replay ok, z[0]=%.4f" % (k, float(z[0])), flush=True)
