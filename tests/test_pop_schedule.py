"""The population-batched launch schedule (gentun_amd/models/pop_schedule.py)
executed by a float64 CPU interpreter -- one conv / pool / fan-out record at a
time, exactly as the HIP step issues them -- against autograd through every
group's own plan (gentun_amd/models/genome.py ``Plan.steps``, the decoding of
gentun/models/keras_models.py:46-118). Pins the DAG gradient fan-out
(write vs accumulate), the ReLU-mask placement (the slot's last writer), the
N-ary input sums the weight gradients read, and the pool source selection."""

import random

import pytest
import torch
import torch.nn.functional as F

from gentun_amd.models.genome import ConvSpec, Plan
from gentun_amd.models.pop_schedule import ACC_SHIFT, MASK_SHIFT, PopulationSchedule, popcount

B = 2


def _plans(nodes, hw, cin, kernels, ksizes, genes_list):
    return [Plan(g, nodes, (hw, hw, cin), kernels, ksizes, 8, 3) for g in genes_list]


def _random_genes(rng, nodes):
    genes = {}
    for s, k in enumerate(nodes):
        nb = k * (k - 1) // 2
        r = rng.random()
        if r < 0.15:
            bits = "0" * nb
        elif r < 0.3:
            bits = "1" * nb
        else:
            bits = "".join(rng.choice("01") for _ in range(nb))
        genes["S_{}".format(s + 1)] = bits
    return genes


def _params(sched, gen):
    """Per layer, per group: weight [cout, cin, KH, KW] and bias (float64)."""
    P = {}
    for L in sched.layers:
        for q, _ in L.rows:
            w = torch.randn(L.cout, L.cin, L.KH, L.KW, generator=gen, dtype=torch.float64) * 0.3
            b = torch.randn(L.cout, generator=gen, dtype=torch.float64) * 0.1
            P[(L.name, q)] = (w, b)
    return P


def _conv(x, w, b):
    return F.conv2d(x, w, b, padding=(w.shape[2] // 2, w.shape[3] // 2))


def _reference(plan, q, x, P, R):
    """Autograd through group q's own plan; returns {layer: (dW, db)}."""
    act = {"input": x}
    leaves = {}
    for st in plan.steps:
        if isinstance(st, ConvSpec):
            w, b = P[(st.name, q)]
            w, b = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
            leaves[st.name] = (w, b)
            xin = act[st.inputs[0]]
            for n in st.inputs[1:]:
                xin = xin + act[n]
            act[st.name] = F.relu(_conv(xin, w, b))
        else:
            act[st.name] = F.max_pool2d(act[st.srcs[0]], 2)
    last = plan.steps[-1].name
    (act[last] * R).sum().backward()
    return {n: (w.grad, b.grad) for n, (w, b) in leaves.items()}


def _run_schedule(sched, x, P, R):
    """Forward then backward through the launch records; returns
    {(layer, group): (dW, db)}."""
    Q = sched.Q
    B = x.shape[0]                     # the batch rows this (data-parallel) rank holds
    act, xin = {"input": x}, {}
    # ---- forward: one launch per superset layer, per group its input set
    for st in sched.stages:
        for L in st.layers:
            out = torch.zeros(Q, B, L.cout, L.H, L.W, dtype=torch.float64)
            xs = torch.zeros(Q, B, L.cin, L.H, L.W, dtype=torch.float64)
            for q, im in L.rows:
                srcs = [act[n] if n == "input" else act[n][q] for k, n in enumerate(L.slots) if (im >> k) & 1]
                s = srcs[0]
                for t in srcs[1:]:
                    s = s + t
                xs[q] = s
                w, b = P[(L.name, q)]
                out[q] = F.relu(_conv(s, w, b))
            act[L.name] = out
            if L.xin is not None:
                xin[L.name] = xs
        sel = sched.pool_source(st)
        x1 = sched.pool_x1(st)
        pooled = []
        for q in range(Q):
            src = act[x1] if sel[q] else act[st.inp]
            pooled.append(F.max_pool2d(src[q], 2))
        act[st.pool] = torch.stack(pooled)
    # ---- backward
    grad = {sched.last: R.clone()}
    out = {}
    for rec in sched.backward():
        kind = rec[0]
        if kind == "pool_bwd":
            st = rec[1]
            sel = sched.pool_source(st)
            for q in range(Q):
                src = sched.pool_x1(st) if sel[q] else st.inp
                a = act[src][q].clone().requires_grad_(True)
                (F.max_pool2d(a, 2) * grad[st.pool][q]).sum().backward()
                g = a.grad * (act[src][q] > 0)            # pool_bwd applies the conv's ReLU mask
                grad.setdefault(src, torch.zeros_like(act[src]))[q] = g
            continue
        L, rows = rec[1], rec[2]
        if kind == "wgrad":
            wslots = L.slots + ([L.xin] if L.xin is not None else [])
            for q, im in rows:
                assert popcount(im) == 1, "wgrad reads exactly one slot"
                k = im.bit_length() - 1
                n = wslots[k]
                xq = xin[L.name][q] if n == L.xin else (act[n] if n == "input" else act[n][q])
                dz = grad[L.name][q]
                w, _ = P[(L.name, q)]
                dW = torch.nn.grad.conv2d_weight(xq, w.shape, dz, padding=(L.KH // 2, L.KW // 2))
                out[(L.name, q)] = (dW, dz.sum((0, 2, 3)))
        else:
            for q, of in rows:
                w, _ = P[(L.name, q)]
                dz = grad[L.name][q]
                dx = torch.nn.grad.conv2d_input((B, L.cin, L.H, L.W), w, dz, padding=(L.KH // 2, L.KW // 2))
                for k, n in enumerate(L.slots):
                    if not (of >> k) & 1:
                        continue
                    g = grad.setdefault(n, torch.zeros_like(act[n]))
                    v = dx + g[q] if (of >> (ACC_SHIFT + k)) & 1 else dx
                    if (of >> (MASK_SHIFT + k)) & 1:
                        v = v * (act[n][q] > 0)
                    g[q] = v
    return out


CASES = [
    # (nodes, hw, cin, kernels, kernel sizes, groups, seed)
    ((3, 5), 8, 3, (4, 6), ((5, 5), (5, 5)), 12, 0),
    ((3, 4, 5), 8, 2, (3, 4, 5), ((3, 3), (5, 5), (3, 3)), 10, 1),
    ((4,), 4, 1, (3,), ((3, 3),), 16, 2),
]


@pytest.mark.parametrize("case", CASES)
def test_schedule_matches_autograd(case):
    nodes, hw, cin, kernels, ksizes, G, seed = case
    rng = random.Random(seed)
    genes = [_random_genes(rng, nodes) for _ in range(G)]
    genes[0] = {"S_{}".format(s + 1): "0" * (k * (k - 1) // 2) for s, k in enumerate(nodes)}
    genes[1] = {"S_{}".format(s + 1): "1" * (k * (k - 1) // 2) for s, k in enumerate(nodes)}
    plans = _plans(nodes, hw, cin, kernels, ksizes, genes)
    sched = PopulationSchedule(plans)
    gen = torch.Generator().manual_seed(seed)
    P = _params(sched, gen)
    x = torch.randn(B, cin, hw, hw, generator=gen, dtype=torch.float64)
    hs = hw >> len(nodes)
    R = torch.randn(G, B, kernels[-1], hs, hs, generator=gen, dtype=torch.float64)
    got = _run_schedule(sched, x, P, R)
    nchecked = 0
    for q, plan in enumerate(plans):
        ref = _reference(plan, q, x, P, R[q])
        have = sorted(n for (n, g) in got if g == q)
        assert have == sorted(ref), (q, plan.genes)
        for n, (dW, db) in ref.items():
            gW, gb = got[(n, q)]
            torch.testing.assert_close(gW, dW, rtol=1e-9, atol=1e-9)
            torch.testing.assert_close(gb, db, rtol=1e-9, atol=1e-9)
            nchecked += 1
    assert nchecked >= G * len(nodes)


def test_schedule_structure():
    nodes = (3, 5)
    plans = _plans(nodes, 8, 3, (4, 6), ((5, 5), (5, 5)),
                   [{"S_1": "000", "S_2": "0000000000"}, {"S_1": "110", "S_2": "1000000001"}])
    sched = PopulationSchedule(plans)
    names = [L.name for L in sched.layers]
    assert names[0] == "s1_in" and "s2_out" in names
    s1 = sched.stages[0]
    assert s1.active == [False, True] and s1.has_out
    assert sched.pool_source(s1) == [0, 1]
    # group 1, S_1 = "110": node1 <- node0, node2 <- node0 (N-ary none): out sums nodes 1, 2
    out = [L for L in sched.layers if L.name == "s1_out"][0]
    assert out.rows == [(1, 0b110)] and out.xin == "s1_out_xin"
    seq = sched.backward()
    assert seq[0][0] == "pool_bwd" and seq[0][1] is sched.stages[-1]
    kinds = [r[0] for r in seq]
    assert kinds[-1] == "wgrad" and seq[-1][1].name == "s1_in"     # the dataset gets no dgrad


def test_schedule_rejects_mixed_spaces():
    a = Plan({"S_1": "101"}, (3,), (8, 8, 1), (4,), ((3, 3),), 8, 3)
    b = Plan({"S_1": "101"}, (3,), (8, 8, 1), (5,), ((3, 3),), 8, 3)
    with pytest.raises(ValueError):
        PopulationSchedule([a, b])
