"""End-to-end parity of the composed HIP train step on DAG genomes (fp32).

One optimizer step of the population-batched executor (every kernel of the
step: gather, fused N-ary Add, conv fwd, pool, dense + head, loss gradient,
pool backward, DAG gradient fan-out with ReLU masks, conv dgrad / wgrad,
dense wgrad) is compared, gradient by gradient, with float64 autograd
through the reference network built directly from the decoded plan
(keras_models.py:97-118 semantics, gentun_amd/models/genome.py). SGD with
lr 1 and zero momentum state makes the optimizer's velocity buffer hold
exactly -grad. Then 50 Adam steps are compared with the torch fp32 oracle
executor started from the same weights on the same batches.

Genes: fan-out, isolated nodes and multiple sinks."""


import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

GENES = [{'S_1': '101', 'S_2': '0101110011'}, {'S_1': '111', 'S_2': '1111111111'},
         {'S_1': '010', 'S_2': '1001001001'}, {'S_1': '000', 'S_2': '0000000000'}]


def _setup(genes, n=240, ntrain=192):
    from gentun_amd.models.genome import make_plan
    from gentun_amd.utils.data import make_cifar_like
    x, y = make_cifar_like(n=n, seed=4)
    idx = np.arange(n)
    fold = (idx[:ntrain], idx[ntrain:])
    plan = make_plan(genes, (3, 5), (32, 32, 3), (20, 50), ((5, 5), (5, 5)), 500, 10)
    return x, y, fold, plan


def _hip_weights(job):
    """{conv name: (w OIHW, b)}, W1 [F_nchw, U], b1, W2, b2 of group 0 (fp32 masters)."""
    out = {}
    for L in job.layers:
        w = L.w[0][0][:L.cout, :, :, :L.cin].permute(0, 3, 1, 2)
        out[L.name] = (w.detach().clone(), L.b[0][0][:L.cout].detach().clone())
        if job.bn:
            out[L.name] += (L.gamma[0][0][:L.cout].detach().clone(), L.beta[0][0][:L.cout].detach().clone())
    hs, ws = job.final_hw
    cp, C, U = job.final_cp, job.plan.kernels_per_layer[-1], job.plan.dense_units
    W1 = job.views["W1"][0][0].view(hs, ws, cp, job.Up)[:, :, :C, :U]          # NHWC features
    W1 = W1.permute(2, 0, 1, 3).reshape(C * hs * ws, U)                          # -> NCHW flatten
    out["W1"] = W1.detach().clone()
    out["b1"] = job.views["b1"][0][0][:U].detach().clone()
    out["W2"] = job.views["W2"][0][0][:U].detach().clone()
    out["b2"] = job.views["b2"][0][0].detach().clone()
    return out


def _hip_grads(job):
    """-velocity of the SGD step = gradient, in the same layout as _hip_weights."""
    g = {}
    for L in job.layers:
        m = L.w[1][0][:L.cout, :, :, :L.cin].permute(0, 3, 1, 2)
        g[L.name] = (-m.detach().clone(), -L.b[1][0][:L.cout].detach().clone())
        if job.bn:
            g[L.name] += (-L.gamma[1][0][:L.cout].detach().clone(), -L.beta[1][0][:L.cout].detach().clone())
    hs, ws = job.final_hw
    cp, C, U = job.final_cp, job.plan.kernels_per_layer[-1], job.plan.dense_units
    M1 = job.views["W1"][1][0].view(hs, ws, cp, job.Up)[:, :, :C, :U].permute(2, 0, 1, 3).reshape(C * hs * ws, U)
    g["W1"] = -M1.detach().clone()
    g["b1"] = -job.views["b1"][1][0][:U].detach().clone()
    g["W2"] = -job.views["W2"][1][0][:U].detach().clone()
    g["b2"] = -job.views["b2"][1][0].detach().clone()
    return g


def _reference_grads(plan, weights, xb, yb, loss, dtype=torch.float64, bn_eps=None, masks=None):
    """autograd through the plan (NCHW) on the CPU, mean loss over the batch;
    ``bn_eps``: conv -> BatchNorm (batch statistics) -> ReLU; ``masks``:
    {layer: NCHW bool} ReLU decisions to use instead of the reference's own."""
    from gentun_amd.models.genome import ConvSpec
    P = {k: (tuple(t.to(dtype).cpu().requires_grad_(True) for t in v) if isinstance(v, tuple)
             else v.to(dtype).cpu().requires_grad_(True)) for k, v in weights.items()}
    yb = yb.to(dtype)
    acts = {"input": xb.to(dtype)}
    for st in plan.steps:
        if isinstance(st, ConvSpec):
            inp = acts[st.inputs[0]]
            for extra in st.inputs[1:]:
                inp = inp + acts[extra]
            w, b = P[st.name][:2]
            z = F.conv2d(inp, w, b, padding=(st.k[0] // 2, st.k[1] // 2))
            if bn_eps is not None:
                gm, bt = P[st.name][2:]
                mean = z.mean((0, 2, 3), keepdim=True)
                var = ((z - mean) ** 2).mean((0, 2, 3), keepdim=True)
                z = (z - mean) / torch.sqrt(var + bn_eps) * gm.view(1, -1, 1, 1) + bt.view(1, -1, 1, 1)
            acts[st.name] = z * masks[st.name].to(dtype) if masks is not None else F.relu(z)
        else:
            acts[st.name] = F.max_pool2d(acts[st.srcs[0]], 2, 2)
    feat = acts[plan.steps[-1].name].reshape(xb.shape[0], -1)
    h = F.relu(feat @ P["W1"] + P["b1"])
    logits = h @ P["W2"] + P["b2"]
    p = torch.softmax(logits, -1)
    if loss == "bce_compat":
        pc = p.clamp(1e-7, 1 - 1e-7)
        per = -(yb * torch.log(pc) + (1 - yb) * torch.log(1 - pc)).mean(-1)
    else:
        per = -(yb * torch.log(p)).sum(-1)
    per.mean().backward()
    out = {}
    for k, v in P.items():
        out[k] = tuple(t.grad for t in v) if isinstance(v, tuple) else v.grad
    return out


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


@pytest.mark.parametrize("loss", ["ce", "bce_compat"])
@pytest.mark.parametrize("gi", range(len(GENES)))
def test_one_step_gradients_match_fp64_autograd(gi, loss):
    _one_step_parity(gi, loss, bn=False)


@pytest.mark.parametrize("gi", range(len(GENES)))
def test_one_step_gradients_with_batchnorm(gi):
    """The optional BatchNorm (conv -> BN -> ReLU, cnn_bn.hip) inside the
    composed step: every conv / gamma / beta / dense gradient vs fp64."""
    _one_step_parity(gi, "ce", bn=True)


def _one_step_parity(gi, loss, bn):
    from gentun_amd.models import cnn_engine as E
    from gentun_amd.models.cnn_hip import HipPopJob
    genes = GENES[gi]
    x, y, fold, plan = _setup(genes)
    dev = torch.device("cuda", 0)
    cfg = E.TrainConfig(epochs=(1,), learning_rate=(1.0,), batch_size=32, dropout=0.0, loss=loss, dtype="fp32",
                        optimizer="sgd", momentum=0.9, use_graph=False, batch_norm=bn)
    job = HipPopJob(plan, x, y, [fold], cfg, dev, fold_ids=[0])
    job.init_params()
    w0 = _hip_weights(job)
    job.reset_optimizer(1.0)
    job._new_epoch_order()
    idx = job.epoch_idx[0, 0].cpu()
    job.train_step()
    torch.cuda.synchronize()
    got = _hip_grads(job)
    xb = torch.from_numpy(np.asarray(x)[idx.numpy()]).permute(0, 3, 1, 2)
    yb = torch.from_numpy(np.asarray(y)[idx.numpy()]).double()
    eps = cfg.bn_eps if bn else None
    # BatchNorm rescales every pre-activation to O(1): a node's BN output lands
    # within fp32 rounding of 0 at a few positions, and a ReLU decision that
    # flips there moves that layer's gradient by O(1e-2). With BN the fp64
    # reference therefore takes the HIP forward's ReLU decisions (the
    # arithmetic is compared, not the tie-breaking).
    # Without BN the same happens at genuine near-ties (the all-ones genome: one
    # flipped decision moves s2_n1.w by 1.6e-2, while torch fp32 flips others
    # there and on genome 2 at 2.3e-2): the strict check below is on the HIP
    # forward's ReLU decisions; the free-running comparison only has to stay
    # within what one flipped decision does.
    hip_masks = {L.name: (job.act[L.name][0][..., :L.cout] > 0).permute(0, 3, 1, 2).cpu() for L in job.layers}
    masks = hip_masks if bn else None
    ref = _reference_grads(plan, w0, xb, yb, loss, bn_eps=eps, masks=masks)
    r32 = _reference_grads(plan, w0, xb, yb, loss, torch.float32, bn_eps=eps, masks=masks)    # torch fp32, same inputs
    if not bn:
        ref_m = _reference_grads(plan, w0, xb, yb, loss, masks=hip_masks)
        r32_m = _reference_grads(plan, w0, xb, yb, loss, torch.float32, masks=hip_masks)

    def errs(g, ref=ref):
        out = {}
        for k, r in ref.items():
            if isinstance(r, tuple):
                out[k + ".w"] = _rel(g[k][0], r[0])
                if r[1].abs().max() > 0 and not bn:         # with BN the conv bias gradient is 0 (+ rounding)
                    out[k + ".b"] = _rel(g[k][1], r[1])
                if bn:
                    out[k + ".gamma"] = _rel(g[k][2], r[2])
                    out[k + ".beta"] = _rel(g[k][3], r[3])
            else:
                out[k] = _rel(g[k], r)
        return out

    worst, worst32 = errs(got), errs(r32)
    kmax = max(worst, key=worst.get)
    print("[parity] genes {} loss {} bn {}: worst rel grad err HIP {:.2e} ({}); torch fp32 there {:.2e}, worst {:.2e}"
          .format(genes, loss, bn, worst[kmax], kmax, worst32[kmax], max(worst32.values())))
    assert set(k.split(".")[0] for k in worst) >= set(L.name for L in job.layers)
    if not bn:
        # free-running: fp32-level, or one flipped near-tie ReLU decision away
        for k, e in worst.items():
            assert e < max(2e-4, 4 * worst32[k], 3e-2), (k, e, worst32[k])
        worst, worst32 = errs(got, ref_m), errs(r32_m, ref_m)
        kmax = max(worst, key=worst.get)
        print("[parity]   on the HIP ReLU decisions: worst rel grad err HIP {:.2e} ({}); torch fp32 there {:.2e}"
              .format(worst[kmax], kmax, worst32[kmax]))
    # fp32-level: within 2e-4 of the fp64 gradient, or no further than torch's
    # own fp32 CPU autograd (max-pool decisions near ties flip in fp32)
    for k, e in worst.items():
        assert e < max(2e-4, 4 * worst32[k]), (k, e, worst32[k])
    # the update itself: p1 = p0 + v = p0 - g
    w1 = _hip_weights(job)
    for k, r in ref.items():
        if isinstance(r, tuple):
            assert torch.allclose(w1[k][0], w0[k][0] - got[k][0], rtol=0, atol=1e-6)


def _copy_into_torch_job(tj, w):
    with torch.no_grad():
        off = 0
        for name, shape, _, _ in tj.shapes:
            n = int(np.prod(shape))
            tj.flat[off:off + n].copy_(_named(w, name).reshape(-1).to(tj.flat.device))
            off += n


def _named(w, name):
    base, kind = name.rsplit(".", 1)
    if base in ("dense1", "dense2"):
        return w[("W" if kind == "w" else "b") + base[-1]]
    return w[base][{"w": 0, "b": 1, "gamma": 2, "beta": 3}[kind]]


def _torch_weights(tj, like):
    out, off = {}, 0
    for name, shape, _, _ in tj.shapes:
        n = int(np.prod(shape))
        out[name] = tj.flat[off:off + n].detach().view(_named(like, name).shape).cpu()
        off += n
    return out


@pytest.mark.parametrize("gi,bn", [(0, False), (1, False), (0, True)])
def test_fifty_steps_track_the_torch_fp32_oracle(gi, bn):
    """50 SGD-momentum steps (no dropout) from identical weights on identical
    batches. Two valid fp32 executions of a 50-step non-convex training run
    drift apart chaotically (ReLU / max-pool decisions near ties flip), so the
    yardstick is torch itself: the HIP fp32 run must stay as close to the
    torch fp32 GPU run as torch's CPU fp32 run of the same steps is."""
    from gentun_amd.models import cnn_engine as E
    from gentun_amd.models.cnn_hip import HipPopJob
    genes = GENES[gi]
    x, y, fold, plan = _setup(genes, n=2000, ntrain=1600)
    dev = torch.device("cuda", 0)
    cfg = E.TrainConfig(epochs=(1,), learning_rate=(0.003,), batch_size=32, dropout=0.0, loss="ce", dtype="fp32",
                        use_graph=False, optimizer="sgd", momentum=0.9, batch_norm=bn)
    hip = HipPopJob(plan, x, y, [fold], cfg, dev, fold_ids=[0])
    tg = E.TorchFoldJob(plan, x, y, [fold], cfg, dev, fold_ids=[0])
    tc = E.TorchFoldJob(plan, x, y, [fold], cfg, torch.device("cpu"), fold_ids=[0])
    hip.init_params()
    w = _hip_weights(hip)
    _copy_into_torch_job(tg, w)
    _copy_into_torch_job(tc, w)
    for job in (hip, tg, tc):
        job.reset_optimizer(0.003)
        job._new_epoch_order()
    tc.epoch_idx.copy_(hip.epoch_idx.cpu())         # the CPU generator draws another order: use the same batches
    assert torch.equal(hip.epoch_idx.cpu(), tg.epoch_idx.cpu())
    for job in (hip, tg, tc):
        for _ in range(job.steps_per_epoch):
            job.train_step()
    torch.cuda.synchronize()
    wh = _hip_weights(hip)
    wg, wc = _torch_weights(tg, w), _torch_weights(tc, w)
    d_hip, d_cpu = {}, {}
    for name in wg:
        if bn and name.endswith(".b") and not name.startswith("dense"):
            continue             # conv bias under BN: zero gradient, a free direction that only drifts with rounding
        scale = max(wg[name].abs().max().item(), 1e-12)
        d_hip[name] = (_named(wh, name).cpu() - wg[name]).abs().max().item() / scale
        d_cpu[name] = (wc[name] - wg[name]).abs().max().item() / scale
    vh, vg, vc = (float(j.evaluate()[0].sum()) / 400 for j in (hip, tg, tc))
    k = max(d_hip, key=d_hip.get)
    print("[parity] 50 SGD steps genes {} bn {}: max |w_hip - w_torchGPU| / max|w| = {:.2e} ({}); torch CPU vs GPU: {:.2e} "
          "(max {:.2e}); val loss hip {:.5f} torchGPU {:.5f} torchCPU {:.5f}".format(
              genes, bn, d_hip[k], k, d_cpu[k], max(d_cpu.values()), vh, vg, vc))
    assert max(d_hip.values()) <= 3 * max(d_cpu.values()) + 1e-5
    if not bn:       # with BN the evaluation uses running statistics that, after 50 steps, are still
        assert abs(vh - vg) <= max(3 * abs(vc - vg), 0.1)      # 60% their (0, 1) start: no stable yardstick
