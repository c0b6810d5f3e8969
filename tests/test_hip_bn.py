"""BatchNorm kernels (csrc/hip/cnn_bn.hip) against torch.nn.BatchNorm2d:
forward (batch and running statistics, fused ReLU), running-stat update,
backward (dz, dgamma, dbeta), population group tables, the Keras short
batch; and the deep S=(3,4,5) space learning at the reference lr 1e-3. The
composed step with BatchNorm is checked gradient by gradient against fp64
autograd and over 50 steps against torch in tests/test_hip_step_parity.py."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _args(K, z, y, gamma, beta, stat, run, part, gg, gb, gtab, valid, st, B, HW, Cp, nchunk, chunk, train, prec):
    a = K.BnArgs()
    a.z, a.y, a.gamma, a.beta = z.data_ptr(), y.data_ptr(), gamma.data_ptr(), beta.data_ptr()
    a.stat, a.run, a.part, a.ggamma, a.gbeta = stat.data_ptr(), run.data_ptr(), part.data_ptr(), gg.data_ptr(), \
        gb.data_ptr()
    a.gtab, a.valid, a.st = gtab.data_ptr(), valid.data_ptr() if valid is not None else 0, st.data_ptr()
    a.ngroups, a.G, a.B, a.HW, a.Cp = gtab.shape[0], z.shape[0], B, HW, Cp
    a.nchunk, a.chunk_px = nchunk, chunk
    a.momentum, a.eps, a.train, a.prec = 0.99, 1e-3, train, prec
    return a


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


@pytest.mark.parametrize("prec", [1, 0])
@pytest.mark.parametrize("shape", [(32, 16, 16, 24, 20), (32, 8, 8, 104, 100), (8, 32, 32, 8, 3),
                                   (32, 8, 8, 256, 250), (32, 16, 16, 128, 120)])
def test_bn_kernels_match_batchnorm2d(prec, shape):
    from gentun_amd.ops import cnn_kernels as K
    L = K.lib()
    dev = torch.device("cuda", 0)
    B, H, W, Cp, C = shape
    Q, HW = 3, H * W
    groups = [2, 0]                                   # group table: a subset, out of order
    nval = [B, B, max(1, B - 5)]                      # group 2: a short batch
    adt = torch.float32 if prec else torch.bfloat16
    torch.manual_seed(0)
    zf = torch.zeros(Q, B, H, W, Cp)
    zf[..., :C] = torch.randn(Q, B, H, W, C) * 2 + 3
    z = zf.to(dev, adt)
    zf = z.float().cpu()                              # what the kernel sees
    gamma = torch.zeros(Q, Cp)
    beta = torch.zeros(Q, Cp)
    gamma[:, :C] = torch.rand(Q, C) + 0.5
    beta[:, :C] = torch.randn(Q, C) * 0.5
    run = torch.stack([torch.randn(Q, Cp) * 0.1, torch.rand(Q, Cp) + 0.5])
    chunk = K.bn_chunk_px(H, W, Cp)                  # the executor's per-shape chunk
    nchunk = -(-(B * HW) // chunk)
    y = torch.zeros_like(z)
    stat = torch.zeros(Q, 2, Cp, device=dev)
    part = torch.zeros(Q, nchunk, 2, Cp, device=dev)
    gg = torch.zeros(Q, Cp, device=dev)
    gb = torch.zeros(Q, Cp, device=dev)
    run_d = run.clone().to(dev)
    gtab = torch.tensor([[g, 0, 0, 0] for g in groups], dtype=torch.int32, device=dev)
    valid = torch.tensor([nval], dtype=torch.int32, device=dev)     # [steps=1][Q]
    st = torch.zeros(8, dtype=torch.int32, device=dev)
    gd, bd = gamma.to(dev), beta.to(dev)
    s = torch.cuda.current_stream().cuda_stream
    a = _args(K, z, y, gd, bd, stat, run_d, part, gg, gb, gtab, valid, st, B, HW, Cp, nchunk, chunk, 1, prec)
    K.check(L.gt_bn_fwd(a, s), "bn_fwd")
    # backward: a ReLU-masked gradient of the BN output, written in place
    gy = torch.randn(Q, B, H, W, Cp) * (torch.rand(Q, B, H, W, Cp) > 0.3)
    gy[..., C:] = 0
    gbuf = gy.to(dev, adt)
    gy = gbuf.float().cpu()
    a.y = gbuf.data_ptr()
    K.check(L.gt_bn_bwd(a, s), "bn_bwd")
    torch.cuda.synchronize()
    tol = 1e-4 if prec else 2e-2
    for g in groups:
        nv = nval[g]
        x = zf[g, :nv, ..., :C].permute(0, 3, 1, 2).double().requires_grad_(True)
        m = torch.nn.BatchNorm2d(C, eps=1e-3, momentum=0.01).double()
        with torch.no_grad():
            m.weight.copy_(gamma[g, :C])
            m.bias.copy_(beta[g, :C])
            m.running_mean.copy_(run[0, g, :C])
            m.running_var.copy_(run[1, g, :C])
        out = m(x)
        yref = torch.relu(out).permute(0, 2, 3, 1)
        assert _rel(y[g, :nv, ..., :C].float(), yref) < tol, "forward"
        assert float(y[g, ..., C:].float().abs().max()) == 0.0          # padding channels stay 0
        assert _rel(run_d[0, g, :C], m.running_mean) < 1e-5
        assert _rel(run_d[1, g, :C], m.running_var) < 1e-5
        out.backward(gy[g, :nv, ..., :C].permute(0, 3, 1, 2).double())
        dz = gbuf[g].float().cpu()
        assert _rel(dz[:nv, ..., :C], x.grad.permute(0, 2, 3, 1)) < tol, "dz"
        if nv < B:
            assert float(dz[nv:].abs().max()) == 0.0                    # padding rows: no gradient
        assert _rel(gg[g, :C], m.weight.grad) < tol, "dgamma"
        assert _rel(gb[g, :C], m.bias.grad) < tol, "dbeta"
    # group 1 is not in the table: untouched
    assert float(y[1].float().abs().max()) == 0.0
    # evaluation: running statistics
    ye = torch.zeros_like(z)
    a.y, a.train = ye.data_ptr(), 0
    K.check(L.gt_bn_fwd(a, s), "bn_fwd(eval)")
    torch.cuda.synchronize()
    for g in groups:
        m = torch.nn.BatchNorm2d(C, eps=1e-3).double().eval()
        with torch.no_grad():
            m.weight.copy_(gamma[g, :C])
            m.bias.copy_(beta[g, :C])
            m.running_mean.copy_(run_d[0, g, :C].cpu())
            m.running_var.copy_(run_d[1, g, :C].cpu())
        ref = torch.relu(m(zf[g, ..., :C].permute(0, 3, 1, 2).double())).permute(0, 2, 3, 1)
        assert _rel(ye[g, ..., :C].float(), ref) < tol, "eval forward"


def test_deep_space_with_batchnorm_learns_at_reference_lr():
    """BASELINE cfg 4 (S=(3,4,5), kernels (20,50,100)) at lr 1e-3: without
    BatchNorm the dense DAG genomes stay at chance (profiles/deep_hip_vs_torch.log);
    with it they learn."""
    from gentun_amd.models import cnn_engine as E
    from gentun_amd.models.genome import make_plan
    from gentun_amd.utils.data import make_cifar_like, stratified_kfold
    dev = torch.device("cuda", 0)
    x, y = make_cifar_like(n=3000, seed=0)
    folds = stratified_kfold(np.argmax(y, 1), 3, seed=0)
    genes = {'S_1': '111', 'S_2': '111111', 'S_3': '1111111111'}
    plan = make_plan(genes, (3, 4, 5), (32, 32, 3), (20, 50, 100), ((5, 5),) * 3, 500, 10)
    # 6 epochs of 63 steps: the running statistics (Keras momentum 0.99) the
    # evaluation uses have forgotten their (0, 1) start
    cfg = E.TrainConfig(epochs=(6,), learning_rate=(1e-3,), batch_size=32, dtype="fp32", loss="ce",
                        batch_norm=True, reset="all")
    r = E.make_job("hip", plan, x, y, folds, cfg, dev).launch().finish()
    print("[bn] deep all-ones genome, lr 1e-3, BN: cat acc", r["categorical_accuracy"])
    assert min(r["categorical_accuracy"]) > 0.3          # chance 0.1
