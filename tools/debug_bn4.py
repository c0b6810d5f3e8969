"""BN step: HIP's ReLU-masked output gradient g of every layer (before the BN
backward) vs the fp64 reference d(bn_out)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np, torch
import torch.nn.functional as F
import test_hip_step_parity as T
from gentun_amd.models import cnn_engine as E
from gentun_amd.models.cnn_hip import HipPopJob
from gentun_amd.models.genome import ConvSpec
from gentun_amd.ops import cnn_kernels as K
gi = 2
genes = T.GENES[gi]
x, y, fold, plan = T._setup(genes)
dev = torch.device("cuda", 0)
cfg = E.TrainConfig(epochs=(1,), learning_rate=(1.0,), batch_size=32, dropout=0.0, loss="ce", dtype="fp32",
                    optimizer="sgd", momentum=0.9, use_graph=False, batch_norm=True)
job = HipPopJob(plan, x, y, [fold], cfg, dev, fold_ids=[0])
job.overlap = False
job.init_params()
w0 = T._hip_weights(job)
job.reset_optimizer(1.0)
job._new_epoch_order()
idx = job.epoch_idx[0, 0].cpu()
# manual step with snapshots of g
Lb = job.L
s = torch.cuda.current_stream().cuda_stream
K.check(Lb.gt_step_begin(job.state.data_ptr(), s), "sb")
job._run_fwd(s, job.fwd_ops)
K.check(Lb.gt_dense_fwd(job.dense_fwd_args, s), "")
K.check(Lb.gt_head(job.head_args, s), "")
K.check(Lb.gt_dense_dgrad(job.dense_dgrad_args, s), "")
K.check(Lb.gt_dense_wgrad_adam(job.dense_wgrad_args, s), "")
gsnap, dzsnap = {}, {}
for kind, a, L in job.bwd_ops:
    if kind == "wgrad":
        K.check(Lb.gt_conv_wgrad(a, s), "")
    elif kind == "conv":
        K.check(Lb.gt_conv_fwd(a, s), "")
    elif kind == "bn_bwd":
        gsnap[L.name] = job.grad[L.name][0].clone()
        K.check(Lb.gt_bn_bwd(a, s), "")
        dzsnap[L.name] = job.grad[L.name][0].clone()
    else:
        K.check(Lb.gt_pool_bwd_mask(*a, s), "")
torch.cuda.synchronize()
# reference with retained grads
xb = torch.from_numpy(np.asarray(x)[idx.numpy()]).permute(0, 3, 1, 2).double()
yb = torch.from_numpy(np.asarray(y)[idx.numpy()]).double()
P = {k: tuple(t.double().cpu().requires_grad_(True) for t in v) if isinstance(v, tuple) else v.double().cpu().requires_grad_(True) for k, v in w0.items()}
acts, outs, zs = {"input": xb}, {}, {}
for st in plan.steps:
    if isinstance(st, ConvSpec):
        inp = acts[st.inputs[0]]
        for e in st.inputs[1:]:
            inp = inp + acts[e]
        w, b, gm, bt = P[st.name]
        z = F.conv2d(inp, w, b, padding=(st.k[0] // 2, st.k[1] // 2))
        z.retain_grad(); zs[st.name] = z
        mean = z.mean((0, 2, 3), keepdim=True)
        var = ((z - mean) ** 2).mean((0, 2, 3), keepdim=True)
        o = (z - mean) / torch.sqrt(var + 1e-3) * gm.view(1, -1, 1, 1) + bt.view(1, -1, 1, 1)
        o.retain_grad(); outs[st.name] = o
        acts[st.name] = F.relu(o)
    else:
        acts[st.name] = F.max_pool2d(acts[st.srcs[0]], 2, 2)
feat = acts[plan.steps[-1].name].reshape(xb.shape[0], -1)
h = F.relu(feat @ P["W1"] + P["b1"])
logits = h @ P["W2"] + P["b2"]
per = -(yb * torch.log_softmax(logits, -1)).sum(-1)
per.mean().backward()
for L in job.layers:
    if L.name not in gsnap:
        continue
    C = L.cout
    g_hip = gsnap[L.name][..., :C].double().cpu()
    g_ref = outs[L.name].grad.permute(0, 2, 3, 1)
    mask_ref = (outs[L.name] > 0).permute(0, 2, 3, 1)
    dz_ref = zs[L.name].grad.permute(0, 2, 3, 1)
    err = (g_hip - g_ref)
    print("{:7s} g err {:.2e} (rel {:.2e}) where-unmasked-err {:.2e} chan-mean-err {:.2e} | dz rel {:.2e} | act>0 mismatch {}".format(
        L.name, err.abs().max().item(), err.abs().max().item() / g_ref.abs().max().item(),
        err[~mask_ref].abs().max().item() if (~mask_ref).any() else 0.0,
        err.mean((0, 1, 2)).abs().max().item(),
        T._rel(dzsnap[L.name][..., :C], dz_ref),
        int(((job.act[L.name][0][..., :C].cpu() > 0) != mask_ref).sum())))
