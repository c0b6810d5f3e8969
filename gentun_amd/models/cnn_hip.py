"""HIP executor of the fold-batched Genetic-CNN train step (MI355X path).

Compiles a decoded :class:`~gentun_amd.models.genome.Plan` into a fixed
sequence of hand-written gfx950 kernel launches (csrc/hip/cnn_conv.hip,
csrc/hip/cnn_dense.hip) over buffers allocated once per job:

  step_begin -> conv_fwd x L (first one gathers the batch from the
  device-resident dataset) / pool_fwd -> dense_fwd (+ReLU+dropout) -> head
  (softmax + loss grad + dW2/db2/db1) -> dense_dgrad -> dense_wgrad_adam
  (W1 gradient consumed in registers by Adam) -> reverse plan: pool_bwd,
  conv_wgrad (split-K partials), conv dgrad (= conv_fwd with flipped weights,
  ReLU mask and DAG fan-out accumulation fused) -> adam_segments.

Layouts: activations NHWC bf16 ``[G][B][H][W][Cp]`` with Cp = C rounded up to
8; fp32 master weights in padded layouts whose padding is zero and stays
zero (zero inputs produce zero gradients); bf16 weight copies written by the
optimizer for the next step. Fold index ``G`` is the outermost dimension of
everything, so one launch trains all folds of the candidate.
"""

import math

import numpy as np
import torch

from ..ops import cnn_kernels as K
from ..utils import rng as _rng
from .cnn_engine import FoldJob
from .genome import ConvSpec


def pad8(c):
    return (c + 7) // 8 * 8


def round_up(x, m):
    return (x + m - 1) // m * m


class _Layer(object):
    pass


class HipFoldJob(FoldJob):
    layout = "nhwc8"

    def __init__(self, *a, **kw):
        super(HipFoldJob, self).__init__(*a, **kw)
        if self.device.type != "cuda":
            raise RuntimeError("the HIP backend needs a GPU device")
        self.L = K.lib()
        if self.cfg.dtype != "bf16":
            raise ValueError("HIP backend computes in bf16 MFMA with fp32 master weights (dtype='bf16')")
        plan, G, B, dev = self.plan, self.G, self.B, self.device
        h0, w0, c0 = plan.input_shape
        if self.data.x.shape[-1] != pad8(c0):
            raise ValueError("dataset channels do not match the plan")
        self.classes = plan.classes
        if plan.classes > 16:
            raise ValueError("HIP head kernel supports at most 16 classes")
        if B > 64:
            raise ValueError("HIP head kernel supports batch_size <= 64")
        # ---- activations -----------------------------------------------------
        self.shapes = {"input": (h0, w0, pad8(c0))}
        self.layers = []
        for st in plan.steps:
            hs, ws = plan.stage_hw(st.stage)
            if isinstance(st, ConvSpec):
                L = _Layer()
                L.spec = st
                L.H, L.W = hs, ws
                L.cin, L.cout = st.cin, st.cout
                L.cinp, L.coutp = pad8(st.cin), pad8(st.cout)
                L.KH, L.KW = st.k
                L.Kdim = L.KH * L.KW * L.cinp
                L.TH = K.conv_tile_rows(L.H, L.W)
                npix = B * L.H * L.W
                L.pps, L.S = K.wgrad_split(npix, L.Kdim, L.coutp, G)
                self.shapes[st.name] = (L.H, L.W, L.coutp)
                self.layers.append(L)
            else:
                src = st.srcs[0]
                hh, ww, cc = self.shapes[src]
                self.shapes[st.name] = (hh // 2, ww // 2, cc)
        last = plan.steps[-1].name
        hs, ws, cp = self.shapes[last]
        self.last = last
        self.Fp = hs * ws * cp
        self.Up = round_up(plan.dense_units, 64)
        self.act = {}
        self.grad = {}
        for name, (hh, ww, cc) in self.shapes.items():
            if name == "input":
                continue
            self.act[name] = torch.zeros((G, B, hh, ww, cc), dtype=torch.bfloat16, device=dev)
            self.grad[name] = torch.zeros((G, B, hh, ww, cc), dtype=torch.bfloat16, device=dev)
        self.hdrop = torch.zeros((G, B, self.Up), dtype=torch.bfloat16, device=dev)
        self.dH = torch.zeros((G, B, self.Up), dtype=torch.float32, device=dev)
        self.dz_head = torch.zeros((G, B, plan.classes), dtype=torch.float32, device=dev)
        self.plog = torch.zeros((G, self.Up // 16, B, plan.classes), dtype=torch.float32, device=dev)
        # ---- parameters (flat fp32 master + Adam moments) --------------------
        segs = []
        for L in self.layers:
            segs.append(("w", L, (G, L.coutp, L.KH, L.KW, L.cinp)))
            segs.append(("b", L, (G, L.coutp)))
        segs.append(("W1", None, (G, self.Fp, self.Up)))
        segs.append(("b1", None, (G, self.Up)))
        segs.append(("W2", None, (G, self.Up, self.classes)))
        segs.append(("b2", None, (G, self.classes)))
        total = sum(int(np.prod(s)) for _, _, s in segs)
        self.flat = torch.zeros(total, dtype=torch.float32, device=dev)
        self.m = torch.zeros_like(self.flat)
        self.v = torch.zeros_like(self.flat)
        off = 0
        self.views = {}
        for kind, L, shape in segs:
            n = int(np.prod(shape))
            view = (self.flat[off:off + n].view(shape), self.m[off:off + n].view(shape),
                    self.v[off:off + n].view(shape))
            if L is not None:
                setattr(L, kind, view)
            else:
                self.views[kind] = view
            off += n
        for L in self.layers:
            L.w_bf = torch.zeros((G, L.coutp, L.KH, L.KW, L.cinp), dtype=torch.bfloat16, device=dev)
            L.wT_bf = torch.zeros((G, L.cinp, L.KH, L.KW, L.coutp), dtype=torch.bfloat16, device=dev)
            L.part_w = torch.zeros((L.S, G, L.coutp, L.Kdim), dtype=torch.float32, device=dev)  # split-K partials
            L.part_b = torch.zeros((L.S, G, L.coutp), dtype=torch.float32, device=dev)
        self.w1t_bf = torch.zeros((G, self.Up, self.Fp), dtype=torch.bfloat16, device=dev)
        self.gW2 = torch.zeros((G, self.Up, self.classes), dtype=torch.float32, device=dev)
        self.gb2 = torch.zeros((G, self.classes), dtype=torch.float32, device=dev)
        self.gb1 = torch.zeros((G, self.Up), dtype=torch.float32, device=dev)
        # ---- step state ------------------------------------------------------
        self.state = torch.zeros(8, dtype=torch.int32, device=dev)
        self.state_f = self.state.view(torch.float32)
        self.step_ctr = self.state[0:1]
        self.eval_state = torch.zeros(8, dtype=torch.int32, device=dev)
        self.fold_ids_t = torch.tensor(self.fold_ids, dtype=torch.int32, device=dev)
        self.drop_seed = _rng.stable_hash(self.base_seed, "dropout") & 0xFFFFFFFF
        self._build_adam_table()
        self._build_args()

    # ------------------------------------------------------------------ setup
    def _build_adam_table(self):
        segs, blocks = [], []
        keep = []

        def add(p, m, v, g, S, gstride, bf=None, bfT=None, tdims=None):
            sg = K.AdamSeg()
            sg.p, sg.m, sg.v, sg.g = p.data_ptr(), m.data_ptr(), v.data_ptr(), g.data_ptr()
            sg.bf = bf.data_ptr() if bf is not None else 0
            sg.bfT = bfT.data_ptr() if bfT is not None else 0
            sg.n = p.numel()
            sg.gstride = gstride
            sg.S = S
            if tdims is not None:
                sg.tG, sg.tCo, sg.tKH, sg.tKW, sg.tCi = tdims
            idx = len(segs)
            segs.append(sg)
            for o in range(0, p.numel(), 256):
                blocks.append((idx, o))

        for L in self.layers:
            p, m, v = L.w
            add(p, m, v, L.part_w, L.S, L.part_w[0].numel(), bf=L.w_bf, bfT=L.wT_bf,
                tdims=(self.G, L.coutp, L.KH, L.KW, L.cinp))
            p, m, v = L.b
            add(p, m, v, L.part_b, L.S, L.part_b[0].numel())
        for name, g in (("b1", self.gb1), ("W2", self.gW2), ("b2", self.gb2)):
            p, m, v = self.views[name]
            add(p, m, v, g, 1, g.numel())
        arr = (K.AdamSeg * len(segs))(*segs)
        raw = bytes(memoryview(arr).cast("B"))
        self.adam_segs = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(self.device)
        self.adam_blocks = torch.tensor(np.asarray(blocks, np.int32).reshape(-1, 2), device=self.device)
        self.adam_nblocks = len(blocks)
        del keep

    def _conv_args(self, L, inputs, outs, acc_flags, w, bias, relu, mask=None, gather=None, st=None, Bn=None):
        a = K.ConvArgs()
        for i, t in enumerate(inputs):
            a.inp[i] = t.data_ptr()
        for i, t in enumerate(outs):
            a.out[i] = t.data_ptr()
        a.n_in, a.n_out, a.acc_flags, a.relu = len(inputs), len(outs), acc_flags, relu
        a.mask = mask.data_ptr() if mask is not None else 0
        a.gather = gather if gather is not None else 0
        a.st = st.data_ptr() if st is not None else self.state.data_ptr()
        a.w = w.data_ptr()
        a.bias = bias.data_ptr() if bias is not None else 0
        a.G, a.B, a.H, a.W = self.G, Bn or self.B, L.H, L.W
        return a

    def _build_args(self):
        """Pre-build every launch's argument struct (pointers are fixed)."""
        G, B = self.G, self.B
        data = self.data.x
        gather_train = self.epoch_idx.data_ptr()
        self.fwd_ops = []
        for st in self.plan.steps:
            if isinstance(st, ConvSpec):
                L = next(l for l in self.layers if l.spec is st)
                if st.inputs == ["input"]:
                    ins, gather = [data], gather_train
                else:
                    ins, gather = [self.act[n] for n in st.inputs], None
                a = self._conv_args(L, ins, [self.act[st.name]], 0, L.w_bf, L.b[0], 1, gather=gather)
                a.Cinp, a.Coutp, a.KH, a.KW, a.TH = L.cinp, L.coutp, L.KH, L.KW, L.TH
                self.fwd_ops.append(("conv", a, L))
            else:
                hh, ww, cc = self.shapes[st.srcs[0]]
                self.fwd_ops.append(("pool", (self.act[st.srcs[0]], self.act[st.name], G * B, hh, ww, cc), None))
        # head
        df = K.DenseFwdArgs()
        df.x, df.wt, df.bias, df.out = (self.act[self.last].data_ptr(), self.w1t_bf.data_ptr(),
                                        self.views["b1"][0].data_ptr(), self.hdrop.data_ptr())
        df.st, df.fold_ids = self.state.data_ptr(), self.fold_ids_t.data_ptr()
        df.G, df.B, df.Fp, df.Up = G, B, self.Fp, self.Up
        df.drop_p, df.train, df.seed = self.cfg.dropout, 1, self.drop_seed
        df.w2, df.plog, df.C = self.views["W2"][0].data_ptr(), self.plog.data_ptr(), self.classes
        self.dense_fwd_args = df
        hd = K.HeadArgs()
        hd.h, hd.w2, hd.b2 = self.hdrop.data_ptr(), self.views["W2"][0].data_ptr(), self.views["b2"][0].data_ptr()
        hd.labels, hd.gather, hd.st = self.data.labels.data_ptr(), gather_train, self.state.data_ptr()
        hd.dH, hd.gw2, hd.gb2, hd.gb1 = self.dH.data_ptr(), self.gW2.data_ptr(), self.gb2.data_ptr(), self.gb1.data_ptr()
        hd.eval_out = 0
        hd.dz = self.dz_head.data_ptr()
        hd.plog = self.plog.data_ptr()
        hd.G, hd.B, hd.Up, hd.C = G, B, self.Up, self.classes
        hd.loss_ce = 1 if self.cfg.loss == "ce" else 0
        hd.drop_scale = 1.0 / (1.0 - self.cfg.dropout) if self.cfg.dropout < 1 else 0.0
        hd.eval = 0
        self.head_args = hd
        dd = K.DenseDgradArgs()
        dd.dH, dd.w1, dd.dx = self.dH.data_ptr(), self.views["W1"][0].data_ptr(), self.grad[self.last].data_ptr()
        dd.G, dd.B, dd.Fp, dd.Up = G, B, self.Fp, self.Up
        self.dense_dgrad_args = dd
        dw = K.DenseWgradAdamArgs()
        p, m, v = self.views["W1"]
        dw.x, dw.dH, dw.p, dw.m, dw.v = self.act[self.last].data_ptr(), self.dH.data_ptr(), p.data_ptr(), \
            m.data_ptr(), v.data_ptr()
        dw.wt, dw.st = self.w1t_bf.data_ptr(), self.state.data_ptr()
        dw.G, dw.B, dw.Fp, dw.Up = G, B, self.Fp, self.Up
        self.dense_wgrad_args = dw
        # backward: the LAST writer of a ReLU layer's gradient (its first consumer
        # in forward order) applies the ReLU mask, so every later reader (wgrad,
        # dgrad) consumes dz = dy * (y > 0) directly
        first_consumer = {}
        for st in self.plan.steps:
            srcs = st.inputs if isinstance(st, ConvSpec) else st.srcs
            for n in srcs:
                first_consumer.setdefault(n, st.name)
        relu_out = {st.name for st in self.plan.steps if isinstance(st, ConvSpec)}
        self.bwd_ops = []
        written = set()
        for st in reversed(self.plan.steps):
            if isinstance(st, ConvSpec):
                L = next(l for l in self.layers if l.spec is st)
                wa = K.WgradArgs()
                first = st.inputs == ["input"]
                ins = [data] if first else [self.act[n] for n in st.inputs]
                for i, t in enumerate(ins):
                    wa.inp[i] = t.data_ptr()
                wa.n_in = len(ins)
                wa.gather = gather_train if first else 0
                wa.st = self.state.data_ptr()
                wa.dz = self.grad[st.name].data_ptr()
                wa.part_w, wa.part_b = L.part_w.data_ptr(), L.part_b.data_ptr()
                wa.G, wa.B, wa.H, wa.W = G, B, L.H, L.W
                wa.Cinp, wa.Coutp, wa.KH, wa.KW, wa.S, wa.pps = L.cinp, L.coutp, L.KH, L.KW, L.S, L.pps
                self.bwd_ops.append(("wgrad", wa, L))
                if not first:
                    outs = [self.grad[n] for n in st.inputs]
                    flags = 0
                    for i, n in enumerate(st.inputs):
                        if n in written:
                            flags |= 1 << i
                        written.add(n)
                    a = self._conv_args(L, [self.grad[st.name]], outs, flags, L.wT_bf, None, 0)
                    for i, n in enumerate(st.inputs):
                        if n in relu_out and first_consumer[n] == st.name:
                            a.out_mask[i] = self.act[n].data_ptr()
                    a.Cinp, a.Coutp, a.KH, a.KW, a.TH = L.coutp, L.cinp, L.KH, L.KW, L.TH
                    self.bwd_ops.append(("conv", a, L))
            else:
                src = st.srcs[0]
                if src in written:
                    raise RuntimeError("pool input with several consumers is not supported")
                written.add(src)
                hh, ww, cc = self.shapes[src]
                self.bwd_ops.append(("pool_bwd", (self.act[src], self.grad[st.name], self.grad[src],
                                                  G * B, hh, ww, cc, int(src in relu_out)), None))
        aa = K.AdamArgs()
        aa.segs, aa.blocks, aa.st = self.adam_segs.data_ptr(), self.adam_blocks.data_ptr(), self.state.data_ptr()
        self.adam_args = aa

    # -------------------------------------------------------------- protocol
    def _build_init_table(self):
        """Segment table of the one-launch Philox Glorot initialiser (K11):
        every conv kernel, W1 and W2 of every fold; biases stay zero."""
        G = self.G
        segs, blocks, seeds = [], [], []

        def add(t, d, r, fan_in, fan_out, name):
            assert t.is_contiguous() and t.numel() == G * int(np.prod(d))
            seeds.append([_rng.stable_hash(self._fold_seed(g), name) & 0x7FFFFFFFFFFFFFFF for g in range(G)])
            sg = K.InitSeg()
            sg.p = t.data_ptr()
            for i in range(4):
                sg.d[i], sg.r[i] = int(d[i]), int(r[i])
            sg.G, sg.tag = G, len(segs)
            sg.limit = math.sqrt(6.0 / (fan_in + fan_out))
            idx = len(segs)
            segs.append(sg)
            for o in range(0, t.numel(), 256):
                blocks.append((idx, o))

        for L in self.layers:
            add(L.w[0], (L.coutp, L.KH, L.KW, L.cinp), (L.cout, L.KH, L.KW, L.cin), L.cin * L.KH * L.KW,
                L.cout * L.KH * L.KW, L.spec.name + ".w")
        hs, ws, cp = self.shapes[self.last]
        add(self.views["W1"][0], (hs, ws, cp, self.Up), (hs, ws, self.plan.final_c, self.plan.dense_units),
            self.plan.flatten, self.plan.dense_units, "dense1.w")
        w2 = self.views["W2"][0]
        add(w2, (1, 1, w2.shape[1], w2.shape[2]), (1, 1, self.plan.dense_units, self.plan.classes),
            self.plan.dense_units, self.plan.classes, "dense2.w")
        self.init_seeds = torch.tensor(np.asarray(seeds, np.int64), device=self.device)
        for k, sg in enumerate(segs):
            sg.seeds = self.init_seeds[k].data_ptr()
        arr = (K.InitSeg * len(segs))(*segs)
        self.init_segs = torch.frombuffer(bytearray(bytes(memoryview(arr).cast("B"))), dtype=torch.uint8
                                          ).to(self.device)
        self.init_blocks = torch.tensor(np.asarray(blocks, np.int32).reshape(-1, 2), device=self.device)
        ia = K.InitArgs()
        ia.segs, ia.blocks = self.init_segs.data_ptr(), self.init_blocks.data_ptr()
        self.init_args = ia
        self.init_nblocks = len(blocks)

    def init_params(self):
        """Glorot-uniform kernels (Philox, keyed by fold id and tensor name),
        zero biases -- Keras defaults, re-drawn per fold."""
        if getattr(self, "init_args", None) is None:
            self._build_init_table()
        self.flat.zero_()
        K.check(K.lib().gt_glorot_init(self.init_args, self.init_nblocks, self._stream()), "glorot_init")
        self._refresh_copies()

    def _refresh_copies(self):
        for L in self.layers:
            w = L.w[0]
            L.w_bf.copy_(w)
            L.wT_bf.copy_(w.flip(2, 3).permute(0, 4, 2, 3, 1))
        self.w1t_bf.copy_(self.views["W1"][0].transpose(1, 2))

    def reset_optimizer(self, lr):
        self.m.zero_()
        self.v.zero_()
        self.state_f[2:3].zero_()
        self.state_f[3:4].fill_(float(lr))
        self.state[6:7].fill_(1 if self.cfg.optimizer == "sgd" else 0)     # StepState.opt
        self.state_f[7:8].fill_(float(self.cfg.momentum))                  # StepState.momentum

    def snapshot(self):
        return (self.flat.clone(), self.m.clone(), self.v.clone(), self.state.clone())

    def restore(self, snap):
        self.flat.copy_(snap[0])
        self.m.copy_(snap[1])
        self.v.copy_(snap[2])
        self.state.copy_(snap[3])
        self._refresh_copies()

    def _stream(self):
        return torch.cuda.current_stream(self.device).cuda_stream

    def _run_fwd(self, s, ops):
        L = self.L
        for kind, a, _ in ops:
            if kind == "conv":
                K.check(L.gt_conv_fwd(a, s), "conv_fwd")
            else:
                x, y, nb, hh, ww, cc = a
                K.check(L.gt_pool_fwd(x.data_ptr(), y.data_ptr(), nb, hh, ww, cc, s), "pool_fwd")

    def train_step(self):
        L, s = self.L, self._stream()
        K.check(L.gt_step_begin(self.state.data_ptr(), s), "step_begin")
        self._run_fwd(s, self.fwd_ops)
        K.check(L.gt_dense_fwd(self.dense_fwd_args, s), "dense_fwd")
        K.check(L.gt_head(self.head_args, s), "head")
        K.check(L.gt_dense_dgrad(self.dense_dgrad_args, s), "dense_dgrad")
        K.check(L.gt_dense_wgrad_adam(self.dense_wgrad_args, s), "dense_wgrad_adam")
        for kind, a, _ in self.bwd_ops:
            if kind == "wgrad":
                K.check(L.gt_conv_wgrad(a, s), "conv_wgrad")
            elif kind == "conv":
                K.check(L.gt_conv_fwd(a, s), "conv_dgrad")
            else:
                x, dy, dx, nb, hh, ww, cc, rm = a
                K.check(L.gt_pool_bwd(x.data_ptr(), dy.data_ptr(), dx.data_ptr(), nb, hh, ww, cc, rm, s),
                        "pool_bwd")
        K.check(L.gt_adam_segments(self.adam_args, self.adam_nblocks, s), "adam")

    def evaluate(self):
        """Forward the validation folds in batches of B (no dropout)."""
        G, B, dev = self.G, self.B, self.device
        maxv = self.val_mat.shape[1]
        nch = -(-maxv // B)
        idx = torch.zeros((G, nch * B), dtype=torch.int64, device=dev)
        mask = torch.zeros((G, nch * B), dtype=torch.float32, device=dev)
        idx[:, :maxv] = self.val_mat
        mask[:, :maxv] = self.val_mask
        table = idx.view(G, nch, B).permute(1, 0, 2).contiguous()        # [nch][G][B]
        out = torch.zeros((nch, G, B, 3), dtype=torch.float32, device=dev)
        self._eval_keep = (table, out)
        s = self._stream()
        L = self.L
        # eval copies of the forward argument structs: gather from the eval table, eval state
        ops = []
        for kind, a, Lr in self.fwd_ops:
            if kind == "conv":
                b = K.ConvArgs.from_buffer_copy(a)
                b.st = self.eval_state.data_ptr()
                ops.append((kind, b, Lr))
            else:
                ops.append((kind, a, Lr))
        df = K.DenseFwdArgs.from_buffer_copy(self.dense_fwd_args)
        df.train = 0
        hd = K.HeadArgs.from_buffer_copy(self.head_args)
        hd.eval, hd.st = 1, self.eval_state.data_ptr()
        for c in range(nch):
            gptr = table[c].data_ptr()
            for kind, b, _ in ops:
                if kind == "conv" and b.gather:
                    b.gather = gptr
            self._run_fwd(s, ops)
            K.check(L.gt_dense_fwd(df, s), "dense_fwd(eval)")
            hd.gather, hd.eval_out = gptr, out[c].data_ptr()
            K.check(L.gt_head(hd, s), "head(eval)")
        res = out.permute(1, 0, 2, 3).reshape(G, nch * B, 3) * mask[:, :, None]
        sums = res.sum(1)
        return sums[:, 0], sums[:, 1], sums[:, 2]
