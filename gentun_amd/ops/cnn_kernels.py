"""ctypes bindings of the Genetic-CNN HIP kernels (csrc/hip/cnn_*.hip).

Every launcher takes raw device pointers and the caller's current
``hipStream_t`` (``torch.cuda.current_stream().cuda_stream``), so launches
interleave with torch's own and are captured by HIP graphs.
"""

import ctypes as C
import os

from . import _lib

P = C.c_void_p
I = C.c_int


MAXSLOT = 8      # GT_MAXSLOT: input / output slots of one conv launch

# precision codes of the kernels (csrc/hip/cnn_args.h ``prec``): activations /
# gradients bf16 with bf16 MFMA, or fp32 with the exact 3-plane split MFMA
PREC = {"bf16": 0, "fp32": 1}
NPL = {"bf16": 1, "fp32": 3}     # bf16 weight planes per precision


class GroupRec(C.Structure):
    """One group (candidate x fold replica) of a population launch:
    ``in_mask`` bit k = input slot k is summed; ``out_mask`` bits 0-7 = output
    slots written, 8-15 = accumulate into them, 16-23 = apply that slot's
    ReLU mask (csrc/hip/cnn_conv.hip GroupRec)."""
    _fields_ = [("g", I), ("in_mask", I), ("out_mask", I), ("pad", I)]


class ConvArgs(C.Structure):
    _fields_ = [("inp", P * MAXSLOT), ("mask", P), ("gather", P), ("st", P), ("out", P * MAXSLOT),
                ("out_mask", P * MAXSLOT), ("w", P), ("bias", P), ("gtab", P),
                ("n_in", I), ("n_out", I), ("acc_flags", I), ("relu", I),
                ("G", I), ("B", I), ("H", I), ("W", I), ("Cinp", I), ("Coutp", I), ("KH", I), ("KW", I),
                ("TH", I), ("ngroups", I), ("xsum", P), ("dbg", I), ("epi_bf16", I), ("prec", I), ("wps", C.c_long),
                ("cbb", I), ("pool_y", P), ("pool_mask", P), ("unpool_x1", P), ("unpool_sel", P),
                ("cout_real", I), ("Hr", I), ("Wr", I), ("wino", I), ("wfrag", I)]


class WinoWSeg(C.Structure):
    """csrc/hip/cnn_conv_wino.hip WinoWSeg: one layer's Winograd weight transform (forward or the
    data gradient's flipped / transposed kernel)."""
    _fields_ = [("w", P), ("u", P), ("ups", C.c_long), ("Q", I), ("Cop", I), ("Cip", I), ("R", I), ("K", I),
                ("dgrad", I), ("pad", I)]


class WinoWArgs(C.Structure):
    _fields_ = [("segs", P), ("blocks", P)]


class FragSeg(C.Structure):
    """csrc/hip/cnn_conv_fast.hip FragSeg: one layer direction's fragment-major weight planes."""
    _fields_ = [("w", P), ("dst", P), ("order", P), ("ps", C.c_long), ("Q", I), ("Cop", I), ("Cip", I), ("KH", I),
                ("KW", I), ("NT", I), ("NKS", I), ("NCBIc", I), ("dgrad", I), ("npl", I)]


class FragArgs(C.Structure):
    _fields_ = [("segs", P), ("blocks", P)]


def frag_order(KH, KW, ncbi, W, prec):
    """Row-major chunk (kk * NCBI + cb) of every entry of a shape-specialised conv's reduction list, in the
    kernel's order (-1 past the list), and the k-step count."""
    nks = (KH * KW * ncbi + 3) // 4
    out = (C.c_int * (nks * 4))()
    lib().gt_conv_frag_order(KH, KW, ncbi, W, prec, out, nks * 4)
    return list(out), nks


class FragTransform(object):
    """One launch that rewrites the fragment-major weight planes (ConvArgs::wfrag) of several layers and
    directions from their fp32 masters -- after every optimizer step and after initialisation."""

    def __init__(self, specs, device):
        """``specs``: (master [Q][Cop][KH][KW][Cip] fp32, planes [npl][Q][NT*NKS*512] bf16, W, prec, dgrad)."""
        import numpy as np
        import torch
        segs, blocks, self._keep = [], [], []
        for master, planes, W, prec, dgrad in specs:
            Q, cop, KH, KW, cip = master.shape
            ncbi = (cop if dgrad else cip) // 8
            nt = -(-(cip if dgrad else cop) // 16)
            order, nks = frag_order(KH, KW, ncbi, W, prec)
            assert tuple(planes.shape) == (planes.shape[0], Q, nt * nks * 512) and planes.is_contiguous()
            ot = torch.tensor(order, dtype=torch.int32, device=device)
            self._keep.append(ot)
            sg = FragSeg()
            sg.w, sg.dst, sg.order, sg.ps = master.data_ptr(), planes.data_ptr(), ot.data_ptr(), planes[0].numel()
            sg.Q, sg.Cop, sg.Cip, sg.KH, sg.KW = Q, cop, cip, KH, KW
            sg.NT, sg.NKS, sg.NCBIc, sg.dgrad, sg.npl = nt, nks, ncbi, 1 if dgrad else 0, planes.shape[0]
            n = Q * nt * nks * 64
            blocks.extend((len(segs), o) for o in range(0, n, 256))
            segs.append(sg)
        arr = (FragSeg * max(1, len(segs)))(*segs)
        self.segs_t = torch.frombuffer(bytearray(bytes(memoryview(arr).cast("B"))), dtype=torch.uint8).to(device)
        self.blocks_t = torch.tensor(np.asarray(blocks, np.int32).reshape(-1, 2), device=device)
        self.args = FragArgs()
        self.args.segs, self.args.blocks = self.segs_t.data_ptr(), self.blocks_t.data_ptr()
        self.nblocks = len(blocks)

    def run(self, stream):
        if self.nblocks:
            check(lib().gt_conv_wfrag(C.addressof(self.args), self.nblocks, stream), "conv_wfrag")


def frag_planes(master, W, prec=1, dgrad=False):
    """Fragment-major planes of ``master`` (tests / one-off use): [npl][Q][NT * NKS * 512] bf16."""
    import torch
    Q, cop, KH, KW, cip = master.shape
    nt = -(-(cip if dgrad else cop) // 16)
    _, nks = frag_order(KH, KW, (cop if dgrad else cip) // 8, W, prec)
    planes = torch.zeros((3 if prec else 1, Q, nt * nks * 512), dtype=torch.bfloat16, device=master.device)
    tr = FragTransform([(master.contiguous(), planes, W, prec, dgrad)], master.device)
    tr.run(torch.cuda.current_stream(master.device).cuda_stream)
    return planes


def wino_dims(cinp, coutp):
    """(rows, columns) of a layer's transformed weight planes [3][Q][16][rows][columns]: output
    channels padded to 16 (one MFMA row tile), input channels to 32 (one k-step)."""
    return -(-coutp // 16) * 16, -(-cinp // 32) * 32


class WgradArgs(C.Structure):
    _fields_ = [("inp", P * MAXSLOT), ("gather", P), ("st", P), ("dz", P), ("part_w", P),
                ("part_b", P), ("gtab", P), ("n_in", I), ("G", I), ("B", I), ("H", I), ("W", I), ("Cinp", I),
                ("Coutp", I), ("KH", I), ("KW", I), ("S", I), ("pps", I), ("ngroups", I), ("prec", I),
                ("cout_real", I)]


class DenseFwdArgs(C.Structure):
    _fields_ = [("x", P), ("wt", P), ("bias", P), ("out", P), ("w2", P), ("plog", P), ("st", P), ("fold_ids", P),
                ("seeds", P), ("G", I), ("B", I), ("Fp", I), ("Up", I), ("drop_p", C.c_float), ("train", I),
                ("seed", C.c_uint), ("C", I), ("prec", I), ("wps", C.c_long), ("row_off", I),
                ("w1", P), ("part", P), ("cnt", P), ("ks", I)]


class HeadArgs(C.Structure):
    _fields_ = [("h", P), ("w2", P), ("b2", P), ("labels", P), ("gather", P), ("st", P), ("dH", P),
                ("gw2", P), ("gb2", P), ("gb1", P), ("eval_out", P), ("dz", P), ("plog", P),
                ("G", I), ("B", I), ("Up", I), ("C", I), ("loss_ce", I), ("drop_scale", C.c_float), ("eval", I),
                ("prec", I), ("valid", P), ("valid_norm", P), ("dHp", P)]


class DenseDgradArgs(C.Structure):
    _fields_ = [("dH", P), ("wt", P), ("dx", P), ("G", I), ("B", I), ("Fp", I), ("Up", I), ("prec", I),
                ("wps", C.c_long), ("unpool_mask", P), ("unpool_x0", P), ("unpool_x1", P), ("unpool_sel", P),
                ("Hs", I), ("Ws", I), ("Cp", I), ("w1", P), ("dHp", P)]


class DenseWgradAdamArgs(C.Structure):
    _fields_ = [("x", P), ("dH", P), ("p", P), ("m", P), ("v", P), ("wt", P), ("st", P),
                ("G", I), ("B", I), ("Fp", I), ("Up", I), ("Cp", I), ("Cr", I), ("Ur", I), ("prec", I),
                ("wps", C.c_long), ("gbuf", P), ("mode", I)]


class AdamSeg(C.Structure):
    _fields_ = [("p", P), ("m", P), ("v", P), ("g", P), ("bf", P), ("bfT", P), ("n", C.c_long),
                ("gstride", C.c_long), ("S", I), ("tG", I), ("tCo", I), ("tKH", I), ("tKW", I), ("tCi", I),
                ("tiled", I), ("npl", I), ("pstride_bf", C.c_long), ("pstride_bfT", C.c_long)]

ADAM_TK = 64        # adam_segments transpose tiles: tCo rows x ADAM_TK reduction columns


ADAM_BLK = 1024     # elements per block of an element-wise Adam segment (cnn_dense.hip ADAM_BLK)


def adam_blocks(n):
    """Block offsets of an element-wise (untiled) Adam segment of ``n`` elements."""
    return range(0, n, ADAM_BLK)


def adam_tiles(tG, tCo, tKH, tKW, tCi):
    """Blocks of a tiled conv-weight segment (csrc/hip/cnn_dense.hip, tiled
    path), or 0 when the segment cannot be tiled (then: ADAM_BLK-element blocks)."""
    if tCo % 8:
        return 0
    kd = tKH * tKW * tCi
    return tG * (-(-tCo // 128)) * (-(-kd // ADAM_TK))


class BnArgs(C.Structure):
    """csrc/hip/cnn_bn.hip BnArgs (optional BatchNorm of the node convs)."""
    _fields_ = [("z", P), ("y", P), ("gamma", P), ("beta", P), ("stat", P), ("run", P), ("part", P),
                ("ggamma", P), ("gbeta", P), ("gtab", P), ("valid", P), ("st", P),
                ("ngroups", I), ("G", I), ("B", I), ("HW", I), ("Cp", I), ("nchunk", I), ("chunk_px", I),
                ("momentum", C.c_float), ("eps", C.c_float), ("train", I), ("prec", I),
                ("pool_y", P), ("pool_mask", P), ("W", I), ("Hr", I), ("Wr", I)]


BN_CHUNK_PX = 512     # pixels per BatchNorm workgroup at most (fixed per shape: batch-invariant sums)
BN_CHUNK_VALUES = 16384


def bn_chunk_px(H, W, Cp):
    """Pixels per BatchNorm workgroup of a layer: 512, halved while a chunk holds more than 16K values and
    the halves still hold whole row pairs (the fused 2x2 pool). A function of the layer shape only, so a
    group's sums do not depend on the other groups of the launch. At 512 pixels a 256-channel 8x8 stage
    had 4 workgroups per group (100 per 25-group launch on 256 CUs: ~1.4 TB/s)."""
    c = BN_CHUNK_PX
    pooled = BN_CHUNK_PX % (2 * W) == 0            # else the pool runs as its own kernel (cnn_hip.py)
    while c * Cp > BN_CHUNK_VALUES and (c // 2 >= 2 * W and (c // 2) % (2 * W) == 0 if pooled else c > 64):
        c //= 2
    return c


class AdamArgs(C.Structure):
    _fields_ = [("segs", P), ("blocks", P), ("st", P)]


class ProgOp(C.Structure):
    """One op of a native step program (csrc/hip/step_prog.hip GtProgOp)."""
    _fields_ = [("kind", C.c_int32), ("stream", C.c_int32), ("event", C.c_int32), ("pad", C.c_int32),
                ("v", C.c_int64 * 14)]


# op kinds of csrc/hip/step_prog.hip, by the name of the launch entry point
PROG_OPS = {"record": 0, "wait": 1, "gt_step_begin": 2, "gt_conv_fwd": 3, "gt_conv_wgrad": 4,
            "gt_wgrad_reduce": 5, "gt_bn_fwd": 6, "gt_bn_bwd": 7, "gt_dense_fwd": 8, "gt_head": 9,
            "gt_dense_dgrad": 10, "gt_dense_wgrad_adam": 11, "gt_adam_segments": 12, "gt_pool_fwd": 13,
            "gt_pool_fwd_mask": 14, "gt_pool_bwd_mask": 15, "gt_wino_wtrans": 16,
            "gt_conv_wfrag": 17}


class InitSeg(C.Structure):
    _fields_ = [("p", P), ("seeds", P), ("d", I * 4), ("r", I * 4), ("G", I), ("tag", I), ("limit", C.c_float),
                ("pad", I)]


class InitArgs(C.Structure):
    _fields_ = [("segs", P), ("blocks", P)]


_TYPED = {}


def lib():
    L = _lib.hip()
    if not _TYPED.get(id(L)):
        for name, argt in (("gt_conv_fwd", C.POINTER(ConvArgs)), ("gt_conv_wgrad", C.POINTER(WgradArgs)),
                           ("gt_dense_fwd", C.POINTER(DenseFwdArgs)), ("gt_head", C.POINTER(HeadArgs)),
                           ("gt_dense_dgrad", C.POINTER(DenseDgradArgs)),
                           ("gt_dense_wgrad_adam", C.POINTER(DenseWgradAdamArgs))):
            fn = getattr(L, name)
            fn.argtypes = [argt, P]
            fn.restype = I
        for name in ("gt_bn_fwd", "gt_bn_bwd"):
            fn = getattr(L, name)
            fn.argtypes = [C.POINTER(BnArgs), P]
            fn.restype = I
        L.gt_adam_segments.argtypes = [C.POINTER(AdamArgs), I, P]
        L.gt_adam_segments.restype = I
        L.gt_step_begin.argtypes = [P, P]
        L.gt_step_begin.restype = I
        L.gt_pool_fwd.argtypes = [P, P, P, P, I, I, I, I, I, I, P]
        L.gt_pool_fwd.restype = I
        L.gt_pool_bwd.argtypes = [P, P, P, P, P, P, I, I, I, I, I, I, I, P]
        L.gt_pool_bwd.restype = I
        L.gt_pool_fwd_mask.argtypes = [P, P, P, P, I, I, I, I, I, P, I, P]
        L.gt_pool_fwd_mask.restype = I
        L.gt_pool_bwd_mask.argtypes = [P, P, P, P, P, I, I, I, I, I, I, I, P]
        L.gt_pool_bwd_mask.restype = I
        L.gt_wgrad_set_nb.argtypes = [I]
        L.gt_wgrad_set_nb.restype = I
        L.gt_wgrad_fast_band.argtypes = [I, I, I, I, I, I, I]
        L.gt_wgrad_fast_splits.argtypes = [I, I, I, I, I, I, I]
        L.gt_wgrad_fast_splits.restype = I
        L.gt_wgrad_fast_band.restype = I
        L.gt_conv_fast_probe.argtypes = [C.POINTER(ConvArgs)]
        L.gt_conv_fast_probe.restype = I
        L.gt_conv_fast_probe_any.argtypes = [C.POINTER(ConvArgs)]
        L.gt_conv_fast_probe_any.restype = I
        L.gt_wgrad_reduce.argtypes = [C.POINTER(WgradArgs), P]
        L.gt_wgrad_reduce.restype = I
        L.gt_conv_frag_order.argtypes = [I, I, I, I, I, C.POINTER(C.c_int), I]
        L.gt_conv_frag_order.restype = I
        L.gt_conv_wfrag.argtypes = [P, I, P]
        L.gt_conv_wfrag.restype = I
        L.gt_sizeof_frag_seg.restype = C.c_size_t
        assert L.gt_sizeof_frag_seg() == C.sizeof(FragSeg), "FragSeg ABI mismatch"
        L.gt_conv_wino_supported.argtypes = [I, I, I, I]
        L.gt_conv_wino_supported.restype = I
        L.gt_wino_wtrans.argtypes = [P, I, P]
        L.gt_wino_wtrans.restype = I
        L.gt_sizeof_wino_wseg.restype = C.c_size_t
        assert L.gt_sizeof_wino_wseg() == C.sizeof(WinoWSeg), "WinoWSeg ABI mismatch"
        L.gt_conv_set_fast.argtypes = [I]
        L.gt_conv_set_fast.restype = I
        L.gt_conv_set_nwv.argtypes = [I]
        L.gt_conv_set_s2in_ct1.restype = I
        L.gt_dense_fwd_splits.argtypes = [I]
        L.gt_dense_fwd_splits.restype = I
        L.gt_conv_set_smallq.argtypes = [I]
        L.gt_conv_set_smallq.restype = I
        L.gt_conv_set_s2in_ct1.argtypes = [I]
        L.gt_conv_set_nwv.restype = I
        L.gt_conv_set_imgs.argtypes = [I]
        L.gt_conv_set_imgs.restype = I
        L.gt_glorot_init.argtypes = [C.POINTER(InitArgs), I, P]
        L.gt_glorot_init.restype = I
        L.gt_glorot_ref.argtypes = [C.c_uint64, C.c_uint64, I, C.c_float]
        L.gt_glorot_ref.restype = C.c_float
        L.gt_prog_create.argtypes = [C.POINTER(ProgOp), I, I, I]
        L.gt_prog_create.restype = P
        L.gt_prog_run.argtypes = [P, P, I, C.POINTER(I)]
        L.gt_prog_run.restype = I
        L.gt_prog_destroy.argtypes = [P]
        L.gt_prog_destroy.restype = None
        L.gt_sizeof_prog_op.restype = C.c_size_t
        assert L.gt_sizeof_prog_op() == C.sizeof(ProgOp), "ProgOp ABI mismatch"
        for name in ("gt_sizeof_conv_args", "gt_sizeof_wgrad_args", "gt_sizeof_adam_seg", "gt_sizeof_init_seg",
                     "gt_sizeof_dense_fwd_args", "gt_sizeof_head_args", "gt_sizeof_dense_dgrad_args",
                     "gt_sizeof_dense_wgrad_args", "gt_sizeof_bn_args"):
            getattr(L, name).restype = C.c_size_t
        assert L.gt_sizeof_conv_args() == C.sizeof(ConvArgs), "ConvArgs ABI mismatch"
        assert L.gt_sizeof_init_seg() == C.sizeof(InitSeg), "InitSeg ABI mismatch"
        assert L.gt_sizeof_wgrad_args() == C.sizeof(WgradArgs), "WgradArgs ABI mismatch"
        assert L.gt_sizeof_adam_seg() == C.sizeof(AdamSeg), "AdamSeg ABI mismatch"
        assert L.gt_adam_block_elems() == ADAM_BLK, "Adam block size mismatch"
        assert L.gt_sizeof_bn_args() == C.sizeof(BnArgs), "BnArgs ABI mismatch"
        for nm, st in (("dense_fwd_args", DenseFwdArgs), ("head_args", HeadArgs),
                       ("dense_dgrad_args", DenseDgradArgs), ("dense_wgrad_args", DenseWgradAdamArgs)):
            assert getattr(L, "gt_sizeof_" + nm)() == C.sizeof(st), nm + " ABI mismatch"
        _TYPED[id(L)] = True
    return L


def check(rc, what):
    if rc != 0:
        raise RuntimeError("HIP kernel launch {} failed with code {}".format(what, rc))


class StepProgram(object):
    """A native step program (csrc/hip/step_prog.hip): ``plan`` is a list of
    ``("k", entry_point, args, stream_key, what)`` launches and ``("rec" |
    "wait", stream_key, event_id)`` edges; stream key ``None`` is the caller's
    stream at :meth:`run` time. Launch operands are ctypes argument structs
    (passed by address) or ints (pool launches)."""

    def __init__(self, plan):
        L = lib()
        self.L = L
        keys, nev = [None], 0
        ops = (ProgOp * len(plan))()
        for o, op in zip(ops, plan):
            st = op[3] if op[0] == "k" else op[1]
            if not any(st is k for k in keys):
                keys.append(st)
            o.stream = next(i for i, k in enumerate(keys) if k is st)
            if op[0] in ("rec", "wait"):
                o.kind = PROG_OPS["record" if op[0] == "rec" else "wait"]
                o.event = int(op[2])
                nev = max(nev, o.event + 1)
                continue
            o.kind = PROG_OPS[op[1]]
            vals = []
            for a in op[2]:
                if isinstance(a, C.Structure):
                    vals.append(C.addressof(a))
                elif a is None:
                    vals.append(0)
                elif isinstance(a, C.c_void_p):
                    vals.append(a.value or 0)
                else:
                    vals.append(int(a))
            if len(vals) > len(o.v):
                raise ValueError("step program: too many operands for " + op[1])
            for i, x in enumerate(vals):
                o.v[i] = x
        self._ops = ops
        self._structs = [a for op in plan if op[0] == "k" for a in op[2] if isinstance(a, C.Structure)]
        self.keys = keys
        self.h = L.gt_prog_create(ops, len(plan), nev, len(keys))
        if not self.h:
            raise RuntimeError("gt_prog_create rejected the step program")
        self._streams = (C.c_void_p * len(keys))()

    def run(self, main_stream, nsteps):
        self._streams[0] = main_stream
        for i, k in enumerate(self.keys[1:], 1):
            self._streams[i] = k.cuda_stream
        bad = I(-1)
        rc = self.L.gt_prog_run(self.h, self._streams, int(nsteps), C.byref(bad))
        if rc != 0:
            raise RuntimeError("HIP step program op {} failed with code {}".format(bad.value, rc))

    def __del__(self):
        h, self.h = getattr(self, "h", None), None
        if h:
            try:
                self.L.gt_prog_destroy(h)
            except Exception:          # interpreter shutdown
                pass


def ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else C.c_void_p(0)


CONV_TILE_PIXELS = 128   # 256-pixel tiles measured slower on every layer (profiles/bench_kernels_tiles.log)


def conv_tile_rows(H, W, tile_pixels=None):
    """Output rows per conv_fwd workgroup (tiles of 64 / 128 / 256 pixels =
    4 waves x 16 / 32 / 64). 128 is the measured optimum for every layer of the
    S=(3,5) space (profiles/conv_tiles.json: 64-pixel tiles are 1.3-2.8x
    slower even when they double the grid)."""
    tp = tile_pixels or CONV_TILE_PIXELS
    if W > tp:
        raise ValueError("image width > {} not supported by conv_fwd tiles".format(tp))
    return max(1, min(H, tp // W))


def wino_segment(master, planes, dgrad):
    """WinoWSeg of one layer: fp32 master weights ``[Q][Cop][3][3][Cip]`` -> transformed bf16 planes
    ``[3][Q][16][R][K]`` (R, K = :func:`wino_dims` of the forward, swapped for the data gradient)."""
    Q, cop, kh, kw, cip = master.shape
    assert (kh, kw) == (3, 3) and master.dtype.is_floating_point and master.is_contiguous()
    R, Kc = (wino_dims(cop, cip) if dgrad else wino_dims(cip, cop))
    assert tuple(planes.shape) == (3, Q, 16, R, Kc) and planes.is_contiguous(), (planes.shape, (3, Q, 16, R, Kc))
    sg = WinoWSeg()
    sg.w, sg.u, sg.ups = master.data_ptr(), planes.data_ptr(), planes[0].numel()
    sg.Q, sg.Cop, sg.Cip, sg.R, sg.K, sg.dgrad = Q, cop, cip, R, Kc, 1 if dgrad else 0
    return sg


class WinoTransform(object):
    """One launch that re-transforms the Winograd weights of several layers (both directions) from
    their fp32 masters -- after every optimizer step and after initialisation."""

    def __init__(self, segs, device):
        import numpy as np
        import torch
        self.nseg = len(segs)
        blocks = []
        for i, sg in enumerate(segs):
            n = sg.Q * sg.R * sg.K
            blocks.extend((i, o) for o in range(0, n, 256))
        arr = (WinoWSeg * max(1, len(segs)))(*segs)
        self.segs_t = torch.frombuffer(bytearray(bytes(memoryview(arr).cast("B"))), dtype=torch.uint8).to(device)
        self.blocks_t = torch.tensor(np.asarray(blocks, np.int32).reshape(-1, 2), device=device)
        self.args = WinoWArgs()
        self.args.segs, self.args.blocks = self.segs_t.data_ptr(), self.blocks_t.data_ptr()
        self.nblocks = len(blocks)

    def run(self, stream):
        if self.nblocks:
            check(lib().gt_wino_wtrans(C.addressof(self.args), self.nblocks, stream), "wino_wtrans")


def wino_unpack(planes):
    """Logical ``[3][Q][16][R][K]`` view of fragment-major transformed planes (the layout
    gt_wino_wtrans writes: per (xi, 16-row tile, 32-column k-step) one 64-lane x 8-value fragment,
    lane = (column % 32) // 8 * 16 + row % 16)."""
    npl, Q, nxi, R, Kc = planes.shape
    f = planes.reshape(npl, Q, nxi, R // 16, Kc // 32, 4, 16, 8)     # [.., rt, ks, kq, l16, e]
    return f.permute(0, 1, 2, 3, 6, 4, 5, 7).reshape(npl, Q, nxi, R, Kc)


def wino_weights(master, dgrad=False, stream=None):
    """Transformed planes of ``master`` (tests / one-off use; jobs keep a :class:`WinoTransform`)."""
    import torch
    Q, cop, _, _, cip = master.shape
    R, Kc = wino_dims(cop, cip) if dgrad else wino_dims(cip, cop)
    planes = torch.zeros((3, Q, 16, R, Kc), dtype=torch.bfloat16, device=master.device)
    tr = WinoTransform([wino_segment(master.contiguous(), planes, dgrad)], master.device)
    tr.run(torch.cuda.current_stream(master.device).cuda_stream if stream is None else stream)
    tr.keep = planes
    return planes


def padded_hw(h, w, nstages, batch_norm=False):
    """(H, W) the HIP executor stores and runs a Genetic-CNN image at.

    The shape-specialised kernels exist for the power-of-two stage widths of
    the search spaces (32 / 16 / 8). An image a little smaller than a power of
    two -- the reference's own MNIST default, 28 x 28 (gentun/individuals.py:221)
    -- is stored zero-padded at the bottom / right to that size, so every stage
    runs those kernels (28 -> 32, 14 -> 16, final 7 x 7 in 8 x 8) instead of
    the generic ones. The forward epilogues write exact zeros outside the real
    rows / columns (ConvArgs::Hr / Wr) and the dense W1 rows of padded pixels
    are initialised to 0 and receive zero gradient, so the padded network IS
    the unpadded one (tests/test_hip_train.py::test_padded_mnist_geometry).
    Conditions: square, every stage's real size even (no floor pooling inside
    the padding), at most 25 % wider. With BatchNorm the statistics count the
    real pixels only and BN writes zeros outside them (cnn_bn.hip BnArgs::Hr /
    Wr); ``batch_norm`` is kept for callers."""
    del batch_norm
    p = 1 << max(0, int(w) - 1).bit_length()
    if (h != w or p == w or p > 1.25 * w or w % (1 << nstages) or p >> nstages < 8):
        return h, w
    return p, p


# channel paddings the shape-specialised conv / wgrad kernels are instantiated for (the narrow (20, 50, 100) and
# wide (64, 128, 256) search spaces' stage widths, padded to 8); other channel counts are padded UP to one of
# these when that puts every layer of the network on the fast kernels (stage_channel_pads)
FAST_PADS = (24, 32, 56, 64, 104, 128, 256)


def _probe_conv(L, KH, KW, cinp, coutp, H, W, prec, ngroups, B, cout_real, fwd):
    a = ConvArgs()
    a.KH, a.KW, a.Cinp, a.Coutp, a.H, a.W = KH, KW, cinp, coutp, H, W
    a.G = a.ngroups = max(1, ngroups)
    a.B, a.prec, a.cout_real = B, prec, cout_real
    a.epi_bf16 = 1 if fwd else 0
    a.TH = conv_tile_rows(H, W)
    return bool(L.gt_conv_fast_probe_any(a))


def layer_fast(KH, KW, cinp, coutp, H, W, prec, ngroups, B, cin_real, cout_real, first):
    """(forward, data gradient, weight gradient) of one layer geometry run on shape-specialised kernels
    (gt_conv_fast / gt_wgrad_fast) -- each probed without launching anything (no GPU needed)."""
    L = lib()
    on = L.gt_conv_set_fast(1)               # the fast path switched off (generic-kernel comparisons): none
    L.gt_conv_set_fast(on)
    if not on:
        return False, False, False
    fwd = _probe_conv(L, KH, KW, cinp, coutp, H, W, prec, ngroups, B, cout_real, True)
    dgr = True if first else _probe_conv(L, KH, KW, coutp, cinp, H, W, prec, ngroups, B, cin_real, False)
    wgr = int(L.gt_wgrad_fast_band(KH, KW, cinp, coutp, H, W, prec)) > 0
    return fwd, dgr, wgr


def stage_channel_pads(c0, kernels, kernel_sizes, h0, w0, prec, ngroups=25, B=32, max_factor=2.0):
    """Channel padding of every stage's tensors (input conv output, node outputs, output conv, pool).

    The reference lets the user choose ``kernels_per_layer`` / ``kernel_sizes`` freely
    (gentun/individuals.py:221-223). The fast kernels exist for a set of padded channel counts
    (FAST_PADS): each stage's count is padded up to one of them -- at most ``max_factor`` x its own
    8-padding -- choosing the cheapest combination (padded multiply-adds) under which EVERY conv
    launch (forward, data gradient, weight gradient) runs a shape-specialised kernel; when no
    combination does, the plain 8-padding (some layers on the generic kernels). Padded channels have
    zero weights, zero bias and zero gradient (they stay exactly 0: the network computes the
    unpadded one)."""
    import itertools
    c0p = (c0 + 7) // 8 * 8
    base = [(c + 7) // 8 * 8 for c in kernels]
    cands = [sorted({b} | {v for v in FAST_PADS if b <= v <= max_factor * b}) for b in base]
    best = None
    for combo in itertools.product(*cands):
        cost, ok = 0.0, True
        cin, cinr = c0p, c0
        for s, (cp, k) in enumerate(zip(combo, kernel_sizes)):
            H, W = h0 >> s, w0 >> s
            kh, kw = tuple(k)
            for (KH, KW, ci, cir, first) in ((kh, kw, cin, cinr, s == 0), (3, 3, cp, kernels[s], False)):
                f = layer_fast(KH, KW, ci, cp, H, W, prec, ngroups, B, cir, kernels[s], first)
                if not all(f):
                    ok = False
                    break
                cost += H * W * KH * KW * ci * cp
            if not ok:
                break
            cin, cinr = cp, kernels[s]
        if ok and (best is None or cost < best[0]):
            best = (cost, combo)
    return list(best[1]) if best is not None else base


def wgrad_blocks(kdim, with_bias=True):
    """Column blocks of conv_wgrad (the bias rides in an extra ones-chunk)."""
    return -(-(kdim + (8 if with_bias else 0)) // 64)


WGRAD_TARGET_BLOCKS = 50     # generic wgrad: ~workgroups per fold
WGRAD_FAST_SPLITS = 0        # shape-specialised wgrad splits: 0 = the per-shape default (tests override it)


def wgrad_band(KH, KW, cinp, coutp, H, W, prec=0):
    """``(pixels per band, preferred splits)`` of the shape-specialised wgrad
    kernel, or ``(0, 0)`` for the generic one."""
    L = lib()
    if not L.gt_conv_set_fast(1):       # probe + restore the fast-path switch
        L.gt_conv_set_fast(0)
        return 0, 0
    band = int(L.gt_wgrad_fast_band(KH, KW, cinp, coutp, H, W, prec))
    splits = int(L.gt_wgrad_fast_splits(KH, KW, cinp, coutp, H, W, prec)) if band else 0
    return band, splits


def wgrad_split(npix, kdim, coutp, G=None, target_blocks=None, band=0):
    """(pixels per split, splits) for conv_wgrad: ~``target_blocks``
    workgroups PER FOLD (the split never depends on how many folds share a
    launch, so a fold's gradient summation order -- and its result -- is the
    same alone or batched), 64-pixel K-steps, >= 2 K-steps per workgroup."""
    band, splits = band if isinstance(band, tuple) else (band, 8)
    if band:
        # specialised kernel: one workgroup per split, splits of whole bands;
        # the split count is a per-shape constant (never depends on how many
        # groups share the launch: a fold's summation order is batch-invariant)
        splits = WGRAD_FAST_SPLITS or splits
        nb = npix // band
        bps = -(-nb // max(1, splits))
        return bps * band, -(-nb // bps)
    if target_blocks is None:
        target_blocks = WGRAD_TARGET_BLOCKS
    nb = wgrad_blocks(kdim)
    mb = -(-coutp // 64)
    per = max(1, nb * mb)
    S = max(1, min(target_blocks // per, npix // 128))
    pps = -(-npix // S)
    pps = max(64, -(-pps // 64) * 64)
    S = -(-npix // pps)
    return pps, S
