"""Fold-batched Genetic-CNN training engine (device side).

One *job* = one candidate architecture trained on ``G`` cross-validation
folds AT ONCE: every parameter carries a leading fold dimension and every
kernel launch processes all folds (SURVEY.md §2.4 "fold-batch", §7.3 hard
part 1). The whole train step (gather -> fwd -> loss -> bwd -> Adam) is
captured once per architecture into a HIP graph and replayed
``epochs x steps`` times; per-epoch shuffles, learning-rate stages and Adam
resets are enqueued asynchronously on the job's own stream, so the host
can enqueue several candidates on different streams and the GPU runs them
concurrently (hard part 1: a single tiny candidate cannot fill 256 CUs).

Training protocol (reference: gentun/models/keras_models.py:120-143, Keras
2.2 semantics -- SURVEY.md §2.2):

* folds (``reset``): ``"kernels"`` (default, the reference:
  folds run one after another and each re-draws only the Glorot kernels,
  so the biases trained on fold k start fold k+1 -- keras_models.py:
  120-125,135; :class:`SequentialFoldJob`), or ``"all"`` (folds train
  CONCURRENTLY as groups of one job, each from fresh kernels and zero
  biases -- the fast mode);
* per ``(epochs_i, lr_i)`` stage a NEW Adam (m, v, t reset), beta1 0.9,
  beta2 0.999, eps 1e-7, Keras bias-corrected step size;
* loss ``bce_compat`` = binary cross-entropy on the softmax output with
  probabilities clipped to [1e-7, 1-1e-7], metric ``binary_accuracy``
  (Keras' resolution of 'accuracy' for that loss), or ``ce`` = categorical
  cross-entropy with categorical accuracy;
* dropout is inverted dropout on the dense layer;
* each epoch visits every training sample once in a fresh random order in
  ``ceil(n_train / B)`` steps (``batching``): ``"keras"`` (default) -- the
  last step is Keras' short batch: the shapes stay fixed (graph capture),
  the padding rows carry zero loss weight and the mean is over the real
  rows; or ``"wrap"`` -- the last batch wraps around to the start of the
  permutation.

Backends: ``hip`` (MI355X kernels, :mod:`gentun_amd.models.cnn_hip`) and
``torch`` (autograd oracle / comparator path (a) of SURVEY.md §6).
"""

import copy
import math
import os

import numpy as np
import torch
import torch.nn.functional as F

from ..utils import rng as _rng
from .genome import ConvSpec, PoolSpec

ADAM_B1, ADAM_B2, ADAM_EPS = 0.9, 0.999, 1e-7
CLIP_EPS = 1e-7



def check_hw_queues(nstreams, env=None):
    """Refuse to capture a step graph over more streams than the process has hardware queues.

    With ``GPU_MAX_HW_QUEUES=3`` the replay of a graph captured over 4 streams segfaults inside
    HIP's graph launch -- reproduced with torch alone (tools/probe_hwq.py: 1 and 2 side streams
    replay, 3 crash; profiles/r5/hwq3_graph_crash_r5.log), so it is the runtime's, not this
    engine's; the population step graph forks onto 1 + WGRAD_STREAMS side streams. A clear error
    instead of the crash (verdict r4 item 6a)."""
    if not hw_queues_ok(nstreams, env):
        v = (os.environ if env is None else env).get("GPU_MAX_HW_QUEUES", "")
        raise RuntimeError(
            "GPU_MAX_HW_QUEUES={} is below the {} streams of the captured step graph: HIP's graph launch "
            "segfaults there (torch-only repro: tools/probe_hwq.py). Use GPU_MAX_HW_QUEUES >= {} (HIP's "
            "default is 4) or eager steps (TrainConfig use_graph=False)".format(int(v), nstreams, nstreams))

def hw_queues_ok(nstreams, env=None):
    """False when ``GPU_MAX_HW_QUEUES`` is set below ``nstreams`` (see :func:`check_hw_queues`)."""
    v = (os.environ if env is None else env).get("GPU_MAX_HW_QUEUES", "")
    return not (v.strip().isdigit() and int(v) < nstreams)


_HWQ_WARNED = []


def graph_or_eager(nstreams, env=None):
    """Whether a job may capture its step graph: with too few hardware queues it trains with eager
    steps instead (same launches, bit-identical results) and says so once per process -- a queue
    setting must not fail every candidate of a search."""
    if hw_queues_ok(nstreams, env):
        return True
    if not _HWQ_WARNED:
        _HWQ_WARNED.append(1)
        import warnings
        v = (os.environ if env is None else env).get("GPU_MAX_HW_QUEUES", "")
        warnings.warn("GPU_MAX_HW_QUEUES={} is below the {} streams of the captured step graph (HIP's graph "
                      "launch segfaults there): training with eager steps instead".format(v.strip(), nstreams),
                      RuntimeWarning, stacklevel=3)
    return False


class TrainConfig(object):
    def __init__(self, epochs=(3,), learning_rate=(1e-3,), batch_size=32, dropout=0.5, loss="bce_compat",
                 dtype="fp32", seed=0, use_graph=None, eval_batch=1000, optimizer="adam", momentum=0.9,
                 reset="kernels", batching="keras", batch_norm=False, bn_momentum=0.99, bn_eps=1e-3,
                 dp_group=None, verbose=False, nfold=None, pad_images=True):
        if isinstance(epochs, int):
            epochs = (epochs,)
        if isinstance(learning_rate, (int, float)):
            learning_rate = (float(learning_rate),)
        epochs, learning_rate = tuple(epochs), tuple(float(x) for x in learning_rate)
        if len(epochs) != len(learning_rate):
            raise ValueError("epochs and learning_rate must have the same length")
        if loss not in ("bce_compat", "ce"):
            raise ValueError("loss must be 'bce_compat' or 'ce'")
        if dtype not in ("bf16", "fp32"):
            raise ValueError("dtype must be 'bf16' or 'fp32'")
        if optimizer not in ("adam", "sgd"):
            raise ValueError("optimizer must be 'adam' or 'sgd'")
        if reset not in ("kernels", "all"):
            raise ValueError("reset must be 'kernels' (reference: sequential folds, biases carried over) or 'all'")
        if batching not in ("keras", "wrap"):
            raise ValueError("batching must be 'keras' (short last batch) or 'wrap'")
        self.reset = reset
        self.batching = batching
        # optional BatchNorm after every conv (conv -> BN -> ReLU; not in the
        # reference network, off by default); Keras BatchNormalization defaults
        self.batch_norm = bool(batch_norm)
        self.bn_momentum = float(bn_momentum)
        self.bn_eps = float(bn_eps)
        # optional intra-candidate data parallelism (torch
        # executor): a torch.distributed process group whose ranks each take a
        # contiguous slice of every batch; gradients are all-reduced (RCCL over
        # xGMI on GPUs) before the identical optimizer step on every rank
        self.dp_group = dp_group
        self.epochs = epochs
        self.learning_rate = learning_rate
        self.batch_size = int(batch_size)
        self.dropout = float(dropout)
        self.loss = loss
        self.dtype = dtype
        self.seed = seed
        self.use_graph = use_graph
        self.eval_batch = int(eval_batch)
        self.optimizer = optimizer
        self.momentum = float(momentum)
        # the reference's progress lines (keras_models.py:134,137): "KFold i/n" as a fold's
        # training is enqueued, "Training N epochs with learning rate lr" per stage
        self.verbose = bool(verbose)
        self.nfold = None if nfold is None else int(nfold)
        # HIP executor: store a slightly-smaller-than-power-of-two image zero-padded so every stage
        # runs the shape-specialised kernels (ops/cnn_kernels.padded_hw: MNIST 28 x 28 -> 32 x 32)
        self.pad_images = bool(pad_images)

    def total_epochs(self):
        return sum(self.epochs)


# ---------------------------------------------------------------------------
# Device-resident dataset cache (no per-batch H2D)
# ---------------------------------------------------------------------------

class DeviceData(object):
    def __init__(self, x, y, device, layout, pad_hw=None):
        x = np.asarray(x)
        y = np.asarray(y)
        self.n = x.shape[0]
        self.hwc = tuple(x.shape[1:])
        self.classes = y.shape[1] if y.ndim == 2 else int(y.max()) + 1
        lab = np.argmax(y, 1) if y.ndim == 2 else y.astype(np.int64)
        self.labels_np = lab.astype(np.int64)
        self.device = device
        self.layout = layout
        xt = torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32))
        if layout == "nchw":
            self.x = xt.permute(0, 3, 1, 2).contiguous().to(device)
        elif layout in ("nhwc8", "nhwc8f"):
            # channels padded to a multiple of 8 so one chunk = 8 channels
            # (nhwc8: bf16 tensors of the bf16 mode; nhwc8f: fp32)
            # pad_hw: the images stored zero-padded at the bottom / right to (H, W) (cnn_kernels.padded_hw)
            n, h, w, c = xt.shape
            hp, wp = pad_hw or (h, w)
            cp = (c + 7) // 8 * 8
            pad = torch.zeros((n, hp, wp, cp), dtype=torch.float32)
            pad[:, :h, :w, :c] = xt
            dt = torch.float32 if layout == "nhwc8f" else torch.bfloat16
            self.x = pad.to(device=device, dtype=dt).contiguous()
        else:
            raise ValueError(layout)
        self.labels = torch.from_numpy(self.labels_np).to(device)
        self.onehot = F.one_hot(self.labels, self.classes).float()


_DATA_CACHE = []


def device_data(x, y, device, layout, pad_hw=None):
    key = (layout, tuple(pad_hw) if pad_hw else None)
    for ent in _DATA_CACHE:
        if ent[0] is x and ent[1] is y and ent[2] == str(device) and ent[3] == key:
            return ent[4]
    dd = DeviceData(x, y, device, layout, pad_hw)
    _DATA_CACHE.append((x, y, str(device), key, dd))
    while len(_DATA_CACHE) > 3:
        _DATA_CACHE.pop(0)
    return dd


# ---------------------------------------------------------------------------
# Shared job driver
# ---------------------------------------------------------------------------

class FoldJob(object):
    """Train one architecture on ``len(folds)`` folds concurrently -- or, with
    ``members``, several architectures ("population batching"): the groups of
    the job are every (member, fold) pair, member-major.

    ``launch()`` only ENQUEUES work on ``self.stream``; ``finish()`` waits and
    returns per-fold metrics (a dict; a list of dicts, one per member, when
    the job was built with ``members``). Subclasses supply the executor.

    Everything random is keyed by (run seed, genes, fold id), never by the
    group's position in the job, so a candidate's result is the same alone or
    batched with any other candidates.
    """

    layout = "nchw"

    def __init__(self, plan, x, y, folds, cfg, device, fold_ids=None, stream=None, members=None):
        self.multi = members is not None
        if members is None:
            members = [(plan, folds, list(range(len(folds))) if fold_ids is None else list(fold_ids))]
        members = [(p, list(f), list(range(len(f))) if ids is None else list(ids)) for p, f, ids in members]
        if not members or any(len(f) != len(ids) or not f for _, f, ids in members):
            raise ValueError("every member needs at least one fold and one fold id per fold")
        self.members = members
        self.plan = members[0][0]
        self.cfg = cfg
        self.device = torch.device(device)
        # groups = (member, fold) pairs, member-major
        self.gmember, self.fold_ids, self.folds = [], [], []
        for c, (_p, f, ids) in enumerate(members):
            for fold, fid in zip(f, ids):
                self.gmember.append(c)
                self.fold_ids.append(int(fid))
                self.folds.append(fold)
        self.G = len(self.folds)
        self.data = device_data(x, y, self.device, self.layout, getattr(self, "pad_hw", None))
        self.stream = stream if stream is not None else torch.cuda.current_stream(self.device) \
            if self.device.type == "cuda" else None
        self.B = cfg.batch_size
        ntr = [len(tr) for tr, _ in self.folds]
        nva = [len(va) for _, va in self.folds]
        self.ntrain = ntr
        self.nval = nva
        self.steps_per_epoch = int(math.ceil(max(ntr) / self.B))
        self.member_seeds = [_rng.stable_hash("cnn", cfg.seed, sorted(p.genes.items())) & 0x7FFFFFFFFFFF
                             for p, _, _ in members]
        self.base_seed = self.member_seeds[0]
        # device index tables
        maxn = max(ntr)
        tm = np.zeros((self.G, maxn), np.int64)
        for g, (tr, _) in enumerate(self.folds):
            tm[g, :len(tr)] = tr
        self.train_mat = torch.from_numpy(tm).to(self.device)
        self.ntrain_t = torch.tensor(ntr, dtype=torch.int64, device=self.device)
        maxv = max(nva)
        vm = np.zeros((self.G, maxv), np.int64)
        vmask = np.zeros((self.G, maxv), np.float32)
        for g, (_, va) in enumerate(self.folds):
            vm[g, :len(va)] = va
            vmask[g, :len(va)] = 1.0
        self.val_mat = torch.from_numpy(vm).to(self.device)
        self.val_mask = torch.from_numpy(vmask).to(self.device)
        # One generator per group, keyed by (member seed, fold id): a fold's data
        # order is the same whether it is trained alone or batched with others.
        self.shuffle_gens = []
        for g, fid in enumerate(self.fold_ids):
            gen = torch.Generator(device=self.device)
            gen.manual_seed(_rng.stable_hash(self.member_seeds[self.gmember[g]], "shuffle", fid) & 0x7FFFFFFF)
            self.shuffle_gens.append(gen)
        self.epoch_idx = torch.zeros((self.steps_per_epoch, self.G, self.B), dtype=torch.int64,
                                     device=self.device)
        # real rows of each (step, group) batch: B, except a Keras short last
        # batch (batching="keras"); padding rows repeat real samples and carry
        # zero loss weight
        self.epoch_valid = torch.full((self.steps_per_epoch, self.G), self.B, dtype=torch.int32, device=self.device)
        if cfg.batching == "keras":
            v = np.zeros((self.steps_per_epoch, self.G), np.int32)
            for g, n in enumerate(ntr):
                for st in range(self.steps_per_epoch):
                    v[st, g] = max(0, min(self.B, n - st * self.B))
            self.epoch_valid.copy_(torch.from_numpy(v))
        self.after_init = None        # callable run right after init_params (sequential folds)
        self.step_ctr = torch.zeros((1,), dtype=torch.int64, device=self.device)
        self.result = None

    # -- sequential folds: one job, re-pointed at the next fold ---------------
    can_rebind = False          # executors whose device state survives a rebind set this

    def rebind(self, folds, fold_ids):
        """Point the job at other folds of the same members (one fold per
        group, in group order) without rebuilding it: index tables, shuffle
        streams and fold ids change; buffers, argument tables and the captured
        step graph stay. Returns False (nothing changed) when the new folds
        need another step count per epoch; the caller then builds a new job."""
        if not self.can_rebind or len(folds) != self.G or len(fold_ids) != self.G:
            return False
        ntr = [len(tr) for tr, _ in folds]
        if int(math.ceil(max(ntr) / self.B)) != self.steps_per_epoch:
            return False
        # the previous fold's launches may still read the old tables: keep them alive
        self._retired = getattr(self, "_retired", []) + [self.train_mat, self.ntrain_t, self.val_mat,
                                                         self.val_mask]
        self.folds = list(folds)
        self.fold_ids = [int(f) for f in fold_ids]
        self.ntrain = ntr
        self.nval = [len(va) for _, va in folds]
        tm = np.zeros((self.G, max(ntr)), np.int64)
        for g, (tr, _) in enumerate(folds):
            tm[g, :len(tr)] = tr
        self.train_mat = torch.from_numpy(tm).to(self.device)
        self.ntrain_t = torch.tensor(ntr, dtype=torch.int64, device=self.device)
        maxv = max(self.nval)
        vm = np.zeros((self.G, maxv), np.int64)
        vmask = np.zeros((self.G, maxv), np.float32)
        for g, (_, va) in enumerate(folds):
            vm[g, :len(va)] = va
            vmask[g, :len(va)] = 1.0
        self.val_mat = torch.from_numpy(vm).to(self.device)
        self.val_mask = torch.from_numpy(vmask).to(self.device)
        self.shuffle_gens = []
        for g, fid in enumerate(self.fold_ids):
            gen = torch.Generator(device=self.device)
            gen.manual_seed(_rng.stable_hash(self.member_seeds[self.gmember[g]], "shuffle", fid) & 0x7FFFFFFF)
            self.shuffle_gens.append(gen)
        if self.cfg.batching == "keras":      # in place: the captured step reads these rows
            v = np.zeros((self.steps_per_epoch, self.G), np.int32)
            for g, n in enumerate(ntr):
                for st in range(self.steps_per_epoch):
                    v[st, g] = max(0, min(self.B, n - st * self.B))
            self.epoch_valid.copy_(torch.from_numpy(v))
        self._rebind_device()
        self.result = None
        return True

    def _rebind_device(self):
        """Executor state keyed by fold id (init seeds, dropout keys)."""

    # -- shuffling -----------------------------------------------------------
    def _new_epoch_order(self):
        G, maxn = self.train_mat.shape
        # each group draws exactly ntrain keys from its own generator, so its
        # order does not depend on the other groups of the job
        keys = torch.full((G, maxn), 2.0, device=self.device)
        for g, gen in enumerate(self.shuffle_gens):
            keys[g, :self.ntrain[g]].uniform_(0.0, 1.0, generator=gen)
        order = torch.argsort(keys, dim=1, stable=True)
        perm = torch.gather(self.train_mat, 1, order)
        pos = torch.arange(self.steps_per_epoch * self.B, device=self.device)[None, :] % self.ntrain_t[:, None]
        idx = torch.gather(perm, 1, pos).view(G, self.steps_per_epoch, self.B)
        self.epoch_idx.copy_(idx.permute(1, 0, 2))
        self.step_ctr.zero_()

    def _fold_seed(self, g):
        return _rng.stable_hash(self.member_seeds[self.gmember[g]], "init", self.fold_ids[g]) & 0x7FFFFFFFFFFF

    # -- to implement ----------------------------------------------------------
    def init_params(self):
        raise NotImplementedError

    def reset_optimizer(self, lr):
        raise NotImplementedError

    def train_step(self):
        """One optimizer step for all folds; must be graph-capturable and read
        its batch from ``epoch_idx[step_ctr]`` then increment ``step_ctr``."""
        raise NotImplementedError

    def evaluate(self):
        """Return device tensors (loss_sum[G], bin_correct[G], cat_correct[G])."""
        raise NotImplementedError

    def snapshot(self):
        raise NotImplementedError

    def restore(self, snap):
        raise NotImplementedError

    def bias_state(self):
        """Clones of everything ``reset_weights`` keeps (biases; BatchNorm
        gamma / beta / running statistics)."""
        raise NotImplementedError

    def load_bias_state(self, state):
        raise NotImplementedError

    def reset_kernels(self):
        """keras_models.py:120-125 ``reset_weights``: re-run the kernel
        initialisers (Glorot, keyed by run seed / genes / fold like a fresh
        job) and keep the biases the job has trained."""
        keep = self.bias_state()
        self.init_params()
        self.load_bias_state(keep)

    # -- driver --------------------------------------------------------------
    def graph_steps(self):
        """Train steps per graph replay: the largest divisor of the epoch's
        step count up to ``cfg.graph_steps`` (default 1). One replay of a
        k-step graph is one host launch for k steps, so at small population
        sizes the host no longer paces the GPU (every step reads its batch
        through the device-side step counter, so k consecutive steps capture
        as k copies of the same launches)."""
        kmax = max(1, int(getattr(self.cfg, "graph_steps", 1) or 1))
        n = self.steps_per_epoch
        return max(d for d in range(1, min(kmax, n) + 1) if n % d == 0)

    def _capture(self):
        check_hw_queues(getattr(self, "graph_streams", 1))
        snap = self.snapshot()
        # warm-up steps read the (still all-zero, i.e. valid) batch table; the
        # shuffle streams are NOT advanced so graph and eager runs are identical
        self.step_ctr.zero_()
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            for _ in range(2):
                self.train_step()
        # Raw capture API: ``torch.cuda.graph`` would device-synchronize on
        # entry and serialise the candidates running on other streams.
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.stream(side):
            graph.capture_begin(capture_error_mode="thread_local")
            try:
                for _ in range(self._k_steps):
                    self.train_step()
            finally:
                graph.capture_end()
        torch.cuda.current_stream(self.device).wait_stream(side)
        self.restore(snap)
        return graph

    def train_steps(self, n):
        """``n`` eager training steps (executors may issue them natively)."""
        for _ in range(n):
            self.train_step()

    def launch(self):
        # use_graph None (default): the captured step graph (cfg.use_graph=False: eager
        # launches, through the native step program: -2..+12 % in a bare population
        # step depending on the box, 2.5 % slower in bench.py on two boxes --
        # profiles/graph_vs_eager_ab_r4.txt)
        ug = True if self.cfg.use_graph is None else bool(self.cfg.use_graph)
        use_graph = ug and self.device.type == "cuda" and getattr(self, "capture_ok", True)
        use_graph = use_graph and graph_or_eager(getattr(self, "graph_streams", 1))
        ctx = torch.cuda.stream(self.stream) if self.stream is not None else _nullctx()
        timed = self.device.type == "cuda"
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)] if timed else None
        with ctx:
            if timed:
                ev[0].record()
            self.init_params()
            if self.after_init is not None:
                self.after_init(self)
            self._k_steps = self.graph_steps() if use_graph else 1
            keep = getattr(self, "_graph_keep", None)
            if use_graph and keep is not None and keep[0] == self._k_steps:
                graph = keep[1]                  # rebound job: same launches, same buffers
            else:
                graph = self._capture() if use_graph else None
                if graph is not None and self.can_rebind:
                    self._graph_keep = (self._k_steps, graph)
            if timed:
                ev[1].record()
            verbose = getattr(self.cfg, "verbose", False)
            if verbose:
                n = getattr(self.cfg, "nfold", None) or (max(self.fold_ids) + 1)
                for fid in sorted(set(self.fold_ids)):
                    print("KFold {}/{}".format(fid + 1, n))
            for epochs, lr in zip(self.cfg.epochs, self.cfg.learning_rate):
                if verbose:
                    print("Training {} epochs with learning rate {}".format(epochs, lr))
                self.reset_optimizer(lr)
                for _ in range(epochs):
                    self._new_epoch_order()
                    if graph is not None:
                        for _ in range(self.steps_per_epoch // self._k_steps):
                            graph.replay()
                    else:
                        self.train_steps(self.steps_per_epoch)
            if timed:
                ev[2].record()
            self._graph = graph
            self._eval = self.evaluate()
            if timed:
                ev[3].record()
            if self.stream is not None:
                self._done = torch.cuda.Event()
                self._done.record(self.stream)
        self._phase_events = ev
        return self

    def finish(self):
        if getattr(self, "_done", None) is not None:
            self._done.synchronize()
        loss, binc, catc = (t.detach().float().cpu().numpy() for t in self._eval)
        ev = getattr(self, "_phase_events", None)
        if ev is not None:
            # device time per phase (HIP events on the job's stream)
            ev[3].synchronize()
            self.phase_ms = {"init_capture": ev[0].elapsed_time(ev[1]), "train": ev[1].elapsed_time(ev[2]),
                             "eval": ev[2].elapsed_time(ev[3])}
            self._phase_events = None
        nval = np.asarray(self.nval, np.float64)
        per = {
            "val_loss": (loss / nval).tolist(),
            "binary_accuracy": (binc / (nval * self.data.classes)).tolist(),
            "categorical_accuracy": (catc / nval).tolist(),
        }
        out = []
        for c in range(len(self.members)):
            gs = [g for g in range(self.G) if self.gmember[g] == c]
            out.append({k: [v[g] for g in gs] for k, v in per.items()})
        self._graph = None
        self.result = out if self.multi else out[0]
        return self.result


# sequential folds of the HIP executor reuse one job (module constant; tests compare both ways)
FOLD_REUSE = True


class SequentialFoldJob(object):
    """The reference's fold protocol (keras_models.py:127-143): the folds of
    the job's candidates train ONE AFTER ANOTHER; fold k+1 re-draws only the
    kernels (Glorot, keyed by fold id) and starts from the biases fold k
    trained (``reset_weights`` re-runs kernel initialisers only,
    keras_models.py:120-125). ``make(fold_index)`` builds the job of one
    fold (all candidates, one group each); everything is enqueued on the
    jobs' stream, so ``launch()`` does not block.

    With ``spec(fold_index) -> (folds, fold_ids)`` (one fold per group) an
    executor that can rebind (the HIP one) trains every fold on ONE job: the
    buffers, argument tables and captured step graph of fold 0 are reused,
    only the index tables and fold-keyed seeds change, and the biases are
    carried in place (``FOLD_REUSE = False``: a new job per fold; results are
    bit-identical either way, tests/test_hip_train.py)."""

    def __init__(self, make, nfolds, multi, spec=None):
        self.make = make
        self.nfolds = nfolds
        self.multi = multi
        self.spec = spec if FOLD_REUSE else None
        self.jobs = []
        self.phase_ms = None

    def launch(self):
        prev = None
        for f in range(self.nfolds):
            job = None
            if prev is not None and self.spec is not None and prev.can_rebind:
                # fold f-1's results stay with a shallow copy (its own eval tensors / events / sizes)
                self.jobs[-1] = copy.copy(prev)
                ctx = torch.cuda.stream(prev.stream) if prev.stream is not None else _nullctx()
                with ctx:                       # ordered after fold f-1's launches on the job stream
                    kept = prev.bias_state()
                    if prev.rebind(*self.spec(f)):
                        job = prev
                        job.after_init = _load_biases(kept)
            if job is None:
                job = self.make(f)
                if prev is not None:
                    job.after_init = _carry_biases(prev)
            job.launch()
            self.jobs.append(job)
            prev = job
        return self

    def finish(self):
        per_fold = [j.finish() for j in self.jobs]
        self.phase_ms = _sum_phases(self.jobs)
        keys = ("val_loss", "binary_accuracy", "categorical_accuracy")
        if not self.multi:
            return {k: [v for r in per_fold for v in r[k]] for k in keys}
        nmem = len(per_fold[0])
        return [{k: [v for r in per_fold for v in r[c][k]] for k in keys} for c in range(nmem)]


def _carry_biases(prev):
    def hook(job):
        job.copy_biases_from(prev)
    return hook


def _load_biases(kept):
    def hook(job):
        job.load_bias_state(kept)
    return hook


def _sum_phases(jobs):
    out = {}
    for j in jobs:
        for k, v in (getattr(j, "phase_ms", None) or {}).items():
            out[k] = out.get(k, 0.0) + v
    return out or None


class _nullctx(object):
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def loss_and_metrics(logits, onehot, mode):
    """Shared oracle of the fused softmax+loss kernel (K9)."""
    p = torch.softmax(logits.float(), dim=-1)
    if mode == "bce_compat":
        pc = p.clamp(CLIP_EPS, 1.0 - CLIP_EPS)
        per = -(onehot * torch.log(pc) + (1.0 - onehot) * torch.log(1.0 - pc)).mean(-1)
    else:
        per = -(onehot * torch.log(p.clamp_min(1e-30))).sum(-1)
    binc = (torch.round(p) == onehot).float().sum(-1)
    catc = (p.argmax(-1) == onehot.argmax(-1)).float()
    return per, binc, catc


# ---------------------------------------------------------------------------
# torch (autograd) oracle executor
# ---------------------------------------------------------------------------

class TorchFoldJob(FoldJob):
    """Stock PyTorch-ROCm ops (MIOpen grouped convs, batched GEMMs, autograd).

    Folds are batched as conv groups: activations live as ``[B, G*C, H, W]``.
    Used as the numerics oracle for the HIP path and as comparator (a).
    """

    layout = "nchw"

    def __init__(self, *a, **kw):
        super(TorchFoldJob, self).__init__(*a, **kw)
        self._check_members()
        plan, G = self.plan, self.G
        shapes = []
        for st in self._conv_specs():
            shapes.append((st.name + ".w", (G, st.cout, st.cin, st.k[0], st.k[1]), "glorot",
                           (st.cin * st.k[0] * st.k[1], st.cout * st.k[0] * st.k[1])))
            shapes.append((st.name + ".b", (G, st.cout), "zero", None))
            if self.cfg.batch_norm:
                shapes.append((st.name + ".gamma", (G, st.cout), "one", None))
                shapes.append((st.name + ".beta", (G, st.cout), "zero", None))
        shapes.append(("dense1.w", (G, plan.flatten, plan.dense_units), "glorot", (plan.flatten, plan.dense_units)))
        shapes.append(("dense1.b", (G, plan.dense_units), "zero", None))
        shapes.append(("dense2.w", (G, plan.dense_units, plan.classes), "glorot", (plan.dense_units, plan.classes)))
        shapes.append(("dense2.b", (G, plan.classes), "zero", None))
        self.shapes = shapes
        total = sum(int(np.prod(s)) for _, s, _, _ in shapes)
        self.flat = torch.zeros(total, device=self.device, requires_grad=True)
        self.m = torch.zeros(total, device=self.device)
        self.v = torch.zeros(total, device=self.device)
        self.t = torch.zeros((), device=self.device)
        self.lr = torch.zeros((), device=self.device)
        self.flat.grad = torch.zeros_like(self.flat)
        # MIOpen's algorithm search is not graph-capture safe: the stock-ops
        # comparator runs eagerly
        self.capture_ok = False
        self.amp = (self.cfg.dtype == "bf16") and self.device.type == "cuda"
        self.drop_gen = None
        # BatchNorm running statistics per conv: [2 (mean, var)][G][C]
        self.bn_run = {st.name: torch.zeros((2, G, st.cout), device=self.device) for st in self._conv_specs()} \
            if self.cfg.batch_norm else {}

    def _check_members(self):
        if len(self.members) != 1:
            raise ValueError("the torch executor trains one architecture per job (TorchPopJob: several)")

    def _conv_specs(self):
        return self.plan.convs()

    def init_params(self):
        with torch.no_grad():
            self.flat.zero_()
            off = 0
            for name, shape, kind, fans in self.shapes:
                n = int(np.prod(shape))
                if kind == "glorot":
                    limit = math.sqrt(6.0 / (fans[0] + fans[1]))
                    per = n // self.G
                    for g in range(self.G):
                        gen = torch.Generator(device=self.device)
                        gen.manual_seed(_rng.stable_hash(self._fold_seed(g), name) & 0x7FFFFFFF)
                        vals = torch.rand(per, generator=gen, device=self.device) * (2 * limit) - limit
                        self.flat[off + g * per: off + (g + 1) * per].copy_(vals)
                elif kind == "one":
                    self.flat[off:off + n].fill_(1.0)
                off += n
            for r in self.bn_run.values():
                r[0].zero_()
                r[1].fill_(1.0)

    def reset_optimizer(self, lr):
        self.m.zero_()
        self.v.zero_()
        self.t.zero_()
        self.lr.fill_(lr)

    def snapshot(self):
        return (self.flat.detach().clone(), self.m.clone(), self.v.clone(), self.t.clone(),
                {k: r.clone() for k, r in self.bn_run.items()})

    def copy_biases_from(self, other):
        """Everything ``reset_weights`` keeps (keras_models.py:120-125 re-runs
        kernel initialisers only): biases and, with BatchNorm, gamma / beta /
        running statistics, from ``other`` (same plan and folds count)."""
        with torch.no_grad():
            a, b = self._views(), other._views()
            for name, _, kind, _ in self.shapes:
                if kind in ("zero", "one"):
                    a[name].copy_(b[name])
            for k, r in self.bn_run.items():
                r.copy_(other.bn_run[k])

    def bias_state(self):
        with torch.no_grad():
            a = self._views()
            return ({name: a[name].clone() for name, _, kind, _ in self.shapes if kind in ("zero", "one")},
                    {k: r.clone() for k, r in self.bn_run.items()})

    def load_bias_state(self, state):
        with torch.no_grad():
            a = self._views()
            for name, t in state[0].items():
                a[name].copy_(t)
            for k, r in state[1].items():
                self.bn_run[k].copy_(r)

    def restore(self, snap):
        with torch.no_grad():
            self.flat.copy_(snap[0])
            self.m.copy_(snap[1])
            self.v.copy_(snap[2])
            self.t.copy_(snap[3])
            for k, r in snap[4].items():
                self.bn_run[k].copy_(r)

    def _views(self):
        # Views are rebuilt per call so their autograd nodes live on the
        # stream that runs the step (graph-capture friendly).
        out, off = {}, 0
        for name, shape, _, _ in self.shapes:
            n = int(np.prod(shape))
            out[name] = self.flat[off:off + n].view(shape)
            off += n
        return out

    def _bn(self, z, name, P, train, nval):
        """BatchNorm of a grouped conv output z [B, G*C, H, W] per group and
        channel; training statistics over the first ``nval[g]`` rows (the
        real rows of a Keras short batch), running stats with Keras momentum
        and the unbiased variance (torch.nn.BatchNorm2d's convention)."""
        G = self.G
        Bn, GC, H, W = z.shape
        C = GC // G
        zz = z.view(Bn, G, C, H, W)
        run = self.bn_run[name]
        if train:
            rows = torch.arange(Bn, device=z.device)[:, None]
            m = (rows < nval[None, :]).to(z.dtype)[:, :, None, None, None]          # [B, G, 1, 1, 1]
            n = (nval.to(z.dtype) * (H * W)).clamp_min(1.0)[None, :, None, None, None]
            mean = (zz * m).sum((0, 3, 4), keepdim=True) / n
            var = ((zz - mean) ** 2 * m).sum((0, 3, 4), keepdim=True) / n
            with torch.no_grad():
                mo = self.cfg.bn_momentum
                nn_ = n.view(1, G, 1)
                run[0].mul_(mo).add_((1.0 - mo) * mean.view(G, C))
                run[1].mul_(mo).add_((1.0 - mo) * (var.view(1, G, C) * nn_ / (nn_ - 1.0).clamp_min(1.0)).view(G, C))
        else:
            mean = run[0].view(1, G, C, 1, 1)
            var = run[1].view(1, G, C, 1, 1)
        xh = (zz - mean) * torch.rsqrt(var + self.cfg.bn_eps)
        out = xh * P[name + ".gamma"].view(1, G, C, 1, 1) + P[name + ".beta"].view(1, G, C, 1, 1)
        return out.reshape(Bn, GC, H, W)

    def _forward(self, xb, train, nval=None):
        """xb: [B, G*C, H, W] -> logits [G, B, classes]."""
        G, plan, P = self.G, self.plan, self._views()
        acts = {"input": xb}
        for st in plan.steps:
            if isinstance(st, ConvSpec):
                inp = acts[st.inputs[0]]
                for extra in st.inputs[1:]:
                    inp = inp + acts[extra]
                w = P[st.name + ".w"].reshape(G * st.cout, st.cin, st.k[0], st.k[1])
                b = P[st.name + ".b"].reshape(G * st.cout)
                z = F.conv2d(inp, w, b, padding=(st.k[0] // 2, st.k[1] // 2), groups=G)
                if self.cfg.batch_norm:
                    if nval is None:
                        nval = torch.full((G,), xb.shape[0], device=xb.device)
                    z = self._bn(z, st.name, P, train, nval)
                acts[st.name] = F.relu(z)
            else:
                src = acts[st.srcs[0]]
                acts[st.name] = F.max_pool2d(src, 2, 2)
        last = acts[plan.steps[-1].name]
        Bn = last.shape[0]
        feat = last.reshape(Bn, G, -1).permute(1, 0, 2)                     # [G, B, F]
        return self._head(feat, train, P)

    def _head(self, feat, train, P):
        """feat [G, B, F] -> logits [G, B, classes] (dense, ReLU, dropout, dense)."""
        G = self.G
        h = torch.baddbmm(P["dense1.b"][:, None, :], feat, P["dense1.w"])
        h = F.relu(h)
        if train and self.cfg.dropout > 0:
            # job-owned generators (not torch's global RNG), one per fold keyed
            # by (candidate seed, fold id): the oracle is deterministic and a
            # fold's masks do not depend on which other folds share the job
            if self.drop_gen is None:
                self.drop_gen = []
                for g in range(G):
                    gen = torch.Generator(device=self.device)
                    gen.manual_seed(_rng.stable_hash(self.member_seeds[self.gmember[g]], "dropout", self.fold_ids[g])
                                    & 0x7FFFFFFF)
                    self.drop_gen.append(gen)
            full = (self.B,) + tuple(h.shape[2:])
            keep = torch.stack([torch.rand(full, generator=gen, device=self.device) for gen in self.drop_gen])
            if keep.shape[1] != h.shape[1]:           # data-parallel slice: the full batch's masks, this rank's rows
                keep = keep[:, self._dp_rows[0]:self._dp_rows[1]]
            h = h * (keep >= self.cfg.dropout).to(h.dtype) / (1.0 - self.cfg.dropout)
        return torch.baddbmm(P["dense2.b"][:, None, :], h, P["dense2.w"])

    def _gather(self, idx):
        """idx [G, B] -> [B, G*C, H, W]."""
        G, Bn = idx.shape
        xb = self.data.x.index_select(0, idx.reshape(-1))                   # [G*B, C, H, W]
        C, H, W = xb.shape[1:]
        return xb.view(G, Bn, C, H, W).permute(1, 0, 2, 3, 4).reshape(Bn, G * C, H, W)

    def _dp(self):
        """(group, rank, world, first row, end row) of the data-parallel slice."""
        grp = self.cfg.dp_group
        if grp is None:
            return None
        if self.cfg.batch_norm:
            raise ValueError("data parallelism with BatchNorm would need synchronised batch statistics")
        import torch.distributed as dist
        world, rank = dist.get_world_size(grp), dist.get_rank(grp)
        r0, r1 = rank * self.B // world, (rank + 1) * self.B // world
        self._dp_rows = (r0, r1)
        return grp, rank, world, r0, r1

    def train_step(self):
        dp = self._dp()
        idx = self.epoch_idx.index_select(0, self.step_ctr).view(self.G, self.B)
        nval = self.epoch_valid.index_select(0, self.step_ctr).view(self.G, 1).float()
        self.step_ctr.add_(1)
        rows = torch.arange(self.B, device=self.device)[None, :].float()
        wt = (rows < nval).float() / nval.clamp_min(1.0)
        if dp is not None:                           # this rank's rows of every group's batch
            idx, wt = idx[:, dp[3]:dp[4]], wt[:, dp[3]:dp[4]]
        xb = self._gather(idx)
        yb = self.data.onehot.index_select(0, idx.reshape(-1)).view(self.G, idx.shape[1], -1)
        self.flat.grad.zero_()
        if self.amp:
            with torch.autocast(device_type="cuda", dtype=torch.bfloat16):
                logits = self._forward(xb, True, nval.view(-1))
        else:
            logits = self._forward(xb, True, nval.view(-1))
        per, _, _ = loss_and_metrics(logits, yb, self.cfg.loss)
        # mean over the real rows of each group's batch (Keras short batch)
        (per * wt).sum().backward()
        with torch.no_grad():
            g = self.flat.grad
            if dp is not None:                       # X5: sum of the slices' gradients = the full batch's
                import torch.distributed as dist
                dist.all_reduce(g, op=dist.ReduceOp.SUM, group=dp[0])
            self.t.add_(1.0)
            if self.cfg.optimizer == "sgd":       # Keras SGD: v = mu v - lr g ; p += v
                self.m.mul_(self.cfg.momentum).sub_(self.lr * g)
                self.flat.add_(self.m)
            else:
                step = self.lr * torch.sqrt(1.0 - ADAM_B2 ** self.t) / (1.0 - ADAM_B1 ** self.t)
                self.m.mul_(ADAM_B1).add_(g, alpha=1.0 - ADAM_B1)
                self.v.mul_(ADAM_B2).addcmul_(g, g, value=1.0 - ADAM_B2)
                self.flat.sub_(step * self.m / (self.v.sqrt() + ADAM_EPS))

    def evaluate(self):
        G = self.G
        loss = torch.zeros(G, device=self.device)
        binc = torch.zeros(G, device=self.device)
        catc = torch.zeros(G, device=self.device)
        maxv = self.val_mat.shape[1]
        eb = self.cfg.eval_batch
        with torch.no_grad():
            for s in range(0, maxv, eb):
                idx = self.val_mat[:, s:s + eb]
                mask = self.val_mask[:, s:s + eb]
                xb = self._gather(idx)
                yb = self.data.onehot.index_select(0, idx.reshape(-1)).view(G, idx.shape[1], -1)
                if self.amp:
                    with torch.autocast(device_type="cuda", dtype=torch.bfloat16):
                        logits = self._forward(xb, False)
                else:
                    logits = self._forward(xb, False)
                per, b, c = loss_and_metrics(logits, yb, self.cfg.loss)
                loss += (per * mask).sum(-1)
                binc += (b * mask).sum(-1)
                catc += (c * mask).sum(-1)
        return loss, binc, catc


class TorchPopJob(TorchFoldJob):
    """Population-batched stock-PyTorch executor (comparator (a) with the
    HIP path's batching): several architectures of one search
    space train in ONE set of grouped convolutions. Every group (member,
    fold) runs the *superset* network of the space -- every node of every
    stage -- and per-group 0/1 masks select its DAG
    (genome.decode_stage): node i reads ``E_i x_in + sum_j A_ij n_j``, the
    output conv reads ``sum_j O_j n_j``, and a stage without a DAG passes
    its input conv through (``D``). Masked terms add exact zeros to the
    ReLU outputs, so an active node computes what the one-architecture
    oracle computes; inactive nodes get zero gradients and Adam leaves
    them at their initial values. Weights are initialised per (member
    seed, fold id, tensor name) like TorchFoldJob. Cost: the superset's
    convolutions for every group (isolated nodes and DAG-less stages are
    computed and discarded)."""

    def _check_members(self):
        p0 = self.members[0][0]
        key = (p0.nodes, p0.input_shape, p0.kernels_per_layer, p0.kernel_sizes, p0.dense_units, p0.classes)
        for p, _, _ in self.members:
            if (p.nodes, p.input_shape, p.kernels_per_layer, p.kernel_sizes, p.dense_units, p.classes) != key:
                raise ValueError("a population job needs one search space (nodes, shapes, kernels, head)")
        self._build_masks()

    def _conv_specs(self):
        p0 = self.plan
        specs, c = [], p0.input_shape[2]
        for s, cout in enumerate(p0.kernels_per_layer):
            specs.append(ConvSpec("s{}_in".format(s + 1), None, c, cout, tuple(p0.kernel_sizes[s]), s))
            if s in self._dag_stages:
                for i in range(p0.nodes[s]):
                    specs.append(ConvSpec("s{}_n{}".format(s + 1, i), None, cout, cout, (3, 3), s))
                specs.append(ConvSpec("s{}_out".format(s + 1), None, cout, cout, (3, 3), s))
            c = cout
        return specs

    def _build_masks(self):
        from .genome import decode_stage
        p0, G = self.plan, self.G
        self._dag_stages, self._masks = set(), {}
        for s, K in enumerate(p0.nodes):
            A = np.zeros((G, K, K), np.float32)
            E = np.zeros((G, K), np.float32)
            O = np.zeros((G, K), np.float32)
            D = np.zeros((G,), np.float32)
            for g in range(G):
                bits = self.members[self.gmember[g]][0].genes["S_{}".format(s + 1)]
                if not any(b == "1" for b in bits):
                    continue
                preds, _succs, active, outputs = decode_stage(bits, K)
                D[g] = 1.0
                for i in range(K):
                    if not active[i]:
                        continue
                    if preds[i]:
                        A[g, i, preds[i]] = 1.0
                    else:
                        E[g, i] = 1.0
                O[g, outputs] = 1.0
            if D.any():
                self._dag_stages.add(s)
            t = lambda v: torch.from_numpy(v).to(self.device)      # noqa: E731
            self._masks[s] = {"A": t(A), "E": t(E), "O": t(O), "D": t(D), "A_np": A, "E_np": E}

    def _forward(self, xb, train, nval=None):
        G, p0, P = self.G, self.plan, self._views()

        def conv(name, inp, k):
            nonlocal nval
            w = P[name + ".w"]
            z = F.conv2d(inp, w.reshape(G * w.shape[1], w.shape[2], k[0], k[1]), P[name + ".b"].reshape(-1),
                         padding=(k[0] // 2, k[1] // 2), groups=G)
            if self.cfg.batch_norm:
                if nval is None:
                    nval = torch.full((G,), xb.shape[0], device=xb.device)
                z = self._bn(z, name, P, train, nval)
            return F.relu(z)

        def scale(t, m):
            Bn, GC, H, W = t.shape
            return (t.view(Bn, G, GC // G, H, W) * m.view(1, G, 1, 1, 1)).view(Bn, GC, H, W)

        cur = xb
        for s, K in enumerate(p0.nodes):
            x_in = conv("s{}_in".format(s + 1), cur, p0.kernel_sizes[s])
            if s in self._dag_stages:
                m = self._masks[s]
                acts = []
                for i in range(K):
                    inp = scale(x_in, m["E"][:, i]) if m["E_np"][:, i].any() else None
                    for j in range(i):
                        if not m["A_np"][:, i, j].any():
                            continue
                        term = scale(acts[j], m["A"][:, i, j])
                        inp = term if inp is None else inp + term
                    if inp is None:                     # isolated in every group: zero input
                        inp = torch.zeros_like(x_in)
                    acts.append(conv("s{}_n{}".format(s + 1, i), inp, (3, 3)))
                out_in = None
                for j in range(K):
                    term = scale(acts[j], m["O"][:, j])
                    out_in = term if out_in is None else out_in + term
                out = conv("s{}_out".format(s + 1), out_in, (3, 3))
                x_in = scale(out, m["D"]) + scale(x_in, 1.0 - m["D"])
            cur = F.max_pool2d(x_in, 2, 2)
        Bn = cur.shape[0]
        feat = cur.reshape(Bn, G, -1).permute(1, 0, 2)
        return self._head(feat, train, P)


def _one_job(backend, plan, x, y, folds, cfg, device, fold_ids, stream):
    if backend == "torch":
        return TorchFoldJob(plan, x, y, folds, cfg, device, fold_ids=fold_ids, stream=stream)
    if backend == "hip":
        from .cnn_hip import HipPopJob
        return HipPopJob(plan, x, y, folds, cfg, device, fold_ids=fold_ids, stream=stream)
    raise ValueError("unknown backend {!r}".format(backend))


def make_job(backend, plan, x, y, folds, cfg, device, fold_ids=None, stream=None):
    """Job training ``folds`` of one architecture: concurrent folds
    (``cfg.reset == "all"``) or the reference's sequential folds with
    carried-over biases (``"kernels"``)."""
    ids = list(range(len(folds))) if fold_ids is None else list(fold_ids)
    if cfg.reset == "all" or len(folds) == 1:
        return _one_job(backend, plan, x, y, folds, cfg, device, ids, stream)
    return SequentialFoldJob(lambda f: _one_job(backend, plan, x, y, [folds[f]], cfg, device, [ids[f]], stream),
                             len(folds), multi=False, spec=lambda f: ([folds[f]], [ids[f]]))


def make_population_job(backend, members, x, y, cfg, device, stream=None):
    """One job training several architectures at once: ``members`` is a list
    of ``(plan, folds, fold_ids)``; ``finish()`` returns one result dict per
    member. The HIP executor batches them into shared launches (with
    ``reset="kernels"`` one launch set per fold position, folds in sequence);
    the torch executor batches them too (:class:`TorchPopJob`: superset
    network + per-group DAG masks, comparator (a))."""
    if backend == "hip":
        from .cnn_hip import HipPopJob as Job
    elif backend == "torch":
        Job = TorchPopJob
    else:
        raise ValueError("unknown backend {!r}".format(backend))
    nf = {len(f) for _, f, _ in members}
    if cfg.reset == "all" or nf == {1}:
        return Job(None, x, y, None, cfg, device, stream=stream, members=members)
    if len(nf) != 1:
        raise ValueError("sequential-fold population jobs need the same number of folds per member")

    def make(k):
        return Job(None, x, y, None, cfg, device, stream=stream,
                   members=[(p, [f[k]], [ids[k]]) for p, f, ids in members])

    def spec(k):
        return [f[k] for _, f, _ in members], [ids[k] for _, _, ids in members]
    return SequentialFoldJob(make, nf.pop(), multi=True, spec=spec)


def default_backend(device):
    dev = torch.device(device)
    if dev.type != "cuda":
        return "torch"
    return "hip"
