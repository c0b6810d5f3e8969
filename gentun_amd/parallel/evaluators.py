"""Local (single-process) evaluation strategies.

The reference evaluates pending individuals one after another, lazily, inside
``max(..., key=get_fitness)`` (gentun/populations.py:55-58). On MI355X one
Genetic-CNN candidate (even fold-batched) is far too small to fill 256 CUs
(SURVEY.md §7.3 hard part 1), so :class:`LocalBatchEvaluator` enqueues the
fold-batched training graphs of several candidates on separate HIP streams
and lets the GPU run them concurrently; the host never blocks until the
results are read back.
"""

import os
import time

import torch

from ..utils import rng as _rng


class SequentialEvaluator(object):
    """Reference behaviour: evaluate one individual at a time."""

    def __init__(self, cache=False, event_log=None):
        self.cache = {} if cache else None
        self.event_log = event_log
        self.evaluations = 0

    def _cached(self, ind):
        if self.cache is None:
            return False
        hit = self.cache.get(ind.genes_key())
        if hit is not None:
            ind.set_fitness(hit[0])
            ind.fold_scores = hit[1]
            return True
        return False

    def _store(self, ind):
        if self.cache is not None:
            self.cache[ind.genes_key()] = (ind.fitness, ind.fold_scores)

    def evaluate(self, individuals):
        n = 0
        for ind in individuals:
            if ind.get_fitness_status() or self._cached(ind):
                continue
            t0 = time.perf_counter()
            ind.evaluate_fitness()
            n += 1
            self._store(ind)
            self._log(ind, time.perf_counter() - t0)
        self.evaluations += n
        return n

    def _log(self, ind, wall):
        if self.event_log is not None:
            self.event_log.write("evaluation", genes=ind.get_genes(), fitness=ind.fitness,
                                 fold_scores=ind.fold_scores, wall_s=wall,
                                 phase_ms=getattr(ind, "phase_ms", None))


class LocalBatchEvaluator(SequentialEvaluator):
    """Evaluate a batch of individuals on ONE GPU.

    Genetic-CNN candidates (species exposing ``build_fitness_model``) on the
    HIP backend are trained as *population jobs*: up to ``pop_batch``
    candidates x all their folds share every kernel launch
    (:class:`~gentun_amd.models.cnn_hip.HipPopJob`); up to ``streams`` such
    jobs run concurrently on separate HIP streams. The torch executor does the
    same with ``torch_pop`` (:class:`~gentun_amd.models.cnn_engine.TorchPopJob`),
    else it runs one fold-batched job per candidate per stream; other species
    fall back to sequential evaluation.
    """

    def __init__(self, device=None, streams=2, cache=False, event_log=None, pop_batch=16, torch_pop=None):
        super(LocalBatchEvaluator, self).__init__(cache=cache, event_log=event_log)
        # population-batch the torch executor too (torch_pop=True: TorchPopJob, comparator (a));
        # otherwise the torch oracle trains one candidate per job
        self.torch_pop = bool(torch_pop)
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
                else torch.device("cpu")
        self.device = torch.device(device)
        self.nstreams = max(1, int(streams))
        self.pop_batch = max(1, int(pop_batch))
        self._streams = None

    def streams(self):
        if self._streams is None:
            if self.device.type == "cuda":
                self._streams = [torch.cuda.Stream(self.device) for _ in range(self.nstreams)]
            else:
                self._streams = [None]
        return self._streams

    def evaluate(self, individuals):
        batch, rest = [], []
        for ind in individuals:
            if ind.get_fitness_status() or self._cached(ind):
                continue
            (batch if hasattr(ind, "build_fitness_model") else rest).append(ind)
        n = super(LocalBatchEvaluator, self).evaluate(rest)
        if batch:
            n += self.evaluate_models(batch)
        return n

    def evaluate_models(self, individuals):
        """Train ``individuals`` (all folds); results land in each individual."""
        def done(ind, model, res, wall, _tag):
            ind.set_fitness(model.collect([res]))
            ind.fold_scores = list(model.fold_scores)
            ind.fold_metrics = dict(model.fold_metrics or {})
            self._store(ind)
            self._log(ind, wall)

        run_cnn_units([(ind, None, None) for ind in individuals], self, done)
        self.evaluations += len(individuals)
        return len(individuals)


def _chunks(units, nchunks):
    """Split cost-sorted units into ``nchunks`` groups of near-equal cost (LPT)."""
    bins = [[] for _ in range(nchunks)]
    load = [0.0] * nchunks
    for u in units:
        k = min(range(nchunks), key=lambda i: (load[i], len(bins[i])))
        bins[k].append(u)
        load[k] += u[3]
    return [b for b in bins if b]





def run_cnn_units(units, evaluator, done):
    """Train Genetic-CNN work units ``(ind, fold_ids or None, tag)`` on the
    evaluator's device and call ``done(ind, model, result, wall_s, tag)`` per unit
    (``result`` = per-fold metric lists of the unit's folds).

    ``units`` may be an iterator (dynamic scheduling claims units lazily):
    units are pulled ``pop_batch`` at a time whenever a stream is free."""
    streams = evaluator.streams() if hasattr(evaluator, "streams") else [None]
    device = getattr(evaluator, "device", None)
    pop_batch = getattr(evaluator, "pop_batch", 1)
    from ..models import cnn_engine as E
    it = iter(units)
    window = []          # (job, [(ind, model, tag)], t0)

    def retire(entry):
        job, items, t0, multi = entry
        res = job.finish()
        res = res if multi else [res]
        wall = time.perf_counter() - t0
        phase = getattr(job, "phase_ms", None) or _merge_phases(getattr(job, "jobs", ()))
        for (ind, model, tag), r in zip(items, res):
            ind.phase_ms = phase            # device ms per phase of the (shared) job
            done(ind, model, r, wall, tag)

    pending = []          # (ind, model, fold_ids, cost, tag, groups)
    k = 0
    exhausted = False

    def groups_of(entries):
        return sum(e[5] for e in entries)

    max_groups = None     # groups (candidate x fold pairs) per population job
    while True:
        if not exhausted and (max_groups is None or groups_of(pending) < max_groups * len(streams)):
            # pull enough units to fill every stream with a batch of groups
            while max_groups is None or groups_of(pending) < max_groups * len(streams):
                nxt = next(it, None)
                if nxt is None:
                    exhausted = True
                    break
                ind, fold_ids, tag = nxt
                model = ind.build_fitness_model(device=device)
                cost = float(ind.cost()) if hasattr(ind, "cost") else 1.0
                nf = len(fold_ids) if fold_ids is not None else model.nfold
                if max_groups is None:
                    max_groups = pop_batch * model.nfold
                pending.append((ind, model, fold_ids, cost * nf, tag, nf))
        if not pending:
            break
        if len(window) >= len(streams):
            retire(window.pop(0))
        pending.sort(key=lambda e: -e[3])
        backends = {e[1].backend for e in pending}
        torch_pop = getattr(evaluator, "torch_pop", False)
        batched = pop_batch > 1 and (backends == {"hip"} or (torch_pop and backends == {"torch"}))
        if batched:
            free = len(streams) - len(window)
            nchunks = min(free, max(1, -(-groups_of(pending) // max_groups))) if exhausted else 1
            take, ng = [], 0
            for e in pending:
                if take and ng + e[5] > max_groups * nchunks:
                    break
                take.append(e)
                ng += e[5]
            pending = pending[len(take):]
            chunks = _chunks(take, nchunks)
            for ch in chunks:
                if len(window) >= len(streams):
                    retire(window.pop(0))
                stream = streams[k % len(streams)]
                k += 1
                _check_shared_settings(ch)
                members, items = [], []
                for ind, model, fold_ids, _c, tag, _g in ch:
                    members.append(model.member(fold_ids))
                    items.append((ind, model, tag))
                m0 = ch[0][1]
                job = E.make_population_job(m0.backend, members, m0.x_train, m0.y_train, m0.cfg, m0.device,
                                            stream=stream)
                t0 = time.perf_counter()
                job.launch()
                window.append((job, items, t0, True))
        else:
            ind, model, fold_ids, _c, tag, _g = pending.pop(0)
            stream = streams[k % len(streams)]
            k += 1
            jobs = model.make_jobs(stream=stream, fold_ids=fold_ids)
            t0 = time.perf_counter()
            for job in jobs:
                job.launch()
            window.append((_MultiJob(jobs), [(ind, model, tag)], t0, False))
    for entry in window:
        retire(entry)


def _settings_key(model):
    """Everything a population job takes from its first member and applies
    to all (training config, dataset identity, search space)."""
    c = model.cfg
    return (id(model.x_train), id(model.y_train), model.backend, str(model.device), model.nfold,
            c.epochs, c.learning_rate, c.batch_size, c.dropout, c.loss, c.dtype, c.seed, c.optimizer, c.momentum,
            getattr(c, "reset", None), getattr(c, "batching", None), getattr(c, "batch_norm", None),
            model.nodes, model.input_shape, model.kernels_per_layer, model.kernel_sizes, model.dense_units,
            model.classes)


def _check_shared_settings(chunk):
    """A population job trains every member with the first member's settings:
    refuse a batch that mixes settings instead of training some candidates
    with another candidate's hyper-parameters."""
    k0 = _settings_key(chunk[0][1])
    for e in chunk[1:]:
        if _settings_key(e[1]) != k0:
            raise ValueError("population job members differ in training settings / dataset / search space; "
                             "evaluate them in separate batches")


def _merge_phases(jobs):
    out = {}
    for j in jobs:
        for k, v in (getattr(j, "phase_ms", None) or {}).items():
            out[k] = out.get(k, 0.0) + v
    return out or None


class _MultiJob(object):
    """Several per-fold-group jobs of one candidate seen as one result."""

    def __init__(self, jobs):
        self.jobs = jobs

    def finish(self):
        merged = {"val_loss": [], "binary_accuracy": [], "categorical_accuracy": []}
        for job in self.jobs:
            r = job.finish()
            for k2 in merged:
                merged[k2].extend(r[k2])
        return merged


def stable_order_key(ind):
    return _rng.stable_hash(ind.genes_key())
