"""Local (single-process) evaluation strategies.

The reference evaluates pending individuals one after another, lazily, inside
``max(..., key=get_fitness)`` (gentun/populations.py:55-58). On MI355X one
Genetic-CNN candidate (even fold-batched) is far too small to fill 256 CUs
(SURVEY.md §7.3 hard part 1), so :class:`LocalBatchEvaluator` enqueues the
fold-batched training graphs of several candidates on separate HIP streams
and lets the GPU run them concurrently; the host never blocks until the
results are read back.
"""

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
                                 fold_scores=ind.fold_scores, wall_s=wall)


class LocalBatchEvaluator(SequentialEvaluator):
    """Evaluate a batch of individuals on ONE GPU with ``streams`` concurrent
    candidates (one HIP stream each; every candidate's training is a graph
    replay loop enqueued asynchronously).

    Species that expose ``build_fitness_model`` (Genetic-CNN) run
    concurrently; other species fall back to sequential evaluation.
    """

    def __init__(self, device=None, streams=4, cache=False, event_log=None):
        super(LocalBatchEvaluator, self).__init__(cache=cache, event_log=event_log)
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
                else torch.device("cpu")
        self.device = torch.device(device)
        self.nstreams = max(1, int(streams))
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

    def evaluate_models(self, individuals, order=None):
        """Run ``individuals`` concurrently; results land in each individual."""
        streams = self.streams()
        # Largest first (LPT) keeps the tail short.
        if order is None:
            order = sorted(range(len(individuals)),
                           key=lambda i: -individuals[i].cost() if hasattr(individuals[i], "cost") else 0)
        window = []          # (ind, model, jobs, t0)
        k = 0

        def retire(entry):
            ind, model, jobs, t0 = entry
            results = [job.finish() for job in jobs]
            ind.set_fitness(model.collect(results))
            ind.fold_scores = list(model.fold_scores)
            self._store(ind)
            self._log(ind, time.perf_counter() - t0)

        for i in order:
            ind = individuals[i]
            if len(window) >= len(streams):
                retire(window.pop(0))
            stream = streams[k % len(streams)]
            k += 1
            model = ind.build_fitness_model(device=self.device)
            jobs = model.make_jobs(stream=stream)
            t0 = time.perf_counter()
            for job in jobs:
                job.launch()
            window.append((ind, model, jobs, t0))
        for entry in window:
            retire(entry)
        self.evaluations += len(individuals)
        return len(individuals)


def stable_order_key(ind):
    return _rng.stable_hash(ind.genes_key())
