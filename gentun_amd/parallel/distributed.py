"""Master/evaluator protocol over collectives (RCCL on MI355X).

Reference: ``DistributedPopulation`` / ``DistributedGridPopulation``
(gentun/master.py:82-145) fan jobs out as JSON over RabbitMQ, one connection
+ one thread per job, and ``GentunWorker`` (gentun/worker.py:13-66) consumes
them. Here every rank is a persistent evaluator
(one per GPU) and rank 0 also runs the GA:

per generation (collectives X2/X3 of SURVEY.md §2.6)
  1. rank 0 broadcasts ``int64[5]`` = (command, generation, P, nfold, blob?),
     the species' ``additional_parameters`` as a JSON blob (X1, only when it
     changed), and the genome table ``float64[U, 4 + width]`` = (candidate
     slot, owner rank, fold mask, population index, encoded genes) for the
     ``U`` work units;
  2. every rank evaluates the units it owns (several concurrently on its GPU,
     :class:`~gentun_amd.parallel.evaluators.LocalBatchEvaluator`);
  3. one ``all_gather`` of ``float64[U, 3 + 2 nfold]`` = (status, fitness,
     wall_s, fold scores, secondary fold scores -- categorical accuracy of a
     Genetic-CNN whose fitness is the reference's binary accuracy) -- a few
     KB, latency-bound on xGMI;
  4. rank 0 merges fold groups per candidate, re-evaluates failed units
     locally once (worst fitness if that fails too) and breeds.

Observability: the reference's progress lines are kept --
" [.] Evaluating individual i" on the evaluating rank (gentun/worker.py:43)
and " [*] Got fitness for individual i" on rank 0 once the gather delivered
it (gentun/master.py:72), ``i`` = the individual's population index -- and
rank 0 writes one ``evaluation`` JSONL event per work unit of every rank
(rank, GA generation, dispatch, population index, genes, folds, fold scores,
fitness, wall_s) from the gathered table, so a distributed run's event log
is as complete as a single-process one's.

Failure handling (:mod:`gentun_amd.parallel.fault`):
per-unit status codes with one local retry on rank 0; a per-rank watchdog
(``GENTUN_WATCHDOG``) that turns a dead or hung peer into a clean process
exit sized from measured generation times; restart of the whole group from
the last generation checkpoint (``torchrun --max-restarts``, CLI
``--resume auto``); fault injection ``GENTUN_FAULT="rank:generation:kind"``,
kind = ``raise`` | ``exit`` | ``hang``.
"""

import json
import os
import time
import warnings

import numpy as np

from ..populations import Population, GridPopulation
from .comm import LocalComm, from_env
from . import fault as _fault
from .evaluators import LocalBatchEvaluator
from .scheduler import balanced_round, lpt_assign, make_units

CMD_STOP, CMD_EVAL, CMD_SYNC = 0, 1, 2
ST_NONE, ST_OK, ST_ERR = 0.0, 1.0, 2.0


# ---------------------------------------------------------------------------
# genome codec
# ---------------------------------------------------------------------------

class GenomeCodec(object):
    """Encode genes as a float64 row (bits -> 0/1, numbers as-is)."""

    def __init__(self, genome):
        self.names = sorted(genome)
        self.genome = genome
        self.kind = []
        self.width = 0
        for n in self.names:
            spec = genome[n]
            if isinstance(spec, int) and not isinstance(spec, bool):      # bit string of `spec` bits
                self.kind.append(("bits", spec))
                self.width += spec
            else:
                is_int = isinstance(spec[0], int) and not isinstance(spec[0], bool)
                self.kind.append(("int" if is_int else "float", 1))
                self.width += 1

    def encode(self, genes):
        row = np.zeros(self.width, np.float64)
        o = 0
        for n, (kind, w) in zip(self.names, self.kind):
            v = genes[n]
            if kind == "bits":
                row[o:o + w] = [1.0 if c == '1' else 0.0 for c in v]
            else:
                row[o] = float(v)
            o += w
        return row

    def decode(self, row):
        genes, o = {}, 0
        for n, (kind, w) in zip(self.names, self.kind):
            if kind == "bits":
                genes[n] = ''.join('1' if x > 0.5 else '0' for x in row[o:o + w])
            elif kind == "int":
                genes[n] = int(round(row[o]))
            else:
                genes[n] = float(row[o])
            o += w
        return genes


def _jsonable(d):
    out = {}
    for k, v in d.items():
        out[k] = list(v) if isinstance(v, tuple) else v
    return out


def _tuplify(v):
    if isinstance(v, list):
        return tuple(_tuplify(x) for x in v)
    return v


def _fault_hook(rank, generation):
    _fault.inject(rank, generation)


class _Unit(object):
    """A (candidate, fold-group) work unit materialised on one rank."""

    def __init__(self, slot, ind, fold_ids):
        self.slot = slot
        self.ind = ind
        self.fold_ids = fold_ids


def evaluate_units(units, evaluator, nfold, rank, generation, on_take=None):
    """Evaluate this rank's units; returns ``{unit_index: row}``.

    ``units`` is a list of ``(unit_index, _Unit)`` (static schedule) or a
    :class:`UnitClaimer` (dynamic schedule: units are claimed from the job-wide
    ticket counter one at a time, whenever this rank has a free slot).
    ``on_take(entry)`` is called as each unit is taken (progress lines)."""
    rows = {}
    source = units if isinstance(units, UnitClaimer) else _StaticSource(units)
    source.on_take = on_take
    try:
        _fault_hook(rank, generation)
    except Exception as exc:     # noqa: BLE001
        # a failed rank takes no work: dynamic units go to the other ranks,
        # its static units come back empty and the master re-evaluates them
        warnings.warn("evaluation failed on rank {}: {}".format(rank, exc))
        return rows
    if source.kind() == "cnn":
        try:
            rows.update(_evaluate_cnn_units(source, evaluator, nfold))
        except Exception as exc:     # noqa: BLE001
            warnings.warn("CNN evaluation failed on rank {}: {}".format(rank, exc))
            for ui, u in source.taken():
                if ui not in rows:
                    rows[ui] = _row(ST_ERR, np.nan, 0.0, [], nfold, u.fold_ids)
        return rows
    for ui, u in source:
        t0 = time.perf_counter()
        try:
            _localize_device(u.ind, evaluator)
            u.ind.evaluate_fitness()
            scores = u.ind.fold_scores or []
            aux = (getattr(u.ind, "fold_metrics", None) or {}).get("categorical_accuracy")
            rows[ui] = _row(ST_OK, u.ind.fitness, time.perf_counter() - t0, scores, nfold, u.fold_ids, aux=aux)
        except Exception as exc:     # noqa: BLE001 -- reported as a status code
            warnings.warn("evaluation failed on rank {}: {}".format(rank, exc))
            rows[ui] = _row(ST_ERR, np.nan, time.perf_counter() - t0, [], nfold, u.fold_ids)
    return rows


class _StaticSource(object):
    """Pre-assigned units, most expensive first (so long jobs start early)."""

    on_take = None

    def __init__(self, units):
        self.units = sorted(units, key=lambda e: -_unit_cost(e[1]))
        self._taken = []

    def kind(self):
        return "cnn" if self.units and hasattr(self.units[0][1].ind, "build_fitness_model") else "other"

    def __iter__(self):
        for e in self.units:
            self._taken.append(e)
            if self.on_take is not None:
                self.on_take(e)
            yield e

    def taken(self):
        return list(self._taken)


class UnitClaimer(object):
    """Dynamic schedule: iterate units by claiming ``comm.ticket(key)``.

    The master orders the unit table by descending cost, so claiming in
    ticket order is on-line LPT: every rank takes the most expensive unit
    nobody has started whenever it has capacity (the pull-queue behaviour of
    the reference's RabbitMQ workers, gentun/worker.py:59-63, without a
    broker)."""

    on_take = None

    def __init__(self, comm, key, n_units, make_unit, kind):
        self.comm = comm
        self.key = key
        self.n = n_units
        self.make_unit = make_unit
        self._kind = kind
        self._taken = []

    def kind(self):
        return self._kind

    def __iter__(self):
        while True:
            k = self.comm.ticket(self.key)
            if k >= self.n:
                return
            e = (k, self.make_unit(k))
            self._taken.append(e)
            if self.on_take is not None:
                self.on_take(e)
            yield e

    def taken(self):
        return list(self._taken)


def _unit_cost(u):
    c = float(u.ind.cost()) if hasattr(u.ind, "cost") else 1.0
    return c * len(u.fold_ids)


def _evaluate_cnn_units(source, evaluator, nfold):
    """Train this rank's units as population jobs (up to ``pop_batch``
    candidates x folds per launch, one job per evaluator stream in flight).
    Units are pulled from ``source`` only when a stream frees up, which is
    what makes dynamic claiming balance the ranks."""
    from .evaluators import run_cnn_units
    rows = {}

    def done(ind, model, res, wall, ui):
        scores = res[model.primary_metric()]
        u = units_by_index[ui]
        rows[ui] = _row(ST_OK, float(np.mean(scores)), wall, scores, nfold, u.fold_ids,
                        aux=res.get("categorical_accuracy"))

    units_by_index = {}

    def gen():
        for ui, u in source:
            units_by_index[ui] = u
            yield (u.ind, u.fold_ids, ui)

    run_cnn_units(gen(), evaluator, done)
    return rows


def row_width(nfold):
    return 3 + 2 * nfold


TABLE_HDR = 4       # genome table columns before the encoded genes: slot, owner, fold mask, population index


def _row(status, fitness, wall, scores, nfold, fold_ids, aux=None):
    row = np.full(row_width(nfold), np.nan, np.float64)
    row[0], row[1], row[2] = status, fitness, wall
    for j, f in enumerate(fold_ids[:len(scores)]):
        row[3 + f] = scores[j]
    for j, f in enumerate(fold_ids[:len(aux or ())]):
        row[3 + nfold + f] = aux[j]
    return row


# ---------------------------------------------------------------------------
# master side
# ---------------------------------------------------------------------------

class AllEvaluationsFailed(RuntimeError):
    """Every candidate of a dispatch failed, on its rank and on the retry
    round: a search on worst-fitness placeholders is meaningless, and resuming
    from the checkpoint would fail the same way (the CLI maps this, and only
    this, to the non-restartable exit code). Raised after the round's
    all_gather, so the evaluator ranks wait in the next broadcast and a STOP
    message reaches them."""


class DistributedPopulation(Population):
    """Population whose pending individuals are evaluated by all ranks.

    Signature-compatible with gentun/master.py:88-90. ``host``/``port`` map
    to ``MASTER_ADDR``/``MASTER_PORT`` when the process group still has to be
    created; ``user``/``password``/``rabbit_queue`` have no meaning without a
    broker and are accepted for compatibility.
    """

    def __init__(self, species, x_train=None, y_train=None, individual_list=None, size=None,
                 crossover_rate=0.5, mutation_rate=0.015, maximize=True, additional_parameters=None,
                 host='localhost', port=5672, user='guest', password='guest', rabbit_queue='rpc_queue',
                 comm=None, evaluator=None, split_folds=True, schedule="auto", event_log=None, verbose=True):
        self.comm = comm if comm is not None else _comm_from_args(host, port)
        # JSONL sink for per-unit evaluation events (the GA attaches its own log when this is None)
        self.event_log = event_log
        self.verbose = verbose
        self.ga_generation = None          # set by the GA: the generation being evaluated
        if evaluator is None:
            evaluator = LocalBatchEvaluator()
        if schedule not in ("auto", "dynamic", "lpt"):
            raise ValueError("schedule must be 'auto', 'dynamic' or 'lpt'")
        if schedule == "auto":
            # a population-batched evaluator trains all of a rank's candidates in
            # shared launches: balance the per-rank SUM of costs up front (LPT);
            # dynamic claiming in cost order would hand one rank the most expensive
            # batch. One-at-a-time evaluators keep the pull-queue behaviour.
            schedule = "lpt" if getattr(evaluator, "pop_batch", 1) > 1 else "dynamic"
        self.local_evaluator = evaluator
        self.split_folds = split_folds
        self.schedule = schedule
        self.credentials = {'host': host, 'port': port, 'user': user, 'password': password,
                            'rabbit_queue': rabbit_queue}
        self.generation_counter = 0
        self.last_dispatch = None
        super(DistributedPopulation, self).__init__(
            species, x_train, y_train, individual_list, size, crossover_rate, mutation_rate, maximize,
            additional_parameters, evaluator=None)

    def empty_like(self, individual_list=None):
        pop = DistributedPopulation.__new__(DistributedPopulation)
        pop.comm = self.comm
        pop.local_evaluator = self.local_evaluator
        pop.split_folds = self.split_folds
        pop.schedule = self.schedule
        pop.credentials = dict(self.credentials)
        pop.generation_counter = self.generation_counter
        pop.last_dispatch = None
        pop.event_log = self.event_log
        pop.verbose = self.verbose
        pop.ga_generation = self.ga_generation
        Population.__init__(pop, self.species, self.x_train, self.y_train,
                            individual_list=[] if individual_list is None else individual_list,
                            crossover_rate=self.crossover_rate, mutation_rate=self.mutation_rate,
                            maximize=self.maximize, additional_parameters=self.additional_parameters)
        return pop

    def get_fittest(self):
        self.evaluate_in_parallel()
        return Population.get_fittest(self)

    def evaluate_pending(self):
        return self.evaluate_in_parallel()

    def evaluate_in_parallel(self, limit=None):
        """Dispatch pending individuals to every rank and collect fitness.
        ``limit``: evaluate at most that many (in population order) -- one
        evaluation *round*; the rest stay pending.

        Failed units (status codes in the gather) are re-queued ONCE as a
        second dispatched round on the ranks that did not fail (SURVEY.md
        §5.3): every rank takes part, so no evaluator sits in a collective
        while rank 0 retrains candidates on its own (their watchdogs stay
        inside one dispatch's budget). A candidate that fails again gets the
        worst fitness. With one rank the retry is a local re-evaluation."""
        todo = self.pending()
        if limit is not None:
            todo = todo[:max(0, int(limit))]
        if not todo:
            return 0
        t0 = time.perf_counter()
        merged, info = self._dispatch(todo)
        failed = [slot for slot in range(len(todo)) if merged[slot][0] != ST_OK]
        if failed and self.comm.world_size > 1:
            again, _ = self._dispatch([todo[slot] for slot in failed], exclude=info["failed_ranks"])
            for slot, res in zip(failed, again):
                merged[slot] = res
        nworst = 0
        for slot, ind in enumerate(todo):
            status, fitness, scores, aux = merged[slot]
            if status != ST_OK:
                if self.comm.world_size == 1:
                    try:
                        ind.set_fitness(None)
                        ind.evaluate_fitness()
                        continue
                    except Exception as exc:   # noqa: BLE001
                        warnings.warn("re-evaluation of slot {} failed: {}".format(slot, exc))
                else:
                    warnings.warn("slot {} failed on its rank and on the retry round".format(slot))
                ind.set_fitness(float("-inf") if self.maximize else float("inf"))
                nworst += 1
            else:
                ind.set_fitness(fitness)
                ind.fold_scores = scores
                if aux is not None:
                    ind.fold_metrics = dict(getattr(ind, "fold_metrics", None) or {}, categorical_accuracy=aux)
            if self.verbose:
                print(" [*] Got fitness for individual {}".format(self._pop_index(ind)))
        if len(todo) > 1 and nworst == len(todo):
            # nothing evaluated anywhere (a lost device, a broken build): a search on worst-fitness
            # placeholders is meaningless -- stop loudly instead of breeding from them
            raise AllEvaluationsFailed("every evaluation of dispatch {} failed (and its retry)".format(
                self.generation_counter))
        self.last_dispatch = {"units": info["units"], "candidates": len(todo), "retried": len(failed),
                              "wall_s": time.perf_counter() - t0, "schedule": info["schedule"],
                              "per_rank_units": info["per_rank_units"]}
        return len(todo)

    def _pop_index(self, ind):
        for i, x in enumerate(self.individuals):
            if x is ind:
                return i
        return -1

    def _dispatch(self, todo, exclude=()):
        """One dispatch of ``todo`` over the ranks (not in ``exclude``):
        broadcast, local evaluation, all_gather. Returns the merged
        ``(status, fitness, fold_scores, aux)`` per candidate and a summary."""
        self.generation_counter += 1
        comm = self.comm
        nfold = int(getattr(todo[0], "nfold", 1) or 1)
        codec = GenomeCodec(todo[0].get_genome())
        costs = [float(ind.cost()) if hasattr(ind, "cost") else 1.0 for ind in todo]
        # a candidate's folds may be split over units only when they train
        # independently (reset="all"); the reference's sequential folds carry
        # biases from fold to fold and stay one unit
        splittable = self.split_folds and hasattr(todo[0], "build_fitness_model") and \
            getattr(todo[0], "reset", "all") == "all"
        # population-batched evaluators take (candidate, fold) units: equal
        # group counts per rank at any generation size
        per_fold = splittable and getattr(self.local_evaluator, "pop_batch", 1) > 1
        allowed = [r for r in range(comm.world_size) if r not in set(exclude)] or list(range(comm.world_size))
        units, ucost = make_units(costs, nfold, len(allowed), splittable, per_fold=per_fold)
        dynamic = self.schedule == "dynamic" and comm.world_size > 1 and len(allowed) == comm.world_size
        if dynamic:
            # table order = claim order: most expensive first (on-line LPT)
            order = sorted(range(len(units)), key=lambda i: (-ucost[i], i))
            units = [units[i] for i in order]
            ucost = [ucost[i] for i in order]
            owner = [-1] * len(units)
        else:
            owner = [allowed[o] for o in lpt_assign(ucost, len(allowed))]
        table = np.zeros((len(units), TABLE_HDR + codec.width), np.float64)
        pidx = [self._pop_index(ind) for ind in todo]
        for k, (slot, fids) in enumerate(units):
            table[k, 0] = slot
            table[k, 1] = owner[k]
            table[k, 2] = sum(1 << f for f in fids)
            table[k, 3] = pidx[slot]
            table[k, TABLE_HDR:] = codec.encode(todo[slot].get_genes())
        wd = _fault.watchdog()
        if wd is not None:
            wd.arm("generation {} (rank 0)".format(self.generation_counter))
        extra = _jsonable(todo[0].get_additional_parameters())
        genome = {k: (list(v) if isinstance(v, tuple) else v) for k, v in todo[0].get_genome().items()}
        blob = json.dumps({"species": self.species.__name__, "extra": extra, "genome": genome}).encode()
        # X1: the config blob travels once (and again only if it changes); the
        # evaluator ranks keep the last one
        send_blob = blob != getattr(comm, "_gentun_last_blob", None)
        # X1 + X2 as ONE message: command header, the config blob when it changed, the genome table
        hdr = np.array([CMD_EVAL, self.generation_counter, len(todo), nfold, int(send_blob)], np.int64)
        comm.broadcast_arrays([hdr, np.frombuffer(blob, np.uint8), table] if send_blob else [hdr, table])
        if send_blob:
            comm._gentun_last_blob = blob

        def make_unit(k):
            slot, fids = units[k]
            return _Unit(slot, todo[slot] if len(fids) == nfold else _clone(todo[slot]), fids)

        if dynamic:
            mine = UnitClaimer(comm, "steal/{}".format(self.generation_counter), len(units), make_unit,
                               "cnn" if splittable else "other")
        else:
            mine = [(k, make_unit(k)) for k in range(len(units)) if owner[k] == comm.rank]
        rows = evaluate_units(mine, self.local_evaluator, nfold, comm.rank, self.generation_counter,
                              on_take=_announcer(table) if self.verbose and comm.world_size > 1 else None)
        local = np.zeros((len(units), row_width(nfold)), np.float64)
        for k, row in rows.items():
            local[k] = row
        gathered = comm.all_gather_array(local)
        if wd is not None:
            wd.disarm()
        merged = _merge(gathered, units, len(todo), nfold)
        log = self.event_log
        if log is not None and comm.world_size > 1:
            self._log_units(log, gathered, units, todo, table, nfold)
        # ranks to leave out of a retry: owners of units that came back empty, ranks that reported errors
        failed_ranks = set()
        for k in range(len(units)):
            got = [r for r, g in enumerate(gathered) if g[k, 0] != ST_NONE]
            if not got and owner[k] >= 0:
                failed_ranks.add(owner[k])
            failed_ranks.update(r for r in got if gathered[r][k, 0] == ST_ERR)
        info = {"units": len(units), "schedule": "dynamic" if dynamic else "lpt", "failed_ranks": failed_ranks,
                "per_rank_units": [int(np.sum(g[:, 0] != ST_NONE)) for g in gathered]}
        return merged, info

    def _log_units(self, log, gathered, units, todo, table, nfold):
        """One ``evaluation`` event per work unit, from whichever rank returned it."""
        for k, (slot, fids) in enumerate(units):
            rank = next((r for r, g in enumerate(gathered) if g[k, 0] != ST_NONE), None)
            row = gathered[rank][k] if rank is not None else None
            ok = row is not None and row[0] == ST_OK
            log.write("evaluation", rank=rank, generation=self.ga_generation, dispatch=self.generation_counter,
                      i=int(table[k, 3]), genes=todo[slot].get_genes(), folds=list(fids),
                      status="ok" if ok else ("error" if row is not None else "missing"),
                      fitness=float(row[1]) if ok else None,
                      fold_scores=[float(row[3 + f]) for f in fids] if ok else None,
                      wall_s=float(row[2]) if row is not None else None)

    def evaluate_round(self, per_rank, slack=1):
        """One balanced evaluation round: about ``per_rank`` candidates per
        rank (up to ``slack`` more when that saves a round), the pending set
        cut into near-equal rounds
        (:func:`~gentun_amd.parallel.scheduler.balanced_round`)."""
        return self.evaluate_in_parallel(
            limit=balanced_round(len(self.pending()), int(per_rank) * self.comm.world_size,
                                 slack=int(slack) * self.comm.world_size))

    def sync_ranks(self):
        """Device-synchronise every rank and barrier (bench timing fence)."""
        if self.comm.world_size > 1:
            self.comm.broadcast_arrays([np.array([CMD_SYNC, self.generation_counter, 0, 0, 0], np.int64)])
        _device_sync(self.local_evaluator)
        self.comm.barrier()

    def shutdown(self):
        """Release the evaluator ranks (they return from ``work()``)."""
        if self.comm.world_size > 1:
            self.comm.broadcast_arrays([np.array([CMD_STOP, self.generation_counter, 0, 0, 0], np.int64)])


def _clone(ind):
    twin = ind.copy()
    twin.set_fitness(None)
    return twin


def _merge(gathered, units, ncand, nfold):
    """Combine per-rank result tables into ``(status, fitness, fold_scores)`` per candidate."""
    per = [{"status": ST_OK, "scores": [np.nan] * nfold, "aux": [np.nan] * nfold, "fit": [], "n": 0}
           for _ in range(ncand)]
    have = [False] * len(units)
    rows = [None] * len(units)
    for table in gathered:
        for k in range(len(units)):
            if table[k, 0] != ST_NONE and not have[k]:
                have[k] = True
                rows[k] = table[k]
    for k, (slot, fids) in enumerate(units):
        row = rows[k]
        p = per[slot]
        if row is None or row[0] != ST_OK:
            p["status"] = ST_ERR
            continue
        p["fit"].append((row[1], len(fids)))
        for f in fids:
            p["scores"][f] = float(row[3 + f])
            p["aux"][f] = float(row[3 + nfold + f])
    out = []
    for p in per:
        if p["status"] != ST_OK or not p["fit"]:
            out.append((ST_ERR, None, None, None))
            continue
        aux = [a for a in p["aux"] if not np.isnan(a)]
        scores = [s for s in p["scores"] if not np.isnan(s)]
        if scores and len(scores) == sum(n for _, n in p["fit"]):
            fit = float(np.mean(scores))
        else:
            tot = sum(n for _, n in p["fit"])
            fit = float(sum(f * n for f, n in p["fit"]) / tot)
        out.append((ST_OK, fit, p["scores"] if scores else None, aux or None))
    return out


class DistributedGridPopulation(DistributedPopulation, GridPopulation):
    """Grid-initialised distributed population (gentun/master.py:132-145)."""

    def __init__(self, species, x_train=None, y_train=None, individual_list=None, genes_grid=None,
                 crossover_rate=0.5, mutation_rate=0.015, maximize=True, additional_parameters=None,
                 host='localhost', port=5672, user='guest', password='guest', rabbit_queue='rpc_queue',
                 comm=None, evaluator=None, split_folds=True):
        if individual_list is None and genes_grid is not None:
            grid = GridPopulation(species, x_train, y_train, genes_grid=genes_grid, crossover_rate=crossover_rate,
                                  mutation_rate=mutation_rate, maximize=maximize,
                                  additional_parameters=additional_parameters)
            individual_list = grid.individuals
        DistributedPopulation.__init__(self, species, x_train, y_train, individual_list, None, crossover_rate,
                                       mutation_rate, maximize, additional_parameters, host, port, user,
                                       password, rabbit_queue, comm, evaluator, split_folds)


# ---------------------------------------------------------------------------
# evaluator ranks
# ---------------------------------------------------------------------------

class GentunWorker(object):
    """Evaluator rank (gentun/worker.py:13-66): serve generations broadcast by
    rank 0 until it broadcasts STOP."""

    def __init__(self, individual, x_train, y_train, host='localhost', port=5672, user='guest',
                 password='guest', rabbit_queue='rpc_queue', comm=None, evaluator=None, verbose=True):
        self.individual = individual
        self.verbose = verbose
        self.x_train = x_train
        self.y_train = y_train
        self.comm = comm if comm is not None else _comm_from_args(host, port)
        self.evaluator = evaluator if evaluator is not None else LocalBatchEvaluator()
        self.served = 0
        self._meta = None           # last config blob (X1) broadcast by rank 0

    def serve_one(self):
        """Handle one broadcast; returns False on STOP."""
        comm = self.comm
        wd = _fault.watchdog()
        if wd is not None:
            wd.arm("evaluator rank {} waiting / evaluating".format(comm.rank))
        msg = comm.broadcast_arrays(None)
        cmd, generation, _ncand, nfold, has_blob = (int(v) for v in msg[0])
        if cmd == CMD_STOP:
            if wd is not None:
                wd.disarm()
            return False
        if cmd == CMD_SYNC:
            _device_sync(self.evaluator)
            comm.barrier()
            if wd is not None:
                wd.disarm()
            return True
        if has_blob:
            self._meta = json.loads(bytes(msg[1].astype(np.uint8)).decode())
        meta = self._meta
        if meta is None:
            raise RuntimeError("evaluator rank {}: generation {} arrived before the config blob".format(
                comm.rank, generation))
        table = msg[-1]
        extra = {k: _tuplify(v) for k, v in meta["extra"].items()}
        # genome spec comes with the broadcast: building a throw-away individual
        # here would draw random genes from the GA stream
        genome = {k: (tuple(v) if isinstance(v, list) else v) for k, v in meta["genome"].items()}
        codec = GenomeCodec(genome)

        def make_unit(k):
            genes = codec.decode(table[k, TABLE_HDR:])
            fids = [f for f in range(nfold) if (int(table[k, 2]) >> f) & 1]
            ind = self.individual(self.x_train, self.y_train, genes=genes, **extra)
            return _Unit(int(table[k, 0]), ind, fids)

        n_units = table.shape[0]
        if n_units and int(table[0, 1]) < 0:
            kind = "cnn" if hasattr(self.individual, "build_fitness_model") else "other"
            mine = UnitClaimer(comm, "steal/{}".format(generation), n_units, make_unit, kind)
        else:
            mine = [(k, make_unit(k)) for k in range(n_units) if int(table[k, 1]) == comm.rank]
        rows = evaluate_units(mine, self.evaluator, nfold, comm.rank, generation,
                              on_take=_announcer(table) if self.verbose else None)
        local = np.zeros((table.shape[0], row_width(nfold)), np.float64)
        for k, row in rows.items():
            local[k] = row
        comm.all_gather_array(local)
        if wd is not None:
            wd.disarm()
        self.served += len(rows)
        return True

    def work(self):
        print(" [x] Evaluator rank {} of {} awaiting generations".format(self.comm.rank, self.comm.world_size))
        try:
            while self.serve_one():
                pass
        except KeyboardInterrupt:
            print()
        print("Good bye!")


def _announcer(table):
    """The reference worker's line per job (gentun/worker.py:43), printed when
    a rank takes a candidate (a candidate split into fold units prints once)."""
    seen = set()

    def on_take(entry):
        i = int(table[entry[0], 3])
        if i not in seen:
            seen.add(i)
            print(" [.] Evaluating individual {}".format(i), flush=True)
    return on_take


def _comm_from_args(host, port):
    if int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        return LocalComm()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1" if host == "localhost" else str(host))
    if port != 5672:
        os.environ.setdefault("MASTER_PORT", str(port))
    return from_env()


def _localize_device(ind, evaluator):
    """A GPU-requesting individual (e.g. ``XgboostIndividual(device='cuda:0')``,
    whose additional parameters come from rank 0's broadcast) runs on the GPU
    of the rank evaluating it, not on rank 0's device."""
    dev = getattr(evaluator, "device", None)
    want = getattr(ind, "device", None)
    if dev is not None and want is not None and str(want).startswith("cuda") and str(dev).startswith("cuda"):
        ind.device = str(dev)


def _device_sync(evaluator):
    dev = getattr(evaluator, "device", None)
    if dev is not None and getattr(dev, "type", "") == "cuda":
        import torch
        torch.cuda.synchronize(dev)
