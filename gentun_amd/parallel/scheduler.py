"""Static work assignment for a generation (SURVEY.md §5.8, §7.3 hard part 3).

The reference load-balances dynamically through a RabbitMQ pull queue with
``prefetch_count=1`` (gentun/worker.py:59-63). Here every rank receives the
whole genome table, so an assignment computed on rank 0 from a cost model
(forward FLOPs per sample, :meth:`Plan.forward_flops`) is broadcast with it.

Work units are ``(candidate, fold-group)``. With a population-batched
evaluator (every (candidate, fold) pair of a rank's share is one group of
shared kernel launches, models/cnn_hip.py) the unit is always ONE fold
(``per_fold``): the ranks then get near-equal numbers of groups even when a
generation re-evaluates only ~14 of 32 candidates on 8 GPUs (SURVEY.md §2.2;
master.py:108-129 dispatches whole candidates). Otherwise a candidate's folds
stay together (one fold-batched launch) unless there are fewer candidates
than ranks. Units are placed Longest-Processing-Time-first on the
least-loaded rank; ties break on rank id, so the result is deterministic.
"""

import heapq


def lpt_assign(costs, world_size):
    """Return ``owner[i]`` for each unit cost (LPT greedy)."""
    order = sorted(range(len(costs)), key=lambda i: (-costs[i], i))
    heap = [(0.0, r) for r in range(world_size)]
    heapq.heapify(heap)
    owner = [0] * len(costs)
    for i in order:
        load, r = heapq.heappop(heap)
        owner[i] = r
        heapq.heappush(heap, (load + costs[i], r))
    return owner


def make_units(costs, nfold, world_size, split_folds=True, per_fold=False):
    """Units ``(candidate, fold_ids)`` with their costs.

    ``per_fold``: one unit per (candidate, fold). Otherwise candidates are
    split into fold groups only while that helps fill the ranks: the number
    of groups per candidate is ``min(nfold, ceil(world/ncand))``.
    """
    n = len(costs)
    if n == 0:
        return [], []
    groups = 1
    if split_folds and nfold > 1 and per_fold and world_size > 1:
        groups = nfold
    elif split_folds and nfold > 1 and n < world_size:
        groups = min(nfold, -(-world_size // n))
    units, ucost = [], []
    base, extra = divmod(nfold, groups)
    for i, c in enumerate(costs):
        f0 = 0
        for k in range(groups):
            size = base + (1 if k < extra else 0)
            fid = list(range(f0, f0 + size))
            f0 += size
            units.append((i, fid))
            ucost.append(c * len(fid) / float(nfold))
    return units, ucost


def balanced_round(n_pending, cap, slack=0):
    """Size of the next evaluation round when at most ``cap`` candidates fit a
    round: the pending set is cut into ``ceil(n / cap)`` near-equal rounds
    (11 pending at cap 5 -> 4, 4, 3 instead of 5, 5, 1; a 1-candidate round
    costs ~40 % of a 5-candidate one on a GPU, so it halves the throughput of
    its time slice). ``slack``: rounds may exceed ``cap`` by up to that many
    candidates when that saves a round (11 at cap 5, slack 1 -> 6, 5: larger
    population launches, and no round below cap - 1)."""
    if n_pending <= 0:
        return 0
    cap = max(1, int(cap))
    rounds = -(-n_pending // cap)
    fewer = n_pending // cap
    if slack > 0 and fewer >= 1 and -(-n_pending // fewer) <= cap + int(slack):
        rounds = fewer
    return -(-n_pending // rounds)


def makespan(costs, owner, world_size):
    loads = [0.0] * world_size
    for c, r in zip(costs, owner):
        loads[r] += c
    return max(loads) if loads else 0.0
