"""MODELLED strong scaling of the headline benchmark (bench.py: RR-GA, population 32 in total over N
evaluator ranks, 5 candidates per rank per round + 1 slack, concurrent folds) -- a planning number from
the measured single-GPU Q-curve, NOT a multi-GPU measurement (no 8-GPU node was available to this
work; the driver measures the real curve, SCALE_rNN.json).

Model: a generation's pending candidates are cut into rounds exactly as bench.py / DistributedPopulation
do (scheduler.balanced_round, make_units, lpt_assign); a round lasts as long as its busiest rank, whose
population job trains 5 x (its candidates) groups for 6,250 steps (epochs (20, 4, 1) of 250 batches) at
the Q-curve's ms/step for that group count (linear interpolation between measured points), plus a fixed
per-round cost (evaluation, initialisation, dispatch; ``--round-overhead``). Collectives (one 32 KB
broadcast + one all_gather per round) are ignored: microseconds against seconds-long rounds.

usage: python tools/scaling_model.py [--qcurve FILE] [--pending 14] [--round-overhead 0.3]
FILE: lines "all P groups ms/step ..." as in profiles/r6/qcurve_fp32_r6.txt (default: that file)."""

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gentun_amd.parallel.scheduler import balanced_round, lpt_assign, make_units  # noqa: E402

STEPS = 6250          # (20 + 4 + 1) epochs x 250 batches of 32 (8,000 training rows per fold)


def load_qcurve(path):
    pts = {}
    for line in open(path):
        f = line.split()
        if len(f) >= 4 and f[0] == "all" and f[1].isdigit():
            pts[int(f[2])] = float(f[3])
    return sorted(pts.items())


def step_ms(curve, groups):
    if groups <= curve[0][0]:
        return curve[0][1] * groups / curve[0][0] if groups < curve[0][0] else curve[0][1]
    for (q0, t0), (q1, t1) in zip(curve, curve[1:]):
        if q0 <= groups <= q1:
            return t0 + (t1 - t0) * (groups - q0) / (q1 - q0)
    (q0, t0), (q1, t1) = curve[-2], curve[-1]
    return t1 + (t1 - t0) * (groups - q1) / (q1 - q0)


def generation_time(curve, pending, world, per_gpu=5, slack=1, nfold=5, overhead=0.3):
    t, rounds = 0.0, []
    while pending > 0:
        n = balanced_round(pending, per_gpu * world, slack=slack * world)
        # the population-batched evaluator takes (candidate, fold) units (DistributedPopulation._dispatch:
        # per_fold when pop_batch > 1 and the folds train concurrently); equal candidate costs here
        units, _ = make_units([1.0] * n, nfold, world, True, per_fold=world > 1)
        folds_per_unit = [len(u[1]) for u in units]
        owner = lpt_assign([float(f) for f in folds_per_unit], world)
        groups = [0] * world
        for f, r in zip(folds_per_unit, owner):
            groups[r] += f
        busiest = max(groups)
        dt = STEPS * step_ms(curve, busiest) / 1000.0 + overhead
        rounds.append((n, busiest, round(dt, 2)))
        t += dt
        pending -= n
    return t, rounds


def main():
    ap = argparse.ArgumentParser()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ap.add_argument("--qcurve", default=os.path.join(root, "profiles", "r6", "qcurve_fp32_r6.txt"))
    ap.add_argument("--pending", type=int, default=14, help="candidates re-evaluated per generation (RR-GA: ~14 of 32)")
    ap.add_argument("--round-overhead", type=float, default=0.3)
    args = ap.parse_args()
    curve = load_qcurve(args.qcurve)
    print("# MODEL, not a measurement: bench.py strong scaling (population 32 total) from the 1-GPU Q-curve")
    print("# Q-curve: {}  (groups -> ms/step: {})".format(os.path.relpath(args.qcurve, root),
                                                         ", ".join("{}: {}".format(q, t) for q, t in curve)))
    print("# steady-state generation: {} pending candidates; per-round overhead {} s".format(
        args.pending, args.round_overhead))
    print("{:>3} {:>10} {:>12} {:>10}  rounds (candidates, busiest rank's groups, s)".format(
        "N", "gen_s", "cand/h", "eff_vs_1"))
    base = None
    for world in (1, 2, 4, 8):
        t, rounds = generation_time(curve, args.pending, world, overhead=args.round_overhead)
        cph = 3600.0 * args.pending / t
        base = base or cph
        print("{:>3} {:>10.1f} {:>12.1f} {:>9.0f}%  {}".format(world, t, cph, 100.0 * cph / (world * base), rounds))


if __name__ == "__main__":
    main()
