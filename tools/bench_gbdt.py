"""GBDT (XGBoost-individual) GA throughput on the MI355X histogram path
(BASELINE.json config 5: synthetic 1M x 256 tabular regression).

Runs the reference's tournament GA (GeneticAlgorithm, tournament 5, elitism;
reference driver tests/test_wine-quality.py:20-25) for ``--gens``
generations over a population of ``--pop`` XgboostIndividuals (5-fold CV,
reg:linear / rmse) evaluated on the GPU histogram / split / partition
kernels, and reports candidates/hour = evaluations (pop + (pop-1)(gens-1):
the elite keeps its fitness) / evaluation wall time. ``--gens 0`` evaluates
one random population only (the round-2 measurement). ``--rounds`` /
``--esr``: num_boost_round / early_stopping_rounds (reference defaults 5000 /
100, gentun/individuals.py:158-160).

usage: python tools/bench_gbdt.py [--rows 1000000] [--features 256] [--pop 10] [--gens 3] [--rounds 5000] [--esr 100]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=1000000)
ap.add_argument("--features", type=int, default=256)
ap.add_argument("--pop", type=int, default=10)
ap.add_argument("--gens", type=int, default=3)
ap.add_argument("--rounds", type=int, default=5000)
ap.add_argument("--esr", type=int, default=100)
ap.add_argument("--seed", type=int, default=0)
ap.add_argument("--nfold", type=int, default=5)
ap.add_argument("--device", default="cuda:0")
args = ap.parse_args()

from gentun_amd import GeneticAlgorithm, Population, XgboostIndividual  # noqa: E402
from gentun_amd.utils import rng  # noqa: E402
from gentun_amd.utils.data import make_regression  # noqa: E402

t0 = time.perf_counter()
x, y = make_regression(n=args.rows, f=args.features, seed=0)
t_data = time.perf_counter() - t0
rng.seed(0)
extra = {"nfold": args.nfold, "num_boost_round": args.rounds, "early_stopping_rounds": args.esr,
         "device": args.device if args.device != "cpu" else None}
pop = Population(XgboostIndividual, x, y, size=args.pop, additional_parameters=extra, maximize=False)
t0 = time.perf_counter()
t_prep = 0.0
if args.device != "cpu":
    # per-dataset quantisation (cached for every later candidate): timed inside eval_s, also reported alone
    from gentun_amd.models import gbdt_hip  # noqa: E402
    gbdt_hip.quantize_device(x)
    t_prep = time.perf_counter() - t0
per = []
evals = [0]
_orig = XgboostIndividual.evaluate_fitness


def _timed(self):
    t1 = time.perf_counter()
    _orig(self)
    evals[0] += 1
    g = self.get_genes()
    per.append({"eval": evals[0], "s": round(time.perf_counter() - t1, 2), "rmse": round(float(self.fitness), 5),
                "eta": round(float(g["eta"]), 5), "max_depth": int(g["max_depth"]),
                "subsample": round(float(g["subsample"]), 4)})
    print("[bench_gbdt] " + json.dumps(per[-1]), file=sys.stderr, flush=True)


XgboostIndividual.evaluate_fitness = _timed
history = []
if args.gens > 0:
    ga = GeneticAlgorithm(pop, tournament_size=min(5, args.pop), elitism=True, seed=args.seed, verbose=False)
    best = ga.run(args.gens)
    history = [{"generation": h["generation"], "best_rmse": h["best_fitness"]} for h in ga.history]
else:
    best = pop.get_fittest()
dt = time.perf_counter() - t0
print(json.dumps({"metric": "candidates/hour (XGB GA, GBDT 5-fold CV)", "value": round(3600 * evals[0] / dt, 2),
                  "algorithm": "GeneticAlgorithm tournament 5 elitism" if args.gens > 0 else "random population",
                  "rows": args.rows, "features": args.features, "pop": args.pop, "gens": args.gens,
                  "evaluations": evals[0], "num_boost_round": args.rounds, "early_stopping_rounds": args.esr,
                  "device": args.device, "eval_s": round(dt, 2), "data_s": round(t_data, 2),
                  "quantize_s": round(t_prep, 2), "best_rmse": best.get_fitness(), "best_by_gen": history,
                  "per_eval": per}), flush=True)
