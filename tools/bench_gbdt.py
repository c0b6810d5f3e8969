"""GBDT (XGBoost-individual) GA throughput on the MI355X histogram path
(BASELINE.json config 5: synthetic 1M x 256 tabular regression).

Evaluates ``--pop`` random XgboostIndividuals (5-fold CV, reg:linear / rmse)
on the GPU histogram / split / partition kernels and reports candidates/hour.
``--rounds`` caps num_boost_round (reference default 5000 with early stopping
100, gentun/individuals.py:158-160); the value used is printed with the result.

usage: python tools/bench_gbdt.py [--rows 1000000] [--features 256] [--pop 4] [--rounds 50] [--esr 10]
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
ap.add_argument("--pop", type=int, default=4)
ap.add_argument("--rounds", type=int, default=50)
ap.add_argument("--esr", type=int, default=10)
ap.add_argument("--nfold", type=int, default=5)
ap.add_argument("--device", default="cuda:0")
args = ap.parse_args()

from gentun_amd import Population, XgboostIndividual  # noqa: E402
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
for i, ind in enumerate(pop):
    t1 = time.perf_counter()
    f = ind.get_fitness()
    per.append({"candidate": i, "s": round(time.perf_counter() - t1, 2), "rmse": round(float(f), 5),
                "eta": round(float(ind.get_genes()["eta"]), 5), "max_depth": int(ind.get_genes()["max_depth"]),
                "rounds": len((getattr(ind, "fold_metrics", None) or {}).get("history", [])) or None})
    print("[bench_gbdt] " + json.dumps(per[-1]), file=sys.stderr, flush=True)
best = pop.get_fittest()
dt = time.perf_counter() - t0
print(json.dumps({"metric": "candidates/hour (XGB GA, GBDT 5-fold CV)", "value": round(3600 * args.pop / dt, 2),
                  "rows": args.rows, "features": args.features, "pop": args.pop, "num_boost_round": args.rounds,
                  "early_stopping_rounds": args.esr, "device": args.device, "eval_s": round(dt, 2),
                  "data_s": round(t_data, 2), "quantize_s": round(t_prep, 2), "best_rmse": best.get_fitness(),
                  "fitness": [round(float(ind.get_fitness()), 5) for ind in pop], "per_candidate": per}), flush=True)
