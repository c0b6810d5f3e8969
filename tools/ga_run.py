"""A long Genetic-CNN search on one GPU with per-generation checkpoints
(BASELINE cfg 2 at config 3's population; verdict r2 item 4): RussianRouletteGA
(pC 0.2 / pM 0.8, qC 0.3 / qM 0.1), population 32, S=(3,5) kernels (20,50),
the full fp32 protocol (5-fold CV on 10k samples, epochs (20,4,1)), whole
generations population-batched. Resumable: ``--resume`` continues from
``<ckpt>/latest.json`` (the GA stream, history and evaluated fitness come
back), so a run longer than one GPU session is split over calls.

usage: python tools/ga_run.py --gens 20 --ckpt DIR [--resume] [--data hard] [--fold-reset all]
                             [--space deep [--kernels 20,50,100] [--batch-norm]]
``--space deep`` is BASELINE config 4's search space: S=(3,4,5), 5x5 stage
convs, kernels (20,50,100) unless ``--kernels`` overrides them.
Prints one JSON line: best categorical / binary val-acc per generation.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ap = argparse.ArgumentParser()
ap.add_argument("--gens", type=int, default=20)
ap.add_argument("--pop", type=int, default=32)
ap.add_argument("--ckpt", required=True)
ap.add_argument("--resume", action="store_true")
ap.add_argument("--data", choices=("hard", "glyph"), default="hard")
ap.add_argument("--fold-reset", choices=("all", "kernels"), default="all")
ap.add_argument("--pop-batch", type=int, default=32)
ap.add_argument("--seed", type=int, default=1234)
ap.add_argument("--space", choices=("default", "deep"), default="default")
ap.add_argument("--kernels", default=None, help="kernels per stage, e.g. 20,50,100")
ap.add_argument("--batch-norm", action="store_true")
ap.add_argument("--time-budget", type=float, default=0.0, help="stop after the generation that passes this many s")
args = ap.parse_args()

import torch  # noqa: E402

from gentun_amd import GeneticCnnIndividual, LocalBatchEvaluator, RussianRouletteGA  # noqa: E402
from gentun_amd.parallel import LocalComm  # noqa: E402
from gentun_amd.parallel.distributed import DistributedPopulation  # noqa: E402
from gentun_amd.utils import rng as grng  # noqa: E402
from gentun_amd.utils.data import make_cifar_hard, make_cifar_like  # noqa: E402

dev = torch.device("cuda", 0)
x, y = (make_cifar_hard if args.data == "hard" else make_cifar_like)(n=10000, seed=0)
nodes, kernels = ((3, 4, 5), (20, 50, 100)) if args.space == "deep" else ((3, 5), (20, 50))
if args.kernels:
    kernels = tuple(int(k) for k in args.kernels.split(","))
extra = dict(nodes=nodes, input_shape=(32, 32, 3), kernels_per_layer=kernels, kernel_sizes=((5, 5),) * len(nodes),
             dense_units=500, dropout_probability=0.5, classes=10, nfold=5, epochs=(20, 4, 1),
             learning_rate=(1e-3, 1e-4, 1e-5), batch_size=32, dtype="fp32", loss="bce_compat", seed=args.seed,
             reset=args.fold_reset, batching="keras", batch_norm=args.batch_norm)
ev = LocalBatchEvaluator(device=dev, streams=1, pop_batch=args.pop_batch)
comm = LocalComm()
latest = os.path.join(args.ckpt, "latest.json")
if args.resume and os.path.exists(latest):
    def factory(inds):
        return DistributedPopulation(GeneticCnnIndividual, x, y, individual_list=inds, additional_parameters=extra,
                                     comm=comm, evaluator=ev, verbose=False)
    ga = RussianRouletteGA.resume(latest, GeneticCnnIndividual, x, y, population_factory=factory,
                                  checkpoint_dir=args.ckpt)
else:
    grng.seed(args.seed)
    pop = DistributedPopulation(GeneticCnnIndividual, x, y, size=args.pop, crossover_rate=0.3, mutation_rate=0.1,
                                additional_parameters=extra, comm=comm, evaluator=ev, verbose=False)
    ga = RussianRouletteGA(pop, crossover_probability=0.2, mutation_probability=0.8, seed=args.seed,
                           checkpoint_dir=args.ckpt, verbose=False)
t0 = time.perf_counter()
while ga.generation <= args.gens:
    ga.evolve_population()
    h = ga.history[-1]
    print("[ga_run] gen {} evals {} best cat {} bin {:.5f} wall {:.1f}s".format(
        h["generation"], h["evals"], h.get("best_cat_acc"), h["best_fitness"], h["wall_s"]), file=sys.stderr,
        flush=True)
    ga.generation += 1
    if args.time_budget and time.perf_counter() - t0 > args.time_budget:
        break
evals = sum(h["evals"] for h in ga.history)
wall = sum(h["wall_s"] for h in ga.history)
print(json.dumps({"generations": len(ga.history), "evals": evals, "eval_wall_s": round(wall, 1),
                  "candidates_per_hour": round(3600 * evals / wall, 1) if wall else None,
                  "data": args.data, "fold_reset": args.fold_reset, "population": args.pop,
                  "space": "S=({}) kernels ({})".format(",".join(map(str, nodes)), ",".join(map(str, kernels))),
                  "batch_norm": args.batch_norm,
                  "best_val_cat_acc_by_gen": [round(h.get("best_cat_acc") or 0.0, 4) for h in ga.history],
                  "best_val_binary_acc_by_gen": [round(h["best_fitness"], 5) for h in ga.history],
                  "mean_val_cat_acc_by_gen": [round(h["mean_cat_acc"], 4) if h.get("mean_cat_acc") is not None
                                              else None for h in ga.history],
                  "mean_fitness_by_gen": [round(h.get("mean_fitness_finite", h["mean_fitness"]) or 0.0, 5)
                                          for h in ga.history],
                  "evals_by_gen": [h["evals"] for h in ga.history],
                  "best_genes_by_gen": [h["best_genes"] for h in ga.history]}), flush=True)
