#!/usr/bin/env python
"""Headline benchmark (BASELINE.json): "candidates/hour + best val-acc@genN,
Genetic-CNN CIFAR-10 1/2/4/8 GPU" -- the reference's paper-replica search
(tests/test_mnist.py:22-34) on CIFAR-10-shaped data, measured on MI355X.

What runs: the real Russian-roulette GA (RussianRouletteGA, pC 0.2 / pM 0.8;
individuals qC 0.3 / qM 0.1) over Genetic-CNN S=(3,5) candidates (kernels
(20,50), 5x5 stage convs, dense 500, dropout 0.5, 10 classes) at BASELINE
config 3's shape: population 32 IN TOTAL over the N evaluator ranks
(``--population``; strong scaling; ``--pop-per-gpu`` gives the weak-scaling
variant). Every evaluation is the reference's training protocol: 5-fold CV on
10,000 synthetic 32x32x3 samples, epochs (20,4,1) with lr (1e-3,1e-4,1e-5),
Adam, batch 32, Keras softmax + binary_crossentropy loss, **fp32** (the
reference's TF float32; HIP kernels compute every product as the exact 3-way
bf16 split on the matrix cores, fp32-level error: tests/test_hip_fp32.py).
Random-init weights, synthetic data (no network).

Fold semantics (``--fold-reset``): ``all`` (default, the fast mode) trains
the 5 folds of a candidate CONCURRENTLY, each from fresh weights;
``kernels`` is the reference's protocol -- folds in sequence, kernels
re-drawn per fold, biases carried over (keras_models.py:120-125,132-142) --
and is the library default. Both train the same number of steps.

One bench *step* = one evaluation round of the GA: the pending individuals of
the current generation are cut into near-equal rounds of at most
``per_gpu x N`` (``DistributedPopulation.evaluate_round``), dispatched over the
N evaluator ranks (one per GPU; RCCL broadcast of the genome table,
all_gather of per-fold scores) and trained population-batched on each GPU.
When a generation has no pending individuals left, rank 0 breeds the next one
(selection / crossover / mutation on the host, milliseconds). ``value`` =
candidates fully evaluated in the K timed rounds / timed hours, over the
whole job; ``best_val_acc_at_gen`` = categorical validation accuracy (5-fold
mean) of the fittest individual of the last completed generation (fitness
itself is the reference's binary accuracy).

Run: ``python bench.py --gpus 1 --steps 2 --warmup 1`` or, for N>1,
``torchrun --nproc-per-node N bench.py --gpus N ...``.
"""

import argparse
import json
import os
import sys
import time

METRIC = "candidates/hour + best val-acc@genN, Genetic-CNN CIFAR-10 1/2/4/8 GPU"


def metric_name(shape):
    """BASELINE.json's metric for the CIFAR-10 shape; other input shapes name their own data set (an
    MNIST-config run must not claim to be the CIFAR-10 headline)."""
    shape = tuple(shape)
    if shape == (32, 32, 3):
        return METRIC
    name = "MNIST" if shape == (28, 28, 1) else "{}-image".format("x".join(map(str, shape)))
    return METRIC.replace("CIFAR-10", name)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--per-gpu", type=int, default=None,
                    help="candidates per GPU per round (default: 5 fp32 / 8 bf16, 16 with --fold-reset kernels; larger rounds = larger population launches: 794 / 862 / 936 candidates/h at 3 / 4 / 6, profiles/bench_round_size_r2.txt)")
    ap.add_argument("--population", type=int, default=32,
                    help="GA population in total (BASELINE cfg 3: 32 on 8 evaluators; strong scaling)")
    ap.add_argument("--pop-per-gpu", type=int, default=None,
                    help="GA population per GPU instead (weak scaling: population = pop_per_gpu x N)")
    ap.add_argument("--streams", type=int, default=1, help="concurrent population jobs per GPU")
    ap.add_argument("--pop-batch", type=int, default=16, help="candidates (x folds) per population job")
    ap.add_argument("--backend", default=None, help="hip (default on GPU) or torch")
    ap.add_argument("--torch-unbatched", action="store_true",
                    help="--backend torch: one candidate per job (default: population-batched TorchPopJob, "
                         "the same batching as the HIP path)")
    ap.add_argument("--epochs", default="20,4,1")
    ap.add_argument("--lr", default="1e-3,1e-4,1e-5")
    ap.add_argument("--samples", type=int, default=10000)
    ap.add_argument("--data", choices=("hard", "glyph"), default="hard",
                    help="hard: base glyphs x tick variants, 30 %% variant-label noise (utils/data.make_cifar_hard: "
                         "learned folds 0.61-0.66 by architecture); glyph: round-2 data (every learned fold ~0.99)")
    ap.add_argument("--nfold", type=int, default=5)
    ap.add_argument("--dtype", default="fp32", choices=("fp32", "bf16"))
    ap.add_argument("--loss", default="bce_compat", choices=("bce_compat", "ce"))
    ap.add_argument("--fold-reset", default="all", choices=("all", "kernels"),
                    help="all: the 5 folds of a candidate train concurrently, each from fresh weights (fast mode); "
                         "kernels: the reference's sequential folds with biases carried over")
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--space", choices=("default", "deep"), default="default",
                    help="default: S=(3,5) kernels (20,50) (headline); deep: BASELINE cfg 4, S=(3,4,5) kernels "
                         "(20,50,100) on 32x32 inputs")
    ap.add_argument("--kernels", default=None, help="override kernels per stage, e.g. 64,128,256")
    ap.add_argument("--batch-norm", action="store_true",
                    help="conv -> BatchNorm -> ReLU in every node (not in the reference network)")
    ap.add_argument("--input-shape", default="32,32,3",
                    help="H,W,C of the synthetic images; 28,28,1 is the reference's MNIST default "
                         "(gentun/individuals.py:221, tests/test_mnist.py)")
    ap.add_argument("--kernel-size", type=int, default=5,
                    help="stage-input conv kernel size of every stage (the reference's kernel_sizes; nodes are 3x3)")
    ap.add_argument("--generic-kernels", action="store_true",
                    help="HIP backend on its generic conv / wgrad kernels only (the comparison figure for the "
                         "shape-specialised fast path)")
    ap.add_argument("--pad-images", type=int, default=1,
                    help="1: a 28x28 image is stored zero-padded to 32x32 so every stage runs the "
                         "shape-specialised kernels (ops/cnn_kernels.padded_hw); 0: the generic kernels")
    return ap.parse_args()


def main():
    args = parse()
    # Library progress lines go to stderr: stdout carries exactly one JSON line.
    real_stdout = sys.stdout
    sys.stdout = sys.stderr
    try:
        out = run(args)
    finally:
        sys.stdout = real_stdout
    if out is not None:
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")


def _teardown(comm):
    """Every rank leaves the RCCL / gloo group explicitly (after the STOP
    broadcast): no communicator is left for interpreter shutdown to tear down."""
    comm.finish()


def run(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    import torch
    if torch.cuda.is_available():
        # one rank per GPU; more ranks than GPUs (a 1-GPU multi-rank rehearsal) share devices
        dev_index = local_rank % max(1, torch.cuda.device_count())
        torch.cuda.set_device(dev_index)
        device = torch.device("cuda", dev_index)
    else:
        device = torch.device("cpu")

    from gentun_amd import GeneticCnnIndividual, LocalBatchEvaluator, RussianRouletteGA
    from gentun_amd.parallel import DistComm, LocalComm
    from gentun_amd.parallel.distributed import DistributedPopulation, GentunWorker
    from gentun_amd.utils import rng as grng
    from gentun_amd.utils.data import (make_cifar_hard, make_cifar_like, make_glyph_classification,
                                       make_variant_classification)

    if world > 1:
        # RCCL (backend "nccl") over xGMI between GPUs; GENTUN_DIST_BACKEND=gloo for rehearsals
        backend = os.environ.get("GENTUN_DIST_BACKEND") or ("nccl" if device.type == "cuda" else "gloo")
        comm = DistComm(backend=backend, device=device)
    else:
        comm = LocalComm()

    epochs = tuple(int(e) for e in args.epochs.split(","))
    lrs = tuple(float(x) for x in args.lr.split(","))
    # sequential folds (kernels) batch candidates only by fold position: a round takes the whole
    # pending generation (up to 16 per GPU) so every fold launch carries ~14-16 groups
    per_gpu = args.per_gpu or (16 if args.fold_reset == "kernels" else 5 if args.dtype == "fp32" else 8)
    shape = tuple(int(v) for v in args.input_shape.split(","))
    if shape == (32, 32, 3):
        x, y = (make_cifar_hard if args.data == "hard" else make_cifar_like)(n=args.samples, seed=0)
    elif args.data == "hard":
        x, y = make_variant_classification(n=args.samples, shape=shape, classes=10, seed=0, noise=0.7,
                                           label_noise=0.3)
    else:
        x, y = make_glyph_classification(n=args.samples, shape=shape, classes=10, seed=0, noise=1.0)
    nodes, kernels = ((3, 4, 5), (20, 50, 100)) if args.space == "deep" else ((3, 5), (20, 50))
    if args.kernels:
        kernels = tuple(int(k) for k in args.kernels.split(","))
    space = "S=({}) kernels ({})".format(",".join(map(str, nodes)), ",".join(map(str, kernels)))
    if args.kernel_size != 5:
        space += " {}x{} stage-input convs".format(args.kernel_size, args.kernel_size)
    ksz = (args.kernel_size, args.kernel_size)
    if args.generic_kernels:
        from gentun_amd.ops import cnn_kernels as _K
        _K.lib().gt_conv_set_fast(0)            # every conv / wgrad on the generic kernels
    fast_path = None
    if device.type == "cuda" and (args.backend or "hip") == "hip":
        # which kernels a superset step of this space runs (probed: cnn_hip.fast_path_report)
        from gentun_amd.models.cnn_hip import fast_path_report
        from gentun_amd.models.genome import make_plan as _mk
        genes_all = {"S_{}".format(i + 1): "1" * (k * (k - 1) // 2) for i, k in enumerate(nodes)}
        rep = fast_path_report(_mk(genes_all, nodes, shape, kernels, (ksz,) * len(nodes), 500, 10), args.dtype,
                               ngroups=per_gpu * args.nfold, B=32, pad_images=bool(args.pad_images),
                               batch_norm=args.batch_norm)
        fast_path = {k: rep[k] for k in ("stored_hw", "stage_channels_padded", "fast_launches", "generic_launches")}
        fast_path["note"] = "launches of a superset step (every node present): fwd + dgrad + wgrad per conv layer"
    extra = dict(nodes=nodes, input_shape=shape, kernels_per_layer=kernels,
                 kernel_sizes=(ksz,) * len(nodes), dense_units=500, dropout_probability=0.5, classes=10,
                 nfold=args.nfold, epochs=epochs, learning_rate=lrs, batch_size=32, dtype=args.dtype,
                 loss=args.loss, seed=args.seed, backend=args.backend, reset=args.fold_reset, batching="keras",
                 batch_norm=args.batch_norm, pad_images=bool(args.pad_images))
    evaluator = LocalBatchEvaluator(device=device, streams=args.streams, pop_batch=args.pop_batch,
                                    torch_pop=not args.torch_unbatched)
    N = comm.world_size
    slack = 1                 # evaluate_round: up to one more per rank when that saves a round
    round_size = (per_gpu + slack) * N

    if comm.rank != 0:
        # evaluator rank: serves EVAL / SYNC (timing fence) / STOP from rank 0
        GentunWorker(GeneticCnnIndividual, x, y, comm=comm, evaluator=evaluator, verbose=False).work()
        _teardown(comm)
        return None

    grng.seed(args.seed)
    population = args.pop_per_gpu * N if args.pop_per_gpu else args.population
    pop = DistributedPopulation(GeneticCnnIndividual, x, y, size=population, crossover_rate=0.3,
                                mutation_rate=0.1, additional_parameters=extra, comm=comm, evaluator=evaluator,
                                verbose=False)
    ga = RussianRouletteGA(pop, crossover_probability=0.2, mutation_probability=0.8, seed=args.seed,
                           verbose=False)
    completed = []          # per completed generation: fittest's fitness / categorical accuracy

    def advance():
        """All of the generation evaluated: record it, breed the next."""
        fittest = ga._evaluate_and_report()
        fm = getattr(fittest, "fold_metrics", None) or {}
        cat = fm.get("categorical_accuracy")
        h = ga.history[-1]
        completed.append({"generation": ga.generation, "best_fitness": fittest.get_fitness(),
                          "best_cat_acc": float(sum(cat) / len(cat)) if cat else None,
                          "best_genes": dict(fittest.get_genes()),
                          "mean_cat_acc": h.get("mean_cat_acc"), "mean_fitness": h.get("mean_fitness_finite")})
        ga.breed()
        ga.generation += 1

    best_seen = {}          # fittest individual evaluated so far (any generation, complete or not)

    def track():
        for ind in ga.population:
            if not ind.get_fitness_status():
                continue
            cat = (getattr(ind, "fold_metrics", None) or {}).get("categorical_accuracy")
            f = ind.get_fitness()
            if cat and (not best_seen or f > best_seen["fitness"]):
                best_seen.update(fitness=f, cat=float(sum(cat) / len(cat)), genes=dict(ind.get_genes()))

    def one_round():
        if not ga.population.pending():
            advance()
        ga.population.ga_generation = ga.generation
        n = ga.population.evaluate_round(per_gpu, slack=slack)
        track()
        return n

    total_evals = 0
    timed_evals = 0
    round_sizes = []
    t_start = None
    for step in range(args.warmup + args.steps):
        if step == args.warmup:
            ga.population.sync_ranks()           # barrier + device sync on every rank
            t_start = time.perf_counter()
        n = one_round()
        total_evals += n
        if step >= args.warmup:
            timed_evals += n
            round_sizes.append(n)
        print("[bench] step {} gen {} evaluated {} ({}) dispatch={}".format(
            step, ga.generation, n, "timed" if step >= args.warmup else "warmup",
            ga.population.last_dispatch), file=sys.stderr, flush=True)
    ga.population.sync_ranks()
    elapsed = time.perf_counter() - t_start
    if not ga.population.pending():
        advance()                                # close the generation the last round finished
    ga.population.shutdown()
    _teardown(comm)

    cph = 3600.0 * timed_evals / elapsed
    last = completed[-1] if completed else None
    out = {
        "metric": metric_name(shape),
        "value": round(cph, 2),
        "unit": "candidates/hour",
        "n_gpus": N,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000.0 * elapsed / max(1, args.steps), 2),
        "higher_is_better": True,
        "scaling": "weak" if args.pop_per_gpu else "strong",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": ("synthetic ({}-shaped {}k x {}: 5 stroke glyphs x 2 tick variants + clutter + noise, "
                 "30% variant-label noise; random-init weights)" if args.data == "hard" else
                 "synthetic ({}-shaped {}k x {} stroke glyphs + clutter + noise; "
                 "random-init weights)").format("CIFAR-10" if shape == (32, 32, 3) else "MNIST" if shape == (28, 28, 1)
                                                else "image", args.samples // 1000, "x".join(map(str, shape))),
        "config": {"model": "Genetic-CNN {} dense 500".format(space), "global_batch": 32 * args.nfold,
                   "seq_len": None,
                   "parallelism": ("population-dp{} ({} genome bcast / score all_gather)".format(
                                       N, "RCCL over xGMI" if getattr(comm, "backend", "") == "nccl"
                                       else getattr(comm, "backend", "?"))
                                   if N > 1 else "population-dp1 (single evaluator, no collectives)"),
                   "algorithm": "RussianRouletteGA pC0.2 pM0.8 qC0.3 qM0.1", "population": population,
                   "population_total": population, "max_candidates_per_round": round_size,
                   "per_gpu": per_gpu, "rounds": round_sizes, "nfold": args.nfold,
                   "epochs": list(epochs), "learning_rate": list(lrs), "samples": args.samples,
                   "loss": args.loss, "backend": args.backend or ("hip" if device.type == "cuda" else "torch"),
                   "fold_reset": args.fold_reset, "batch_norm": args.batch_norm, "batching": "keras (8000 = 250 x 32: no short batch)",
                   "fp32_impl": ("fp32 tensors, 3-way exact bf16 split x 6 MFMA terms per product"
                                 if device.type == "cuda" and (args.backend or "hip") == "hip"
                                 else "stock PyTorch fp32 ops (MIOpen / hipBLASLt)") if args.dtype == "fp32" else None,
                   "torch_population_batched": (not args.torch_unbatched) if args.backend == "torch" else None,
                   "streams_per_gpu": args.streams, "pop_batch": args.pop_batch,
                   "kernels": "generic only" if args.generic_kernels else "shape-specialised where available",
                   "fast_path": fast_path},
        "generations": len(completed),
        "evals": total_evals,
        "timed_candidates": timed_evals,
        "elapsed_s": round(elapsed, 3),
        "best_val_acc_at_gen": round(last["best_cat_acc"], 5) if last and last["best_cat_acc"] is not None else None,
        "best_val_binary_acc_at_gen": round(last["best_fitness"], 5) if last else None,
        "best_gen": last["generation"] if last else None,
        "best_genes": last["best_genes"] if last else None,
        "best_val_cat_acc_by_gen": [round(c["best_cat_acc"], 4) if c["best_cat_acc"] is not None else None
                                    for c in completed],
        # population means per completed generation (the search signal: RR-GA keeps no elite, so the
        # best-by-generation curve is not monotone; the mean shows whether selection moves the population)
        "mean_val_cat_acc_by_gen": [round(c["mean_cat_acc"], 4) if c["mean_cat_acc"] is not None else None
                                    for c in completed],
        "mean_fitness_by_gen": [round(c["mean_fitness"], 5) if c["mean_fitness"] is not None else None
                                for c in completed],
        # the fittest individual evaluated in the run (also when no generation completed)
        "best_val_acc_evaluated": round(best_seen["cat"], 5) if best_seen else None,
        "best_genes_evaluated": best_seen.get("genes"),
    }
    return out


if __name__ == "__main__":
    main()
