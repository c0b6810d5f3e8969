#!/usr/bin/env python
"""Headline benchmark: Genetic-CNN candidates/hour on MI355X (BASELINE.json).

Config (BASELINE.md protocol, reference driver tests/test_mnist.py:22-34 on
CIFAR-10-shaped data): S=(3,5) nodes, kernels (20,50), 5x5 stage convs,
dense 500, dropout 0.5, 10 classes; each candidate = 5-fold CV on 10,000
synthetic 32x32x3 samples, epochs (20,4,1) with lr (1e-3,1e-4,1e-5), Adam,
batch 32 -- i.e. the full reference per-candidate protocol, nothing
skipped. Random-init weights, synthetic learnable data (no network).

One bench *step* = one GA generation of ``per_gpu x N`` freshly sampled
candidates, dispatched over the N evaluator ranks (one per GPU, RCCL
broadcast of the genome table + all_gather of fold scores) and trained
fold-batched + stream-concurrent on each GPU. Per-GPU work is fixed as N
grows (weak scaling). ``value`` = candidates evaluated in the K timed
steps / timed hours, over the whole job.

Run: ``python bench.py --gpus 1 --steps 2 --warmup 1`` or, for N>1,
``torchrun --nproc-per-node N bench.py --gpus N ...``.
"""

import argparse
import json
import os
import sys
import time


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--per-gpu", type=int, default=16, help="candidates per GPU per generation")
    ap.add_argument("--streams", type=int, default=1, help="concurrent population jobs per GPU")
    ap.add_argument("--pop-batch", type=int, default=16, help="candidates per population job (shared launches)")
    ap.add_argument("--backend", default=None, help="hip (default on GPU) or torch")
    ap.add_argument("--epochs", default="20,4,1")
    ap.add_argument("--lr", default="1e-3,1e-4,1e-5")
    ap.add_argument("--samples", type=int, default=10000)
    ap.add_argument("--nfold", type=int, default=5)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--space", choices=("default", "deep"), default="default",
                    help="default: S=(3,5) kernels (20,50) (headline); deep: BASELINE cfg 4, S=(3,4,5) kernels "
                         "(20,50,100) on 32x32 inputs")
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


def run(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
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

    from gentun_amd import GeneticCnnIndividual, LocalBatchEvaluator
    from gentun_amd.parallel import DistComm, LocalComm
    from gentun_amd.parallel.distributed import DistributedPopulation, GentunWorker
    from gentun_amd.utils import rng as grng
    from gentun_amd.utils.data import make_cifar_like

    if world > 1:
        # RCCL (backend "nccl") over xGMI between GPUs; GENTUN_DIST_BACKEND=gloo for rehearsals
        backend = os.environ.get("GENTUN_DIST_BACKEND") or ("nccl" if device.type == "cuda" else "gloo")
        comm = DistComm(backend=backend, device=device)
    else:
        comm = LocalComm()

    epochs = tuple(int(e) for e in args.epochs.split(","))
    lrs = tuple(float(x) for x in args.lr.split(","))
    x, y = make_cifar_like(n=args.samples, seed=0)
    nodes, kernels = ((3, 4, 5), (20, 50, 100)) if args.space == "deep" else ((3, 5), (20, 50))
    space = "S=({}) kernels ({})".format(",".join(map(str, nodes)), ",".join(map(str, kernels)))
    extra = dict(nodes=nodes, input_shape=(32, 32, 3), kernels_per_layer=kernels,
                 kernel_sizes=((5, 5),) * len(nodes), dense_units=500, dropout_probability=0.5, classes=10,
                 nfold=args.nfold, epochs=epochs, learning_rate=lrs, batch_size=32, dtype=args.dtype,
                 seed=args.seed, backend=args.backend)
    evaluator = LocalBatchEvaluator(device=device, streams=args.streams, pop_batch=args.pop_batch)
    P = args.per_gpu * comm.world_size

    if comm.rank != 0:
        # evaluator rank: serves EVAL / SYNC (timing fence) / STOP from rank 0
        GentunWorker(GeneticCnnIndividual, x, y, comm=comm, evaluator=evaluator).work()
        return None

    def make_pop(step):
        grng.seed(args.seed * 1000 + step)
        return DistributedPopulation(GeneticCnnIndividual, x, y, size=P, crossover_rate=0.3, mutation_rate=0.1,
                                     additional_parameters=extra, comm=comm, evaluator=evaluator)

    best = {"fitness": -1.0, "cat_acc": None, "genes": None}
    timed_evals = 0
    t_start = None
    pop = None
    for step in range(args.warmup + args.steps):
        pop = make_pop(step)
        if step == args.warmup:
            pop.sync_ranks()                     # barrier + device sync on every rank
            t_start = time.perf_counter()
        n = pop.evaluate_in_parallel()
        if step >= args.warmup:
            timed_evals += n
        for ind in pop:
            if ind.fitness is not None and ind.fitness > best["fitness"]:
                best = {"fitness": ind.fitness, "genes": dict(ind.get_genes())}
        print("[bench] step {} evaluated {} candidates ({}) dispatch={}".format(
            step, n, "timed" if step >= args.warmup else "warmup", pop.last_dispatch), file=sys.stderr, flush=True)
    pop.sync_ranks()
    elapsed = time.perf_counter() - t_start
    pop.shutdown()

    cph = 3600.0 * timed_evals / elapsed
    out = {
        "metric": "candidates/hour (Genetic-CNN {}, CIFAR-10-shaped, {}-fold CV, epochs ({}))".format(
            space.split(" kernels")[0], args.nfold, ",".join(str(e) for e in epochs)),
        "value": round(cph, 2),
        "unit": "candidates/hour",
        "n_gpus": comm.world_size,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000.0 * elapsed / max(1, args.steps), 2),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (CIFAR-10-shaped {}k x 32x32x3 coloured stroke glyphs + clutter + noise; "
                "random-init weights)".format(args.samples // 1000),
        "config": {"model": "Genetic-CNN {} dense 500".format(space), "global_batch": 32 * args.nfold,
                   "seq_len": None, "parallelism": "population-dp{}".format(comm.world_size),
                   "candidates_per_step": P, "per_gpu": args.per_gpu, "nfold": args.nfold,
                   "epochs": list(epochs), "learning_rate": list(lrs), "samples": args.samples,
                   "backend": args.backend or ("hip" if device.type == "cuda" else "torch"),
                   "streams_per_gpu": args.streams, "pop_batch": args.pop_batch},
        "best_val_binary_acc": round(best["fitness"], 5),
        "best_genes": best["genes"],
        "timed_candidates": timed_evals,
        "elapsed_s": round(elapsed, 3),
    }
    return out


if __name__ == "__main__":
    main()
