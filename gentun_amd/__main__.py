"""Command line entry points (the reference has none).

    python -m gentun_amd cnn   [--pop 20 --gens 50 --nodes 3,5 ...]   Genetic-CNN search
    python -m gentun_amd xgb   [--data iris|wine|PATH.csv --target COL]  GBDT hyper-parameter search
    python -m gentun_amd info                                            build / device summary

Multi-GPU: launch the same command under ``torchrun --nproc-per-node N``;
rank 0 runs the GA, every rank is an evaluator (RCCL over xGMI). Runs are
checkpointed per generation with ``--checkpoint-dir`` and resumed with
``--resume``.
"""

import argparse
import json
import os
import sys


def _ints(s):
    return tuple(int(v) for v in s.split(",")) if s else ()


def _floats(s):
    return tuple(float(v) for v in s.split(",")) if s else ()


class SearchFailed(SystemExit):
    """A search that cannot continue (every evaluation failed): exit code
    parallel.fault.EXIT_SEARCH_FAILED, which the restart supervisor does not retry."""

    def __init__(self):
        from .parallel.fault import EXIT_SEARCH_FAILED
        super(SearchFailed, self).__init__(EXIT_SEARCH_FAILED)


def _common(ap):
    from .config import RunConfig
    d = RunConfig.from_env()          # GENTUN_* environment over the defaults; flags win over both
    ap.add_argument("--pop", type=int, default=20)
    ap.add_argument("--gens", type=int, default=10)
    ap.add_argument("--algorithm", choices=("roulette", "tournament"), default="roulette")
    ap.add_argument("--seed", type=int, default=d.seed)
    ap.add_argument("--checkpoint-dir", default=d.checkpoint_dir)
    ap.add_argument("--resume", default=None,
                    help="checkpoint file or directory to continue from; 'auto': <checkpoint-dir>/latest.json if "
                         "it exists (restarted runs), else a fresh start")
    ap.add_argument("--watchdog", default=os.environ.get("GENTUN_WATCHDOG", ""),
                    help="per-generation deadline first_s[:factor[:min_s]]: a rank stuck past it (dead / hung "
                         "peer) exits with code 75 so the launcher can restart the group from the checkpoint")
    ap.add_argument("--events", default=d.events, help="JSONL event log path")
    ap.add_argument("--streams", type=int, default=d.streams, help="concurrent population jobs per GPU")
    ap.add_argument("--pop-batch", type=int, default=d.pop_batch,
                    help="Genetic-CNN candidates sharing each kernel launch")
    ap.add_argument("--pairing", choices=RunConfig.CHOICES["pairing"], default=d.pairing,
                    help="RussianRouletteGA pairs: reference (overlapping) or disjoint")
    ap.add_argument("--schedule", choices=RunConfig.CHOICES["schedule"], default=d.schedule,
                    help="distributed (candidate, fold) unit schedule")
    ap.add_argument("--collective-timeout", type=int, default=d.collective_timeout_s,
                    help="seconds before a collective with a dead rank fails the run")
    ap.add_argument("--backend", choices=("nccl", "gloo"), default=d.backend)


def _config(args):
    from .config import RunConfig
    return RunConfig(seed=args.seed, checkpoint_dir=args.checkpoint_dir, events=args.events,
                     collective_timeout_s=args.collective_timeout, dtype=getattr(args, "dtype", "fp32"),
                     loss=getattr(args, "loss", "bce_compat"), pairing=args.pairing, streams=args.streams,
                     pop_batch=args.pop_batch, schedule=args.schedule, backend=args.backend)


def _device():
    import torch
    if torch.cuda.is_available():
        lr = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(lr)
        return torch.device("cuda", lr)
    return torch.device("cpu")


def _release_evaluators(population, timeout_s):
    """Best-effort CMD_STOP to the evaluator ranks from a daemon thread, waited for at most
    ``timeout_s`` (returns whether it completed)."""
    import threading
    done = []

    def stop():
        try:
            population.shutdown()
            done.append(True)
        except Exception:  # noqa: BLE001 -- the original error is what gets reported
            pass

    t = threading.Thread(target=stop, daemon=True)
    t.start()
    t.join(timeout_s)
    if done:
        sys.stderr.write("[gentun] search aborted; evaluators released\n")
    return bool(done)


def _run_search(args, species, x, y, extra, maximize):
    from . import GeneticAlgorithm, RussianRouletteGA
    from .metrics import EventLog
    from .parallel import LocalBatchEvaluator, from_env
    from .parallel.distributed import DistributedPopulation, GentunWorker
    from .utils import rng
    cfg = _config(args)
    from .parallel.fault import parse_watchdog
    parse_watchdog(args.watchdog)             # malformed spec: one clear error at startup, on every rank
    if args.watchdog and args.watchdog.strip():
        os.environ["GENTUN_WATCHDOG"] = args.watchdog
    else:
        os.environ.pop("GENTUN_WATCHDOG", None)
    if args.resume == "auto":
        latest = os.path.join(cfg.checkpoint_dir or "", "latest.json")
        args.resume = latest if cfg.checkpoint_dir and os.path.exists(latest) else None
    device = _device()
    comm = from_env(backend=cfg.backend, timeout_s=cfg.collective_timeout_s, device=device)
    evaluator = LocalBatchEvaluator(device=device, streams=cfg.streams, pop_batch=cfg.pop_batch)
    if comm.rank != 0:
        GentunWorker(species, x, y, comm=comm, evaluator=evaluator).work()
        comm.finish()
        return None
    roulette = args.algorithm == "roulette"
    cls = RussianRouletteGA if roulette else GeneticAlgorithm
    ga_kw = {"pairing": cfg.pairing} if roulette else {}
    log = EventLog(cfg.events) if cfg.events else None
    if log is not None:
        log.write("config", **cfg.to_dict())
    if args.resume:
        def factory(inds):
            return DistributedPopulation(species, x, y, individual_list=inds, maximize=maximize,
                                         additional_parameters=extra, comm=comm, evaluator=evaluator,
                                         schedule=cfg.schedule)
        ga = cls.resume(args.resume, species, x, y, population_factory=factory, checkpoint_dir=cfg.checkpoint_dir,
                        event_log=log)
    else:
        rng.seed(cfg.seed)
        pop = DistributedPopulation(species, x, y, size=args.pop, maximize=maximize, additional_parameters=extra,
                                    comm=comm, evaluator=evaluator, schedule=cfg.schedule)
        ga = cls(pop, seed=cfg.seed, checkpoint_dir=cfg.checkpoint_dir, event_log=log, **ga_kw)
    from .parallel.distributed import AllEvaluationsFailed
    try:
        best = ga.run(args.gens)
    except AllEvaluationsFailed:
        import traceback
        traceback.print_exc()
        # every evaluator rank waits in the next dispatch broadcast: release them (CMD_STOP) before
        # failing, and exit with a code the restart supervisor does not retry (a failed search is
        # not a transient rank fault: resuming from the checkpoint would fail the same way). Any
        # other exception (a HIP launch failure, a checkpoint OSError, a dead peer's collective
        # error) propagates: a non-zero exit the supervisor restarts from the last checkpoint.
        try:
            ga.population.shutdown()
            comm.finish()
        finally:
            sys.stderr.write("[gentun] search failed; evaluators released\n")
        raise SearchFailed()
    except Exception:
        # Under torchrun the agent tears the group down. A plain MASTER_ADDR / RANK launch has no
        # agent: the evaluator ranks would wait in the next dispatch broadcast until the collective
        # timeout, so try to release them (bounded: a dead peer can make the broadcast hang too).
        if not os.environ.get("TORCHELASTIC_USE_AGENT_STORE"):
            _release_evaluators(ga.population, timeout_s=30.0)
        raise
    ga.population.shutdown()
    comm.finish()
    out = {"best_fitness": best.get_fitness(), "best_genes": best.get_genes(),
           "history": [{k: h[k] for k in ("generation", "best_fitness", "evals", "wall_s", "candidates_per_hour")}
                       for h in ga.history]}
    print(json.dumps(out, default=str))
    return out


def cmd_cnn(args):
    from . import GeneticCnnIndividual
    from .utils.data import make_glyph_classification, make_variant_classification
    shape = _ints(args.input_shape)
    if args.data == "hard":
        x, y = make_variant_classification(n=args.samples, shape=shape, classes=args.classes, seed=args.data_seed,
                                           noise=0.7 if args.noise is None else args.noise, label_noise=0.3)
    else:
        x, y = make_glyph_classification(n=args.samples, shape=shape, classes=args.classes, seed=args.data_seed,
                                         noise=1.0 if args.noise is None else args.noise)
    nodes = _ints(args.nodes)
    kernels = _ints(args.kernels)
    ks = tuple((k, k) for k in _ints(args.kernel_sizes))
    extra = dict(nodes=nodes, input_shape=shape, kernels_per_layer=kernels, kernel_sizes=ks,
                 dense_units=args.dense, dropout_probability=args.dropout, classes=args.classes, nfold=args.nfold,
                 epochs=_ints(args.epochs), learning_rate=_floats(args.lr), batch_size=args.batch, loss=args.loss,
                 seed=args.seed, optimizer=args.optimizer, momentum=args.momentum, dtype=args.dtype,
                 reset=args.fold_reset, batching=args.batching, batch_norm=args.batch_norm)
    return _run_search(args, GeneticCnnIndividual, x, y, extra, maximize=True)


def cmd_xgb(args):
    from . import XgboostIndividual
    from .utils import data
    if args.data == "iris":
        x, y = data.load_iris_xy()
    elif args.data == "wine":
        x, y = data.load_wine_quality()
    elif args.data == "synthetic":
        x, y = data.make_regression(n=args.rows, f=args.features)
    else:
        import pandas as pd
        df = pd.read_csv(args.data, sep=None, engine="python")
        y = df.pop(args.target).to_numpy()
        x = df.to_numpy()
    extra = dict(nfold=args.nfold, num_boost_round=args.rounds, early_stopping_rounds=args.early_stopping,
                 objective=args.objective, eval_metric=args.metric,
                 device="cuda:{}".format(os.environ.get("LOCAL_RANK", "0")) if args.gpu else None)
    return _run_search(args, XgboostIndividual, x, y, extra, maximize=False)


def cmd_info(_args):
    import torch
    from .ops import _lib
    info = {"torch": torch.__version__, "hip": getattr(torch.version, "hip", None),
            "gpu": torch.cuda.is_available()}
    libs = _lib.load_all(require_gpu=False)
    info["native"] = sorted(libs)
    if torch.cuda.is_available():
        info["device"] = torch.cuda.get_device_name(0)
    print(json.dumps(info))


def _env_default(name):
    from .config import RunConfig
    return getattr(RunConfig.from_env(), name)


def main(argv=None):
    ap = argparse.ArgumentParser(prog="python -m gentun_amd")
    sub = ap.add_subparsers(dest="cmd", required=True)
    c = sub.add_parser("cnn", help="Genetic-CNN architecture search")
    _common(c)
    c.add_argument("--nodes", default="3,5")
    c.add_argument("--kernels", default="20,50")
    c.add_argument("--kernel-sizes", default="5,5")
    c.add_argument("--input-shape", default="32,32,3")
    c.add_argument("--classes", type=int, default=10)
    c.add_argument("--samples", type=int, default=10000)
    c.add_argument("--noise", type=float, default=None, help="image noise (default 1.0 glyph / 0.7 hard)")
    c.add_argument("--data", choices=("glyph", "hard"), default="glyph",
                   help="glyph: stroke glyphs (every learned fold ~0.99); hard: glyph x tick variants with 30 %% "
                        "variant-label noise (accuracy depends on the architecture; the bench data)")
    c.add_argument("--data-seed", type=int, default=0)
    c.add_argument("--dense", type=int, default=500)
    c.add_argument("--dropout", type=float, default=0.5)
    c.add_argument("--nfold", type=int, default=5)
    c.add_argument("--epochs", default="20,4,1")
    c.add_argument("--lr", default="1e-3,1e-4,1e-5")
    c.add_argument("--batch", type=int, default=32)
    c.add_argument("--loss", choices=("bce_compat", "ce"), default=_env_default("loss"))
    c.add_argument("--dtype", choices=("bf16", "fp32"), default=_env_default("dtype"),
                   help="fp32 (reference precision; HIP: exact split-fp32 MFMA) or bf16 (fast mode)")
    c.add_argument("--optimizer", choices=("adam", "sgd"), default="adam")
    c.add_argument("--fold-reset", choices=("kernels", "all"), default="kernels",
                   help="kernels: reference sequential folds (biases carried over); all: concurrent folds (fast)")
    c.add_argument("--batching", choices=("keras", "wrap"), default="keras",
                   help="keras: short last batch; wrap: the last batch wraps around the epoch permutation")
    c.add_argument("--momentum", type=float, default=0.9, help="SGD momentum")
    c.add_argument("--batch-norm", action="store_true",
                   help="conv -> BatchNorm -> ReLU in every node (not in the reference network; off by default)")
    c.set_defaults(fn=cmd_cnn)
    x = sub.add_parser("xgb", help="GBDT (XGBoost-style) hyper-parameter search")
    _common(x)
    x.add_argument("--data", default="iris", help="iris | wine | synthetic | path to a CSV")
    x.add_argument("--target", default="quality")
    x.add_argument("--rows", type=int, default=100000)
    x.add_argument("--features", type=int, default=32)
    x.add_argument("--nfold", type=int, default=5)
    x.add_argument("--rounds", type=int, default=5000)
    x.add_argument("--early-stopping", type=int, default=100)
    x.add_argument("--objective", default="reg:linear")
    x.add_argument("--metric", default="rmse")
    x.add_argument("--gpu", action="store_true", help="run the GBDT histograms on the GPU")
    x.set_defaults(fn=cmd_xgb)
    i = sub.add_parser("info", help="build / device summary")
    i.set_defaults(fn=cmd_info)
    args = ap.parse_args(argv)
    return args.fn(args)


if __name__ == "__main__":
    sys.exit(0 if main() is not None or True else 1)
