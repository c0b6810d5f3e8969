"""bf16 vs fp32 fitness of the same candidates: N random
S=(3,5) genomes, the bench protocol (5 folds, epochs (20,4,1), Adam, batch 32,
bce_compat loss, concurrent folds), trained once with fp32 tensors (exact
split-fp32 MFMA) and once in bf16. Prints per-candidate fitness and the
summary (mean / max |delta|, Spearman rank correlation, top-1 agreement).

usage: python tools/fitness_delta.py [N] [samples]"""
import json, os, random, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from gentun_amd.models import cnn_engine as E
from gentun_amd.models.genome import make_plan
from gentun_amd.utils.data import make_cifar_like, stratified_kfold
N = int(sys.argv[1]) if len(sys.argv) > 1 else 16
n = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
dev = torch.device("cuda", 0)
x, y = make_cifar_like(n=n, seed=0)
folds = stratified_kfold(np.argmax(y, 1), 5, seed=0)
rnd = random.Random(7)
genes = [{"S_1": "".join(rnd.choice("01") for _ in range(3)), "S_2": "".join(rnd.choice("01") for _ in range(10))}
         for _ in range(N)]
plans = [make_plan(g, (3, 5), (32, 32, 3), (20, 50), ((5, 5), (5, 5)), 500, 10) for g in genes]
res = {}
for dtype in ("fp32", "bf16"):
    cfg = E.TrainConfig(epochs=(20, 4, 1), learning_rate=(1e-3, 1e-4, 1e-5), batch_size=32, dtype=dtype,
                        loss="bce_compat", reset="all")
    t = time.perf_counter()
    out = E.make_population_job("hip", [(p, folds, list(range(5))) for p in plans], x, y, cfg, dev).launch().finish()
    res[dtype] = out
    print("[delta] {} trained {} candidates in {:.1f} s".format(dtype, N, time.perf_counter() - t), flush=True)


def spearman(a, b):
    ra, rb = np.argsort(np.argsort(a)), np.argsort(np.argsort(b))
    return float(np.corrcoef(ra, rb)[0, 1])


f32 = np.array([np.mean(r["binary_accuracy"]) for r in res["fp32"]])
b16 = np.array([np.mean(r["binary_accuracy"]) for r in res["bf16"]])
c32 = np.array([np.mean(r["categorical_accuracy"]) for r in res["fp32"]])
c16 = np.array([np.mean(r["categorical_accuracy"]) for r in res["bf16"]])
for i, g in enumerate(genes):
    print(json.dumps({"genes": "-".join(g[k] for k in sorted(g)), "fitness_fp32": round(float(f32[i]), 5),
                      "fitness_bf16": round(float(b16[i]), 5), "cat_fp32": round(float(c32[i]), 4),
                      "cat_bf16": round(float(c16[i]), 4)}))
print(json.dumps({"summary": True, "candidates": N, "mean_abs_delta_fitness": round(float(np.abs(f32 - b16).mean()), 6),
                  "max_abs_delta_fitness": round(float(np.abs(f32 - b16).max()), 6),
                  "mean_abs_delta_cat_acc": round(float(np.abs(c32 - c16).mean()), 5),
                  "max_abs_delta_cat_acc": round(float(np.abs(c32 - c16).max()), 5),
                  "spearman_fitness": round(spearman(f32, b16), 4), "spearman_cat_acc": round(spearman(c32, c16), 4),
                  "top1_same": int(np.argmax(f32)) == int(np.argmax(b16)),
                  "best_fp32": round(float(f32.max()), 5), "best_bf16": round(float(b16.max()), 5)}))
