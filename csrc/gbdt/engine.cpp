// Native histogram GBDT engine with xgboost-style k-fold cross-validation.
//
// Replaces the XGBoost 0.72 `DMatrix` + `xgb.cv` call of the reference
// (gentun/models/xgboost_models.py:28-37):
//   * G1 quantise: per feature <= 256 bins (exact unique values when they fit,
//     so small fixtures such as Iris / wine split exactly like exact-greedy);
//   * G2 grad/hess per objective (reg:linear|squarederror, reg:logistic,
//     binary:logistic|logitraw with scale_pos_weight, multi:softmax|softprob);
//   * G3 histograms with the subtraction trick (build the smaller child);
//   * G4 best split with lambda, alpha (L1 soft threshold), gamma,
//     min_child_weight, max_delta_step (xgboost's CalcGain/CalcWeight math);
//   * G5 partition, G6 leaf update (eta), G7 subsample / colsample_bytree /
//     colsample_bylevel, G8 metrics (rmse, mae, logloss, error, auc, merror,
//     mlogloss) per fold, mean/std over folds, early stopping on the mean
//     test value of the last metric; history truncated to the best round.
//
// Folds advance in lock-step (one boosting round of every fold, then the
// early-stopping check), each fold on its own thread. Deterministic: all
// sampling comes from a splitmix64 stream keyed by (seed, fold, round, node).
// The HIP kernels in hist.hip implement G3/G4 on MI355X for large data; the
// host engine owns the tree bookkeeping for both.

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <numeric>
#include <thread>
#include <vector>

namespace {

constexpr int kMaxBin = 256;

enum Objective { OBJ_SQUARED = 0, OBJ_LOGISTIC = 1, OBJ_BINARY_LOGISTIC = 2, OBJ_BINARY_LOGITRAW = 3,
                 OBJ_MULTI_SOFTMAX = 4, OBJ_MULTI_SOFTPROB = 5 };
enum Metric { M_RMSE = 0, M_MAE = 1, M_LOGLOSS = 2, M_ERROR = 3, M_AUC = 4, M_MERROR = 5, M_MLOGLOSS = 6 };

struct Params {
  double eta, min_child_weight, max_depth, gamma, max_delta_step, subsample, colsample_bytree,
      colsample_bylevel, lambda, alpha, scale_pos_weight, base_score;
};

inline uint64_t splitmix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed) {}
  uint64_t next() { s = splitmix(s); return s; }
  double uniform() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
};

inline double row_uniform(uint64_t key, uint64_t row) {
  return (splitmix(key ^ splitmix(row)) >> 11) * (1.0 / 9007199254740992.0);
}

inline double threshold_l1(double g, double alpha) {
  if (g > alpha) return g - alpha;
  if (g < -alpha) return g + alpha;
  return 0.0;
}
inline double calc_weight(const Params& p, double G, double H) {
  if (H < p.min_child_weight || H <= 0.0) return 0.0;
  double w = -threshold_l1(G, p.alpha) / (H + p.lambda);
  if (p.max_delta_step != 0.0 && std::fabs(w) > p.max_delta_step) w = std::copysign(p.max_delta_step, w);
  return w;
}
inline double calc_gain(const Params& p, double G, double H) {
  if (H < p.min_child_weight || H <= 0.0) return 0.0;
  if (p.max_delta_step == 0.0) {
    double t = threshold_l1(G, p.alpha);
    return t * t / (H + p.lambda);
  }
  double w = calc_weight(p, G, H);
  double ret = -(2.0 * G * w + (H + p.lambda) * w * w);
  return p.alpha == 0.0 ? ret : ret + p.alpha * std::fabs(w);
}

struct Quantized {
  int n = 0, F = 0;
  std::vector<uint8_t> bins;            // row-major [n][F]
  std::vector<int> nbins;               // per feature
};

// One feature column -> bins (exact: <= kMaxBin distinct values keep one bin
// each, otherwise kMaxBin equal-count quantile cuts). Writes bin b of row i
// at out[i * stride].
static int quantize_column(const float* X, int n, int F, int f, uint8_t* out, size_t stride,
                           std::vector<float>& col, std::vector<float>& sorted) {
  for (int i = 0; i < n; ++i) {
    float v = X[(size_t)i * F + f];
    col[i] = std::isnan(v) ? -std::numeric_limits<float>::infinity() : v;
  }
  sorted = col;
  std::sort(sorted.begin(), sorted.end());
  std::vector<float> uniq;
  uniq.reserve(256);
  for (int i = 0; i < n; ++i)
    if (uniq.empty() || sorted[i] != uniq.back()) {
      uniq.push_back(sorted[i]);
      if ((int)uniq.size() > kMaxBin) break;
    }
  std::vector<float> upper;           // bin b holds values <= upper[b]
  if ((int)uniq.size() <= kMaxBin) {
    upper = uniq;
  } else {
    // quantile cuts: kMaxBin bins of ~equal counts
    upper.reserve(kMaxBin);
    for (int b = 1; b <= kMaxBin; ++b) {
      size_t idx = std::min<size_t>((size_t)n - 1, (size_t)((double)b * n / kMaxBin) - (b == kMaxBin ? 1 : 0));
      float v = sorted[idx];
      if (upper.empty() || v > upper.back()) upper.push_back(v);
    }
    upper.back() = sorted[n - 1];
  }
  for (int i = 0; i < n; ++i) {
    int b = (int)(std::lower_bound(upper.begin(), upper.end(), col[i]) - upper.begin());
    if (b >= (int)upper.size()) b = (int)upper.size() - 1;
    out[(size_t)i * stride] = (uint8_t)b;
  }
  return (int)upper.size();
}

// Columns are independent: one thread per stripe of features (the per-column
// sort dominates: ~n log n per feature). feature_major: bins[f][n] (the GPU
// histogram layout) instead of bins[n][F].
static void quantize_into(const float* X, int n, int F, uint8_t* bins, int* nbins, bool feature_major) {
  int nt = (int)std::max(1u, std::thread::hardware_concurrency());
  nt = std::min(nt, std::max(1, F));
  auto work = [&](int t) {
    std::vector<float> col(n), sorted;
    for (int f = t; f < F; f += nt)
      nbins[f] = feature_major ? quantize_column(X, n, F, f, bins + (size_t)f * n, 1, col, sorted)
                               : quantize_column(X, n, F, f, bins + f, (size_t)F, col, sorted);
  };
  if (nt == 1 || (size_t)n * F < (1u << 16)) {
    nt = 1;
    work(0);
    return;
  }
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t) th.emplace_back(work, t);
  for (auto& x : th) x.join();
}

Quantized quantize(const float* X, int n, int F) {
  Quantized q;
  q.n = n; q.F = F;
  q.bins.resize((size_t)n * F);
  q.nbins.resize(F);
  quantize_into(X, n, F, q.bins.data(), q.nbins.data(), false);
  return q;
}

struct Node {
  int feature = -1, split_bin = -1, left = -1, right = -1;
  double value = 0.0;
};

struct GH { double g, h; };

struct Tree {
  std::vector<Node> nodes;
  double predict(const uint8_t* row) const {
    int k = 0;
    while (nodes[k].left >= 0) k = (row[nodes[k].feature] <= nodes[k].split_bin) ? nodes[k].left : nodes[k].right;
    return nodes[k].value;
  }
};

struct SplitResult {
  double gain = 0.0; int feature = -1, bin = -1; double GL = 0, HL = 0;
};

// Build one tree on rows `rows` (indices into the dataset) with grad/hess `gh`.
Tree build_tree(const Quantized& q, const std::vector<GH>& gh, std::vector<int>& rows, const Params& p,
                Rng& rng) {
  const int F = q.F;
  const int max_depth = std::max(0, (int)p.max_depth);
  Tree tree;
  // colsample_bytree
  std::vector<int> feats(F);
  std::iota(feats.begin(), feats.end(), 0);
  if (p.colsample_bytree < 1.0) {
    int k = std::max(1, (int)std::floor(p.colsample_bytree * F + 1e-9));
    for (int i = 0; i < F; ++i) std::swap(feats[i], feats[i + (int)(rng.next() % (uint64_t)(F - i))]);
    feats.resize(k);
    std::sort(feats.begin(), feats.end());
  }
  // colsample_bylevel: one draw keys the level streams (level d shuffles with
  // its own stream), so the tree stream's draw count does not depend on how
  // deep the tree grows -- the GPU engine precomputes every level's features
  const uint64_t level_key = p.colsample_bylevel < 1.0 ? rng.next() : 0ull;
  struct Work { int node; int begin, end; std::vector<GH> hist; double G, H; };
  auto build_hist = [&](int b, int e, std::vector<GH>& hist) {
    hist.assign((size_t)F * kMaxBin, GH{0.0, 0.0});
    for (int r = b; r < e; ++r) {
      const int i = rows[r];
      const uint8_t* row = &q.bins[(size_t)i * F];
      const GH v = gh[i];
      for (int f : feats) { GH& c = hist[(size_t)f * kMaxBin + row[f]]; c.g += v.g; c.h += v.h; }
    }
  };
  std::vector<Work> level;
  {
    Work root;
    root.node = 0; root.begin = 0; root.end = (int)rows.size();
    tree.nodes.emplace_back();
    build_hist(root.begin, root.end, root.hist);
    double G = 0, H = 0;
    for (int r = root.begin; r < root.end; ++r) { G += gh[rows[r]].g; H += gh[rows[r]].h; }
    root.G = G; root.H = H;
    level.push_back(std::move(root));
  }
  for (int depth = 0; depth <= max_depth && !level.empty(); ++depth) {
    std::vector<Work> next;
    // colsample_bylevel
    std::vector<int> lfeats = feats;
    if (p.colsample_bylevel < 1.0 && (int)lfeats.size() > 1) {
      int m = (int)lfeats.size();
      int k = std::max(1, (int)std::floor(p.colsample_bylevel * m + 1e-9));
      Rng lrng(splitmix(level_key ^ splitmix((uint64_t)depth + 1)));
      for (int i = 0; i < m; ++i) std::swap(lfeats[i], lfeats[i + (int)(lrng.next() % (uint64_t)(m - i))]);
      lfeats.resize(k);
    }
    for (Work& w : level) {
      Node& nd = tree.nodes[w.node];
      nd.value = calc_weight(p, w.G, w.H) * p.eta;
      if (depth == max_depth || w.end - w.begin < 2) continue;
      const double parent_gain = calc_gain(p, w.G, w.H);
      SplitResult best;
      for (int f : lfeats) {
        const GH* hf = &w.hist[(size_t)f * kMaxBin];
        double GL = 0, HL = 0;
        for (int b = 0; b + 1 < q.nbins[f]; ++b) {
          GL += hf[b].g; HL += hf[b].h;
          const double GR = w.G - GL, HR = w.H - HL;
          if (HL < p.min_child_weight || HR < p.min_child_weight || HL <= 0.0 || HR <= 0.0) continue;
          const double chg = calc_gain(p, GL, HL) + calc_gain(p, GR, HR) - parent_gain;
          if (chg > best.gain + 1e-12 || (best.feature < 0 && chg > 1e-12)) {
            best.gain = chg; best.feature = f; best.bin = b; best.GL = GL; best.HL = HL;
          }
        }
      }
      if (best.feature < 0 || best.gain < p.gamma || best.gain <= 1e-12) continue;
      // partition rows[w.begin, w.end) stably: left (bin <= split) first
      const int f = best.feature, sb = best.bin;
      auto mid_it = std::stable_partition(rows.begin() + w.begin, rows.begin() + w.end,
                                          [&](int i) { return q.bins[(size_t)i * F + f] <= sb; });
      const int mid = (int)(mid_it - rows.begin());
      const int li = (int)tree.nodes.size();
      tree.nodes.emplace_back();
      tree.nodes.emplace_back();
      Node& pn = tree.nodes[w.node];
      pn.feature = f; pn.split_bin = sb; pn.left = li; pn.right = li + 1;
      Work L, R;
      L.node = li; L.begin = w.begin; L.end = mid; L.G = best.GL; L.H = best.HL;
      R.node = li + 1; R.begin = mid; R.end = w.end; R.G = w.G - best.GL; R.H = w.H - best.HL;
      if (depth + 1 < max_depth) {
        // subtraction trick: build the smaller child, derive the larger
        Work& small = (L.end - L.begin <= R.end - R.begin) ? L : R;
        Work& large = (&small == &L) ? R : L;
        build_hist(small.begin, small.end, small.hist);
        large.hist = std::move(w.hist);
        for (size_t k = 0; k < large.hist.size(); ++k) {
          large.hist[k].g -= small.hist[k].g; large.hist[k].h -= small.hist[k].h;
        }
      }
      next.push_back(std::move(L));
      next.push_back(std::move(R));
    }
    level = std::move(next);
  }
  return tree;
}

inline double sigmoid(double x) { return 1.0 / (1.0 + std::exp(-x)); }

struct FoldState {
  std::vector<int> train, test;
  std::vector<double> margin;   // [n * K]
};

double auc_score(const std::vector<double>& s, const std::vector<double>& y) {
  const size_t n = s.size();
  std::vector<size_t> idx(n);
  std::iota(idx.begin(), idx.end(), 0);
  std::sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return s[a] < s[b]; });
  double npos = 0, nneg = 0, rank_sum = 0;
  size_t i = 0;
  while (i < n) {
    size_t j = i;
    while (j + 1 < n && s[idx[j + 1]] == s[idx[i]]) ++j;
    const double avg_rank = 0.5 * (i + j) + 1.0;
    for (size_t k = i; k <= j; ++k) if (y[idx[k]] > 0.5) { rank_sum += avg_rank; npos += 1; } else nneg += 1;
    i = j + 1;
  }
  if (npos == 0 || nneg == 0) return 0.5;
  return (rank_sum - npos * (npos + 1) / 2) / (npos * nneg);
}

double eval_metric(int metric, int obj, int K, const std::vector<int>& rows, const std::vector<double>& margin,
                   const float* y) {
  const double n = (double)std::max<size_t>(1, rows.size());
  const double eps = 1e-15;
  switch (metric) {
    case M_RMSE: case M_MAE: {
      double acc = 0;
      for (int i : rows) {
        double pred = margin[(size_t)i * K];
        if (obj == OBJ_LOGISTIC || obj == OBJ_BINARY_LOGISTIC) pred = sigmoid(pred);
        const double d = pred - y[i];
        acc += metric == M_RMSE ? d * d : std::fabs(d);
      }
      return metric == M_RMSE ? std::sqrt(acc / n) : acc / n;
    }
    case M_LOGLOSS: {
      double acc = 0;
      for (int i : rows) {
        double pr = std::min(1 - eps, std::max(eps, sigmoid(margin[(size_t)i * K])));
        acc += -(y[i] * std::log(pr) + (1 - y[i]) * std::log(1 - pr));
      }
      return acc / n;
    }
    case M_ERROR: {
      double acc = 0;
      for (int i : rows) {
        const double pr = (obj == OBJ_BINARY_LOGITRAW) ? margin[(size_t)i * K] : sigmoid(margin[(size_t)i * K]);
        const double thr = (obj == OBJ_BINARY_LOGITRAW) ? 0.0 : 0.5;
        acc += ((pr > thr) ? 1.0 : 0.0) != (y[i] > 0.5 ? 1.0 : 0.0);
      }
      return acc / n;
    }
    case M_AUC: {
      std::vector<double> s, yy;
      for (int i : rows) { s.push_back(margin[(size_t)i * K]); yy.push_back(y[i]); }
      return auc_score(s, yy);
    }
    case M_MERROR: case M_MLOGLOSS: {
      double acc = 0;
      for (int i : rows) {
        const double* m = &margin[(size_t)i * K];
        int arg = 0;
        double mx = m[0];
        for (int k = 1; k < K; ++k) if (m[k] > mx) { mx = m[k]; arg = k; }
        if (metric == M_MERROR) { acc += (arg != (int)y[i]); continue; }
        double z = 0;
        for (int k = 0; k < K; ++k) z += std::exp(m[k] - mx);
        const int c = (int)y[i];
        const double pr = std::max(eps, std::exp(m[c] - mx) / z);
        acc += -std::log(pr);
      }
      return acc / n;
    }
  }
  return 0.0;
}

bool higher_better(int metric) { return metric == M_AUC; }

}  // namespace

extern "C" {

#ifndef GT_SRC_HASH
#define GT_SRC_HASH "unhashed"
#endif
// content hash of the sources this library was compiled from (tools/build_native.py)
const char* gt_build_hash() { return GT_SRC_HASH; }

// params: eta, min_child_weight, max_depth, gamma, max_delta_step, subsample,
//         colsample_bytree, colsample_bylevel, lambda, alpha, scale_pos_weight, base_score
// out_hist: [num_boost_round][n_metrics][4] = train-mean, train-std, test-mean, test-std
// returns the number of rows of history kept (best round + 1), or <0 on error.
int gbdt_cv(const float* X, int n, int F, const float* y, const int* fold_of, int nfold, const double* params,
            int objective, int num_class, const int* metrics, int n_metrics, int num_boost_round,
            int early_stopping_rounds, unsigned long long seed, int nthreads, double* out_hist) {
  if (n <= 0 || F <= 0 || nfold <= 0 || n_metrics <= 0) return -1;
  Params p;
  std::memcpy(&p, params, sizeof(Params));
  const bool multi = (objective == OBJ_MULTI_SOFTMAX || objective == OBJ_MULTI_SOFTPROB);
  const int K = multi ? std::max(2, num_class) : 1;
  Quantized q = quantize(X, n, F);
  std::vector<FoldState> folds(nfold);
  double base_margin = p.base_score;
  if (objective == OBJ_LOGISTIC || objective == OBJ_BINARY_LOGISTIC) {
    const double b = std::min(1 - 1e-7, std::max(1e-7, p.base_score));
    base_margin = std::log(b / (1 - b));
  }
  for (int k = 0; k < nfold; ++k) {
    for (int i = 0; i < n; ++i) (fold_of[i] == k ? folds[k].test : folds[k].train).push_back(i);
    folds[k].margin.assign((size_t)n * K, base_margin);
  }
  if (nthreads <= 0) nthreads = (int)std::max(1u, std::thread::hardware_concurrency());
  const int eval_metric_id = metrics[n_metrics - 1];
  double best_score = higher_better(eval_metric_id) ? -INFINITY : INFINITY;
  int best_round = 0, rounds_done = 0;
  std::vector<double> train_vals((size_t)nfold * n_metrics), test_vals((size_t)nfold * n_metrics);

  auto round_fold = [&](int k, int round) {
    FoldState& fs = folds[k];
    const uint64_t fold_round = splitmix(seed ^ splitmix((uint64_t)k * 1000003ull + (uint64_t)round * 7919ull + 17));
    for (int c = 0; c < K; ++c) {
      // one stream per tree (class c of fold k, round): a fixed number of draws
      // per tree (row key, colsample_bytree, level key), so the GPU engine
      // (csrc/hip/gbdt_hist.hip) derives every tree's draws up front
      Rng rng(c == 0 ? fold_round : splitmix(fold_round ^ splitmix((uint64_t)c * 0x51ED27ull + 3)));
      std::vector<GH> gh(n, GH{0.0, 0.0});
      for (int i : fs.train) {
        const double* m = &fs.margin[(size_t)i * K];
        double g, h;
        if (objective == OBJ_SQUARED) { g = m[0] - y[i]; h = 1.0; }
        else if (!multi) {
          const double pr = sigmoid(m[0]);
          g = pr - y[i]; h = std::max(pr * (1 - pr), 1e-16);
          if (y[i] > 0.5 && objective != OBJ_LOGISTIC) { g *= p.scale_pos_weight; h *= p.scale_pos_weight; }
        } else {
          double mx = m[0];
          for (int j = 1; j < K; ++j) mx = std::max(mx, m[j]);
          double z = 0;
          for (int j = 0; j < K; ++j) z += std::exp(m[j] - mx);
          const double pr = std::exp(m[c] - mx) / z;
          g = pr - ((int)y[i] == c ? 1.0 : 0.0); h = std::max(2.0 * pr * (1 - pr), 1e-16);
        }
        gh[i] = GH{g, h};
      }
      std::vector<int> rows;
      rows.reserve(fs.train.size());
      if (p.subsample < 1.0) {
        // counter-based Bernoulli per row, keyed by one draw of the stream: the
        // GPU path (csrc/hip/gbdt_hist.hip root_rows_kernel) samples the same rows in parallel
        const uint64_t key = rng.next();
        for (int i : fs.train) if (row_uniform(key, (uint64_t)i) < p.subsample) rows.push_back(i);
      } else {
        rows = fs.train;
      }
      Tree t = build_tree(q, gh, rows, p, rng);
      for (int i = 0; i < n; ++i) fs.margin[(size_t)i * K + c] += t.predict(&q.bins[(size_t)i * F]);
    }
    for (int m = 0; m < n_metrics; ++m) {
      train_vals[(size_t)k * n_metrics + m] = eval_metric(metrics[m], objective, K, fs.train, fs.margin, y);
      test_vals[(size_t)k * n_metrics + m] = eval_metric(metrics[m], objective, K, fs.test, fs.margin, y);
    }
  };

  for (int round = 0; round < num_boost_round; ++round) {
    if (nthreads > 1 && nfold > 1) {
      std::vector<std::thread> th;
      std::atomic<int> next{0};
      const int nt = std::min(nthreads, nfold);
      for (int t = 0; t < nt; ++t)
        th.emplace_back([&]() { for (int k; (k = next.fetch_add(1)) < nfold;) round_fold(k, round); });
      for (auto& t : th) t.join();
    } else {
      for (int k = 0; k < nfold; ++k) round_fold(k, round);
    }
    for (int m = 0; m < n_metrics; ++m) {
      double trm = 0, tem = 0;
      for (int k = 0; k < nfold; ++k) { trm += train_vals[(size_t)k * n_metrics + m]; tem += test_vals[(size_t)k * n_metrics + m]; }
      trm /= nfold; tem /= nfold;
      double trs = 0, tes = 0;
      for (int k = 0; k < nfold; ++k) {
        const double a = train_vals[(size_t)k * n_metrics + m] - trm, b = test_vals[(size_t)k * n_metrics + m] - tem;
        trs += a * a; tes += b * b;
      }
      double* o = &out_hist[((size_t)round * n_metrics + m) * 4];
      o[0] = trm; o[1] = std::sqrt(trs / nfold); o[2] = tem; o[3] = std::sqrt(tes / nfold);
    }
    rounds_done = round + 1;
    const double score = out_hist[((size_t)round * n_metrics + (n_metrics - 1)) * 4 + 2];
    const bool better = higher_better(eval_metric_id) ? score > best_score : score < best_score;
    if (better) { best_score = score; best_round = round; }
    if (early_stopping_rounds > 0 && round - best_round >= early_stopping_rounds) break;
  }
  return early_stopping_rounds > 0 ? best_round + 1 : rounds_done;
}

// Quantise only (exposed for the HIP path and tests): bins out [n][F], nbins out [F].
int gbdt_quantize(const float* X, int n, int F, uint8_t* bins_out, int* nbins_out) {
  quantize_into(X, n, F, bins_out, nbins_out, false);
  return 0;
}

// Feature-major bins [F][n] for the GPU histogram path.
int gbdt_quantize_fm(const float* X, int n, int F, uint8_t* bins_out, int* nbins_out) {
  quantize_into(X, n, F, bins_out, nbins_out, true);
  return 0;
}

}  // extern "C"
