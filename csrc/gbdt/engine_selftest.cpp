// Stand-alone driver of the C++ GBDT engine for host sanitizer builds
// (the reference has no race detection or sanitizers; its
// xgb.cv is an opaque library call, gentun/models/xgboost_models.py:28-37).
//
// Built by tests/test_sanitizers.py together with engine.cpp under
//   -fsanitize=address,undefined   (heap / stack bounds, UB in the split math)
//   -fsanitize=thread              (the multi-threaded histogram / quantiser)
// and run without Python in the process, so every report is the engine's.
// It walks the code paths the GA reaches: every objective family, every
// metric, row / column sampling, L1 / max_delta_step / gamma, early stopping,
// tiny folds (empty leaves) and both quantiser layouts.

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

extern "C" {
int gbdt_cv(const float* X, int n, int F, const float* y, const int* fold_of, int nfold, const double* params,
            int objective, int num_class, const int* metrics, int n_metrics, int num_boost_round,
            int early_stopping_rounds, unsigned long long seed, int nthreads, double* out_hist);
int gbdt_quantize(const float* X, int n, int F, uint8_t* bins_out, int* nbins_out);
int gbdt_quantize_fm(const float* X, int n, int F, uint8_t* bins_out, int* nbins_out);
}

namespace {

int failures = 0;

void check(bool ok, const char* what) {
  if (!ok) {
    std::fprintf(stderr, "FAIL: %s\n", what);
    ++failures;
  }
}

struct Data {
  int n, F;
  std::vector<float> X, y;
  std::vector<int> fold_of;
};

// kind 0: regression, 1: binary, 2: 3-class
Data make(int n, int F, int kind, int nfold, unsigned seed) {
  std::mt19937 g(seed);
  std::normal_distribution<float> nd(0.f, 1.f);
  Data d{n, F, std::vector<float>(size_t(n) * F), std::vector<float>(n), std::vector<int>(n)};
  for (int i = 0; i < n; ++i) {
    for (int f = 0; f < F; ++f) {
      float v = nd(g);
      if (f % 3 == 2) v = float(int(v * 2.f));      // few distinct values
      d.X[size_t(i) * F + f] = v;
    }
    const float* r = &d.X[size_t(i) * F];
    float s = r[0] - 0.5f * r[1] + 0.25f * r[F - 1] + 0.1f * nd(g);
    d.y[i] = kind == 0 ? s : kind == 1 ? float(s > 0.f) : float(s < -0.5f ? 0 : s < 0.5f ? 1 : 2);
    d.fold_of[i] = i % nfold;
  }
  return d;
}

//           eta  mcw  depth gamma mds  sub  cs_t cs_l lambda alpha spw  base
double P_default[12] = {0.3, 1, 6, 0, 0, 1, 1, 1, 1, 0, 1, 0.5};

int run(const Data& d, int nfold, const double* p, int obj, int ncls, std::vector<int> metrics, int rounds,
        int es, int threads) {
  std::vector<double> hist(size_t(rounds) * metrics.size() * 4, -1.0);
  int kept = gbdt_cv(d.X.data(), d.n, d.F, d.y.data(), d.fold_of.data(), nfold, p, obj, ncls, metrics.data(),
                     int(metrics.size()), rounds, es, 1234ull, threads, hist.data());
  check(kept > 0 && kept <= rounds, "gbdt_cv kept rows");
  for (int r = 0; r < kept; ++r)
    for (size_t j = 0; j < metrics.size() * 4; ++j) check(std::isfinite(hist[r * metrics.size() * 4 + j]), "finite");
  return kept;
}

}  // namespace

int main() {
  // quantiser, both layouts
  {
    Data d = make(5000, 13, 0, 5, 1);
    std::vector<uint8_t> b(size_t(d.n) * d.F), bfm(size_t(d.n) * d.F);
    std::vector<int> nb(d.F), nbfm(d.F);
    check(gbdt_quantize(d.X.data(), d.n, d.F, b.data(), nb.data()) == 0, "quantize rc");
    check(gbdt_quantize_fm(d.X.data(), d.n, d.F, bfm.data(), nbfm.data()) == 0, "quantize_fm rc");
    for (int f = 0; f < d.F; ++f) {
      check(nb[f] == nbfm[f] && nb[f] >= 1 && nb[f] <= 256, "bin counts");
      for (int i = 0; i < d.n; i += 97) check(b[size_t(i) * d.F + f] == bfm[size_t(f) * d.n + i], "layouts agree");
    }
  }
  // regression: sampling, L1, gamma, max_delta_step, early stopping, threads
  {
    Data d = make(3000, 9, 0, 5, 2);
    double p[12];
    std::memcpy(p, P_default, sizeof p);
    p[0] = 0.1; p[2] = 8; p[3] = 0.05; p[4] = 2; p[5] = 0.7; p[6] = 0.6; p[7] = 0.5; p[9] = 0.5;
    run(d, 5, p, 0, 0, {0, 1}, 200, 10, 4);
    run(d, 5, P_default, 1, 0, {0}, 20, 0, 1);        // reg:logistic on unscaled targets still finite
  }
  // binary: weights, logloss / error / auc
  {
    Data d = make(2000, 6, 1, 3, 3);
    double p[12];
    std::memcpy(p, P_default, sizeof p);
    p[10] = 3.0; p[1] = 0; p[8] = 0.1;
    run(d, 3, p, 2, 0, {2, 3, 4}, 50, 5, 3);
    run(d, 3, p, 3, 0, {2}, 10, 0, 2);                 // logitraw
  }
  // multiclass softprob / softmax
  {
    Data d = make(1500, 5, 2, 4, 4);
    run(d, 4, P_default, 5, 3, {5, 6}, 30, 5, 4);
    run(d, 4, P_default, 4, 3, {5}, 10, 0, 1);
  }
  // tiny data: folds of 2-3 rows, deep trees, empty children
  {
    Data d = make(7, 3, 0, 3, 5);
    double p[12];
    std::memcpy(p, P_default, sizeof p);
    p[1] = 0; p[2] = 10; p[8] = 0.0;
    run(d, 3, p, 0, 0, {0}, 5, 0, 8);
  }
  if (failures) {
    std::fprintf(stderr, "%d failure(s)\n", failures);
    return 1;
  }
  std::printf("selftest ok\n");
  return 0;
}
