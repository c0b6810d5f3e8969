// GBDT on MI355X: histogram / split / partition / predict kernels plus the
// host driver that runs xgboost-style k-fold CV with them (SURVEY.md §2.4
// G2-G8; reference call site gentun/models/xgboost_models.py:32-36).
//
// Device layout: feature-major uint8 bins binsT[F][n] (a workgroup reading
// one feature for consecutive rows is coalesced), per-fold margins, grad/hess
// and a row -> node map. One tree level = one histogram launch:
//   grid (feature blocks of FB features, row chunks); each workgroup keeps a
//   private LDS histogram [FB][nodes_in_group][256 bins] of (G, H), filled
//   with LDS float atomics, then flushed with one global float atomic per
//   (feature, node, bin) it touched (Guideline 12: partial reduce first).
// Split search: one wave per (node, feature) scans the 256-bin prefix sums
// with xgboost's CalcGain (lambda, alpha L1 soft-threshold, max_delta_step,
// min_child_weight) and reduces the best gain with shuffles; the host picks
// the best feature per node (gamma pruning) and issues the partition kernel.
// Histogram float atomics make the last bits order-dependent (like
// xgboost's gpu_hist); the CPU engine (csrc/gbdt/engine.cpp) is the
// bit-reproducible reference.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#define GB_BINS 256
#define GB_FB 2          // features per histogram workgroup
#define GB_NG 16         // nodes per histogram pass

namespace {

struct DevParams {
  float min_child_weight, lambda, alpha, max_delta_step;
};

__device__ __forceinline__ float thr_l1(float g, float a) { return g > a ? g - a : (g < -a ? g + a : 0.f); }

__device__ __forceinline__ float dev_weight(const DevParams& p, float G, float H) {
  if (H < p.min_child_weight || H <= 0.f) return 0.f;
  float w = -thr_l1(G, p.alpha) / (H + p.lambda);
  if (p.max_delta_step != 0.f && fabsf(w) > p.max_delta_step) w = copysignf(p.max_delta_step, w);
  return w;
}

__device__ __forceinline__ float dev_gain(const DevParams& p, float G, float H) {
  if (H < p.min_child_weight || H <= 0.f) return 0.f;
  if (p.max_delta_step == 0.f) {
    const float t = thr_l1(G, p.alpha);
    return t * t / (H + p.lambda);
  }
  const float w = dev_weight(p, G, H);
  const float r = -(2.f * G * w + (H + p.lambda) * w * w);
  return p.alpha == 0.f ? r : r + p.alpha * fabsf(w);
}

// ---- G2: gradients ---------------------------------------------------------
// obj 0 squared error, 1 reg:logistic, 2 binary:logistic (scale_pos_weight)
__global__ void grad_kernel(const float* __restrict__ margin, const float* __restrict__ y,
                            const int* __restrict__ node_of_row, float2* __restrict__ gh, int n, int obj,
                            float spw) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    if (node_of_row[i] < 0) { gh[i] = make_float2(0.f, 0.f); continue; }
    float g, h;
    if (obj == 0) { g = margin[i] - y[i]; h = 1.f; }
    else {
      const float p = 1.f / (1.f + expf(-margin[i]));
      g = p - y[i]; h = fmaxf(p * (1.f - p), 1e-16f);
      if (obj == 2 && y[i] > 0.5f) { g *= spw; h *= spw; }
    }
    gh[i] = make_float2(g, h);
  }
}

// ---- G3: histograms ---------------------------------------------------------
// node_of_row holds the level-local node index (0 .. nodes-1) or -1.
__global__ void __launch_bounds__(256) hist_kernel(const uint8_t* __restrict__ binsT, const float2* __restrict__ gh,
                                                   const int* __restrict__ node_of_row, float2* __restrict__ hist,
                                                   int n, int F, int node_lo, int nodes_in_pass, int rows_per_block) {
  __shared__ float2 lh[GB_FB][GB_NG][GB_BINS];
  const int f0 = blockIdx.x * GB_FB;
  for (int i = threadIdx.x; i < GB_FB * GB_NG * GB_BINS; i += 256) (&lh[0][0][0])[i] = make_float2(0.f, 0.f);
  __syncthreads();
  const int r0 = blockIdx.y * rows_per_block;
  const int r1 = min(n, r0 + rows_per_block);
  for (int r = r0 + threadIdx.x; r < r1; r += 256) {
    const int nd = node_of_row[r] - node_lo;
    if (nd < 0 || nd >= nodes_in_pass) continue;
    const float2 v = gh[r];
#pragma unroll
    for (int j = 0; j < GB_FB; ++j) {
      if (f0 + j >= F) break;
      const int b = binsT[(long)(f0 + j) * n + r];
      atomicAdd(&lh[j][nd][b].x, v.x);
      atomicAdd(&lh[j][nd][b].y, v.y);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < GB_FB * nodes_in_pass * GB_BINS; i += 256) {
    const int j = i / (nodes_in_pass * GB_BINS);
    const int rem = i % (nodes_in_pass * GB_BINS);
    const int nd = rem / GB_BINS, b = rem % GB_BINS;
    if (f0 + j >= F) continue;
    const float2 v = lh[j][nd][b];
    if (v.x != 0.f || v.y != 0.f) {
      float2* dst = &hist[(((long)(node_lo + nd)) * F + f0 + j) * GB_BINS + b];
      atomicAdd(&dst->x, v.x);
      atomicAdd(&dst->y, v.y);
    }
  }
}

// ---- G4: best split per (node, feature): one wave each -----------------------
struct SplitOut { float gain; int bin; float GL, HL; };

__global__ void __launch_bounds__(64) split_kernel(const float2* __restrict__ hist, const int* __restrict__ nbins,
                                                   const uint8_t* __restrict__ feat_ok, const float2* __restrict__ tot,
                                                   SplitOut* __restrict__ out, int F, DevParams p) {
  const int node = blockIdx.y, f = blockIdx.x, lane = threadIdx.x;
  SplitOut best = {0.f, -1, 0.f, 0.f};
  if (feat_ok[f]) {
    const float2* h = hist + ((long)node * F + f) * GB_BINS;
    // each lane owns 4 consecutive bins; wave prefix over lane sums
    float2 v[4];
    float sg = 0.f, sh = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) { v[k] = h[lane * 4 + k]; sg += v[k].x; sh += v[k].y; }
    float pg = sg, ph = sh;                       // inclusive scan across lanes
    for (int o = 1; o < 64; o <<= 1) {
      const float tg = __shfl_up(pg, o), th = __shfl_up(ph, o);
      if (lane >= o) { pg += tg; ph += th; }
    }
    float GL = pg - sg, HL = ph - sh;             // exclusive prefix
    const float G = tot[node].x, H = tot[node].y;
    const float parent = dev_gain(p, G, H);
    const int nb = nbins[f];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      GL += v[k].x; HL += v[k].y;
      const int b = lane * 4 + k;
      if (b + 1 >= nb) continue;
      const float GR = G - GL, HR = H - HL;
      if (HL < p.min_child_weight || HR < p.min_child_weight || HL <= 0.f || HR <= 0.f) continue;
      const float chg = dev_gain(p, GL, HL) + dev_gain(p, GR, HR) - parent;
      if (chg > best.gain) { best.gain = chg; best.bin = b; best.GL = GL; best.HL = HL; }
    }
    for (int o = 32; o > 0; o >>= 1) {           // argmax, ties -> lower bin
      const float og = __shfl_xor(best.gain, o);
      const int ob = __shfl_xor(best.bin, o);
      const float oG = __shfl_xor(best.GL, o), oH = __shfl_xor(best.HL, o);
      if (og > best.gain || (og == best.gain && ob >= 0 && (best.bin < 0 || ob < best.bin))) {
        best.gain = og; best.bin = ob; best.GL = oG; best.HL = oH;
      }
    }
  }
  if (lane == 0) out[(long)node * F + f] = best;
}

// per-node totals: sum of hist over bins of feature 0 (all features give the same sum)
__global__ void totals_kernel(const float2* __restrict__ hist, float2* __restrict__ tot, int F) {
  const int node = blockIdx.x, lane = threadIdx.x;
  const float2* h = hist + (long)node * F * GB_BINS;
  float g = 0.f, hh = 0.f;
  for (int b = lane; b < GB_BINS; b += 64) { g += h[b].x; hh += h[b].y; }
  for (int o = 32; o > 0; o >>= 1) { g += __shfl_xor(g, o); hh += __shfl_xor(hh, o); }
  if (lane == 0) tot[node] = make_float2(g, hh);
}

// ---- G5: partition: level-local node -> child index of the next level --------
// split table per level node: (feature, bin, left_child_next, right_child_next) or feature < 0 = leaf
__global__ void partition_kernel(const uint8_t* __restrict__ binsT, int* __restrict__ node_of_row,
                                 const int4* __restrict__ split, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int nd = node_of_row[i];
    if (nd < 0) continue;
    const int4 s = split[nd];
    if (s.x < 0) { node_of_row[i] = -1; continue; }
    node_of_row[i] = (binsT[(long)s.x * n + i] <= s.y) ? s.z : s.w;
  }
}

// ---- G6: prediction update by tree traversal (all rows, train and test) -----
__global__ void predict_kernel(const uint8_t* __restrict__ binsT, const int4* __restrict__ tree,
                               const float* __restrict__ leaf, float* __restrict__ margin, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    int k = 0;
    int4 t = tree[0];
    while (t.x >= 0) { k = (binsT[(long)t.x * n + i] <= t.y) ? t.z : t.w; t = tree[k]; }
    margin[i] += leaf[k];
  }
}

// ---- G8: metric partial sums over a fold's train / test rows -----------------
// out[0..3] = (train sum, train count, test sum, test count); metric 0 rmse, 1 mae, 2 logloss, 3 error
__global__ void metric_kernel(const float* __restrict__ margin, const float* __restrict__ y,
                              const int* __restrict__ fold_of, int fold, int n, int metric, int obj,
                              double* __restrict__ out) {
  __shared__ double red[4][256];
  double s[4] = {0, 0, 0, 0};
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    float pred = margin[i];
    if (obj != 0 && metric != 3) pred = 1.f / (1.f + expf(-pred));
    float v;
    if (metric == 0) { const float d = pred - y[i]; v = d * d; }
    else if (metric == 1) v = fabsf(pred - y[i]);
    else if (metric == 2) {
      const float pc = fminf(fmaxf(pred, 1e-15f), 1.f - 1e-15f);
      v = -(y[i] * logf(pc) + (1.f - y[i]) * logf(1.f - pc));
    } else {
      const float pp = (obj == 0) ? pred : 1.f / (1.f + expf(-pred));
      v = ((pp > 0.5f) ? 1.f : 0.f) != (y[i] > 0.5f ? 1.f : 0.f) ? 1.f : 0.f;
    }
    const int k = (fold_of[i] == fold) ? 2 : 0;
    s[k] += v; s[k + 1] += 1.0;
  }
  for (int k = 0; k < 4; ++k) red[k][threadIdx.x] = s[k];
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o)
      for (int k = 0; k < 4; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x < 4) atomicAdd(&out[threadIdx.x], red[threadIdx.x][0]);
}

inline double h_thr(double g, double a) { return g > a ? g - a : (g < -a ? g + a : 0.0); }
inline double h_weight(const double* P, double G, double H) {
  // P: eta, mcw, depth, gamma, mds, subsample, cbt, cbl, lambda, alpha, spw, base
  if (H < P[1] || H <= 0.0) return 0.0;
  double w = -h_thr(G, P[9]) / (H + P[8]);
  if (P[4] != 0.0 && std::fabs(w) > P[4]) w = std::copysign(P[4], w);
  return w;
}

uint64_t smix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

#define HC(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return -100 - (int)e_; } while (0)

}  // namespace

extern "C" {

// Same contract as gbdt_cv (csrc/gbdt/engine.cpp) for objectives 0-3 and
// metrics rmse/mae/logloss/error; bins are precomputed on the host,
// FEATURE-MAJOR [F][n] (gbdt_quantize_fm; cached per dataset by the caller).
int gbdt_cv_hip(const uint8_t* binsT, const int* nbins_h, int n, int F, const float* y_h,
                const int* fold_h, int nfold, const double* P, int objective, const int* metrics, int n_metrics,
                int num_boost_round, int early_stopping_rounds, unsigned long long seed, double* out_hist) {
  if (objective > 3 || n_metrics != 1 || metrics[0] > 3) return -1;
  const int obj = objective == 0 ? 0 : (objective == 1 ? 1 : 2);
  const int metric = metrics[0];
  const int max_depth = std::max(0, (int)P[2]);
  // ---- device buffers
  uint8_t *d_bins, *d_fok;
  float *d_y, *d_margin, *d_leaf;
  int *d_fold, *d_node, *d_nb;
  float2 *d_gh, *d_hist, *d_tot;
  int4 *d_split, *d_tree;
  SplitOut* d_best;
  double* d_met;
  const int max_nodes = 1 << std::min(max_depth, 12);
  HC(hipMalloc(&d_bins, (size_t)n * F));
  HC(hipMalloc(&d_y, sizeof(float) * n));
  HC(hipMalloc(&d_fold, sizeof(int) * n));
  HC(hipMalloc(&d_node, sizeof(int) * n));
  HC(hipMalloc(&d_margin, sizeof(float) * (size_t)n * nfold));
  HC(hipMalloc(&d_gh, sizeof(float2) * n));
  HC(hipMalloc(&d_hist, sizeof(float2) * (size_t)max_nodes * F * GB_BINS));
  HC(hipMalloc(&d_tot, sizeof(float2) * max_nodes));
  HC(hipMalloc(&d_best, sizeof(SplitOut) * (size_t)max_nodes * F));
  HC(hipMalloc(&d_nb, sizeof(int) * F));
  HC(hipMalloc(&d_fok, F));
  HC(hipMalloc(&d_split, sizeof(int4) * max_nodes));
  HC(hipMalloc(&d_tree, sizeof(int4) * 2 * max_nodes * 2));
  HC(hipMalloc(&d_leaf, sizeof(float) * 2 * max_nodes * 2));
  HC(hipMalloc(&d_met, sizeof(double) * 4));
  HC(hipMemcpy(d_bins, binsT, (size_t)n * F, hipMemcpyHostToDevice));
  HC(hipMemcpy(d_y, y_h, sizeof(float) * n, hipMemcpyHostToDevice));
  HC(hipMemcpy(d_fold, fold_h, sizeof(int) * n, hipMemcpyHostToDevice));
  HC(hipMemcpy(d_nb, nbins_h, sizeof(int) * F, hipMemcpyHostToDevice));
  double base = P[11];
  if (obj != 0) { const double b = std::min(1 - 1e-7, std::max(1e-7, P[11])); base = std::log(b / (1 - b)); }
  {
    std::vector<float> m((size_t)n * nfold, (float)base);
    HC(hipMemcpy(d_margin, m.data(), sizeof(float) * m.size(), hipMemcpyHostToDevice));
  }
  DevParams dp{(float)P[1], (float)P[8], (float)P[9], (float)P[4]};
  const int blocks = std::min(2048, (n + 255) / 256);
  const int rows_per_block = std::max(4096, (n + 1023) / 1024);
  const int row_chunks = (n + rows_per_block - 1) / rows_per_block;
  std::vector<int> node0(n);
  std::vector<uint8_t> fok(F);
  std::vector<SplitOut> best((size_t)max_nodes * F);
  std::vector<float2> tot(max_nodes);
  const bool lower_better = true;
  double best_score = INFINITY;
  int best_round = 0, rounds_done = 0;
  for (int round = 0; round < num_boost_round; ++round) {
    double trv[64], tev[64];
    for (int k = 0; k < nfold; ++k) {
      // same splitmix stream and draw order as the CPU engine (engine.cpp round_fold / build_tree)
      uint64_t rs = smix(seed ^ smix((uint64_t)k * 1000003ull + (uint64_t)round * 7919ull + 17));
      auto next = [&]() { rs = smix(rs); return rs; };
      auto uni = [&]() { return (next() >> 11) * (1.0 / 9007199254740992.0); };
      // row sample of the fold's training rows -> level-0 node map
      for (int i = 0; i < n; ++i) node0[i] = (fold_h[i] != k && (P[5] >= 1.0 || uni() < P[5])) ? 0 : -1;
      HC(hipMemcpy(d_node, node0.data(), sizeof(int) * n, hipMemcpyHostToDevice));
      // colsample_bytree
      std::vector<int> feats(F);
      for (int f = 0; f < F; ++f) feats[f] = f;
      if (P[6] < 1.0) {
        const int kk = std::max(1, (int)std::floor(P[6] * F + 1e-9));
        for (int i = 0; i < F; ++i) std::swap(feats[i], feats[i + (int)(next() % (uint64_t)(F - i))]);
        feats.resize(kk);
        std::sort(feats.begin(), feats.end());
      }
      float* margin = d_margin + (size_t)k * n;
      hipLaunchKernelGGL(grad_kernel, dim3(blocks), dim3(256), 0, 0, margin, d_y, d_node, d_gh, n, obj,
                         (float)P[10]);
      // tree nodes in BFS order; level-local ids map to global node ids
      std::vector<int4> tree(1, make_int4(-1, 0, 0, 0));
      std::vector<float> leaf(1, 0.f);
      std::vector<int> level_nodes(1, 0);
      for (int depth = 0; depth <= max_depth && !level_nodes.empty(); ++depth) {
        const int L = (int)level_nodes.size();
        HC(hipMemset(d_hist, 0, sizeof(float2) * (size_t)L * F * GB_BINS));
        for (int lo = 0; lo < L; lo += GB_NG) {
          dim3 grid((F + GB_FB - 1) / GB_FB, row_chunks);
          hipLaunchKernelGGL(hist_kernel, grid, dim3(256), 0, 0, d_bins, d_gh, d_node, d_hist, n, F, lo,
                             std::min(GB_NG, L - lo), rows_per_block);
        }
        hipLaunchKernelGGL(totals_kernel, dim3(L), dim3(64), 0, 0, d_hist, d_tot, F);
        std::fill(fok.begin(), fok.end(), 0);
        std::vector<int> lf = feats;
        if (P[7] < 1.0 && lf.size() > 1) {
          const int m = (int)lf.size();
          const int kk = std::max(1, (int)std::floor(P[7] * m + 1e-9));
          for (int i = 0; i < m; ++i) std::swap(lf[i], lf[i + (int)(next() % (uint64_t)(m - i))]);
          lf.resize(kk);
        }
        for (int f : lf) fok[f] = 1;
        HC(hipMemcpy(d_fok, fok.data(), F, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(split_kernel, dim3(F, L), dim3(64), 0, 0, d_hist, d_nb, d_fok, d_tot, d_best, F, dp);
        HC(hipMemcpy(best.data(), d_best, sizeof(SplitOut) * (size_t)L * F, hipMemcpyDeviceToHost));
        HC(hipMemcpy(tot.data(), d_tot, sizeof(float2) * L, hipMemcpyDeviceToHost));
        std::vector<int4> split(L);
        std::vector<int> next;
        for (int j = 0; j < L; ++j) {
          const int gnode = level_nodes[j];
          const double G = tot[j].x, H = tot[j].y;
          leaf[gnode] = (float)(h_weight(P, G, H) * P[0]);
          int bf = -1;
          SplitOut bs = {0.f, -1, 0.f, 0.f};
          if (depth < max_depth) {
            for (int f = 0; f < F; ++f) {
              const SplitOut& c = best[(size_t)j * F + f];
              if (c.bin >= 0 && c.gain > bs.gain + 1e-12f) { bs = c; bf = f; }
            }
          }
          if (bf < 0 || bs.gain < P[3] || bs.gain <= 1e-12) {
            split[j] = make_int4(-1, 0, 0, 0);
            continue;
          }
          const int li = (int)tree.size();
          tree.push_back(make_int4(-1, 0, 0, 0));
          tree.push_back(make_int4(-1, 0, 0, 0));
          leaf.push_back(0.f);
          leaf.push_back(0.f);
          tree[gnode] = make_int4(bf, bs.bin, li, li + 1);
          split[j] = make_int4(bf, bs.bin, (int)next.size(), (int)next.size() + 1);
          next.push_back(li);
          next.push_back(li + 1);
        }
        if (next.empty()) break;
        HC(hipMemcpy(d_split, split.data(), sizeof(int4) * L, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(partition_kernel, dim3(blocks), dim3(256), 0, 0, d_bins, d_node, d_split, n);
        level_nodes = next;
      }
      HC(hipMemcpy(d_tree, tree.data(), sizeof(int4) * tree.size(), hipMemcpyHostToDevice));
      HC(hipMemcpy(d_leaf, leaf.data(), sizeof(float) * leaf.size(), hipMemcpyHostToDevice));
      hipLaunchKernelGGL(predict_kernel, dim3(blocks), dim3(256), 0, 0, d_bins, d_tree, d_leaf, margin, n);
      HC(hipMemset(d_met, 0, sizeof(double) * 4));
      hipLaunchKernelGGL(metric_kernel, dim3(std::min(blocks, 1024)), dim3(256), 0, 0, margin, d_y, d_fold, k, n,
                         metric, obj, d_met);
      double met[4];
      HC(hipMemcpy(met, d_met, sizeof(met), hipMemcpyDeviceToHost));
      double tr = met[0] / std::max(1.0, met[1]), te = met[2] / std::max(1.0, met[3]);
      if (metric == 0) { tr = std::sqrt(tr); te = std::sqrt(te); }
      trv[k] = tr; tev[k] = te;
    }
    double trm = 0, tem = 0, trs = 0, tes = 0;
    for (int k = 0; k < nfold; ++k) { trm += trv[k]; tem += tev[k]; }
    trm /= nfold; tem /= nfold;
    for (int k = 0; k < nfold; ++k) { trs += (trv[k] - trm) * (trv[k] - trm); tes += (tev[k] - tem) * (tev[k] - tem); }
    double* o = &out_hist[(size_t)round * 4];
    o[0] = trm; o[1] = std::sqrt(trs / nfold); o[2] = tem; o[3] = std::sqrt(tes / nfold);
    rounds_done = round + 1;
    if (lower_better ? tem < best_score : tem > best_score) { best_score = tem; best_round = round; }
    if (early_stopping_rounds > 0 && round - best_round >= early_stopping_rounds) break;
  }
  for (void* p : {(void*)d_bins, (void*)d_y, (void*)d_fold, (void*)d_node, (void*)d_margin, (void*)d_gh,
                  (void*)d_hist, (void*)d_tot, (void*)d_best, (void*)d_nb, (void*)d_fok, (void*)d_split,
                  (void*)d_tree, (void*)d_leaf, (void*)d_met})
    (void)hipFree(p);
  return early_stopping_rounds > 0 ? best_round + 1 : rounds_done;
}

}  // extern "C"
