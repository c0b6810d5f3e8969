// GBDT on MI355X: histogram / split / partition / predict kernels plus the
// host driver that runs xgboost-style k-fold CV with them (SURVEY.md §2.4
// G2-G8; reference call site gentun/models/xgboost_models.py:32-36).
//
// Layout: ROW-major uint8 bins [n][Fs] (Fs = F rounded up to 4), so one row's
// bins are a contiguous 32-byte run per 32-feature block. Each tree level keeps
// the active rows grouped by node in an index list (one contiguous segment per
// node, partitioned level by level), which gives the gpu_hist structure:
//   * histograms are built only for the SMALLER child of every split (its own
//     rows, gathered through the index list); the sibling is parent - built
//     (subtraction trick), so a level touches <= n/2 rows, not n per 16 nodes;
//   * a histogram workgroup = one row chunk of one node x 32 features: 8 lanes
//     read a row's 32 bins as 4-byte words, LDS float atomics into a
//     [32][257] float2 histogram (+1 float2 pad per feature spreads the banks),
//     then one global float atomic per non-zero entry (Guideline 12);
//   * the partition is one pass: left rows fill the parent's segment from its
//     start, right rows from its end (workgroup ballot scans + one cursor
//     atomic per wave side), so child segments need no count pre-pass.
// Split search: one wave per (node, feature) scans the 256-bin prefix sums with
// xgboost's CalcGain (lambda, alpha L1 soft-threshold, max_delta_step,
// min_child_weight); a per-node reduction picks the best feature on the device
// and the host only applies gamma pruning and lays out the next level.
// Histogram float atomics make the last bits order-dependent (like xgboost's
// gpu_hist); the CPU engine (csrc/gbdt/engine.cpp) is the bit-reproducible
// reference.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <vector>

#include "gbdt_cache.h"

#define GB_BINS 256
#define HB_F 16          // features per histogram workgroup
#define HB_STRIDE 514    // int64 per feature in the LDS histogram (256 (G,H) pairs + 1 pad pair)

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

// ---- G2: gradients (all rows; only indexed rows are ever read) -------------
// obj 0 squared error, 1 reg:logistic, 2 binary:logistic (scale_pos_weight)
__global__ void grad_kernel(const float* __restrict__ margin, const float* __restrict__ y,
                            float2* __restrict__ gh, int n, int obj, float spw) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
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

// multi:softmax / multi:softprob, class c of K: softmax over the row's K
// margins (engine.cpp: g = p_c - [y == c], h = max(2 p_c (1 - p_c), 1e-16))
__global__ void grad_multi_kernel(const float* __restrict__ margin, const float* __restrict__ y,
                                  float2* __restrict__ gh, int n, int K, int c) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const float* m = margin + (size_t)i * K;
    float mx = m[0];
    for (int k = 1; k < K; ++k) mx = fmaxf(mx, m[k]);
    float z = 0.f;
    for (int k = 0; k < K; ++k) z += expf(m[k] - mx);
    const float p = expf(m[c] - mx) / z;
    gh[i] = make_float2(p - ((int)y[i] == c ? 1.f : 0.f), fmaxf(2.f * p * (1.f - p), 1e-16f));
  }
}

// ---- G3: histograms -----------------------------------------------------------
// Fixed-point LDS accumulation: LDS float atomics measured 7x slower than the
// same loop with plain adds (profiles/gbdt_probe_depth6_10.log), so every
// row's (g, h) is scaled by a power of two chosen from the tree's max |g|,
// |h| and the row count (no overflow for any node) and summed with 64-bit
// integer LDS atomics: exact, order-independent sums -> the histograms (and
// with the fixed-order partial reduction, the whole GPU boosting run) are
// bitwise reproducible, unlike float atomics.

// max |g|, max |h| over all rows (bit patterns of non-negative floats order as ints)
__global__ void gh_max_kernel(const float2* __restrict__ gh, int n, unsigned int* __restrict__ mx) {
  unsigned int mg = 0, mh = 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const float2 v = gh[i];
    mg = max(mg, __float_as_uint(fabsf(v.x)));
    mh = max(mh, __float_as_uint(fabsf(v.y)));
  }
  for (int o = 32; o > 0; o >>= 1) { mg = max(mg, __shfl_xor(mg, o)); mh = max(mh, __shfl_xor(mh, o)); }
  if ((threadIdx.x & 63) == 0) { atomicMax(&mx[0], mg); atomicMax(&mx[1], mh); }
}

// scale exponent: max * 2^se * n < 2^62
__device__ __forceinline__ int fx_exp(unsigned int maxbits, int lg_n) {
  int e = 0;
  (void)frexpf(__uint_as_float(maxbits), &e);          // max < 2^e
  return min(100, 61 - e - lg_n);
}

// grid (chunks, feature blocks of HB_F), HB_T threads = HB_T/4 row lanes x 4 word
// lanes (16 features = 4 x 4 bin bytes per row); each lane keeps HB_U rows' loads in flight
#define HB_T 512
#define HB_U 4
__global__ void __launch_bounds__(HB_T) hist_kernel(const uint8_t* __restrict__ bins, int Fs, int F,
                                                    const int* __restrict__ rows, const float2* __restrict__ gh,
                                                    const int4* __restrict__ chunks, float2* __restrict__ hist,
                                                    unsigned long long* __restrict__ hist_part,
                                                    const unsigned int* __restrict__ mx, int lg_n) {
  __shared__ unsigned long long lh[HB_F * HB_STRIDE];
  const int4 c = chunks[blockIdx.x];
  const int fb = blockIdx.y * HB_F, tid = threadIdx.x;
  constexpr int RL = HB_T / 4;                  // row lanes
  for (int i = tid; i < HB_F * HB_STRIDE; i += HB_T) lh[i] = 0ull;
  const int seg = fx_exp(mx[0], lg_n), seh = fx_exp(mx[1], lg_n);
  const float sg = ldexpf(1.f, seg), sh = ldexpf(1.f, seh);
  __syncthreads();
  const int wl = tid & 3, rl = tid >> 2;
  const int f4 = fb + wl * 4;
  if (f4 < F) {
    const int* rp = rows + c.y;
    unsigned long long* my = lh + wl * 4 * HB_STRIDE;
    int i = rl;
    for (; i + (HB_U - 1) * RL < c.z; i += HB_U * RL) {
      int r[HB_U];
      float2 g[HB_U];
      uint32_t w[HB_U];
#pragma unroll
      for (int u = 0; u < HB_U; ++u) r[u] = rp[i + RL * u];
#pragma unroll
      for (int u = 0; u < HB_U; ++u) {
        g[u] = gh[r[u]];
        w[u] = *reinterpret_cast<const uint32_t*>(bins + (size_t)r[u] * Fs + f4);
      }
#pragma unroll
      for (int u = 0; u < HB_U; ++u) {
        const unsigned long long qg = (unsigned long long)llrintf(g[u].x * sg);
        const unsigned long long qh = (unsigned long long)llrintf(g[u].y * sh);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          unsigned long long* d = my + k * HB_STRIDE + 2 * ((w[u] >> (8 * k)) & 255u);
          atomicAdd(d, qg);
          atomicAdd(d + 1, qh);
        }
      }
    }
    for (; i < c.z; i += RL) {
      const int r = rp[i];
      const float2 g = gh[r];
      const uint32_t w = *reinterpret_cast<const uint32_t*>(bins + (size_t)r * Fs + f4);
      const unsigned long long qg = (unsigned long long)llrintf(g.x * sg);
      const unsigned long long qh = (unsigned long long)llrintf(g.y * sh);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        unsigned long long* d = my + k * HB_STRIDE + 2 * ((w >> (8 * k)) & 255u);
        atomicAdd(d, qg);
        atomicAdd(d + 1, qh);
      }
    }
  }
  __syncthreads();
  // flush with plain stores, no global atomics: a node that fits one chunk is
  // written straight into its (float) histogram, otherwise its exact integer
  // sums go to partial slot c.w (reduce_kernel adds a node's slots exactly,
  // so the result does not depend on which rows a chunk got)
  const int nf = min(HB_F, F - fb);
  if (c.w < 0) {
    float* dst = reinterpret_cast<float*>(hist + (size_t)c.x * F * GB_BINS) + (size_t)fb * 2 * GB_BINS;
    const float ig = ldexpf(1.f, -seg), ih = ldexpf(1.f, -seh);
    for (int i = tid; i < nf * 2 * GB_BINS; i += HB_T) {
      const int fl = i >> 9, j = i & 511;
      const long long v = (long long)lh[fl * HB_STRIDE + j];
      dst[(size_t)fl * 2 * GB_BINS + j] = (float)v * ((j & 1) ? ih : ig);
    }
  } else {
    unsigned long long* dst = hist_part + ((size_t)c.w * F + fb) * 2 * GB_BINS;
    for (int i = tid; i < nf * 2 * GB_BINS; i += HB_T) {
      const int fl = i >> 9, j = i & 511;
      dst[(size_t)fl * 2 * GB_BINS + j] = lh[fl * HB_STRIDE + j];
    }
  }
}

// node histogram = sum of its partial slots; red = (node, first slot, slots)
__global__ void __launch_bounds__(256) reduce_kernel(const unsigned long long* __restrict__ part,
                                                     float* __restrict__ hist, const int4* __restrict__ red, int F,
                                                     const unsigned int* __restrict__ mx, int lg_n) {
  const int4 rd = red[blockIdx.x];
  const size_t per = (size_t)F * 2 * GB_BINS;
  const float ig = ldexpf(1.f, -fx_exp(mx[0], lg_n)), ih = ldexpf(1.f, -fx_exp(mx[1], lg_n));
  for (size_t e = threadIdx.x + (size_t)blockIdx.y * 256; e < per; e += (size_t)gridDim.y * 256) {
    unsigned long long acc = 0;
    for (int sl = 0; sl < rd.z; ++sl) acc += part[(size_t)(rd.y + sl) * per + e];
    hist[(size_t)rd.x * per + e] = (float)(long long)acc * ((e & 1) ? ih : ig);
  }
}

// root rows of fold k: rows of the other folds, Bernoulli(subsample) by a
// counter-based hash keyed by one draw of the tree's stream (engine.cpp
// row_uniform); unordered compaction (ballot + one counter atomic per wave)
__global__ void __launch_bounds__(256) root_rows_kernel(const int* __restrict__ fold_of, int fold, int n,
                                                        unsigned long long key, double subsample,
                                                        int* __restrict__ rows, int* __restrict__ count) {
  const int lane = threadIdx.x & 63;
  const unsigned long long below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int base = blockIdx.x * blockDim.x; base < n; base += gridDim.x * blockDim.x) {
    const int i = base + threadIdx.x;
    bool keep = i < n && fold_of[i] != fold;
    if (keep && subsample < 1.0) {
      unsigned long long x = (unsigned long long)i + 0x9E3779B97F4A7C15ull;
      x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull; x = (x ^ (x >> 27)) * 0x94D049BB133111EBull; x ^= x >> 31;
      x = (key ^ x) + 0x9E3779B97F4A7C15ull;
      x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull; x = (x ^ (x >> 27)) * 0x94D049BB133111EBull; x ^= x >> 31;
      keep = (double)(x >> 11) * (1.0 / 9007199254740992.0) < subsample;
    }
    const unsigned long long m = __ballot(keep);
    int b0 = 0;
    if (lane == 0 && m) b0 = atomicAdd(count, __popcll(m));
    b0 = __shfl(b0, 0);
    if (keep) rows[b0 + __popcll(m & below)] = i;
  }
}

// sibling = parent (previous level) - built child; pairs (other, parent_prev, built)
__global__ void __launch_bounds__(256) subtract_kernel(const float2* __restrict__ prev, float2* __restrict__ cur,
                                                       const int4* __restrict__ pairs, int F) {
  const int4 pr = pairs[blockIdx.x];
  const size_t per = (size_t)F * GB_BINS;
  const float2* P = prev + (size_t)pr.y * per;
  const float2* B = cur + (size_t)pr.z * per;
  float2* O = cur + (size_t)pr.x * per;
  for (size_t i = threadIdx.x + (size_t)blockIdx.y * 256; i < per; i += (size_t)gridDim.y * 256) {
    const float2 a = P[i], b = B[i];
    O[i] = make_float2(a.x - b.x, a.y - b.y);
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

// best feature per node: ties -> lower feature (the host scan order of the CPU engine)
struct NodeBest { float gain; int bin; float GL, HL; int feature; int pad[3]; };

__global__ void __launch_bounds__(256) best_kernel(const SplitOut* __restrict__ cand, NodeBest* __restrict__ out,
                                                   int F) {
  __shared__ float sg[256];
  __shared__ int sf[256];
  const int node = blockIdx.x, tid = threadIdx.x;
  float bg = 0.f;
  int bf = -1;
  for (int f = tid; f < F; f += 256) {
    const SplitOut& c = cand[(size_t)node * F + f];
    if (c.bin >= 0 && c.gain > bg) { bg = c.gain; bf = f; }
  }
  sg[tid] = bg; sf[tid] = bf;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) {
      const float og = sg[tid + o];
      const int of = sf[tid + o];
      if (of >= 0 && (sf[tid] < 0 || og > sg[tid] || (og == sg[tid] && of < sf[tid]))) { sg[tid] = og; sf[tid] = of; }
    }
    __syncthreads();
  }
  if (tid == 0) {
    NodeBest b = {0.f, -1, 0.f, 0.f, -1, {0, 0, 0}};
    if (sf[0] >= 0) {
      const SplitOut& c = cand[(size_t)node * F + sf[0]];
      b.gain = c.gain; b.bin = c.bin; b.GL = c.GL; b.HL = c.HL; b.feature = sf[0];
    }
    out[node] = b;
  }
}

// ---- G5: partition ---------------------------------------------------------------
// chunks of split nodes' rows: (node, first index, count); split[node] = (feature, bin);
// cursors[node] = (next left slot, end of the right region); left grows up, right grows down
__global__ void __launch_bounds__(256) partition_kernel(const uint8_t* __restrict__ bins, int Fs,
                                                        const int* __restrict__ rows_in, int* __restrict__ rows_out,
                                                        const int4* __restrict__ chunks,
                                                        const int2* __restrict__ split, int2* __restrict__ cursors) {
  __shared__ int wl_cnt[4], wr_cnt[4], wl_base[4], wr_base[4];
  const int4 c = chunks[blockIdx.x];
  const int2 sp = split[c.x];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const unsigned long long below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int base = 0; base < c.z; base += 256) {
    const int i = base + tid;
    const bool valid = i < c.z;
    const int r = valid ? rows_in[c.y + i] : 0;
    const bool left = valid && bins[(size_t)r * Fs + sp.x] <= (uint8_t)sp.y;
    const bool right = valid && !left;
    const unsigned long long lm = __ballot(left), rm = __ballot(right);
    if (lane == 0) { wl_cnt[wv] = __popcll(lm); wr_cnt[wv] = __popcll(rm); }
    __syncthreads();
    if (tid == 0) {
      int tl = 0, tr = 0;
      for (int w = 0; w < 4; ++w) { tl += wl_cnt[w]; tr += wr_cnt[w]; }
      const int l0 = atomicAdd(&cursors[c.x].x, tl);
      const int r0 = atomicSub(&cursors[c.x].y, tr) - tr;
      int al = l0, ar = r0;
      for (int w = 0; w < 4; ++w) { wl_base[w] = al; al += wl_cnt[w]; wr_base[w] = ar; ar += wr_cnt[w]; }
    }
    __syncthreads();
    if (left) rows_out[wl_base[wv] + __popcll(lm & below)] = r;
    if (right) rows_out[wr_base[wv] + __popcll(rm & below)] = r;
    __syncthreads();
  }
}

// ---- G6: prediction update by tree traversal (all rows, train and test) -----
__global__ void predict_kernel(const uint8_t* __restrict__ bins, int Fs, const int4* __restrict__ tree,
                               const float* __restrict__ leaf, float* __restrict__ margin, int n, int K, int c) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    int k = 0;
    int4 t = tree[0];
    const uint8_t* row = bins + (size_t)i * Fs;
    while (t.x >= 0) { k = (row[t.x] <= t.y) ? t.z : t.w; t = tree[k]; }
    margin[(size_t)i * K + c] += leaf[k];
  }
}

// ---- G8: metric partial sums over a fold's train / test rows -----------------
// out[0..3] = (train sum, train count, test sum, test count); metric 0 rmse, 1 mae, 2 logloss, 3 error
__global__ void metric_kernel(const float* __restrict__ margin, const float* __restrict__ y,
                              const int* __restrict__ fold_of, int fold, int n, int metric, int objective, int K,
                              double* __restrict__ out) {
  // engine.cpp eval_metric: rmse/mae on sigmoid(margin) for reg:logistic / binary:logistic,
  // logloss on sigmoid, error thresholds margin 0 for binary:logitraw, merror / mlogloss over K
  __shared__ double red[4][256];
  double s[4] = {0, 0, 0, 0};
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const float* m = margin + (size_t)i * K;
    const float sig = 1.f / (1.f + expf(-m[0]));
    float v;
    if (metric == 0 || metric == 1) {
      const float d = ((objective == 1 || objective == 2) ? sig : m[0]) - y[i];
      v = metric == 0 ? d * d : fabsf(d);
    } else if (metric == 2) {
      const float pc = fminf(fmaxf(sig, 1e-15f), 1.f - 1e-15f);
      v = -(y[i] * logf(pc) + (1.f - y[i]) * logf(1.f - pc));
    } else if (metric == 3) {
      const bool pos = (objective == 3) ? (m[0] > 0.f) : (sig > 0.5f);
      v = (pos != (y[i] > 0.5f)) ? 1.f : 0.f;
    } else {
      int arg = 0;
      float mx = m[0];
      for (int k = 1; k < K; ++k) if (m[k] > mx) { mx = m[k]; arg = k; }
      if (metric == 5) v = (arg != (int)y[i]) ? 1.f : 0.f;
      else {
        float z = 0.f;
        for (int k = 0; k < K; ++k) z += expf(m[k] - mx);
        v = -logf(fmaxf(1e-15f, expf(m[(int)y[i]] - mx) / z));
      }
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
  if (threadIdx.x < 4) out[blockIdx.x * 4 + threadIdx.x] = red[threadIdx.x][0];   // host sums in block order
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

namespace gbdt_cache {
uint8_t* bins = nullptr;
long long key = 0;
size_t bytes = 0;
std::mutex mu;
}  // namespace gbdt_cache

extern "C" {

// Same contract as gbdt_cv (csrc/gbdt/engine.cpp) for every objective
// (reg:linear/squarederror, reg:logistic, binary:logistic/logitraw,
// multi:softmax/softprob: one tree per class) and every metric but auc
// (rmse, mae, logloss, error, merror, mlogloss; early stopping on the last).
// bins_h may be null when gbdt_quantize_hip already left the dataset's bins
// on the device under cache_key (returns -7 if they were evicted). bins: ROW-major [n][Fs] uint8 (Fs >= F,
// Fs % 4 == 0), precomputed on the host. cache_key != 0 keeps the device copy
// of the bins across calls for the same key (one dataset, many candidates).
int gbdt_cv_hip(const uint8_t* bins_h, int Fs, const int* nbins_h, int n, int F, const float* y_h,
                const int* fold_h, int nfold, const double* P, int objective, int num_class, const int* metrics,
                int n_metrics, int num_boost_round, int early_stopping_rounds, unsigned long long seed,
                long long cache_key, double* out_hist) {
  if (objective < 0 || objective > 5 || n_metrics < 1 || Fs % 4 || Fs < F || n <= 0 || nfold <= 0) return -1;
  for (int mi = 0; mi < n_metrics; ++mi)
    if (metrics[mi] < 0 || metrics[mi] > 6 || metrics[mi] == 4) return -1;   // auc: CPU engine
  const bool multi = objective >= 4;
  const int K = multi ? std::max(2, num_class) : 1;
  const int obj = objective == 0 ? 0 : (objective == 1 ? 1 : 2);
  const int max_depth = std::max(0, std::min((int)P[2], 12));
  std::lock_guard<std::mutex> lock(gbdt_cache::mu);   // one GBDT call at a time per process (bins cache)
  // ---- device buffers
  const size_t nbytes = (size_t)n * Fs;
  if (cache_key == 0 || cache_key != gbdt_cache::key || gbdt_cache::bytes != nbytes || gbdt_cache::bins == nullptr) {
    if (bins_h == nullptr) return -7;      // device copy evicted: the caller quantises again
    if (gbdt_cache::bins) (void)hipFree(gbdt_cache::bins);
    gbdt_cache::bins = nullptr; gbdt_cache::key = 0; gbdt_cache::bytes = 0;
    HC(hipMalloc(&gbdt_cache::bins, nbytes));
    HC(hipMemcpy(gbdt_cache::bins, bins_h, nbytes, hipMemcpyHostToDevice));
    gbdt_cache::key = cache_key; gbdt_cache::bytes = nbytes;
  }
  const uint8_t* d_bins = gbdt_cache::bins;
  float *d_y, *d_margin, *d_leaf;
  int *d_fold, *d_nb, *d_rows[3];
  float2 *d_gh, *d_hist[2], *d_tot;
  uint8_t* d_fok;
  int4 *d_chunks, *d_tree, *d_pairs;
  int2 *d_split, *d_cur;
  SplitOut* d_cand;
  NodeBest* d_best;
  double* d_met;
  const int max_level_nodes = 1 << max_depth;                         // nodes on the deepest level
  const int max_hist_nodes = 1 << std::max(0, max_depth - 1);         // levels that are split searched
  const size_t hist_node = (size_t)F * GB_BINS;
  HC(hipMalloc(&d_y, sizeof(float) * n));
  HC(hipMalloc(&d_fold, sizeof(int) * n));
  for (int b = 0; b < 3; ++b) HC(hipMalloc(&d_rows[b], sizeof(int) * n));
  HC(hipMalloc(&d_margin, sizeof(float) * (size_t)n * nfold * K));
  HC(hipMalloc(&d_gh, sizeof(float2) * n));
  for (int b = 0; b < 2; ++b) HC(hipMalloc(&d_hist[b], sizeof(float2) * (size_t)max_hist_nodes * hist_node));
  HC(hipMalloc(&d_tot, sizeof(float2) * max_level_nodes));
  HC(hipMalloc(&d_cand, sizeof(SplitOut) * (size_t)max_hist_nodes * F));
  HC(hipMalloc(&d_best, sizeof(NodeBest) * max_hist_nodes));
  HC(hipMalloc(&d_nb, sizeof(int) * F));
  HC(hipMalloc(&d_fok, F));
  const int max_chunks = 4096 + 2 * max_level_nodes;
  HC(hipMalloc(&d_chunks, sizeof(int4) * max_chunks));
  HC(hipMalloc(&d_pairs, sizeof(int4) * max_level_nodes));
  int4* d_reds;
  HC(hipMalloc(&d_reds, sizeof(int4) * max_chunks));
  HC(hipMalloc(&d_split, sizeof(int2) * max_level_nodes));
  HC(hipMalloc(&d_cur, sizeof(int2) * max_level_nodes));
  HC(hipMalloc(&d_tree, sizeof(int4) * 2 * max_level_nodes * 2));
  HC(hipMalloc(&d_leaf, sizeof(float) * 2 * max_level_nodes * 2));
  HC(hipMalloc(&d_met, sizeof(double) * 4 * 1024));
  HC(hipMemcpy(d_y, y_h, sizeof(float) * n, hipMemcpyHostToDevice));
  HC(hipMemcpy(d_fold, fold_h, sizeof(int) * n, hipMemcpyHostToDevice));
  HC(hipMemcpy(d_nb, nbins_h, sizeof(int) * F, hipMemcpyHostToDevice));
  double base = P[11];
  if (objective == 1 || objective == 2) {   // engine.cpp: logit base margin for the logistic objectives only
    const double b = std::min(1 - 1e-7, std::max(1e-7, P[11]));
    base = std::log(b / (1 - b));
  }
  {
    std::vector<float> m((size_t)n * nfold * K, (float)base);
    HC(hipMemcpy(d_margin, m.data(), sizeof(float) * m.size(), hipMemcpyHostToDevice));
  }
  DevParams dp{(float)P[1], (float)P[8], (float)P[9], (float)P[4]};
  const int blocks = std::min(2048, (n + 255) / 256);
  const int nfb = (F + HB_F - 1) / HB_F;
  int* d_count;
  HC(hipMalloc(&d_count, sizeof(int)));
  unsigned int* d_mx;                      // max |g|, |h| of the current tree (fixed-point scale)
  HC(hipMalloc(&d_mx, 2 * sizeof(unsigned int)));
  int lg_n = 0;
  while ((1ll << lg_n) < (long long)n + 1) ++lg_n;
  unsigned long long* d_part = nullptr;    // exact partial histograms of multi-chunk nodes
  int part_cap = 0;
  std::vector<int4> reds;
  std::vector<uint8_t> fok(F);
  std::vector<NodeBest> best(max_hist_nodes);
  std::vector<int4> chunks, pairs;
  std::vector<int2> split, cur;
  std::vector<float2> tot;

  struct Node { int gnode, start, count, parent; float G, H; bool built; };
  // chunk a set of (node, start, count) segments into row chunks of <= R rows
  auto add_chunks = [&](std::vector<int4>& out, int node, int start, int count, int R) {
    for (int o = 0; o < count; o += R) out.push_back(make_int4(node, start + o, std::min(R, count - o), 0));
  };
  const bool lower_better = true;
  double best_score = INFINITY;
  int best_round = 0, rounds_done = 0;
  // GENTUN_GBDT_TIMING=1: host wall time per phase (each phase ends in a blocking copy)
  static const bool timing = std::getenv("GENTUN_GBDT_TIMING") != nullptr;
  double ph[6] = {0, 0, 0, 0, 0, 0};    // rows, hist, split, partition, predict+metric, trees
  auto now = []() { return std::chrono::steady_clock::now(); };
  auto since = [&](std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double>(now() - t).count();
  };
  for (int round = 0; round < num_boost_round; ++round) {
    std::vector<double> trv((size_t)nfold * n_metrics), tev((size_t)nfold * n_metrics);
    for (int k = 0; k < nfold; ++k) {
      auto t0 = now();
      // same splitmix stream and draw order as the CPU engine (engine.cpp round_fold / build_tree)
      uint64_t rs = smix(seed ^ smix((uint64_t)k * 1000003ull + (uint64_t)round * 7919ull + 17));
      auto next = [&]() { rs = smix(rs); return rs; };
      auto uni = [&]() { return (next() >> 11) * (1.0 / 9007199254740992.0); };
      float* margin = d_margin + (size_t)k * n * K;
      for (int c = 0; c < K; ++c) {     // one tree per class (engine.cpp round_fold), margins updated in turn
        const unsigned long long row_key = P[5] < 1.0 ? next() : 0ull;   // engine.cpp: one draw keys the rows
        HC(hipMemsetAsync(d_count, 0, sizeof(int), 0));
        hipLaunchKernelGGL(root_rows_kernel, dim3(blocks), dim3(256), 0, 0, d_fold, k, n, row_key, P[5], d_rows[0],
                           d_count);
        int nroot = 0;
        HC(hipMemcpy(&nroot, d_count, sizeof(int), hipMemcpyDeviceToHost));
        ph[0] += since(t0);
        ph[5] += 1;
        // colsample_bytree
        std::vector<int> feats(F);
        for (int f = 0; f < F; ++f) feats[f] = f;
        if (P[6] < 1.0) {
          const int kk = std::max(1, (int)std::floor(P[6] * F + 1e-9));
          for (int i = 0; i < F; ++i) std::swap(feats[i], feats[i + (int)(next() % (uint64_t)(F - i))]);
          feats.resize(kk);
          std::sort(feats.begin(), feats.end());
        }
        if (multi)
          hipLaunchKernelGGL(grad_multi_kernel, dim3(blocks), dim3(256), 0, 0, margin, d_y, d_gh, n, K, c);
        else
          hipLaunchKernelGGL(grad_kernel, dim3(blocks), dim3(256), 0, 0, margin, d_y, d_gh, n, obj, (float)P[10]);
        HC(hipMemsetAsync(d_mx, 0, 2 * sizeof(unsigned int), 0));
        hipLaunchKernelGGL(gh_max_kernel, dim3(std::min(blocks, 512)), dim3(256), 0, 0, d_gh, n, d_mx);
        std::vector<int4> tree(1, make_int4(-1, 0, 0, 0));
        std::vector<float> leaf(1, 0.f);
        std::vector<Node> level(1, Node{0, 0, nroot, -1, 0.f, 0.f, true});
        int rb = 0;                   // row-list buffer holding this level's segments
        int hb = 0;                   // histogram buffer of this level
        for (int depth = 0; depth <= max_depth && !level.empty(); ++depth) {
          const int L = (int)level.size();
          if (depth == max_depth && depth > 0) {   // deepest level: leaves only, totals from the parent splits
            for (const Node& nd : level) leaf[nd.gnode] = (float)(h_weight(P, nd.G, nd.H) * P[0]);
            break;
          }
          // ---- histograms: built children over their rows, siblings by subtraction
          auto t1 = now();
          float2* hcur = d_hist[hb];
          chunks.clear(); pairs.clear(); reds.clear();
          long long built_rows = 0;
          for (const Node& nd : level) if (nd.built) built_rows += nd.count;
          const int R = std::max(2048, (int)((built_rows + 63) / 64));
          int nslots = 0;
          for (int j = 0; j < L; ++j) {
            const Node& nd = level[j];
            if (!nd.built) {
              pairs.push_back(make_int4(j, nd.parent, j ^ 1, 0));   // siblings are adjacent (2i, 2i+1)
            } else if (nd.count <= R) {                             // one chunk: written in place
              chunks.push_back(make_int4(j, nd.start, nd.count, -1));
            } else {                                                // partial slots + reduction
              const int first = nslots;
              for (int o = 0; o < nd.count; o += R)
                chunks.push_back(make_int4(j, nd.start + o, std::min(R, nd.count - o), nslots++));
              reds.push_back(make_int4(j, first, nslots - first, 0));
            }
          }
          if ((int)chunks.size() > max_chunks || (int)reds.size() > max_chunks) return -3;
          if (nslots > part_cap) {
            if (d_part) (void)hipFree(d_part);
            part_cap = std::max(nslots, 2 * part_cap);
            HC(hipMalloc(&d_part, sizeof(unsigned long long) * 2 * (size_t)part_cap * hist_node));
          }
          if (!chunks.empty()) {
            HC(hipMemcpy(d_chunks, chunks.data(), sizeof(int4) * chunks.size(), hipMemcpyHostToDevice));
            hipLaunchKernelGGL(hist_kernel, dim3((unsigned)chunks.size(), nfb), dim3(HB_T), 0, 0, d_bins, Fs, F,
                               d_rows[rb], d_gh, d_chunks, hcur, d_part, d_mx, lg_n);
          }
          if (!reds.empty()) {
            HC(hipMemcpy(d_reds, reds.data(), sizeof(int4) * reds.size(), hipMemcpyHostToDevice));
            hipLaunchKernelGGL(reduce_kernel, dim3((unsigned)reds.size(), std::max(1, (int)(hist_node * 2 / 4096))),
                               dim3(256), 0, 0, d_part, reinterpret_cast<float*>(hcur), d_reds, F, d_mx, lg_n);
          }
          if (!pairs.empty()) {
            HC(hipMemcpy(d_pairs, pairs.data(), sizeof(int4) * pairs.size(), hipMemcpyHostToDevice));
            hipLaunchKernelGGL(subtract_kernel, dim3((unsigned)pairs.size(), std::max(1, (int)(hist_node / 2048))),
                               dim3(256), 0, 0, d_hist[hb ^ 1], hcur, d_pairs, F);
          }
          // ---- node totals: root from its histogram, children from the parent's split
          if (depth == 0) {
            hipLaunchKernelGGL(totals_kernel, dim3(1), dim3(64), 0, 0, hcur, d_tot, F);
            float2 t0;
            HC(hipMemcpy(&t0, d_tot, sizeof(float2), hipMemcpyDeviceToHost));
            level[0].G = t0.x; level[0].H = t0.y;
          } else {
            tot.resize(L);
            for (int j = 0; j < L; ++j) tot[j] = make_float2(level[j].G, level[j].H);
            HC(hipMemcpy(d_tot, tot.data(), sizeof(float2) * L, hipMemcpyHostToDevice));
          }
          if (timing) { HC(hipDeviceSynchronize()); ph[1] += since(t1); t1 = now(); }
          // ---- split search (colsample_bylevel draw as in the CPU engine)
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
          hipLaunchKernelGGL(split_kernel, dim3(F, L), dim3(64), 0, 0, hcur, d_nb, d_fok, d_tot, d_cand, F, dp);
          hipLaunchKernelGGL(best_kernel, dim3(L), dim3(256), 0, 0, d_cand, d_best, F);
          HC(hipMemcpy(best.data(), d_best, sizeof(NodeBest) * L, hipMemcpyDeviceToHost));
          if (timing) { ph[2] += since(t1); t1 = now(); }
          // ---- host: leaves, gamma pruning, next level layout
          split.assign(L, make_int2(-1, 0));
          cur.assign(L, make_int2(0, 0));
          chunks.clear();
          std::vector<Node> nextl;
          std::vector<int> split_of;       // level node -> index of its left child in nextl (or -1)
          split_of.assign(L, -1);
          for (int j = 0; j < L; ++j) {
            Node& nd = level[j];
            leaf[nd.gnode] = (float)(h_weight(P, nd.G, nd.H) * P[0]);
            const NodeBest& b = best[j];
            if (depth >= max_depth || b.feature < 0 || b.bin < 0 || b.gain < P[3] || b.gain <= 1e-12f ||
                nd.count <= 0)
              continue;
            const int li = (int)tree.size();
            tree.push_back(make_int4(-1, 0, 0, 0));
            tree.push_back(make_int4(-1, 0, 0, 0));
            leaf.push_back(0.f);
            leaf.push_back(0.f);
            tree[nd.gnode] = make_int4(b.feature, b.bin, li, li + 1);
            split[j] = make_int2(b.feature, b.bin);
            cur[j] = make_int2(nd.start, nd.start + nd.count);
            split_of[j] = (int)nextl.size();
            nextl.push_back(Node{li, nd.start, 0, j, b.GL, b.HL, false});
            nextl.push_back(Node{li + 1, 0, 0, j, nd.G - b.GL, nd.H - b.HL, false});
            add_chunks(chunks, j, nd.start, nd.count, 4096);
          }
          if (nextl.empty()) break;
          if ((int)chunks.size() > max_chunks) return -3;
          // ---- partition the split nodes' rows into the other row buffer
          const int ob = (rb == 1) ? 2 : 1;
          HC(hipMemcpy(d_split, split.data(), sizeof(int2) * L, hipMemcpyHostToDevice));
          HC(hipMemcpy(d_cur, cur.data(), sizeof(int2) * L, hipMemcpyHostToDevice));
          HC(hipMemcpy(d_chunks, chunks.data(), sizeof(int4) * chunks.size(), hipMemcpyHostToDevice));
          hipLaunchKernelGGL(partition_kernel, dim3((unsigned)chunks.size()), dim3(256), 0, 0, d_bins, Fs,
                             d_rows[rb], d_rows[ob], d_chunks, d_split, d_cur);
          HC(hipMemcpy(cur.data(), d_cur, sizeof(int2) * L, hipMemcpyDeviceToHost));
          for (int j = 0; j < L; ++j) {
            if (split_of[j] < 0) continue;
            const Node& nd = level[j];
            const int lc = cur[j].x - nd.start;
            Node& l = nextl[split_of[j]];
            Node& r = nextl[split_of[j] + 1];
            l.count = lc;
            r.start = nd.start + lc; r.count = nd.count - lc;
            l.parent = r.parent = j;
            (l.count <= r.count ? l : r).built = true;     // smaller child: histogram; sibling: subtraction
          }
          if (timing) ph[3] += since(t1);
          level.swap(nextl);
          rb = ob;
          hb ^= 1;
        }
        auto t4 = now();
        HC(hipMemcpy(d_tree, tree.data(), sizeof(int4) * tree.size(), hipMemcpyHostToDevice));
        HC(hipMemcpy(d_leaf, leaf.data(), sizeof(float) * leaf.size(), hipMemcpyHostToDevice));
        hipLaunchKernelGGL(predict_kernel, dim3(blocks), dim3(256), 0, 0, d_bins, Fs, d_tree, d_leaf, margin, n, K, c);
      }
      auto t4 = now();
      const int mblocks = std::min(blocks, 1024);
      std::vector<double> mpart((size_t)mblocks * 4);
      for (int mi = 0; mi < n_metrics; ++mi) {
        const int metric = metrics[mi];
        hipLaunchKernelGGL(metric_kernel, dim3(mblocks), dim3(256), 0, 0, margin, d_y, d_fold, k, n, metric,
                           objective, K, d_met);
        HC(hipMemcpy(mpart.data(), d_met, sizeof(double) * mpart.size(), hipMemcpyDeviceToHost));
        double met[4] = {0, 0, 0, 0};
        for (int b = 0; b < mblocks; ++b)
          for (int q = 0; q < 4; ++q) met[q] += mpart[(size_t)b * 4 + q];
        double tr = met[0] / std::max(1.0, met[1]), te = met[2] / std::max(1.0, met[3]);
        if (metric == 0) { tr = std::sqrt(tr); te = std::sqrt(te); }
        trv[k * n_metrics + mi] = tr; tev[k * n_metrics + mi] = te;
      }
      ph[4] += since(t4);
    }
    double tem_last = 0;
    for (int mi = 0; mi < n_metrics; ++mi) {
      double trm = 0, tem = 0, trs = 0, tes = 0;
      for (int k = 0; k < nfold; ++k) { trm += trv[k * n_metrics + mi]; tem += tev[k * n_metrics + mi]; }
      trm /= nfold; tem /= nfold;
      for (int k = 0; k < nfold; ++k) {
        const double a = trv[k * n_metrics + mi] - trm, b = tev[k * n_metrics + mi] - tem;
        trs += a * a; tes += b * b;
      }
      double* o = &out_hist[((size_t)round * n_metrics + mi) * 4];
      o[0] = trm; o[1] = std::sqrt(trs / nfold); o[2] = tem; o[3] = std::sqrt(tes / nfold);
      tem_last = tem;                  // early stopping on the last metric (engine.cpp)
    }
    rounds_done = round + 1;
    if (lower_better ? tem_last < best_score : tem_last > best_score) { best_score = tem_last; best_round = round; }
    if (early_stopping_rounds > 0 && round - best_round >= early_stopping_rounds) break;
  }
  if (timing)
    std::fprintf(stderr, "[gbdt_hip] trees %.0f  rows %.3fs  hist %.3fs  split %.3fs  partition %.3fs  "
                 "predict+metric %.3fs\n", ph[5], ph[0], ph[1], ph[2], ph[3], ph[4]);
  (void)hipFree(d_count);
  (void)hipFree(d_mx);
  (void)hipFree(d_reds);
  if (d_part) (void)hipFree(d_part);
  for (void* p : {(void*)d_y, (void*)d_fold, (void*)d_rows[0], (void*)d_rows[1], (void*)d_rows[2],
                  (void*)d_margin, (void*)d_gh, (void*)d_hist[0], (void*)d_hist[1], (void*)d_tot, (void*)d_cand,
                  (void*)d_best, (void*)d_nb, (void*)d_fok, (void*)d_chunks, (void*)d_pairs, (void*)d_split,
                  (void*)d_cur, (void*)d_tree, (void*)d_leaf, (void*)d_met})
    (void)hipFree(p);
  return early_stopping_rounds > 0 ? best_round + 1 : rounds_done;
}

}  // extern "C"
