// GBDT on MI355X: xgboost-style k-fold CV with every fold's trees built
// TOGETHER and every tree level decided ON THE DEVICE (SURVEY.md §2.4 G2-G8;
// reference call site gentun/models/xgboost_models.py:32-36).
//
// Fold batching: the nfold boosters of a CV run advance in lock step; every
// launch covers all folds (grid z / y = fold), so one level of one round is a
// fixed sequence of ~8 launches whatever nfold is, and the launches are nfold
// times larger (fills 256 CUs at small n).
//
// Device-resident level loop: the level structure of a depth-D tree is static
// (level d has at most 2^d nodes, heap-indexed), so every grid is a host-known
// upper bound and the device decides which nodes exist. Per level:
//   hist      : (XCD-grouped workgroups) histograms of the "built" nodes (the root; then the smaller
//               child of every split) over their row segments, chunk lists
//               written by the previous level's plan kernel (blocks past the
//               fold's chunk count exit at once);
//   reduce    : multi-chunk nodes: exact sum of their partial slots;
//   subtract  : the sibling of every built node = parent - built (exact; on the
//               last histogram level the split search reads the difference
//               directly instead);
//   split     : one wave per (node, feature): 256-bin prefix scan, xgboost's
//               CalcGain (lambda, alpha L1 soft threshold, max_delta_step,
//               min_child_weight) in fp64; best: per-node argmax;
//   plan      : leaf weight (eta), gamma pruning, the split table, the tree
//               arrays, the children's totals;
//   partition : one pass over the level's row positions: left rows fill the
//               parent's segment from its start, right rows from its end
//               (wave-uniform ballot + one cursor atomic per side; per-lane
//               atomics at segment boundaries);
//   plan_next : children's segments, which child is built (the smaller, the
//               CPU engine's rule), the next level's chunk / reduction lists.
// No host round trip inside a round: the only blocking copy per round is the
// metric read-back that early stopping needs. The per-tree random draws
// (row-subsample key, colsample_bytree / _bylevel feature orders) do not
// depend on the data, so the host derives them up front (same streams as the
// CPU engine, csrc/gbdt/engine.cpp round_fold / build_tree) and uploads them
// with one asynchronous copy per round.
//
// Histograms are fixed point: every row's (g, h) is scaled by a power of two
// chosen from the fold's max |g|, |h| and the row count (no overflow for any
// node) and summed with 64-bit integer LDS atomics. Sums, the subtraction
// trick and the partial-slot reduction are exact and order independent, and
// the split search reads the exact integers into fp64: the GPU run is bitwise
// reproducible and follows the CPU engine (fp64 sums) to rounding level.
//
// Layout: ROW-major uint8 bins [n][Fs] (Fs = F rounded up to 4): a histogram
// lane reads 4 features of a row as one 4-byte word.

#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

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
// features per histogram workgroup: gradient-only packed image (constant hessian) / (g, h) pairs
#define HB_FC 32
#define HB_FG 16
#define HB_STRIDE 514    // int64 per feature in the LDS histogram (256 (G,H) pairs + 1 pad pair)
#define HB_T 512
#define HB_U 8           // rows in flight per thread
// rows per histogram chunk. 16K since round 5: with the reduce grid bounded by the nodes that can have
// partial slots, more chunks (= more histogram workgroups at the shallow levels) won: depth-6 level time
// -7.5 %, depth 10 even (r5/gbdt_chunk_ab_r5.txt; 64K had been chosen in round 3 against the old reduce)
#define GB_R 16384
#define GB_MAXD 12       // deepest supported tree

namespace {
typedef long long i64;
typedef unsigned long long u64;

struct DevParams {
  double min_child_weight, lambda, alpha, max_delta_step, eta, gamma;
};

__device__ __forceinline__ double thr_l1(double g, double a) { return g > a ? g - a : (g < -a ? g + a : 0.0); }

__device__ __forceinline__ double dev_weight(const DevParams& p, double G, double H) {
  if (H < p.min_child_weight || H <= 0.0) return 0.0;
  double w = -thr_l1(G, p.alpha) / (H + p.lambda);
  if (p.max_delta_step != 0.0 && fabs(w) > p.max_delta_step) w = copysign(p.max_delta_step, w);
  return w;
}

__device__ __forceinline__ double dev_gain(const DevParams& p, double G, double H) {
  if (H < p.min_child_weight || H <= 0.0) return 0.0;
  if (p.max_delta_step == 0.0) {
    const double t = thr_l1(G, p.alpha);
    return t * t / (H + p.lambda);
  }
  const double w = dev_weight(p, G, H);
  const double r = -(2.0 * G * w + (H + p.lambda) * w * w);
  return p.alpha == 0.0 ? r : r + p.alpha * fabs(w);
}

// one node of a level (per fold): row segment [start, start + count) in the
// level's row list; exact fixed-point totals; built = histogram from rows
// (else parent - sibling). Segments of a level are ordered by node index and
// (start + count) is non-decreasing: nodes that do not exist have count 0.
struct LNode {
  int start, count;
  i64 G, H;
  int exists, built, parent, pad;
};
struct Chunk { int node, start, count, slot; };      // slot -1: one chunk, written in place
struct Red { int node, first, nslots, pad; };
struct SplitOut { double gain; i64 GL, HL; int bin, order; };
struct NodeBest { double gain; i64 GL, HL; int feature, bin; };

// geometry of one CV call (kernel argument)
struct Geo {
  int n, F, Fs, nfold, K, max_depth;
  int Lmax;      // nodes of the deepest level (2^max_depth)
  int Lh;        // nodes with a histogram per level (2^(max_depth-1), >= 1)
  int maxch;     // chunk records per fold
  int maxslot;   // partial histogram slots per fold
  int lg_n;
  int rch;       // rows per histogram chunk (GB_R)
};

// ---- G2: gradients of every fold (all rows; only indexed rows are read) ----
// obj 0 squared error, 1 reg:logistic, 2 binary:logistic (scale_pos_weight), 3 multi (class c of K)
__global__ void grad_kernel(const float* __restrict__ margin, const float* __restrict__ y, float2* __restrict__ gh,
                            int n, int K, int c, int obj, float spw) {
  const int k = blockIdx.y;
  const float* mk = margin + (size_t)k * n * K;
  float2* gk = gh + (size_t)k * n;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    float g, h;
    if (obj == 0) {
      g = mk[i] - y[i]; h = 1.f;
    } else if (obj == 3) {
      const float* m = mk + (size_t)i * K;
      float mx = m[0];
      for (int q = 1; q < K; ++q) mx = fmaxf(mx, m[q]);
      float z = 0.f;
      for (int q = 0; q < K; ++q) z += expf(m[q] - mx);
      const float p = expf(m[c] - mx) / z;
      g = p - ((int)y[i] == c ? 1.f : 0.f); h = fmaxf(2.f * p * (1.f - p), 1e-16f);
    } else {
      const float p = 1.f / (1.f + expf(-mk[i]));
      g = p - y[i]; h = fmaxf(p * (1.f - p), 1e-16f);
      if (obj == 2 && y[i] > 0.5f) { g *= spw; h *= spw; }
    }
    gk[i] = make_float2(g, h);
  }
}

// max |g|, max |h| per fold (bit patterns of non-negative floats order as ints)
__global__ void gh_max_kernel(const float2* __restrict__ gh, int n, unsigned int* __restrict__ mx) {
  const int k = blockIdx.y;
  const float2* gk = gh + (size_t)k * n;
  unsigned int mg = 0, mh = 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const float2 v = gk[i];
    mg = max(mg, __float_as_uint(fabsf(v.x)));
    mh = max(mh, __float_as_uint(fabsf(v.y)));
  }
  for (int o = 32; o > 0; o >>= 1) { mg = max(mg, __shfl_xor(mg, o)); mh = max(mh, __shfl_xor(mh, o)); }
  __shared__ unsigned int sm[2][4];             // one atomic per workgroup (not per wave: they serialise at L2)
  if ((threadIdx.x & 63) == 0) { sm[0][threadIdx.x >> 6] = mg; sm[1][threadIdx.x >> 6] = mh; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) { mg = max(mg, sm[0][w]); mh = max(mh, sm[1][w]); }
    atomicMax(&mx[2 * k], mg);
    atomicMax(&mx[2 * k + 1], mh);
  }
}

// fixed-point exponent: max * 2^se * n < 2^62
__device__ __forceinline__ int fx_exp(unsigned int maxbits, int lg_n) {
  int e = 0;
  (void)frexpf(__uint_as_float(maxbits), &e);          // max < 2^e
  return min(100, 61 - e - lg_n);
}

// root rows of fold k: rows of the other folds, Bernoulli(subsample) by the
// counter-based hash of the CPU engine (engine.cpp row_uniform) keyed by one
// draw of the tree's stream. Unordered compaction with ONE cursor atomic per
// workgroup and 4096 rows (a per-wave atomic on the fold's single counter
// serialised at L2: 0.9 ms per fold at 1M rows)
#define RR_PER 16
__global__ void __launch_bounds__(256) root_rows_kernel(const int* __restrict__ fold_of, int n,
                                                        const u64* __restrict__ keys, double subsample,
                                                        int* __restrict__ rows, int* __restrict__ counts) {
  __shared__ int wtot[4];
  __shared__ int base_s;
  const int k = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const u64 key = keys[k];
  int* rk = rows + (size_t)k * n;
  for (long s0 = (long)blockIdx.x * 256 * RR_PER; s0 < n; s0 += (long)gridDim.x * 256 * RR_PER) {
    uint32_t keepm = 0;
#pragma unroll
    for (int j = 0; j < RR_PER; ++j) {
      const long i = s0 + (long)j * 256 + tid;
      bool keep = i < n && fold_of[i] != k;
      if (keep && subsample < 1.0) {
        u64 x = (u64)i + 0x9E3779B97F4A7C15ull;
        x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull; x = (x ^ (x >> 27)) * 0x94D049BB133111EBull; x ^= x >> 31;
        x = (key ^ x) + 0x9E3779B97F4A7C15ull;
        x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull; x = (x ^ (x >> 27)) * 0x94D049BB133111EBull; x ^= x >> 31;
        keep = (double)(x >> 11) * (1.0 / 9007199254740992.0) < subsample;
      }
      if (keep) keepm |= 1u << j;
    }
    const int cnt = __popc(keepm);
    int incl = cnt;                                // inclusive scan over the wave
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(incl, o);
      if (lane >= o) incl += t;
    }
    if (lane == 63) wtot[wv] = incl;
    __syncthreads();
    if (tid == 0) {
      const int tot = wtot[0] + wtot[1] + wtot[2] + wtot[3];
      base_s = tot ? atomicAdd(&counts[k], tot) : 0;
    }
    __syncthreads();
    int pos = base_s + incl - cnt;
    for (int w = 0; w < wv; ++w) pos += wtot[w];
#pragma unroll
    for (int j = 0; j < RR_PER; ++j)
      if ((keepm >> j) & 1u) rk[pos++] = (int)(s0 + (long)j * 256 + tid);
    __syncthreads();                               // wtot / base_s reused by the next slice
  }
}

// feature-major copy of the bins [Fs][n] for the partition's per-row
// lookups (row-major bins: every lookup its own cache line)
__global__ void __launch_bounds__(256) transpose_bins_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                             int n, int Fs) {
  __shared__ uint8_t t[64][65];
  const long r0 = (long)blockIdx.x * 64;
  const int f0 = blockIdx.y * 64;
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int r = i >> 6, f = i & 63;
    if (r0 + r < n && f0 + f < Fs) t[r][f] = in[(r0 + r) * Fs + f0 + f];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int f = i >> 6, r = i & 63;
    if (r0 + r < n && f0 + f < Fs) out[(long)(f0 + f) * n + r0 + r] = t[r][f];
  }
}

// chunk records of one built node (thread-serial; plan kernels)
__device__ void emit_node(Chunk* ch, Red* rd, int& nch, int& nrd, int& nslot, int node, int start, int count,
                          int rch) {
  if (count <= rch) {
    ch[nch++] = Chunk{node, start, count, -1};
    return;
  }
  const int first = nslot;
  for (int o = 0; o < count; o += rch) ch[nch++] = Chunk{node, start + o, min(rch, count - o), nslot++};
  rd[nrd++] = Red{node, first, nslot - first, 0};
}

// level 0 of every fold: the root over all its rows
__global__ void level0_kernel(Geo geo, const int* __restrict__ nroot, LNode* __restrict__ cur,
                              Chunk* __restrict__ chunks, Red* __restrict__ reds, int* __restrict__ counts) {
  const int k = blockIdx.x;
  if (threadIdx.x != 0) return;
  LNode r;
  r.start = 0; r.count = nroot[k]; r.G = 0; r.H = 0; r.exists = 1; r.built = 1; r.parent = -1; r.pad = 0;
  cur[(size_t)k * geo.Lmax] = r;
  int nch = 0, nrd = 0, nslot = 0;
  emit_node(chunks + (size_t)k * geo.maxch, reds + (size_t)k * geo.maxch, nch, nrd, nslot, 0, 0, r.count, geo.rch);
  counts[2 * k] = nch;
  counts[2 * k + 1] = nrd;
}

// ---- G3: histograms (grid: chunks x feature blocks x folds) -----------------
// HC (constant hessian: squared error, h = 1 for every row): the hessian sum of a bin is its row
// count times the one fixed-point value every row carries, and the count rides in the low 17 bits of
// the gradient's own 64-bit LDS word: ONE atomic of (qg << 17) + 1 per row and feature. Exact: a
// chunk has at most GB_R = 2^14 rows, so the count never carries into the gradient bits, and with
// |qg| < 2^29 per row (geo.lg_n >= 32 on this path) the chunk's gradient sum stays below 2^43,
// shifted 2^60. Decode: count = word & (2^17 - 1), sum qg = word >> 17 (arithmetic). The image is
// 32 features x 258 words = 66 KB (2 workgroups per CU): twice the features per workgroup of the
// (g, h) image halves the row-id / gradient gathers per bin row (round 5: 590 -> 380 us per level).
// Resolution: lg_n >= 32 puts each row's gradient on a grid of 2^-29 * 2^ceil(log2 max|g|) (fx_exp),
// instead of 2^-(61 - lg_n) at the real row count -- 2^12 coarser at 1M rows. A gradient 10^6 times
// smaller than the largest one still keeps ~9 significant bits; rounding is to nearest, so the
// per-bin error is unbiased and at most n_bin / 2 grid steps. Histograms stay exact integer sums of
// those values (bitwise-reproducible). tests/test_gbdt_gpu.py::test_hip_outlier_gradients_match_cpu
// pins a target whose gradients span 5 orders of magnitude against the CPU engine's fp64 sums.
#define HB_GSTRIDE 258   // int64 per feature in the gradient-only image (256 bins + pad)
#define HB_CBITS 17
static_assert(GB_R < (1 << HB_CBITS), "packed counts must not carry into the gradient bits");
template <bool HC>
__global__ void __launch_bounds__(HB_T) hist_kernel(Geo geo, const uint8_t* __restrict__ bins,
                                                    const int* __restrict__ rows, const float2* __restrict__ gh,
                                                    const Chunk* __restrict__ chunks, const int* __restrict__ counts,
                                                    i64* __restrict__ hist, i64* __restrict__ part,
                                                    const unsigned int* __restrict__ mx) {
  // XCD-aware order: the hardware deals consecutive workgroups to the 8 XCDs round-robin; remap so
  // that the feature blocks of one row chunk are CONSECUTIVE workgroups of ONE XCD. They gather the
  // same rows (row ids, gradients, and 16-byte slices of the same 256-byte bin rows), so all but the
  // first of them hit that XCD's L2 instead of each XCD fetching every line from HBM (round-4 PMC:
  // 24 % L2 hits, the kernel waited on memory half of its cycles)
  constexpr int NF = HC ? HB_FC : HB_FG;
  int cx = blockIdx.x, cy = blockIdx.y, cz = blockIdx.z;
  {
    const int gx = gridDim.x, gy = gridDim.y;
    const int total = gx * gy * gridDim.z;
    int t = cx + gx * (cy + gy * cz);
    if ((total & 7) == 0) t = (t & 7) * (total >> 3) + (t >> 3);
    cy = t % gy;
    t /= gy;
    cx = t % gx;
    cz = t / gx;
  }
  const int k = cz;
  if (cx >= counts[2 * k]) return;
  constexpr int LHN = HC ? NF * HB_GSTRIDE : NF * HB_STRIDE;
  __shared__ u64 lh[LHN];
  const Chunk c = chunks[(size_t)k * geo.maxch + cx];
  const int F = geo.F, Fs = geo.Fs;
  const int fb = cy * NF, tid = threadIdx.x;
  constexpr int LPR = NF / 4;                 // lanes per row (4 features each)
  constexpr int RL = HB_T / LPR;                // row lanes
  for (int i = tid; i < LHN; i += HB_T) lh[i] = 0ull;
  const float sg = ldexpf(1.f, fx_exp(mx[2 * k], geo.lg_n)), sh = ldexpf(1.f, fx_exp(mx[2 * k + 1], geo.lg_n));
  __syncthreads();
  const int wl = tid % LPR, rl = tid / LPR;
  const int f4 = fb + wl * 4;
  const float2* gk = gh + (size_t)k * geo.n;
  auto add = [&](uint32_t w, u64 qg, u64 qh) {
    if constexpr (HC) {
      u64* my = lh + wl * 4 * HB_GSTRIDE;
      const u64 v = (qg << HB_CBITS) + 1ull;
#pragma unroll
      for (int q = 0; q < 4; ++q) atomicAdd(my + q * HB_GSTRIDE + ((w >> (8 * q)) & 255u), v);
    } else {
      u64* my = lh + wl * 4 * HB_STRIDE;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        u64* d = my + q * HB_STRIDE + 2 * ((w >> (8 * q)) & 255u);
        atomicAdd(d, qg);
        atomicAdd(d + 1, qh);
      }
    }
  };
  if (f4 < F) {
    const int* rp = rows + (size_t)k * geo.n + c.start;
    int i = rl;
    for (; i + (HB_U - 1) * RL < c.count; i += HB_U * RL) {
      int r[HB_U];
      float2 g[HB_U];
      uint32_t w[HB_U];
#pragma unroll
      for (int u = 0; u < HB_U; ++u) r[u] = rp[i + RL * u];
#pragma unroll
      for (int u = 0; u < HB_U; ++u) {
        g[u] = gk[r[u]];
        w[u] = *reinterpret_cast<const uint32_t*>(bins + (size_t)r[u] * Fs + f4);
      }
#pragma unroll
      for (int u = 0; u < HB_U; ++u) add(w[u], (u64)llrintf(g[u].x * sg), HC ? 0ull : (u64)llrintf(g[u].y * sh));
    }
    for (; i < c.count; i += RL) {
      const int r = rp[i];
      const float2 g = gk[r];
      const uint32_t w = *reinterpret_cast<const uint32_t*>(bins + (size_t)r * Fs + f4);
      add(w, (u64)llrintf(g.x * sg), HC ? 0ull : (u64)llrintf(g.y * sh));
    }
  }
  __syncthreads();
  // exact integer sums: in place for a one-chunk node, else partial slot c.slot
  const int nf = min(NF, F - fb);
  i64* dst = c.slot < 0 ? hist + (((size_t)k * geo.Lh + c.node) * F + fb) * 2 * GB_BINS
                        : part + (((size_t)k * geo.maxslot + c.slot) * F + fb) * 2 * GB_BINS;
  const i64 qh1 = (i64)llrintf(1.0f * sh);     // every row's hessian (h = 1) in fixed point
  for (int i = tid; i < nf * 2 * GB_BINS; i += HB_T) {
    const int fl = i >> 9, j = i & 511;
    if constexpr (HC) {
      const i64 v = (i64)lh[fl * HB_GSTRIDE + (j >> 1)];
      dst[(size_t)fl * 2 * GB_BINS + j] = (j & 1) ? (v & ((1ll << HB_CBITS) - 1)) * qh1 : v >> HB_CBITS;
    } else
      dst[(size_t)fl * 2 * GB_BINS + j] = (i64)lh[fl * HB_STRIDE + j];
  }
}

// node histogram = sum of its partial slots (grid: reductions x y x folds)
__global__ void __launch_bounds__(256) reduce_kernel(Geo geo, const i64* __restrict__ part, i64* __restrict__ hist,
                                                     const Red* __restrict__ reds, const int* __restrict__ counts) {
  const int k = blockIdx.z;
  if ((int)blockIdx.x >= counts[2 * k + 1]) return;
  const Red rd = reds[(size_t)k * geo.maxch + blockIdx.x];
  const size_t per = (size_t)geo.F * 2 * GB_BINS;
  const i64* pk = part + (size_t)k * geo.maxslot * per;
  i64* h = hist + ((size_t)k * geo.Lh + rd.node) * per;
  for (size_t e = threadIdx.x + (size_t)blockIdx.y * 256; e < per; e += (size_t)gridDim.y * 256) {
    // 8 slot loads in flight per step (the one-at-a-time loop was latency-bound: a root
    // node of ~50 slots waited ~50 HBM round trips per element, 0.2 TB/s)
    i64 acc = 0;
    int sl = 0;
    const i64* p0 = pk + (size_t)rd.first * per + e;
    for (; sl + 8 <= rd.nslots; sl += 8) {
      i64 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = p0[(size_t)(sl + u) * per];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; sl < rd.nslots; ++sl) acc += p0[(size_t)sl * per];
    h[e] = acc;
  }
}

// sibling = parent (previous level) - built child (grid: level nodes x y x folds)
__global__ void __launch_bounds__(256) subtract_kernel(Geo geo, const LNode* __restrict__ cur,
                                                       const i64* __restrict__ prev, i64* __restrict__ hist) {
  const int k = blockIdx.z, j = blockIdx.x;
  const LNode nd = cur[(size_t)k * geo.Lmax + j];
  if (!nd.exists || nd.built) return;
  const size_t per = (size_t)geo.F * 2 * GB_BINS;
  const i64* P = prev + ((size_t)k * geo.Lh + nd.parent) * per;
  const i64* B = hist + ((size_t)k * geo.Lh + (j ^ 1)) * per;
  i64* O = hist + ((size_t)k * geo.Lh + j) * per;
  for (size_t i = threadIdx.x + (size_t)blockIdx.y * 256; i < per; i += (size_t)gridDim.y * 256) O[i] = P[i] - B[i];
}

// root totals: sum over the bins of feature 0 (exact)
__global__ void root_totals_kernel(Geo geo, const i64* __restrict__ hist, LNode* __restrict__ cur) {
  const int k = blockIdx.x, lane = threadIdx.x;
  const i64* h = hist + (size_t)k * geo.Lh * geo.F * 2 * GB_BINS;
  i64 g = 0, hh = 0;
  for (int b = lane; b < GB_BINS; b += 64) { g += h[2 * b]; hh += h[2 * b + 1]; }
  for (int o = 32; o > 0; o >>= 1) { g += __shfl_xor(g, o); hh += __shfl_xor(hh, o); }
  if (lane == 0) { cur[(size_t)k * geo.Lmax].G = g; cur[(size_t)k * geo.Lmax].H = hh; }
}

// the CPU engine's scan rule (build_tree): a candidate later in the scan
// replaces an earlier one only if better by more than 1e-12
__device__ __forceinline__ bool later_wins(double g_early, bool early_ok, double g_late, bool late_ok) {
  if (!late_ok) return false;
  if (!early_ok) return true;
  return g_late > g_early + 1e-12;
}

// ---- G4: best split per (node, feature): one wave each (grid F x L x folds) --
// order[(k * (D+1) + depth) * F + f] = position of f in the level's feature
// scan (colsample_bytree / _bylevel), 0 = not sampled
// prev != null (the last histogram level): the histograms of the non-built nodes were not materialised
// (no later level subtracts from them) -- read as parent (prev) - built sibling, the same exact integers
__global__ void __launch_bounds__(64) split_kernel(Geo geo, int depth, const i64* __restrict__ hist,
                                                   const i64* __restrict__ prev,
                                                   const int* __restrict__ nbins, const int* __restrict__ order,
                                                   const LNode* __restrict__ cur, const unsigned int* __restrict__ mx,
                                                   SplitOut* __restrict__ out, DevParams p) {
  const int f = blockIdx.x, j = blockIdx.y, k = blockIdx.z, lane = threadIdx.x, F = geo.F;
  const LNode nd = cur[(size_t)k * geo.Lmax + j];
  const int ord = order[((size_t)k * (geo.max_depth + 1) + depth) * F + f] - 1;
  double bg = 0.0;
  int bb = -1;
  i64 bGL = 0, bHL = 0;
  if (nd.exists && nd.count >= 2 && ord >= 0) {
    const double ig = ldexp(1.0, -fx_exp(mx[2 * k], geo.lg_n)), ih = ldexp(1.0, -fx_exp(mx[2 * k + 1], geo.lg_n));
    const bool virt = prev != nullptr && !nd.built;
    const i64* h = hist + (((size_t)k * geo.Lh + (virt ? (j ^ 1) : j)) * F + f) * 2 * GB_BINS;
    const i64* hp = virt ? prev + (((size_t)k * geo.Lh + nd.parent) * F + f) * 2 * GB_BINS : nullptr;
    i64 vg[4], vh[4], sg = 0, sh = 0;
    {
      const longlong2* h2 = reinterpret_cast<const longlong2*>(h) + lane * 4;
      longlong2 v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = h2[q];
      if (virt) {
        const longlong2* p2 = reinterpret_cast<const longlong2*>(hp) + lane * 4;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const longlong2 pv = p2[q];
          v[q].x = pv.x - v[q].x;
          v[q].y = pv.y - v[q].y;
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) { vg[q] = v[q].x; vh[q] = v[q].y; sg += vg[q]; sh += vh[q]; }
    }
    i64 pg = sg, ph = sh;                       // inclusive scan across lanes (exact)
    for (int o = 1; o < 64; o <<= 1) {
      const i64 tg = __shfl_up(pg, o), th = __shfl_up(ph, o);
      if (lane >= o) { pg += tg; ph += th; }
    }
    i64 GLf = pg - sg, HLf = ph - sh;           // exclusive prefix
    const double G = (double)nd.G * ig, H = (double)nd.H * ih;
    const double parent = dev_gain(p, G, H);
    const int nb = nbins[f];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      GLf += vg[q]; HLf += vh[q];
      const int b = lane * 4 + q;
      if (b + 1 >= nb) continue;
      const double GL = (double)GLf * ig, HL = (double)HLf * ih;
      const double GR = G - GL, HR = H - HL;
      if (HL < p.min_child_weight || HR < p.min_child_weight || HL <= 0.0 || HR <= 0.0) continue;
      const double chg = dev_gain(p, GL, HL) + dev_gain(p, GR, HR) - parent;
      if (chg > bg + 1e-12 || (bb < 0 && chg > 1e-12)) { bg = chg; bb = b; bGL = GLf; bHL = HLf; }
    }
    for (int o = 1; o < 64; o <<= 1) {          // combine lane groups in bin (scan) order
      const double og = __shfl_xor(bg, o);
      const int ob = __shfl_xor(bb, o);
      const i64 oG = __shfl_xor(bGL, o), oH = __shfl_xor(bHL, o);
      const bool partner_early = (lane & o) != 0;  // the partner holds the lower bins
      const bool take = partner_early ? !later_wins(og, ob >= 0, bg, bb >= 0) && ob >= 0
                                      : later_wins(bg, bb >= 0, og, ob >= 0);
      if (take) { bg = og; bb = ob; bGL = oG; bHL = oH; }
    }
  }
  if (lane == 0) out[((size_t)k * geo.Lh + j) * F + f] = SplitOut{bg, bGL, bHL, bb, ord};
}

// best feature per node, in the CPU engine's feature scan order (grid L x folds)
__global__ void __launch_bounds__(256) best_kernel(Geo geo, const SplitOut* __restrict__ cand,
                                                   NodeBest* __restrict__ out) {
  __shared__ double sg[256];
  __shared__ int so[256], sf[256];
  const int j = blockIdx.x, k = blockIdx.y, tid = threadIdx.x, F = geo.F;
  const SplitOut* c = cand + ((size_t)k * geo.Lh + j) * F;
  // per thread: its features in scan order (sequential rule), then a tree over threads by order
  double bg = 0.0;
  int bo = -1, bf = -1;
  for (int f = tid; f < F; f += 256) {
    const SplitOut s = c[f];
    if (s.bin < 0 || s.order < 0) continue;
    if (bf < 0 || (s.order < bo ? !(bg > s.gain + 1e-12) : s.gain > bg + 1e-12)) { bg = s.gain; bo = s.order; bf = f; }
  }
  sg[tid] = bg; so[tid] = bo; sf[tid] = bf;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o && sf[tid + o] >= 0) {
      const double og = sg[tid + o];
      const int oo = so[tid + o];
      bool take;
      if (sf[tid] < 0) take = true;
      else if (oo < so[tid]) take = !(sg[tid] > og + 1e-12);
      else take = og > sg[tid] + 1e-12;
      if (take) { sg[tid] = og; so[tid] = oo; sf[tid] = sf[tid + o]; }
    }
    __syncthreads();
  }
  if (tid == 0) {
    NodeBest b{0.0, 0, 0, -1, -1};
    if (sf[0] >= 0) {
      const SplitOut& s = c[sf[0]];
      b = NodeBest{s.gain, s.GL, s.HL, sf[0], s.bin};
    }
    out[(size_t)k * geo.Lh + j] = b;
  }
}

// ---- plan: leaves, gamma pruning, split table, children totals (grid folds) --
__global__ void __launch_bounds__(256) plan_split_kernel(Geo geo, int depth, const LNode* __restrict__ cur,
                                                         const NodeBest* __restrict__ best,
                                                         const unsigned int* __restrict__ mx, int2* __restrict__ tree,
                                                         float* __restrict__ leaf, int2* __restrict__ splitv,
                                                         int2* __restrict__ cursor, LNode* __restrict__ nxt,
                                                         DevParams p) {
  const int k = blockIdx.x, L = 1 << depth;
  const int tsz = (2 << geo.max_depth) - 1;
  const double ig = ldexp(1.0, -fx_exp(mx[2 * k], geo.lg_n)), ih = ldexp(1.0, -fx_exp(mx[2 * k + 1], geo.lg_n));
  for (int j = threadIdx.x; j < L; j += blockDim.x) {
    const LNode nd = cur[(size_t)k * geo.Lmax + j];
    const int id = L - 1 + j;
    bool split = false;
    NodeBest b{0.0, 0, 0, -1, -1};
    if (nd.exists) {
      leaf[(size_t)k * tsz + id] = (float)(dev_weight(p, (double)nd.G * ig, (double)nd.H * ih) * p.eta);
      tree[(size_t)k * tsz + id] = make_int2(-1, 0);
      if (depth < geo.max_depth && nd.count >= 2) {
        b = best[(size_t)k * geo.Lh + j];
        split = b.feature >= 0 && b.bin >= 0 && b.gain >= p.gamma && b.gain > 1e-12;
      }
    }
    splitv[(size_t)k * geo.Lmax + j] = split ? make_int2(b.feature, b.bin) : make_int2(-1, 0);
    cursor[(size_t)k * geo.Lmax + j] = make_int2(nd.start, nd.start + nd.count);
    if (split) tree[(size_t)k * tsz + id] = make_int2(b.feature, b.bin);
    if (depth < geo.max_depth) {
      const int end = nd.start + nd.count;
      LNode l, r;
      l.start = r.start = end; l.count = r.count = 0;
      l.G = l.H = r.G = r.H = 0;
      l.exists = r.exists = split ? 1 : 0;
      l.built = r.built = 0;
      l.parent = r.parent = j;
      l.pad = r.pad = 0;
      if (split) { l.G = b.GL; l.H = b.HL; r.G = nd.G - b.GL; r.H = nd.H - b.HL; }
      nxt[(size_t)k * geo.Lmax + 2 * j] = l;
      nxt[(size_t)k * geo.Lmax + 2 * j + 1] = r;
    }
  }
}

// ---- G5: partition of the level's row positions (grid: position blocks x folds)
// A workgroup owns PT_PER x 256 consecutive positions. When they all lie in
// one node (the common case: segments are long), the block reserves its left
// and right ranges with ONE cursor atomic per side (per-wave atomics on the
// root's single cursor serialised at L2: 1 ms per level at 4M rows); blocks
// that straddle segment boundaries use per-wave ballots, per-lane atomics
// where a wave straddles one.
#define PT_PER 16
__global__ void __launch_bounds__(256) partition_kernel(Geo geo, int depth, const uint8_t* __restrict__ binsT,
                                                        const int* __restrict__ nroot, const LNode* __restrict__ cur,
                                                        const int2* __restrict__ splitv,
                                                        const int* __restrict__ rows_in, int* __restrict__ rows_out,
                                                        int2* __restrict__ cursor) {
  __shared__ int ends[1 << GB_MAXD];
  __shared__ int wl[4], wr[4], jfl[2], base_l, base_r;
  const int k = blockIdx.y, L = 1 << depth, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int nr = nroot[k];
  const int p0 = blockIdx.x * 256 * PT_PER;
  if (p0 >= nr) return;
  for (int j = tid; j < L; j += 256) {
    const LNode nd = cur[(size_t)k * geo.Lmax + j];
    ends[j] = nd.start + nd.count;
  }
  __syncthreads();
  auto node_of = [&](int p) {                  // node whose segment holds position p, or -1
    int lo = 0, hi = L;
    while (lo < hi) { const int mid = (lo + hi) >> 1; if (ends[mid] > p) hi = mid; else lo = mid + 1; }
    return (lo < L && cur[(size_t)k * geo.Lmax + lo].start <= p) ? lo : -1;
  };
  if (tid == 0) {
    jfl[0] = node_of(p0);
    jfl[1] = node_of(min(p0 + 256 * PT_PER, nr) - 1);
  }
  __syncthreads();
  const int* rin = rows_in + (size_t)k * geo.n;
  int* out = rows_out + (size_t)k * geo.n;
  const u64 below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  if (jfl[0] == jfl[1]) {
    if (jfl[0] < 0) return;
    const int j0 = jfl[0];
    const int2 sp = splitv[(size_t)k * geo.Lmax + j0];
    if (sp.x < 0) return;                      // a leaf: its rows leave the tree
    const uint8_t* col = binsT + (size_t)sp.x * geo.n;
    int rr[PT_PER];
    uint32_t lm = 0, vm = 0;
#pragma unroll
    for (int q = 0; q < PT_PER; ++q) {
      const int p = p0 + q * 256 + tid;
      rr[q] = 0;
      if (p < nr) {
        rr[q] = rin[p];
        vm |= 1u << q;
        if (col[rr[q]] <= (uint8_t)sp.y) lm |= 1u << q;
      }
    }
    const int cl = __popc(lm), cr = __popc(vm & ~lm);
    int il = cl, ir = cr;                      // inclusive wave scans
    for (int o = 1; o < 64; o <<= 1) {
      const int tl = __shfl_up(il, o), tr = __shfl_up(ir, o);
      if (lane >= o) { il += tl; ir += tr; }
    }
    if (lane == 63) { wl[wv] = il; wr[wv] = ir; }
    __syncthreads();
    if (tid == 0) {
      const int tl = wl[0] + wl[1] + wl[2] + wl[3], tr = wr[0] + wr[1] + wr[2] + wr[3];
      int2* cu = cursor + (size_t)k * geo.Lmax + j0;
      base_l = tl ? atomicAdd(&cu->x, tl) : 0;
      base_r = tr ? atomicSub(&cu->y, tr) - tr : 0;
    }
    __syncthreads();
    int pl = base_l + il - cl, pr = base_r + ir - cr;
    for (int w = 0; w < wv; ++w) { pl += wl[w]; pr += wr[w]; }
#pragma unroll
    for (int q = 0; q < PT_PER; ++q) {
      if (!((vm >> q) & 1u)) continue;
      if ((lm >> q) & 1u) out[pl++] = rr[q];
      else out[pr++] = rr[q];
    }
    return;
  }
  // segment boundary inside the block
  for (int q = 0; q < PT_PER; ++q) {
    const int p = p0 + q * 256 + tid;
    bool valid = p < nr;
    int j = valid ? node_of(p) : -1;
    valid = valid && j >= 0;
    int2 sp = make_int2(-1, 0);
    if (valid) sp = splitv[(size_t)k * geo.Lmax + j];
    valid = valid && sp.x >= 0;
    int r = 0;
    bool left = false;
    if (valid) {
      r = rin[p];
      left = binsT[(size_t)sp.x * geo.n + r] <= (uint8_t)sp.y;
    }
    const u64 vmw = __ballot(valid);
    if (!vmw) continue;
    const int lead = __builtin_ctzll(vmw);
    const int jw = __shfl(j, lead);
    const bool uniform = __ballot(valid && j != jw) == 0ull;
    if (uniform) {
      const u64 lmw = __ballot(valid && left), rmw = __ballot(valid && !left);
      int l0 = 0, r0 = 0;
      if (lane == lead) {
        int2* cu = cursor + (size_t)k * geo.Lmax + jw;
        l0 = atomicAdd(&cu->x, __popcll(lmw));
        r0 = atomicSub(&cu->y, __popcll(rmw)) - __popcll(rmw);
      }
      l0 = __shfl(l0, lead);
      r0 = __shfl(r0, lead);
      if (valid) out[left ? l0 + __popcll(lmw & below) : r0 + __popcll(rmw & below)] = r;
    } else if (valid) {
      int2* cu = cursor + (size_t)k * geo.Lmax + j;
      const int pos = left ? atomicAdd(&cu->x, 1) : atomicSub(&cu->y, 1) - 1;
      out[pos] = r;
    }
  }
}

// children segments, built flags, next level's chunk / reduction lists (grid folds)
__global__ void __launch_bounds__(256) plan_next_kernel(Geo geo, int depth, const LNode* __restrict__ cur,
                                                        const int2* __restrict__ splitv,
                                                        const int2* __restrict__ cursor, LNode* __restrict__ nxt,
                                                        Chunk* __restrict__ chunks, Red* __restrict__ reds,
                                                        int* __restrict__ counts) {
  const int k = blockIdx.x, L = 1 << depth;
  for (int j = threadIdx.x; j < L; j += blockDim.x) {
    if (splitv[(size_t)k * geo.Lmax + j].x < 0) continue;
    const LNode nd = cur[(size_t)k * geo.Lmax + j];
    const int lc = cursor[(size_t)k * geo.Lmax + j].x - nd.start;
    LNode* l = nxt + (size_t)k * geo.Lmax + 2 * j;
    LNode* r = l + 1;
    l->start = nd.start; l->count = lc;
    r->start = nd.start + lc; r->count = nd.count - lc;
    l->built = lc <= nd.count - lc ? 1 : 0;     // smaller child (engine.cpp: left on ties)
    r->built = 1 - l->built;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  int nch = 0, nrd = 0, nslot = 0;
  if (depth + 1 < geo.max_depth) {
    Chunk* ch = chunks + (size_t)k * geo.maxch;
    Red* rd = reds + (size_t)k * geo.maxch;
    for (int j = 0; j < 2 * L; ++j) {
      const LNode c = nxt[(size_t)k * geo.Lmax + j];
      if (c.exists && c.built) emit_node(ch, rd, nch, nrd, nslot, j, c.start, c.count, geo.rch);
    }
  }
  counts[2 * k] = nch;
  counts[2 * k + 1] = nrd;
}

// ---- G6: prediction update by tree traversal (all rows of every fold) ------
// A workgroup stages R consecutive bin rows in LDS (coalesced 4-byte loads, row stride Fs + 4 bytes:
// the lookups of R threads at one feature fall on distinct banks) and the trees of nk folds (split
// table + leaf values, 2^(D+1) - 1 nodes each); each staged row is then walked through every staged
// fold's tree from LDS. A row's bins leave HBM once per round for all folds, and the D dependent
// lookups per row and tree are LDS reads: the walk with the tree in global memory and one byte load
// per lookup moved a 128-byte line from L2 per lookup (0.65 ms per round at 1M rows x 5 folds,
// depth 10). R = 0 (rows wider than the LDS budget): lookups straight from global memory.
__global__ void __launch_bounds__(256) predict_kernel(Geo geo, const uint8_t* __restrict__ bins,
                                                      const int2* __restrict__ tree, const float* __restrict__ leaf,
                                                      float* __restrict__ margin, int c, int nk, int R) {
  extern __shared__ uint32_t psm[];
  const int k0 = blockIdx.y * nk, tsz = (2 << geo.max_depth) - 1, tid = threadIdx.x;
  const int Fs = geo.Fs, rs = Fs / 4 + 1;           // LDS row stride in dwords
  nk = min(nk, geo.nfold - k0);
  uint32_t* prow = psm;
  int2* ptree = reinterpret_cast<int2*>(psm + (size_t)R * rs + ((R * rs) & 1));
  float* pleaf = reinterpret_cast<float*>(ptree + (size_t)nk * tsz);
  for (int i = tid; i < nk * tsz; i += 256) {
    ptree[i] = tree[(size_t)k0 * tsz + i];
    pleaf[i] = leaf[(size_t)k0 * tsz + i];
  }
  auto walk = [&](const uint8_t* row, int rstride, int kk) {   // leaf of one row in fold k0 + kk's tree
    const int2* tk = ptree + (size_t)kk * tsz;
    int id = 0;
    int2 t = tk[0];
    while (t.x >= 0) {
      id = (row[(size_t)t.x * rstride] <= t.y) ? 2 * id + 1 : 2 * id + 2;
      t = tk[id];
    }
    return pleaf[(size_t)kk * tsz + id];
  };
  if (R == 0) {
    __syncthreads();
    for (int i = blockIdx.x * 256 + tid; i < geo.n; i += gridDim.x * 256)
      for (int kk = 0; kk < nk; ++kk)
        margin[((size_t)(k0 + kk) * geo.n + i) * geo.K + c] += walk(bins + (size_t)i * Fs, 1, kk);
    return;
  }
  const int tpr = 256 / R;                           // threads per row (folds split among them)
  const int fd = Fs / 4;
  for (long i0 = (long)blockIdx.x * R; i0 < geo.n; i0 += (long)gridDim.x * R) {
    __syncthreads();                                 // the previous rows (and, first, the trees) are ready
    const int rows = (int)min((long)R, geo.n - i0);
    const uint32_t* src = reinterpret_cast<const uint32_t*>(bins + (size_t)i0 * Fs);
    for (int v = tid; v < rows * fd; v += 256) {
      const int r = v / fd;
      prow[r * rs + (v - r * fd)] = src[v];
    }
    __syncthreads();
    const int r = tid % R;
    if (r < rows) {
      const uint8_t* row = reinterpret_cast<const uint8_t*>(prow + r * rs);
      for (int kk = tid / R; kk < nk; kk += tpr)
        margin[((size_t)(k0 + kk) * geo.n + i0 + r) * geo.K + c] += walk(row, 1, kk);
    }
  }
}

// ---- G8: metric partial sums over every fold's train / test rows -------------
// out[(k * gridDim.x + block) * 4 + (train sum, train count, test sum, test count)];
// metric 0 rmse, 1 mae, 2 logloss, 3 error, 5 merror, 6 mlogloss (engine.cpp eval_metric)
__global__ void __launch_bounds__(256) metric_kernel(Geo geo, const float* __restrict__ margin,
                                                     const float* __restrict__ y, const int* __restrict__ fold_of,
                                                     int metric, int objective, double* __restrict__ out) {
  __shared__ double red[4][256];
  const int k = blockIdx.y, K = geo.K;
  const float* mk = margin + (size_t)k * geo.n * K;
  double s[4] = {0, 0, 0, 0};
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < geo.n; i += gridDim.x * blockDim.x) {
    const float* m = mk + (size_t)i * K;
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
      float mxv = m[0];
      for (int q = 1; q < K; ++q) if (m[q] > mxv) { mxv = m[q]; arg = q; }
      if (metric == 5) v = (arg != (int)y[i]) ? 1.f : 0.f;
      else {
        float z = 0.f;
        for (int q = 0; q < K; ++q) z += expf(m[q] - mxv);
        v = -logf(fmaxf(1e-15f, expf(m[(int)y[i]] - mxv) / z));
      }
    }
    const int q = (fold_of[i] == k) ? 2 : 0;
    s[q] += v; s[q + 1] += 1.0;
  }
  for (int q = 0; q < 4; ++q) red[q][threadIdx.x] = s[q];
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o)
      for (int q = 0; q < 4; ++q) red[q][threadIdx.x] += red[q][threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x < 4) out[((size_t)k * gridDim.x + blockIdx.x) * 4 + threadIdx.x] = red[threadIdx.x][0];
}

// ---- G8 auc: tie-averaged rank sum of the positives per (fold, train / test) segment ----------
// engine.cpp auc_score sorts every fold's margins and gives a tie group its average rank. Here one
// radix sort orders all nfold * n rows at once by key = seg << 33 | ordered(margin) << 1 | positive
// (seg = 2 k + [row in fold k's test set]); a positive then finds its tie group [a, b] and its
// segment's start by binary search in the sorted keys (negatives of the group sort first, which does
// not change its bounds). Each positive adds (a + b) / 2 + 1 - start, a multiple of 1/2 below 2^52,
// so the fp64 sums are exact and independent of the atomic order: the result is deterministic.
__global__ void __launch_bounds__(256) auc_keys_kernel(Geo geo, const float* __restrict__ margin,
                                                       const float* __restrict__ y,
                                                       const int* __restrict__ fold_of, u64* __restrict__ keys) {
  const int k = blockIdx.y;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < geo.n; i += gridDim.x * blockDim.x) {
    const unsigned int b = __float_as_uint(margin[((size_t)k * geo.n + i) * geo.K] + 0.f);   // -0 -> +0
    const unsigned int ord = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
    const u64 seg = 2u * (unsigned)k + (fold_of[i] == k ? 1u : 0u);
    keys[(size_t)k * geo.n + i] = (seg << 33) | ((u64)ord << 1) | (y[i] > 0.5f ? 1u : 0u);
  }
}

__device__ __forceinline__ size_t lower_bound_u64(const u64* __restrict__ a, size_t n, u64 x) {
  size_t lo = 0;
  while (n > 0) {
    const size_t h = n >> 1;
    if (a[lo + h] < x) { lo += h + 1; n -= h + 1; } else n = h;
  }
  return lo;
}

// acc[seg * 2 + {0: rank sum of the positives, 1: positives}], zeroed before the launch; nseg <= 64.
// Segment starts: one binary search per segment per workgroup (LDS); tie-group bounds: a positive whose
// neighbours carry other margins is its own group (the common case once trees separate the rows), else
// binary search.
__global__ void __launch_bounds__(256) auc_rank_kernel(const u64* __restrict__ sorted, size_t N, int nseg,
                                                       double* __restrict__ acc) {
  __shared__ double s[128];
  __shared__ size_t st[64];
  for (int t = threadIdx.x; t < 2 * nseg; t += blockDim.x) s[t] = 0.0;
  for (int t = threadIdx.x; t < nseg; t += blockDim.x) st[t] = lower_bound_u64(sorted, N, (u64)t << 33);
  __syncthreads();
  for (size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x; p < N; p += (size_t)gridDim.x * blockDim.x) {
    const u64 key = sorted[p];
    if (!(key & 1u)) continue;
    const u64 seg = key >> 33, m = key >> 1;
    const bool lo_tie = p > 0 && (sorted[p - 1] >> 1) == m;
    const bool hi_tie = p + 1 < N && (sorted[p + 1] >> 1) == m;
    const size_t a = lo_tie ? lower_bound_u64(sorted, N, key & ~1ull) : p;
    const size_t b = hi_tie ? lower_bound_u64(sorted, N, key + 1) - 1 : p;     // key | 1 == key: last of the group
    atomicAdd(&s[2 * seg], 0.5 * (double)(a + b) + 1.0 - (double)st[seg]);
    atomicAdd(&s[2 * seg + 1], 1.0);
  }
  __syncthreads();
  for (int t = threadIdx.x; t < 2 * nseg; t += blockDim.x)
    if (s[t] != 0.0) atomicAdd(&acc[t], s[t]);
}

uint64_t smix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

#define HC(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { rc = -100 - (int)e_; goto done; } } while (0)

}  // namespace

// feature-major copy of the cached bins (partition), rebuilt when the cache changes
static uint8_t* g_binsT = nullptr;
static const uint8_t* g_binsT_src = nullptr;
static long long g_binsT_key = 0;
static size_t g_binsT_bytes = 0;

namespace gbdt_cache {
uint8_t* bins = nullptr;
long long key = 0;
size_t bytes = 0;
std::mutex mu;
void invalidate_derived() { g_binsT_key = 0; }
}  // namespace gbdt_cache

extern "C" {

// Same contract as gbdt_cv (csrc/gbdt/engine.cpp) for every objective
// (reg:linear/squarederror, reg:logistic, binary:logistic/logitraw,
// multi:softmax/softprob: one tree per class) and every metric (rmse, mae,
// logloss, error, auc, merror, mlogloss; early stopping on the last, auc
// maximised). auc needs nfold <= 32 (64 sort segments).
// bins_h may be null when gbdt_quantize_hip already left the dataset's bins
// on the device under cache_key (returns -7 if they were evicted). bins:
// ROW-major [n][Fs] uint8 (Fs >= F, Fs % 4 == 0). cache_key != 0 keeps the
// device copy of the bins across calls for the same key (one dataset, many
// candidates).
int gbdt_cv_hip(const uint8_t* bins_h, int Fs, const int* nbins_h, int n, int F, const float* y_h,
                const int* fold_h, int nfold, const double* P, int objective, int num_class, const int* metrics,
                int n_metrics, int num_boost_round, int early_stopping_rounds, unsigned long long seed,
                long long cache_key, double* out_hist) {
  if (objective < 0 || objective > 5 || n_metrics < 1 || Fs % 4 || Fs < F || n <= 0 || nfold <= 0 || F <= 0)
    return -1;
  bool want_auc = false;
  for (int mi = 0; mi < n_metrics; ++mi) {
    if (metrics[mi] < 0 || metrics[mi] > 6) return -1;
    want_auc = want_auc || metrics[mi] == 4;
  }
  if (want_auc && nfold > 32) return -1;
  const bool multi = objective >= 4;
  const int K = multi ? std::max(2, num_class) : 1;
  const int obj = multi ? 3 : (objective == 0 ? 0 : (objective == 1 ? 1 : 2));
  // squared error: h = 1 for every row -> count histograms for the hessian (hist_kernel<true>)
  const bool hconst = obj == 0;
  const int D = std::max(0, std::min((int)P[2], GB_MAXD));
  std::lock_guard<std::mutex> lock(gbdt_cache::mu);   // one GBDT call at a time per process (bins cache)
  int rc = 0;
  Geo geo;
  geo.n = n; geo.F = F; geo.Fs = Fs; geo.nfold = nfold; geo.K = K; geo.max_depth = D;
  geo.Lmax = 1 << D;
  geo.Lh = 1 << std::max(0, D - 1);
  // rows per histogram chunk: fewer, longer chunks = fewer partial slots for the reduce to sum
  geo.rch = GB_R;
  const int rchunks = (n + geo.rch - 1) / geo.rch;
  geo.maxch = rchunks + geo.Lh + 2;
  geo.maxslot = 2 * rchunks + 2;
  geo.lg_n = 0;
  while ((1ll << geo.lg_n) < (long long)n + 1) ++geo.lg_n;
  if (hconst) geo.lg_n = std::max(geo.lg_n, 32);   // |qg| < 2^29 per row (packed counts)
  const int tsz = (2 << D) - 1;
  const size_t per_node = (size_t)F * 2 * GB_BINS;      // int64 per histogram node
  DevParams dp{P[1], P[8], P[9], P[4], P[0], P[3]};
  const int blocks = std::min(2048, (n + 255) / 256);
  const int pblocks = (n + 256 * PT_PER - 1) / (256 * PT_PER);
  const int mblocks = std::min(blocks, 256);
  // predict: R staged rows (a power of two, 32 KB of LDS) + as many folds' trees as fit 96 KB more
  int pr_rows = 0;
  if (Fs + 4 <= 32768 / 4) {
    pr_rows = 256;
    while (pr_rows > 4 && (size_t)pr_rows * (Fs + 4) > 32768) pr_rows >>= 1;
  }
  const int pk = (int)std::max<size_t>(1, std::min<size_t>(nfold, (96u << 10) / ((size_t)tsz * 12)));
  const size_t pred_lds = (size_t)pr_rows * (Fs + 4) + 8 + (size_t)pk * tsz * 12;
  if (pred_lds > 65536)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(predict_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)pred_lds);
  const int nfb = hconst ? (F + HB_FC - 1) / HB_FC : (F + HB_FG - 1) / HB_FG;
  const int ylen = std::max(1, (int)(per_node / 4096));
  const int rlen = std::max(1, (int)(per_node / 512));       // reduce: 2 elements per thread, ~256 workgroups per node
  // device buffers
  float *d_y = nullptr, *d_margin = nullptr, *d_leaf = nullptr;
  int *d_fold = nullptr, *d_nb = nullptr, *d_rows[2] = {nullptr, nullptr}, *d_order = nullptr, *d_counts = nullptr,
      *d_nroot = nullptr;
  float2* d_gh = nullptr;
  i64 *d_hist[2] = {nullptr, nullptr}, *d_part = nullptr;
  LNode* d_lvl[2] = {nullptr, nullptr};
  Chunk* d_chunks = nullptr;
  Red* d_reds = nullptr;
  SplitOut* d_cand = nullptr;
  NodeBest* d_best = nullptr;
  int2 *d_tree = nullptr, *d_split = nullptr, *d_cur = nullptr;
  unsigned int* d_mx = nullptr;
  u64* d_keys = nullptr;
  double* d_met = nullptr;
  void* h_up = nullptr;           // pinned upload block: keys [K][nfold] u64, orders [K][nfold][D+1][F] int
  double* h_met = nullptr;        // pinned metric read-back
  const size_t keys_bytes = sizeof(u64) * K * nfold;
  const size_t order_elems = (size_t)nfold * (D + 1) * F;
  const size_t up_bytes = keys_bytes + sizeof(int) * K * order_elems;
  const size_t met_elems = (size_t)n_metrics * nfold * mblocks * 4;
  const uint8_t* d_bins = nullptr;
  double base = P[11];
  const bool lower_better = metrics[n_metrics - 1] != 4;      // engine.cpp higher_better: auc
  double best_score = lower_better ? INFINITY : -INFINITY;
  // auc: sort keys (two buffers + rocprim scratch) and [2 nfold][2] rank sums; rows per test fold
  u64 *d_akeys = nullptr, *d_asorted = nullptr;
  void* d_atmp = nullptr;
  size_t atmp_bytes = 0;
  double* d_aacc = nullptr;
  const size_t aN = (size_t)nfold * n;
  const int aseg_bits = 33 + [](int s) { int b = 0; while ((1 << b) < s) ++b; return b; }(2 * nfold);
  std::vector<double> h_aacc(4 * (size_t)nfold);
  std::vector<double> ntest(nfold, 0.0);
  for (int i = 0; i < n; ++i)
    if (fold_h[i] >= 0 && fold_h[i] < nfold) ntest[fold_h[i]] += 1.0;
  int best_round = 0, rounds_done = 0;
  static const bool timing = std::getenv("GENTUN_GBDT_TIMING") != nullptr;
  static const int progress = std::getenv("GENTUN_GBDT_PROGRESS") ? std::atoi(std::getenv("GENTUN_GBDT_PROGRESS")) : 0;
  const auto t_start = std::chrono::steady_clock::now();

  {
    const size_t nbytes = (size_t)n * Fs;
    if (cache_key == 0 || cache_key != gbdt_cache::key || gbdt_cache::bytes != nbytes || gbdt_cache::bins == nullptr) {
      if (bins_h == nullptr) return -7;      // device copy evicted: the caller quantises again
      if (gbdt_cache::bins) (void)hipFree(gbdt_cache::bins);
      gbdt_cache::bins = nullptr; gbdt_cache::key = 0; gbdt_cache::bytes = 0;
      if (hipMalloc(&gbdt_cache::bins, nbytes) != hipSuccess) return -100;
      if (hipMemcpy(gbdt_cache::bins, bins_h, nbytes, hipMemcpyHostToDevice) != hipSuccess) return -100;
      gbdt_cache::key = cache_key; gbdt_cache::bytes = nbytes;
    }
    d_bins = gbdt_cache::bins;
    if (g_binsT == nullptr || g_binsT_key == 0 || g_binsT_key != gbdt_cache::key || g_binsT_src != d_bins ||
        g_binsT_bytes != nbytes) {
      if (g_binsT) (void)hipFree(g_binsT);
      g_binsT = nullptr;
      if (hipMalloc(&g_binsT, nbytes) != hipSuccess) return -100;
      hipLaunchKernelGGL(transpose_bins_kernel, dim3((n + 63) / 64, (Fs + 63) / 64), dim3(256), 0, 0, d_bins, g_binsT,
                         n, Fs);
      g_binsT_src = d_bins; g_binsT_key = gbdt_cache::key; g_binsT_bytes = nbytes;
    }
  }
  HC(hipMalloc(&d_y, sizeof(float) * n));
  HC(hipMalloc(&d_fold, sizeof(int) * n));
  HC(hipMalloc(&d_nb, sizeof(int) * F));
  for (int b = 0; b < 2; ++b) HC(hipMalloc(&d_rows[b], sizeof(int) * (size_t)nfold * n));
  HC(hipMalloc(&d_margin, sizeof(float) * (size_t)nfold * n * K));
  HC(hipMalloc(&d_gh, sizeof(float2) * (size_t)nfold * n));
  for (int b = 0; b < 2; ++b) HC(hipMalloc(&d_hist[b], sizeof(i64) * (size_t)nfold * geo.Lh * per_node));
  HC(hipMalloc(&d_part, sizeof(i64) * (size_t)nfold * geo.maxslot * per_node));
  for (int b = 0; b < 2; ++b) HC(hipMalloc(&d_lvl[b], sizeof(LNode) * (size_t)nfold * geo.Lmax));
  HC(hipMalloc(&d_chunks, sizeof(Chunk) * (size_t)nfold * geo.maxch));
  HC(hipMalloc(&d_reds, sizeof(Red) * (size_t)nfold * geo.maxch));
  HC(hipMalloc(&d_counts, sizeof(int) * 2 * nfold));
  HC(hipMalloc(&d_nroot, sizeof(int) * nfold));
  HC(hipMalloc(&d_cand, sizeof(SplitOut) * (size_t)nfold * geo.Lh * F));
  HC(hipMalloc(&d_best, sizeof(NodeBest) * (size_t)nfold * geo.Lh));
  HC(hipMalloc(&d_tree, sizeof(int2) * (size_t)nfold * tsz));
  HC(hipMalloc(&d_leaf, sizeof(float) * (size_t)nfold * tsz));
  HC(hipMalloc(&d_split, sizeof(int2) * (size_t)nfold * geo.Lmax));
  HC(hipMalloc(&d_cur, sizeof(int2) * (size_t)nfold * geo.Lmax));
  HC(hipMalloc(&d_mx, sizeof(unsigned int) * 2 * nfold));
  HC(hipMalloc(&d_keys, keys_bytes));
  HC(hipMalloc(&d_order, sizeof(int) * K * order_elems));
  HC(hipMalloc(&d_met, sizeof(double) * met_elems));
  if (want_auc) {
    HC(hipMalloc(&d_akeys, sizeof(u64) * aN));
    HC(hipMalloc(&d_asorted, sizeof(u64) * aN));
    HC(hipMalloc(&d_aacc, sizeof(double) * 4 * nfold));
    HC(rocprim::radix_sort_keys(nullptr, atmp_bytes, d_akeys, d_asorted, aN, 0u, (unsigned)aseg_bits));
    HC(hipMalloc(&d_atmp, std::max<size_t>(atmp_bytes, 1)));
  }
  HC(hipHostMalloc(&h_up, up_bytes, hipHostMallocDefault));
  HC(hipHostMalloc((void**)&h_met, sizeof(double) * met_elems, hipHostMallocDefault));
  HC(hipMemcpy(d_y, y_h, sizeof(float) * n, hipMemcpyHostToDevice));
  HC(hipMemcpy(d_fold, fold_h, sizeof(int) * n, hipMemcpyHostToDevice));
  HC(hipMemcpy(d_nb, nbins_h, sizeof(int) * F, hipMemcpyHostToDevice));
  if (objective == 1 || objective == 2) {   // engine.cpp: logit base margin for the logistic objectives only
    const double b = std::min(1 - 1e-7, std::max(1e-7, P[11]));
    base = std::log(b / (1 - b));
  }
  {
    std::vector<float> m((size_t)nfold * n * K, (float)base);
    HC(hipMemcpy(d_margin, m.data(), sizeof(float) * m.size(), hipMemcpyHostToDevice));
  }

  for (int round = 0; round < num_boost_round; ++round) {
    // ---- host: every tree's random draws (engine.cpp round_fold / build_tree streams)
    u64* h_keys = reinterpret_cast<u64*>(h_up);
    int* h_order = reinterpret_cast<int*>(reinterpret_cast<char*>(h_up) + keys_bytes);
    std::memset(h_order, 0, sizeof(int) * K * order_elems);
    for (int k = 0; k < nfold; ++k) {
      const uint64_t fold_round = smix(seed ^ smix((uint64_t)k * 1000003ull + (uint64_t)round * 7919ull + 17));
      for (int c = 0; c < K; ++c) {
        uint64_t rs = c == 0 ? fold_round : smix(fold_round ^ smix((uint64_t)c * 0x51ED27ull + 3));
        auto next = [&]() { rs = smix(rs); return rs; };
        h_keys[(size_t)c * nfold + k] = P[5] < 1.0 ? next() : 0ull;
        std::vector<int> feats(F);
        for (int f = 0; f < F; ++f) feats[f] = f;
        if (P[6] < 1.0) {
          const int kk = std::max(1, (int)std::floor(P[6] * F + 1e-9));
          for (int i = 0; i < F; ++i) std::swap(feats[i], feats[i + (int)(next() % (uint64_t)(F - i))]);
          feats.resize(kk);
          std::sort(feats.begin(), feats.end());
        }
        const uint64_t level_key = P[7] < 1.0 ? next() : 0ull;
        for (int d = 0; d <= D; ++d) {
          std::vector<int> lf = feats;
          if (P[7] < 1.0 && lf.size() > 1) {
            const int m = (int)lf.size();
            const int kk = std::max(1, (int)std::floor(P[7] * m + 1e-9));
            uint64_t ls = smix(level_key ^ smix((uint64_t)d + 1));
            for (int i = 0; i < m; ++i) {
              ls = smix(ls);
              std::swap(lf[i], lf[i + (int)(ls % (uint64_t)(m - i))]);
            }
            lf.resize(kk);
          }
          int* o = h_order + (size_t)c * order_elems + ((size_t)k * (D + 1) + d) * F;
          for (int i = 0; i < (int)lf.size(); ++i) o[lf[i]] = i + 1;
        }
      }
    }
    HC(hipMemcpyAsync(d_keys, h_keys, keys_bytes, hipMemcpyHostToDevice, 0));
    HC(hipMemcpyAsync(d_order, h_order, sizeof(int) * K * order_elems, hipMemcpyHostToDevice, 0));
    // ---- device: one tree per class for every fold, levels decided on the device
    for (int c = 0; c < K; ++c) {
      hipLaunchKernelGGL(grad_kernel, dim3(blocks, nfold), dim3(256), 0, 0, d_margin, d_y, d_gh, n, K, c, obj,
                         (float)P[10]);
      HC(hipMemsetAsync(d_mx, 0, sizeof(unsigned int) * 2 * nfold, 0));
      hipLaunchKernelGGL(gh_max_kernel, dim3(std::min(blocks, 256), nfold), dim3(256), 0, 0, d_gh, n, d_mx);
      HC(hipMemsetAsync(d_nroot, 0, sizeof(int) * nfold, 0));
      hipLaunchKernelGGL(root_rows_kernel, dim3(std::max(1, std::min(1024, (n + 256 * RR_PER - 1) / (256 * RR_PER))), nfold),
                         dim3(256), 0, 0, d_fold, n, d_keys + (size_t)c * nfold,
                         P[5], d_rows[0], d_nroot);
      hipLaunchKernelGGL(level0_kernel, dim3(nfold), dim3(64), 0, 0, geo, d_nroot, d_lvl[0], d_chunks, d_reds,
                         d_counts);
      const int* order_c = d_order + (size_t)c * order_elems;
      for (int d = 0; d <= D; ++d) {
        const int L = 1 << d;
        LNode* cur = d_lvl[d & 1];
        LNode* nxt = d_lvl[(d + 1) & 1];
        i64* hcur = d_hist[d & 1];
        if (d < D || d == 0) {
          if (hconst)
            hipLaunchKernelGGL(hist_kernel<true>, dim3(geo.maxch, nfb, nfold), dim3(HB_T), 0, 0, geo, d_bins,
                               d_rows[d & 1], d_gh, d_chunks, d_counts, hcur, d_part, d_mx);
          else
            hipLaunchKernelGGL(hist_kernel<false>, dim3(geo.maxch, nfb, nfold), dim3(HB_T), 0, 0, geo, d_bins,
                               d_rows[d & 1], d_gh, d_chunks, d_counts, hcur, d_part, d_mx);
          // a reduced node has more than rch rows: at most n / (rch + 1) of them per fold
          hipLaunchKernelGGL(reduce_kernel, dim3(std::max(1, n / (geo.rch + 1)), rlen, nfold), dim3(256), 0, 0, geo,
                             d_part, hcur, d_reds, d_counts);
          // siblings = parent - built child, materialised only where a later level subtracts from them
          // (the last histogram level's split reads them as the difference)
          if (d == 0)
            hipLaunchKernelGGL(root_totals_kernel, dim3(nfold), dim3(64), 0, 0, geo, hcur, cur);
          else if (d + 1 < D)
            hipLaunchKernelGGL(subtract_kernel, dim3(L, ylen, nfold), dim3(256), 0, 0, geo, cur, d_hist[(d - 1) & 1],
                               hcur);
        }
        if (d < D) {
          hipLaunchKernelGGL(split_kernel, dim3(F, L, nfold), dim3(64), 0, 0, geo, d, hcur,
                             (d > 0 && d + 1 == D) ? d_hist[(d - 1) & 1] : nullptr, d_nb, order_c, cur, d_mx, d_cand,
                             dp);
          hipLaunchKernelGGL(best_kernel, dim3(L, nfold), dim3(256), 0, 0, geo, d_cand, d_best);
        }
        hipLaunchKernelGGL(plan_split_kernel, dim3(nfold), dim3(256), 0, 0, geo, d, cur, d_best, d_mx, d_tree, d_leaf,
                           d_split, d_cur, nxt, dp);
        if (d < D) {
          hipLaunchKernelGGL(partition_kernel, dim3(pblocks, nfold), dim3(256), 0, 0, geo, d, g_binsT, d_nroot, cur,
                             d_split, d_rows[d & 1], d_rows[(d + 1) & 1], d_cur);
          hipLaunchKernelGGL(plan_next_kernel, dim3(nfold), dim3(256), 0, 0, geo, d, cur, d_split, d_cur, nxt,
                             d_chunks, d_reds, d_counts);
        }
      }
      hipLaunchKernelGGL(predict_kernel, dim3(std::min(blocks, 512), (nfold + pk - 1) / pk), dim3(256), pred_lds, 0,
                         geo, d_bins, d_tree, d_leaf, d_margin, c, pk, pr_rows);
    }
    for (int mi = 0; mi < n_metrics; ++mi)
      if (metrics[mi] != 4)
        hipLaunchKernelGGL(metric_kernel, dim3(mblocks, nfold), dim3(256), 0, 0, geo, d_margin, d_y, d_fold,
                           metrics[mi], objective, d_met + (size_t)mi * nfold * mblocks * 4);
    if (want_auc) {
      hipLaunchKernelGGL(auc_keys_kernel, dim3(mblocks, nfold), dim3(256), 0, 0, geo, d_margin, d_y, d_fold, d_akeys);
      HC(rocprim::radix_sort_keys(d_atmp, atmp_bytes, d_akeys, d_asorted, aN, 0u, (unsigned)aseg_bits));
      HC(hipMemsetAsync(d_aacc, 0, sizeof(double) * 4 * nfold, 0));
      hipLaunchKernelGGL(auc_rank_kernel, dim3((unsigned)std::min<size_t>(1024, (aN + 255) / 256)), dim3(256), 0, 0,
                         d_asorted, aN, 2 * nfold, d_aacc);
    }
    HC(hipGetLastError());
    // the round's blocking copies: early stopping needs the test metric
    HC(hipMemcpy(h_met, d_met, sizeof(double) * met_elems, hipMemcpyDeviceToHost));
    if (want_auc) HC(hipMemcpy(h_aacc.data(), d_aacc, sizeof(double) * 4 * nfold, hipMemcpyDeviceToHost));
    double tem_last = 0;
    for (int mi = 0; mi < n_metrics; ++mi) {
      std::vector<double> trv(nfold), tev(nfold);
      for (int k = 0; k < nfold; ++k) {
        if (metrics[mi] == 4) {         // engine.cpp auc_score: (R+ - n+(n+ + 1)/2) / (n+ n-), 0.5 if one class
          auto auc = [](double r, double np, double nn) {
            return (np == 0 || nn <= 0) ? 0.5 : (r - np * (np + 1) / 2) / (np * nn);
          };
          const double* a = &h_aacc[4 * (size_t)k];
          trv[k] = auc(a[0], a[1], (double)n - ntest[k] - a[1]);
          tev[k] = auc(a[2], a[3], ntest[k] - a[3]);
          continue;
        }
        double met[4] = {0, 0, 0, 0};
        const double* pm = h_met + ((size_t)mi * nfold + k) * mblocks * 4;
        for (int b = 0; b < mblocks; ++b)
          for (int q = 0; q < 4; ++q) met[q] += pm[(size_t)b * 4 + q];
        double tr = met[0] / std::max(1.0, met[1]), te = met[2] / std::max(1.0, met[3]);
        if (metrics[mi] == 0) { tr = std::sqrt(tr); te = std::sqrt(te); }
        trv[k] = tr; tev[k] = te;
      }
      double trm = 0, tem = 0, trs = 0, tes = 0;
      for (int k = 0; k < nfold; ++k) { trm += trv[k]; tem += tev[k]; }
      trm /= nfold; tem /= nfold;
      for (int k = 0; k < nfold; ++k) {
        const double a = trv[k] - trm, b = tev[k] - tem;
        trs += a * a; tes += b * b;
      }
      double* o = &out_hist[((size_t)round * n_metrics + mi) * 4];
      o[0] = trm; o[1] = std::sqrt(trs / nfold); o[2] = tem; o[3] = std::sqrt(tes / nfold);
      tem_last = tem;                  // early stopping on the last metric (engine.cpp)
    }
    rounds_done = round + 1;
    if (progress > 0 && rounds_done % progress == 0)
      std::fprintf(stderr, "[gbdt_hip] round %d  test metric %.6g  %.2f s\n", rounds_done, tem_last,
                   std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count());
    if (lower_better ? tem_last < best_score : tem_last > best_score) { best_score = tem_last; best_round = round; }
    if (early_stopping_rounds > 0 && round - best_round >= early_stopping_rounds) break;
  }
  if (timing)
    std::fprintf(stderr, "[gbdt_hip] %d rounds x %d folds in %.3f s (fold-batched device levels, depth %d)\n",
                 rounds_done, nfold,
                 std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count(), D);
  rc = early_stopping_rounds > 0 ? best_round + 1 : rounds_done;
done:
  for (void* p : {(void*)d_y, (void*)d_fold, (void*)d_nb, (void*)d_rows[0], (void*)d_rows[1], (void*)d_margin,
                  (void*)d_gh, (void*)d_hist[0], (void*)d_hist[1], (void*)d_part, (void*)d_lvl[0], (void*)d_lvl[1],
                  (void*)d_chunks, (void*)d_reds, (void*)d_counts, (void*)d_nroot, (void*)d_cand, (void*)d_best,
                  (void*)d_tree, (void*)d_leaf, (void*)d_split, (void*)d_cur, (void*)d_mx, (void*)d_keys,
                  (void*)d_order, (void*)d_met, (void*)d_akeys, (void*)d_asorted, (void*)d_atmp, (void*)d_aacc})
    if (p) (void)hipFree(p);
  if (h_up) (void)hipHostFree(h_up);
  if (h_met) (void)hipHostFree(h_met);
  return rc;
}

}  // extern "C"
