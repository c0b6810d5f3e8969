// Optional BatchNorm of the Genetic-CNN node convs (TrainConfig.batch_norm,
// off by default: the reference network has none, keras_models.py:97-118).
//
//   conv (bias, no ReLU) -> z  ->  y = relu(gamma * (z - mean) * rstd + beta)
//
// Per group (candidate x fold replica) and channel, statistics over the
// batch's real rows (B, or the short last batch of batching="keras") and all
// pixels; running mean / unbiased variance with Keras' momentum (0.99) and
// epsilon (1e-3) for evaluation. Population-batched like the convs: a launch
// covers the groups of a GroupRec table, the grid is (chunks, groups).
//
// Two kernels per direction, both deterministic (fixed chunk geometry per
// layer shape, fixed-order reductions: a group's result does not depend on
// which other groups share the launch):
//   forward  : bn_stats  -> per-chunk shifted sums S1 = sum(z - k), S2 = sum((z - k)^2)
//              bn_apply  -> reduce the chunk partials, save (mean, rstd), update
//                           the running stats (chunk 0), write y (ReLU fused)
//   backward : bn_bwd_stats -> per-chunk sum(g), sum(g * xhat) of the ReLU-masked
//                              output gradient g (the consumers' dgrad applied the mask)
//              bn_bwd_apply -> dgamma / dbeta (chunk 0) and, in place,
//                              dz = gamma rstd (g - sum g / N - xhat sum(g xhat) / N)
//                              (0 on padding rows of a short batch and on the padded pixels of a
//                              zero-padded image: BnArgs::Hr / Wr)
// The shift k = z at pixel 0 of the group keeps S2 / N - (S1 / N)^2 free of
// cancellation when |mean| >> std. Pixels per chunk: cnn_kernels.bn_chunk_px (a function of the layer
// shape; at most 16K values per chunk so wide stages launch enough workgroups).
// Measured and not kept (round 6, profiles/r6/bn_chunk_r6.txt): 4 pixels' loads in flight per thread in
// the statistics kernels and 4 chunks' loads before the stores in the apply kernels (no gain).
#include "common.h"
#include "cnn_args.h"

struct BnArgs {
  void* z;                  // [Q][B][H][W][Cp] pre-activation (conv output with bias)
  void* y;                  // fwd: [Q][B][H][W][Cp] relu(bn(z)) out; bwd: ReLU-masked grad in, dz out (in place)
  const float* gamma;       // [Q][Cp]
  const float* beta;        // [Q][Cp]
  float* stat;              // [Q][2][Cp] saved mean, rstd of the training forward
  float* run;               // [2][Q][Cp] running mean, running (unbiased) variance
  float* part;              // [Q][nchunk][2][Cp] chunk partials
  float* ggamma;            // [Q][Cp] (bwd)
  float* gbeta;             // [Q][Cp] (bwd)
  const GroupRec* gtab;     // [ngroups]
  const int* valid;         // [steps][Q] real rows per training batch, or null = B
  const StepState* st;
  int ngroups, G, B, HW, Cp, nchunk, chunk_px;
  float momentum, eps;
  int train;                // 1: batch statistics (training forward); 0: running statistics
  int prec;
  // fused 2x2 max-pool (K1/K4 with BatchNorm: conv -> BN -> ReLU -> pool): groups whose GroupRec
  // out_mask bit 24 is set pool this layer's output into pool_y [Q][B][H/2][W/2][Cp] and the argmax
  // mask (pool_fwd_kernel's format; null in evaluation). Chunks hold whole row pairs (chunk_px % 2W == 0).
  void* pool_y;
  uint8_t* pool_mask;
  int W;
  // real extent of a zero-padded image (ConvArgs::Hr / Wr; 0: not padded): statistics count the real
  // pixels only, and y / dz are exact zeros outside them (the padded network IS the unpadded one)
  int Hr, Wr;
};

// pixel p (flat over the group's images) lies outside the real extent of a zero-padded image
__device__ __forceinline__ bool bn_pad_px(const BnArgs& a, long p) {
  if (a.Hr <= 0) return false;
  const int pi = (int)(p % a.HW);
  return pi / a.W >= a.Hr || pi % a.W >= a.Wr;
}

// real pixels per image (the statistics' count)
__device__ __forceinline__ long bn_real_hw(const BnArgs& a) {
  return a.Hr > 0 ? (long)a.Hr * a.Wr : (long)a.HW;
}

#define BN_THREADS 256

// sum over the nch chunk partials of channel t (stride 2 Cp), in chunk order, 8 loads in flight: the
// apply kernels' prologue (a dependent load per chunk made it ~0.7 us per chunk on every workgroup)
__device__ __forceinline__ void bn_sum_parts(const float* __restrict__ part, int nch, int Cp, int t, float& s1,
                                             float& s2) {
  s1 = 0.f; s2 = 0.f;
  int c = 0;
  for (; c + 8 <= nch; c += 8) {
    float x1[8], x2[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      x1[k] = part[(long)(c + k) * 2 * Cp + t];
      x2[k] = part[(long)(c + k) * 2 * Cp + Cp + t];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) { s1 += x1[k]; s2 += x2[k]; }
  }
  for (; c < nch; ++c) {
    s1 += part[(long)c * 2 * Cp + t];
    s2 += part[(long)c * 2 * Cp + Cp + t];
  }
}

__device__ __forceinline__ int bn_rows(const BnArgs& a, int g) {
  if (!a.train || !a.valid) return a.B;
  const int step = a.st ? a.st->cur_step : 0;
  const int nv = a.valid[(long)step * a.G + g];
  return nv < 0 ? 0 : (nv > a.B ? a.B : nv);
}

// Two per-channel sums over a pixel range, reduced in a fixed order: threads
// t < nact own channel chunk t % nc8 and pixels (t / nc8) + k * (nact / nc8).
// acc[0..7] / acc[8..15] are the two sums of the thread's 8 channels; the
// result for channel c lands in out[0][c], out[1][c] (threads c < Cp).
__device__ __forceinline__ void bn_block_reduce(float (*red)[17], const float* acc, int nc8, int nact,
                                                float* out0, float* out1, int Cp) {
  const int t = threadIdx.x;
  if (t < nact) {
#pragma unroll
    for (int e = 0; e < 16; ++e) red[t][e] = acc[e];
  }
  __syncthreads();
  if (t < Cp) {
    const int c8 = t >> 3, e = t & 7, np = nact / nc8;
    float s0 = 0.f, s1 = 0.f;
    for (int p = 0; p < np; ++p) {
      s0 += red[p * nc8 + c8][e];
      s1 += red[p * nc8 + c8][8 + e];
    }
    out0[t] = s0;
    out1[t] = s1;
  }
}

template <int PREC>
__global__ void __launch_bounds__(BN_THREADS) bn_stats_kernel(BnArgs a) {
  typedef typename ActT<PREC>::T AT;
  __shared__ float red[BN_THREADS][17];
  const GroupRec r = a.gtab[blockIdx.y];
  const int g = r.g, Cp = a.Cp, nc8 = Cp >> 3;
  const int nact = (BN_THREADS / nc8) * nc8, t = threadIdx.x;
  const long npx = (long)bn_rows(a, g) * a.HW;
  const long p0 = (long)blockIdx.x * a.chunk_px;
  const long p1 = p0 + a.chunk_px < npx ? p0 + a.chunk_px : npx;
  const AT* z = reinterpret_cast<const AT*>(a.z) + (long)g * a.B * a.HW * Cp;
  float acc[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = 0.f;
  if (t < nact) {
    const int c8 = t % nc8;
    float k[8], v[8];
    ld_chunk(z + c8 * 8, k);                       // shift: the group's pixel 0
    for (long p = p0 + t / nc8; p < p1; p += nact / nc8) {
      if (bn_pad_px(a, p)) continue;
      ld_chunk(z + p * Cp + c8 * 8, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = v[e] - k[e];
        acc[e] += d;
        acc[8 + e] += d * d;
      }
    }
  }
  float* part = a.part + ((long)g * a.nchunk + blockIdx.x) * 2 * Cp;
  bn_block_reduce(red, acc, nc8, nact, part, part + Cp, Cp);
}

template <int PREC>
__global__ void __launch_bounds__(BN_THREADS) bn_apply_kernel(BnArgs a) {
  typedef typename ActT<PREC>::T AT;
  __shared__ float sc[256], sh[256];
  const GroupRec r = a.gtab[blockIdx.y];
  const int g = r.g, Cp = a.Cp, nc8 = Cp >> 3, t = threadIdx.x;
  const AT* z = reinterpret_cast<const AT*>(a.z) + (long)g * a.B * a.HW * Cp;
  AT* y = reinterpret_cast<AT*>(a.y) + (long)g * a.B * a.HW * Cp;
  if (t < Cp) {
    const float gm = a.gamma[(long)g * Cp + t], bt = a.beta[(long)g * Cp + t];
    float mean, rstd;
    if (a.train) {
      const long npx = (long)bn_rows(a, g) * a.HW;
      const int nch = (int)((npx + a.chunk_px - 1) / a.chunk_px);
      const float* part = a.part + (long)g * a.nchunk * 2 * Cp;
      float s1, s2;
      bn_sum_parts(part, nch, Cp, t, s1, s2);
      const long nreal = (long)bn_rows(a, g) * bn_real_hw(a);
      const float n = nreal > 0 ? (float)nreal : 1.f;
      const float m1 = s1 / n;
      const float var = fmaxf(s2 / n - m1 * m1, 0.f);
      float k;                                     // the shift of bn_stats: the group's pixel 0
      if constexpr (PREC) k = z[t]; else k = bf2f(z[t]);
      mean = k + m1;
      rstd = rsqrtf(var + a.eps);
      if (blockIdx.x == 0 && npx > 0) {
        a.stat[(long)g * 2 * Cp + t] = mean;
        a.stat[(long)g * 2 * Cp + Cp + t] = rstd;
        float* rm = a.run + (long)g * Cp + t;
        float* rv = a.run + (long)a.G * Cp + (long)g * Cp + t;
        const float unb = nreal > 1 ? var * n / (n - 1.f) : var;
        *rm = a.momentum * *rm + (1.f - a.momentum) * mean;
        *rv = a.momentum * *rv + (1.f - a.momentum) * unb;
      }
    } else {
      mean = a.run[(long)g * Cp + t];
      rstd = rsqrtf(a.run[(long)a.G * Cp + (long)g * Cp + t] + a.eps);
    }
    sc[t] = gm * rstd;
    sh[t] = bt - mean * gm * rstd;
  }
  __syncthreads();
  const long npx = (long)a.B * a.HW;              // every row (padding rows too: finite values, zero loss weight)
  const long p0 = (long)blockIdx.x * a.chunk_px;
  const long p1 = p0 + a.chunk_px < npx ? p0 + a.chunk_px : npx;
  const long n8 = (p1 - p0) * nc8;
  for (long i = t; i < n8; i += BN_THREADS) {
    const long p = p0 + i / nc8;
    const int c8 = (int)(i % nc8);
    float v[8];
    ld_chunk(z + p * Cp + c8 * 8, v);
    const bool pad = bn_pad_px(a, p);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = pad ? 0.f : fmaxf(v[e] * sc[c8 * 8 + e] + sh[c8 * 8 + e], 0.f);
    st_chunk(y + p * Cp + c8 * 8, v);
  }
  if (!a.pool_y || !((r.out_mask >> 24) & 1)) return;
  // pooled cells of this chunk, from z (the values exactly as stored in y: bf16-rounded in prec 0);
  // first strict maximum over (0,0), (0,1), (1,0), (1,1), bit 2 = maximum > 0
  const int W = a.W, Wo = W >> 1;
  AT* py = reinterpret_cast<AT*>(a.pool_y) + (long)g * a.B * (a.HW >> 2) * Cp;
  uint8_t* pm = a.pool_mask ? a.pool_mask + (long)g * a.B * (a.HW >> 2) * Cp : nullptr;
  const long rp0 = p0 / (2 * W);                   // first row pair of the chunk (flat over images)
  const long ncell = (p1 - p0) >> 2;
  for (long i = t; i < ncell * nc8; i += BN_THREADS) {
    const long k = i / nc8;
    const int c8 = (int)(i % nc8);
    const long rp = rp0 + k / Wo;
    const int pc = (int)(k % Wo);
    const long ptl = rp * 2 * W + 2 * pc;          // top-left pixel
    const long offs[4] = {0, 1, (long)W, (long)W + 1};
    float m[8], v[8];
    int arg[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      ld_chunk(z + (ptl + offs[q]) * Cp + c8 * 8, v);
      const bool pad = bn_pad_px(a, ptl + offs[q]);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float o = pad ? 0.f : fmaxf(v[e] * sc[c8 * 8 + e] + sh[c8 * 8 + e], 0.f);
        if constexpr (!PREC) o = bf2f(f2bf(o));
        if (q == 0) m[e] = o;
        else if (o > m[e]) { m[e] = o; arg[e] = q; }
      }
    }
    const long o = (rp * Wo + pc) * Cp + c8 * 8;
    st_chunk(py + o, m);
    if (pm) {
      uint32_t lo = 0, hi = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) lo |= (uint32_t)(arg[j] | (m[j] > 0.f ? 4 : 0)) << (8 * j);
#pragma unroll
      for (int j = 0; j < 4; ++j) hi |= (uint32_t)(arg[4 + j] | (m[4 + j] > 0.f ? 4 : 0)) << (8 * j);
      *reinterpret_cast<uint2*>(pm + o) = make_uint2(lo, hi);
    }
  }
}

template <int PREC>
__global__ void __launch_bounds__(BN_THREADS) bn_bwd_stats_kernel(BnArgs a) {
  typedef typename ActT<PREC>::T AT;
  __shared__ float red[BN_THREADS][17];
  const GroupRec r = a.gtab[blockIdx.y];
  const int g = r.g, Cp = a.Cp, nc8 = Cp >> 3;
  const int nact = (BN_THREADS / nc8) * nc8, t = threadIdx.x;
  const long npx = (long)bn_rows(a, g) * a.HW;
  const long p0 = (long)blockIdx.x * a.chunk_px;
  const long p1 = p0 + a.chunk_px < npx ? p0 + a.chunk_px : npx;
  const AT* z = reinterpret_cast<const AT*>(a.z) + (long)g * a.B * a.HW * Cp;
  const AT* gy = reinterpret_cast<const AT*>(a.y) + (long)g * a.B * a.HW * Cp;
  const float* stat = a.stat + (long)g * 2 * Cp;
  float acc[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = 0.f;
  if (t < nact) {
    const int c8 = t % nc8;
    float mean[8], rstd[8], v[8], d[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      mean[e] = stat[c8 * 8 + e];
      rstd[e] = stat[Cp + c8 * 8 + e];
    }
    for (long p = p0 + t / nc8; p < p1; p += nact / nc8) {
      if (bn_pad_px(a, p)) continue;
      ld_chunk(z + p * Cp + c8 * 8, v);
      ld_chunk(gy + p * Cp + c8 * 8, d);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        acc[e] += d[e];
        acc[8 + e] += d[e] * ((v[e] - mean[e]) * rstd[e]);
      }
    }
  }
  float* part = a.part + ((long)g * a.nchunk + blockIdx.x) * 2 * Cp;
  bn_block_reduce(red, acc, nc8, nact, part, part + Cp, Cp);
}

template <int PREC>
__global__ void __launch_bounds__(BN_THREADS) bn_bwd_apply_kernel(BnArgs a) {
  typedef typename ActT<PREC>::T AT;
  __shared__ float cg[256], cm[256], cx[256], mu[256], rs[256];
  const GroupRec r = a.gtab[blockIdx.y];
  const int g = r.g, Cp = a.Cp, nc8 = Cp >> 3, t = threadIdx.x;
  const long nvpx = (long)bn_rows(a, g) * a.HW;
  const AT* z = reinterpret_cast<const AT*>(a.z) + (long)g * a.B * a.HW * Cp;
  AT* gy = reinterpret_cast<AT*>(a.y) + (long)g * a.B * a.HW * Cp;
  if (t < Cp) {
    const int nch = (int)((nvpx + a.chunk_px - 1) / a.chunk_px);
    const float* part = a.part + (long)g * a.nchunk * 2 * Cp;
    float sg, sgx;
    bn_sum_parts(part, nch, Cp, t, sg, sgx);
    if (blockIdx.x == 0) {
      a.gbeta[(long)g * Cp + t] = sg;
      a.ggamma[(long)g * Cp + t] = sgx;
    }
    const long nreal = (long)bn_rows(a, g) * bn_real_hw(a);
    const float inv_n = nreal > 0 ? 1.f / (float)nreal : 0.f;
    const float rstd = a.stat[(long)g * 2 * Cp + Cp + t];
    cg[t] = a.gamma[(long)g * Cp + t] * rstd;
    cm[t] = sg * inv_n;
    cx[t] = sgx * inv_n;
    mu[t] = a.stat[(long)g * 2 * Cp + t];
    rs[t] = rstd;
  }
  __syncthreads();
  const long npx = (long)a.B * a.HW;
  const long p0 = (long)blockIdx.x * a.chunk_px;
  const long p1 = p0 + a.chunk_px < npx ? p0 + a.chunk_px : npx;
  const long n8 = (p1 - p0) * nc8;
  for (long i = t; i < n8; i += BN_THREADS) {
    const long p = p0 + i / nc8;
    const int c8 = (int)(i % nc8);
    float v[8], d[8];
    if (p < nvpx && !bn_pad_px(a, p)) {
      ld_chunk(z + p * Cp + c8 * 8, v);
      ld_chunk(gy + p * Cp + c8 * 8, d);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = c8 * 8 + e;
        const float xh = (v[e] - mu[c]) * rs[c];
        d[e] = cg[c] * (d[e] - cm[c] - xh * cx[c]);
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) d[e] = 0.f;
    }
    st_chunk(gy + p * Cp + c8 * 8, d);
  }
}

static bool bn_shape_ok(const BnArgs* a) {
  return a->Cp > 0 && a->Cp % 8 == 0 && a->Cp <= 256 && a->ngroups > 0 && a->nchunk > 0 && a->chunk_px > 0 &&
         (long)a->nchunk * a->chunk_px >= (long)a->B * a->HW && a->gtab && a->part;
}

extern "C" {

int gt_bn_fwd(const BnArgs* a, hipStream_t s) {
  if (!bn_shape_ok(a)) return (int)hipErrorInvalidValue;
  const dim3 grid(a->nchunk, a->ngroups);
  if (a->train) {
    if (a->prec) hipLaunchKernelGGL(bn_stats_kernel<1>, grid, dim3(BN_THREADS), 0, s, *a);
    else hipLaunchKernelGGL(bn_stats_kernel<0>, grid, dim3(BN_THREADS), 0, s, *a);
  }
  if (a->prec) hipLaunchKernelGGL(bn_apply_kernel<1>, grid, dim3(BN_THREADS), 0, s, *a);
  else hipLaunchKernelGGL(bn_apply_kernel<0>, grid, dim3(BN_THREADS), 0, s, *a);
  return (int)hipGetLastError();
}

int gt_bn_bwd(const BnArgs* a, hipStream_t s) {
  if (!bn_shape_ok(a) || !a->ggamma || !a->gbeta) return (int)hipErrorInvalidValue;
  const dim3 grid(a->nchunk, a->ngroups);
  if (a->prec) {
    hipLaunchKernelGGL(bn_bwd_stats_kernel<1>, grid, dim3(BN_THREADS), 0, s, *a);
    hipLaunchKernelGGL(bn_bwd_apply_kernel<1>, grid, dim3(BN_THREADS), 0, s, *a);
  } else {
    hipLaunchKernelGGL(bn_bwd_stats_kernel<0>, grid, dim3(BN_THREADS), 0, s, *a);
    hipLaunchKernelGGL(bn_bwd_apply_kernel<0>, grid, dim3(BN_THREADS), 0, s, *a);
  }
  return (int)hipGetLastError();
}

size_t gt_sizeof_bn_args() { return sizeof(BnArgs); }

}  // extern "C"
