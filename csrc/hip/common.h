// Shared helpers for the gfx950 (MI355X / CDNA4) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;

#define GT_WAVE 64

// Step state shared by every kernel of one captured train step (int32 words):
//  [0] step_ctr (index into the epoch's batch table, ++ per step)
//  [1] cur_step (step_ctr snapshot for this step)
//  [2] t        (Adam step, float bits)
//  [3] lr       (float bits)
//  [4] lr_t     (bias-corrected step size, float bits)
//  [5] global_step (never reset; keys the dropout stream)
struct StepState {
  int step_ctr, cur_step;
  float t, lr, lr_t;
  int global_step;
  int opt;          // 0: Adam (Keras defaults), 1: SGD with momentum (Keras SGD, nesterov=False)
  float momentum;   // SGD momentum
};

// One parameter update. Adam: m, v moments, lr_t bias-corrected step.
// SGD-momentum (Keras 2.2 SGD): m is the velocity, v unused:
//   m = momentum * m - lr * g ;  p += m
__device__ __forceinline__ float opt_update(const StepState* st, float p, float g, float& m, float& v,
                                            float lr_t) {
  if (st->opt == 1) {
    m = st->momentum * m - lr_t * g;
    return p + m;
  }
  m = 0.9f * m + (1.f - 0.9f) * g;
  v = 0.999f * v + (1.f - 0.999f) * g * g;
  return p - lr_t * m / (sqrtf(v) + 1e-7f);
}

__device__ __forceinline__ float bf2f(uint16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

// round to nearest even; a plain conversion compiles to the gfx950
// v_cvt_pk_bf16_f32 (one instruction per pair, NaN stays NaN)
__device__ __forceinline__ uint16_t f2bf(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }

typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;

__device__ __forceinline__ uint32_t pack2bf(float a, float b) {
  const bf16x2_t v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}

__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 v;
  v.x = pack2bf(f[0], f[1]);
  v.y = pack2bf(f[2], f[3]);
  v.z = pack2bf(f[4], f[5]);
  v.w = pack2bf(f[6], f[7]);
  return v;
}

__device__ __forceinline__ uint2 pack4(const float* f) {
  uint2 v;
  v.x = pack2bf(f[0], f[1]);
  v.y = pack2bf(f[2], f[3]);
  return v;
}

__device__ __forceinline__ bf16x8_t as_frag(const uint4& v) { return __builtin_bit_cast(bf16x8_t, v); }

__device__ __forceinline__ f32x4_t mfma16(const uint4& a, const uint4& b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(a), as_frag(b), c, 0, 0, 0);
}

// ---------------------------------------------------------------------------
// fp32 precision on bf16 matrix cores: exact 3-way split ("bf16x6")
//
// Every fp32 value a (24-bit significand) is the EXACT sum of three bf16
// values a = a0 + a1 + a2: a0 = rne(a), a1 = rne(a - a0), a2 = a - a0 - a1
// (each residual is exact in fp32; the last has <= 8 significant bits, so it
// is a bf16 -- valid while a2 does not underflow, |a| > ~1e-33). A product
//   a*b = sum_{i+j<=2} ai*bj  +  (a1 b2 + a2 b1 + a2 b2)
// keeps six terms; every ai*bj is exact in fp32 (8x8-bit significands) and
// the MFMA accumulates in fp32, so the only error beyond fp32 accumulation is
// the three dropped terms: |a1 b2 + a2 b1 + a2 b2| <= (2^-24 + 2^-24 + 2^-32)|ab|
// ~= 2^-23 |ab| = 2 fp32 ulps of the product -- fp32-level by construction
// (tests/test_hip_fp32.py measures it against an fp64 oracle next to torch's
// own fp32). Cost: 6 v_mfma_f32_16x16x32_bf16 per 32-deep k-step, i.e. 2.7x
// cheaper than the native v_mfma_f32_16x16x4_f32 (8 x 32 cycles vs 6 x 16).
// ---------------------------------------------------------------------------
#define GT_NPL_F32 3     // bf16 planes of an fp32 operand

// bf16 / fp32 storage type of a precision (0 / 1)
template <int PREC> struct ActT { typedef uint16_t T; };
template <> struct ActT<1> { typedef float T; };

// 8 fp32 -> three bf16x8 planes with f = p0 + p1 + p2 exactly
__device__ __forceinline__ void split8(const float* f, uint4& p0, uint4& p1, uint4& p2) {
  float t[8], r[8];
  p0 = pack8(f);
  unpack8(p0, t);
#pragma unroll
  for (int e = 0; e < 8; ++e) r[e] = f[e] - t[e];
  p1 = pack8(r);
  unpack8(p1, t);
#pragma unroll
  for (int e = 0; e < 8; ++e) r[e] = r[e] - t[e];
  p2 = pack8(r);
}

// the fp32 value of three planes (exact: the inverse of split8)
__device__ __forceinline__ void join8(const uint4& p0, const uint4& p1, const uint4& p2, float* f) {
  float t[8];
  unpack8(p0, f);
  unpack8(p1, t);
#pragma unroll
  for (int e = 0; e < 8; ++e) f[e] += t[e];
  unpack8(p2, t);
#pragma unroll
  for (int e = 0; e < 8; ++e) f[e] += t[e];
}

// 8 consecutive fp32 (one 32-byte chunk of an fp32 activation)
__device__ __forceinline__ void load8f(const float* p, float* f) {
  const float4 q0 = reinterpret_cast<const float4*>(p)[0];
  const float4 q1 = reinterpret_cast<const float4*>(p)[1];
  f[0] = q0.x; f[1] = q0.y; f[2] = q0.z; f[3] = q0.w;
  f[4] = q1.x; f[5] = q1.y; f[6] = q1.z; f[7] = q1.w;
}

// 32 zero bytes in global memory: the source of out-of-image patch chunks
__device__ __attribute__((aligned(32), weak)) float gt_zero8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};

// load8f of p, or 8 zeros when !ok -- without a branch: the address is
// selected, the two loads always issue (a load under a per-chunk branch makes
// hipcc wait vmcnt(0) at each branch, serialising a thread's whole staging)
__device__ __forceinline__ void load8f_or0(const float* p, bool ok, float* f) {
  load8f(ok ? p : gt_zero8, f);
}

__device__ __forceinline__ void store8f(float* p, const float* f) {
  reinterpret_cast<float4*>(p)[0] = make_float4(f[0], f[1], f[2], f[3]);
  reinterpret_cast<float4*>(p)[1] = make_float4(f[4], f[5], f[6], f[7]);
}

// one 16x16 x 32-deep k-step of a split-precision product: A and B each in
// NPL bf16 planes (NPL = 1: plain bf16 MFMA; 3: the six-term fp32 product,
// smallest terms first)
template <int NPL>
__device__ __forceinline__ f32x4_t mfma_np(const uint4* a, const uint4* b, f32x4_t c) {
  if (NPL == 1) return mfma16(a[0], b[0], c);
  c = mfma16(a[2], b[0], c);
  c = mfma16(a[1], b[1], c);
  c = mfma16(a[0], b[2], c);
  c = mfma16(a[1], b[0], c);
  c = mfma16(a[0], b[1], c);
  return mfma16(a[0], b[0], c);
}

// element loads/stores of an activation chunk (8 channels) in either storage
// type: bf16 (uint16_t) or fp32 (float)
__device__ __forceinline__ void ld_chunk(const uint16_t* p, float* f) { unpack8(*reinterpret_cast<const uint4*>(p), f); }
__device__ __forceinline__ void ld_chunk(const float* p, float* f) { load8f(p, f); }
__device__ __forceinline__ void st_chunk(uint16_t* p, const float* f) { *reinterpret_cast<uint4*>(p) = pack8(f); }
__device__ __forceinline__ void st_chunk(float* p, const float* f) { store8f(p, f); }

// Counter-based hash -> uniform in [0,1): keyed dropout (deterministic per
// (seed, fold, step, row, col), independent of launch geometry).
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t hash4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  uint32_t h = mix32(a ^ 0x9e3779b9U);
  h = mix32(h ^ b);
  h = mix32(h ^ (c * 0x85ebca6bU));
  return mix32(h ^ (d * 0xc2b2ae35U));
}

// Exact unsigned division by a runtime divisor d via one mul-hi, valid
// whenever n * d < 2^32 (all index math here): m = ceil(2^32 / d).
struct FastDiv {
  uint32_t d, m;
  __device__ __forceinline__ explicit FastDiv(uint32_t dd) : d(dd), m(dd > 1 ? 0xFFFFFFFFu / dd + 1u : 0u) {}
  __device__ __forceinline__ uint32_t div(uint32_t n) const { return d > 1 ? __umulhi(n, m) : n; }
  __device__ __forceinline__ void divmod(uint32_t n, uint32_t& q, uint32_t& r) const { q = div(n); r = n - q * d; }
};

// Philox4x32-10 counter-based RNG (Salmon et al., SC'11): stateless, so any
// element of any tensor can be drawn independently by any thread.
__host__ __device__ inline void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[1] = (uint32_t)p1;
    c[3] = (uint32_t)p0;
    c[0] = n0;
    c[2] = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}
