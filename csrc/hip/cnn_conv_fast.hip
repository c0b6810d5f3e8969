// Shape-specialised implicit-GEMM convolution (forward and data-gradient) and weight gradient:
// host dispatch of the search-space shapes. The kernel templates (and the design notes) are in
// conv_fast_impl.h; user-chosen architectures dispatch in cnn_conv_fast_ext.hip.
#include "conv_fast_host.h"

// ---------------------------------------------------------------------------
// dispatch: (KH, KW, Cinp, W, Coutp-tiles) -> instantiation; -100 = no match
// (the caller then uses the generic kernel)
// ---------------------------------------------------------------------------

static int g_conv_nwv = 0;   // waves per workgroup override for the 8-wave-capable shapes (0: per-shape default)

extern "C" int gt_conv_set_nwv(int n) {
  const int old = g_conv_nwv;
  g_conv_nwv = n;
  return old;
}


// probe mode (gt_conv_fast_probe): report the tile rows of the instantiation
// that would run instead of launching it (0: none that fuses the pool)
static int g_probe = 0;


// The S=(3,5) s2 input-conv dgrad (5x5, 50 -> 20) with one co tile per wave and 4 pixel groups each
// instead of the packed tile's 2 tiles x 2 groups: 33 % more MFMAs but half the weight loads per MFMA;
// same-box A/B 126 -> 114 us per launch at 25 groups, population step -1.6 % (profiles/conv_s2in_dgrad_ct1_ab_r3.txt).
// Runtime setter (gt_conv_set_s2in_ct1, tests only) so both variants are compared against the fp64
// oracle on one launch in one process (tests/test_hip_fp32.py::test_s2in_dgrad_variants): both 1.3e-6 of
// the output range (torch fp32: 7.1e-7), channels 0-15 bitwise equal, deterministic; the 2-rank DP
// trajectory stays within the derived summation-order bound (tests/test_hip_dp.py). On by default since
// round 4 (profiles/conv_s2in_dgrad_ct1_r4.txt).
static int g_s2in_ct1 = -1;
static bool s2in_ct1_on() {
  if (g_s2in_ct1 < 0) g_s2in_ct1 = 1;
  return g_s2in_ct1 != 0;
}
extern "C" int gt_conv_set_s2in_ct1(int on) {
  s2in_ct1_on();
  const int old = g_s2in_ct1;
  g_s2in_ct1 = on;
  return old;
}

// fp32 register-direct epilogue in the tile kernel (gt_conv_set_regepi: tests compare it with the LDS tile):
// no LDS output tile, no second barrier, the pool from lane shuffles
static int g_regepi = -1;
static bool regepi_on() {
  // on by default: 2-19 % faster per fp32 conv launch, bit-identical (profiles/conv_f32_regepi_ab_r3.txt)
  if (g_regepi < 0) g_regepi = 1;
  return g_regepi != 0;
}
extern "C" int gt_conv_set_regepi(int on) {
  regepi_on();
  const int old = g_regepi;
  g_regepi = on;
  return old;
}



// Small launches (few groups per launch: the reference's sequential folds, one
// rank's share of a config-3 generation): at 2 groups the 8-row tiles of the
// 16x16 stage make 128 workgroups for 256 CUs. Shorter tiles (4 or 2 rows;
// 2 rows = one co tile per wave, so a wave still holds whole row pairs for the
// fused pool) multiply the grid. Every output's k loop (order of k-steps and
// of the six split terms) is the same for any tile height: results are
// bit-identical to the 8-row tiles (tests/test_hip_kernels.py), so a
// candidate's result still does not depend on how many groups share its
// launch. gt_conv_set_smallq(0) disables (tests compare both).
static int g_smallq = -1;
extern "C" int gt_conv_set_smallq(int on) {
  const int old = g_smallq;
  g_smallq = on;
  return old;
}
// tile rows for a launch whose default tile has TH rows: halve while the grid
// is below 300 workgroups (default 300: about one per CU; at 5 and 10 groups the
// 8-row tiles measured faster than 4-row ones, profiles/conv_tile_threshold_ab_r4.txt), down to THMIN
static long g_smallq_wg = -1;
static int smallq_th(const ConvArgs* a, int TH, int THMIN) {
  if (g_smallq < 0) g_smallq = 1;
  if (g_smallq_wg < 0)
    g_smallq_wg = 300;
  if (!g_smallq) return TH;
  int th = TH;
  while (th > THMIN && (long)a->ngroups * a->B * (a->H / th) < g_smallq_wg) th >>= 1;
  return th;
}

#ifndef GT_KERNELS_ONLY   // (tools/isa_one.sh: one explicit instantiation, no dispatch tables)
extern "C" int gt_conv_wino(const ConvArgs* a, hipStream_t stream, int probe);
extern "C" int gt_conv_fast_ext(const ConvArgs* a, hipStream_t stream, int probe);
extern "C" int gt_wgrad_fast_ext(const WgradArgs* a, hipStream_t stream);
extern "C" int gt_wgrad_rows_ext(int KH, int KW, int Cinp, int Coutp, int H, int W, int prec);

// dispatch state for cnn_conv_fast_ext.hip (its launch macros read the same switches)
extern "C" int gt_conv_regepi_on() { return regepi_on() ? 1 : 0; }
extern "C" int gt_conv_smallq_th(const ConvArgs* a, int TH, int THMIN) { return smallq_th(a, TH, THMIN); }

extern "C" int gt_conv_fast(const ConvArgs* a_in, hipStream_t stream) {
  const ConvArgs* a = a_in;
  if (a->wino) return gt_conv_wino(a, stream, g_probe);   // Winograd 3x3 layers (cnn_conv_wino.hip)
  if (a->mask) return -100;                  // staged ReLU mask: generic kernel only
  if (a->prec == 1) {
    // small launches: shorter tiles of the S=(3,5) shapes (see smallq_th)
    if (CONV_FAST_MATCH(5, 5, 1, 32, 8, 2, 3) && smallq_th(a, 8, 4) == 4) {      // s1 input conv
      if (pk_ok(a, 2)) CONV_FAST_LAUNCH_PK(5, 5, 1, 32, 4, 2, 3, 2, 1, 1)
      CONV_FAST_LAUNCH(5, 5, 1, 32, 4, 2, 3, 2, 1)
    }
    if (CONV_FAST_MATCH(3, 3, 3, 32, 8, 2, 3) && smallq_th(a, 8, 4) == 4) {      // s1 nodes / dgrad
      if (pk_ok(a, 2)) CONV_FAST_LAUNCH_PK(3, 3, 3, 32, 4, 2, 3, 2, 1, 1)
      CONV_FAST_LAUNCH(3, 3, 3, 32, 4, 2, 3, 2, 1)
    }
    if (CONV_FAST_MATCH(5, 5, 3, 16, 8, 4, 7)) {                                  // s2 input conv
      const int th = smallq_th(a, 8, 2);
      if (th == 4) CONV_FAST_LAUNCH(5, 5, 3, 16, 4, 4, 7, 4, 1)
      if (th == 2) CONV_FAST_LAUNCH_CT1(5, 5, 3, 16, 2, 4, 7, 4)
    }
    if (CONV_FAST_MATCH(3, 3, 7, 16, 8, 4, 7)) {                                  // s2 nodes / dgrad
      const int th = smallq_th(a, 8, 2);
      if (th == 4) CONV_FAST_LAUNCH(3, 3, 7, 16, 4, 4, 7, 4, 1)
      if (th == 2) CONV_FAST_LAUNCH_CT1(3, 3, 7, 16, 2, 4, 7, 4)
    }
    if (s2in_ct1_on() && CONV_FAST_MATCH(5, 5, 7, 16, 8, 2, 3) && smallq_th(a, 8, 4) == 4)   // s2 input dgrad
      CONV_FAST_LAUNCH_CT1(5, 5, 7, 16, 4, 2, 3, 4)
    // Genetic-CNN CIFAR-shaped S=(3,5) space, kernels (20, 50), 5x5 stage convs
    // (8-wave workgroups for these fp32 tiles: 35-40 % slower per launch, r5/conv_f32_nwv8_ab_r5.txt)
    CONV_FAST_CASE_F32_PK(5, 5, 1, 32, 8, 2, 3, 4)   // s1 input conv (3 -> 20)
    CONV_FAST_CASE_F32_PK(3, 3, 3, 32, 8, 2, 3, 4)   // s1 nodes / output conv, and their dgrad (20 -> 20)
    // s2 input conv (20 -> 50): one co tile per wave as well (fwd 84-85 vs 86-90 us, r5/conv_s2n_ct1_ab_r5.txt)
    if (CONV_FAST_MATCH(5, 5, 3, 16, 8, 4, 7)) CONV_FAST_LAUNCH_CT1S(5, 5, 3, 16, 8, 4, 7, 4, 0)
    // (a packed tile here needs every wave to own all 4 co tiles: 2x the weight traffic per MFMA,
    // measured 20 % slower than the 2 + 2 split -- profiles/conv_f32_packed_tile_ab_r2.txt)
    // s2 nodes / output conv, and their dgrad (50 -> 50): one co tile per wave, all 8 pixel groups (170 VGPRs
    // at 2 waves/SIMD): half the weight-fragment loads per MFMA of the 2 co x 4 group split, -1 % per
    // population step at 25 and 80 groups (r5/conv_s2n_ct1_ab_r5.txt; the enforced-pipeline build spills here)
    if (CONV_FAST_MATCH(3, 3, 7, 16, 8, 4, 7)) CONV_FAST_LAUNCH_CT1S(3, 3, 7, 16, 8, 4, 7, 4, 0)
    if (s2in_ct1_on() && CONV_FAST_MATCH(5, 5, 7, 16, 8, 2, 3)) CONV_FAST_LAUNCH_CT1(5, 5, 7, 16, 8, 2, 3, 4)
    CONV_FAST_CASE_F32_PK(5, 5, 7, 16, 8, 2, 3, 4)   // s2 input conv dgrad (50 -> 20)
    // deep S=(3,4,5) space, kernels (20, 50, 100): stage 3 at 8x8, one image per workgroup
    CONV_FAST_CASE_F32_NARROW(5, 5, 7, 8, 8, 7, 13, 7)   // s3 input conv (50 -> 100): one co tile per wave, 7 waves
    CONV_FAST_CASE_F32_NARROW(3, 3, 13, 8, 8, 7, 13, 7)  // s3 nodes / output conv, and their dgrad (100 -> 100)
    CONV_FAST_CASE_F32_NARROW(5, 5, 13, 8, 8, 4, 7, 4)   // s3 input conv dgrad (100 -> 50)
    // wide deep space S=(3,4,5), kernels (64, 128, 256): the whole Cin patch in LDS (up to 154 KB: one
    // workgroup of 8 waves per CU for stages 2-3), 2 co tiles x 4 pixel groups per wave
    CONV_FAST_CASE_F32_NARROW(5, 5, 1, 32, 8, 4, 8, 4)     // s1 input conv (3 -> 64)
    // s1 nodes / output conv, and their dgrad (64 -> 64): one co tile per wave (-0.7 % per wide step)
    if (CONV_FAST_MATCH(3, 3, 8, 32, 4, 4, 8)) CONV_FAST_LAUNCH_CT1S(3, 3, 8, 32, 4, 4, 8, 4, 0)
    // stage 2 (s2 input conv 64 -> 128; nodes / output conv and their dgrad 128 -> 128): one co tile per wave
    // over all 8 pixel groups (-4.3 % per wide population step, r5/conv_s2n_ct1_ab_r5.txt)
    if (CONV_FAST_MATCH(5, 5, 8, 16, 8, 8, 16)) CONV_FAST_LAUNCH_CT1S(5, 5, 8, 16, 8, 8, 16, 8, 0)
    if (CONV_FAST_MATCH(3, 3, 16, 16, 8, 8, 16)) CONV_FAST_LAUNCH_CT1S(3, 3, 16, 16, 8, 8, 16, 8, 0)
    CONV_FAST_CASE_F32_NARROW(5, 5, 16, 16, 4, 4, 8, 4)    // s2 input conv dgrad (128 -> 64)
    CONV_FAST_CASE_F32_NARROW(5, 5, 16, 8, 8, 16, 32, 8)   // s3 input conv (128 -> 256)
    CONV_FAST_CASE_F32_NARROW(3, 3, 32, 8, 8, 16, 32, 8)   // s3 nodes / output conv, and their dgrad (256 -> 256)
    CONV_FAST_CASE_F32_NARROW(5, 5, 32, 8, 4, 8, 16, 4)    // s3 input conv dgrad (256 -> 128)
    {   // user-chosen architectures (cnn_conv_fast_ext.hip: 32/64-channel stages, 3x3 stage-input kernels)
      const int rc = gt_conv_fast_ext(a, stream, g_probe);
      if (rc != -100) return rc;
    }
    return -100;
  }
  if (a->prec != 0) return -1;
  // Genetic-CNN CIFAR-shaped S=(3,5) space, kernels (20, 50), 5x5 stage convs
  CONV_FAST_CASE2(5, 5, 1, 32, 8, 2, 3, 4)   // s1 input conv (3 -> 20)
  CONV_FAST_CASE2(3, 3, 3, 32, 8, 2, 3, 4)   // s1 nodes / output conv, and their dgrad (20 -> 20)
  CONV_FAST_CASE2(5, 5, 3, 16, 16, 4, 7, 4)  // s2 input conv (20 -> 50)
  CONV_FAST_CASE2(3, 3, 7, 16, 16, 4, 7, 8)  // s2 nodes / output conv, and their dgrad (50 -> 50)
  CONV_FAST_CASE2(5, 5, 7, 16, 16, 2, 3, 4)  // s2 input conv dgrad (50 -> 20)
  // deep S=(3,4,5) space, kernels (20, 50, 100): stage 3 at 8x8 (one image per workgroup)
  CONV_FAST_CASE_NW(5, 5, 7, 8, 8, 7, 13, 7)    // s3 input conv (50 -> 100)
  CONV_FAST_CASE_NW(3, 3, 13, 8, 8, 7, 13, 7)   // s3 nodes / output conv, and their dgrad (100 -> 100)
  CONV_FAST_CASE2(5, 5, 13, 8, 8, 4, 7, 4)      // s3 input conv dgrad (100 -> 50)
  return -100;
}

// rows of the shape-specialised tile gt_conv_fast would launch for these
// arguments when that kernel can fuse the 2x2 pool (even rows), else 0
extern "C" int gt_conv_fast_probe(const ConvArgs* a) {
  g_probe = 1;
  const int rc = gt_conv_fast(a, nullptr);
  g_probe = 0;
  const int th = rc >= 1000 ? rc - 1000 : 0;
  return th % 2 == 0 ? th : 0;
}

// 1 when gt_conv_fast would run these (data-gradient) arguments on a
// shape-specialised kernel, which can un-pool its output (fused pool backward)
extern "C" int gt_conv_fast_probe_any(const ConvArgs* a) {
  g_probe = 1;
  const int rc = gt_conv_fast(a, nullptr);
  g_probe = 0;
  return rc >= 1000 ? 1 : 0;
}

#endif  // GT_KERNELS_ONLY


__global__ void __launch_bounds__(256) wgrad_reduce_kernel(WgradArgs a) {
  const GroupRec gr = group_rec(a.gtab, blockIdx.y, a.n_in, 0, 0, nullptr);
  const int g = gr.g;
  const long kd = (long)a.KH * a.KW * a.Cinp;
  const long n = (long)a.Coutp * kd;
  const long gs = (long)a.G * n;                   // split stride of part_w
  float* pw = a.part_w + (long)g * n;
  const long i4 = ((long)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i4 < n) {                                    // n % 4 == 0 (Cinp % 8 == 0)
    // 8 partials in flight per batch (a dependent load-add chain waited for
    // each one: ~20 us per call); summed in split order
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    int sp = 0;
    for (; sp + 8 <= a.S; sp += 8) {
      float4 v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = *reinterpret_cast<const float4*>(pw + (long)(sp + k) * gs + i4);
#pragma unroll
      for (int k = 0; k < 8; ++k) { acc.x += v[k].x; acc.y += v[k].y; acc.z += v[k].z; acc.w += v[k].w; }
    }
    for (; sp < a.S; ++sp) {
      const float4 v = *reinterpret_cast<const float4*>(pw + (long)sp * gs + i4);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    *reinterpret_cast<float4*>(pw + i4) = acc;
  }
  if (blockIdx.x == 0 && a.part_b) {
    float* pb = a.part_b + (long)g * a.Coutp;
    for (int i = threadIdx.x; i < a.Coutp; i += 256) {
      float acc = 0.f;
      for (int sp = 0; sp < a.S; ++sp) acc += pb[(long)sp * a.G * a.Coutp + i];
      pb[i] = acc;
    }
  }
}

extern "C" int gt_wgrad_reduce(const WgradArgs* a, hipStream_t stream) {
  const long n = (long)a->Coutp * a->KH * a->KW * a->Cinp;
  if (n % 4 || a->S < 2) return -1;
  dim3 grid((unsigned)((n / 4 + 255) / 256), a->ngroups);
  hipLaunchKernelGGL(wgrad_reduce_kernel, grid, dim3(256), 0, stream, *a);
  return (int)hipGetLastError();
}

static int g_wgrad_nb = 0;   // 0: per-shape default, 1 / 2: force band buffers (gt_wgrad_set_nb, tests)

extern "C" int gt_wgrad_set_nb(int nb) {
  const int old = g_wgrad_nb;
  g_wgrad_nb = nb;
  return old;
}


// Small launches (few groups x splits: a population job of 1-5 groups, the
// reference's sequential folds or a rank's share on 8 GPUs): the k-column
// tiles are sliced over NZ workgroups that stage the same bands, so the
// grid fills more CUs and each workgroup's serial band loop carries 1/NZ of
// the MFMAs. Every weight's sum runs in the same band / k-step order in any
// slice: results are bit-identical for any NZ (tests/test_hip_kernels.py).
// gt_wgrad_set_nz (tests): 0 auto (default), 1 / 2 / 4 / 8 forced (8: 4-wave workgroups).
static int g_wgrad_nz = 0;

extern "C" int gt_wgrad_set_nz(int nz) {
  const int old = g_wgrad_nz;
  g_wgrad_nz = nz;
  return old;
}

static int wgrad_nz(const WgradArgs* a) {
  const int force = g_wgrad_nz;
  if (force == 1 || force == 2 || force == 4 || force == 8) return force;
  // (an 8-slice variant below ~32 blocks measured neutral at 2 groups: profiles/wgrad_nz8_ab_r4.txt)
  const int blocks = a->S * a->ngroups;
  return blocks < 64 ? 4 : blocks < 160 ? 2 : 1;
}


// band rows of the specialised wgrad per precision (the host sizes the split
// in whole bands: pps multiple of R*W); 0 = generic kernel
extern "C" int gt_wgrad_rows_ext(int KH, int KW, int Cinp, int Coutp, int H, int W, int prec);
extern "C" int gt_wgrad_nb_force() { return g_wgrad_nb; }
extern "C" int gt_wgrad_nz_of(const WgradArgs* a) { return wgrad_nz(a); }

static int wgrad_rows(int KH, int KW, int Cinp, int Coutp, int H, int W, int prec) {
  if (prec == 1) {
    if (KH == 5 && KW == 5 && Cinp == 8 && Coutp == 24 && W == 32 && H % 8 == 0) return 8;
    if (KH == 3 && KW == 3 && Cinp == 24 && Coutp == 24 && W == 32 && H % 4 == 0) return 4;
    if (KH == 5 && KW == 5 && Cinp == 24 && Coutp == 56 && W == 16 && H % 4 == 0) return 4;
    if (KH == 3 && KW == 3 && Cinp == 56 && Coutp == 56 && W == 16 && H % 4 == 0) return 4;
    if (KH == 5 && KW == 5 && Cinp == 56 && Coutp == 104 && W == 8 && H % 4 == 0) return 4;    // deep s3
    if (KH == 3 && KW == 3 && Cinp == 104 && Coutp == 104 && W == 8 && H % 4 == 0) return 4;
    // wide deep space
    if (KH == 5 && KW == 5 && Cinp == 8 && Coutp == 64 && W == 32 && H % 4 == 0) return 4;
    if (KH == 3 && KW == 3 && Cinp == 64 && Coutp == 64 && W == 32 && H % 2 == 0) return 2;
    if (KH == 5 && KW == 5 && Cinp == 64 && Coutp == 128 && W == 16 && H % 2 == 0) return 2;
    if (KH == 3 && KW == 3 && Cinp == 128 && Coutp == 128 && W == 16 && H % 2 == 0) return 2;
    if (KH == 5 && KW == 5 && Cinp == 128 && Coutp == 256 && W == 8 && H % 4 == 0) return 4;
    if (KH == 3 && KW == 3 && Cinp == 256 && Coutp == 256 && W == 8 && H % 4 == 0) return 4;
    return gt_wgrad_rows_ext(KH, KW, Cinp, Coutp, H, W, prec);
  }
  if (KH == 5 && KW == 5 && Cinp == 8 && Coutp == 24 && W == 32 && H % 8 == 0) return 8;
  if (KH == 3 && KW == 3 && Cinp == 24 && Coutp == 24 && W == 32 && H % 8 == 0) return 8;
  if (KH == 5 && KW == 5 && Cinp == 24 && Coutp == 56 && W == 16 && H % 16 == 0) return 16;
  if (KH == 3 && KW == 3 && Cinp == 56 && Coutp == 56 && W == 16 && H % 16 == 0) return 16;
  return 0;
}

// pixels per band of the specialised wgrad for this geometry, or 0
extern "C" int gt_wgrad_fast_band(int KH, int KW, int Cinp, int Coutp, int H, int W, int prec) {
  return wgrad_rows(KH, KW, Cinp, Coutp, H, W, prec) * W;
}

// Preferred splits per group (measured, profiles/wgrad_splits.txt): many small
// workgroups for the 32-wide stage (single LDS buffer, 4+ per CU), few large
// ones for the 16-wide stage (double-buffered: 128 KB of LDS, one workgroup per
// CU). 3 splits x 80 groups of a 16-candidate population = 240 workgroups, one
// round on 256 CUs; 4 splits left a 64-workgroup second round (population step
// 2-3 % slower, same-box sweep).
// fp32 (prec 1): the band work is ~6x the bf16 one, and a bench round
// trains only ~10 groups per launch: 8 / 32 splits keep >= 80 / 320
// workgroups busy at 10 groups (3 splits left 30 workgroups on 256 CUs:
// 199 us per call, 34 % of a 10-group step) for 2.7x the partial-sum bytes.
extern "C" int gt_wgrad_fast_splits(int KH, int KW, int Cinp, int Coutp, int H, int W, int prec) {
  (void)KH; (void)KW; (void)Cinp; (void)Coutp; (void)H;
  if (prec == 1) {
    // 8-wide (deep stage 3): 4 splits x 4 column slices per group
    // (12 or 16 splits for the 16-wide stage: 0.4-1.8 % slower steps at 25 and 80 groups,
    // profiles/r5/wgrad_splits_ab_r5.txt)
    return W >= 32 ? 32 : W <= 8 ? 4 : 8;
  }
  return W >= 32 ? 16 : 3;
}

#ifndef GT_KERNELS_ONLY
extern "C" int gt_wgrad_fast(const WgradArgs* a, hipStream_t stream) {
  if (a->prec == 1) {
    WGRAD_FAST_CASE_F32(5, 5, 1, 3, 32, 8, 4, 1)      // s1 input conv (3 -> 20)
    WGRAD_FAST_CASE_F32(3, 3, 3, 3, 32, 4, 4, 1)      // s1 nodes / output conv (20 -> 20)
    // s2: ONE band buffer (57 KB of LDS instead of 115): in the population step the wgrads run beside the
    // data-gradient convs, and a single-buffered wgrad workgroup leaves room on its CU for a conv
    // workgroup (60 KB) -- 1.1-1.6 % per step from 25 groups up although the wgrad alone is slower
    // (profiles/wgrad_nb_ab_r4.txt)
    WGRAD_FAST_CASE_F32(5, 5, 3, 7, 16, 4, 8, 1)      // s2 input conv (20 -> 50)
    WGRAD_FAST_CASE_F32(3, 3, 7, 7, 16, 4, 8, 1)      // s2 nodes / output conv (50 -> 50)
    WGRAD_FAST_CASE_F32Z(5, 5, 7, 13, 8, 4, 8, 4)     // deep s3 input conv (50 -> 100)
    WGRAD_FAST_CASE_F32Z(3, 3, 13, 13, 8, 4, 8, 4)    // deep s3 nodes / output conv (100 -> 100)
    // wide deep space (64, 128, 256): column slices so each workgroup's dW slice fits its registers
    WGRAD_FAST_CASE_F32(5, 5, 1, 8, 32, 4, 4, 1)      // s1 input conv (3 -> 64)
    WGRAD_FAST_CASE_F32(3, 3, 8, 8, 32, 2, 8, 1)      // s1 nodes / output conv (64 -> 64)
    WGRAD_FAST_CASE_F32Z(5, 5, 8, 16, 16, 2, 8, 7)    // s2 input conv (64 -> 128)
    WGRAD_FAST_CASE_F32Z(3, 3, 16, 16, 16, 2, 8, 4)   // s2 nodes / output conv (128 -> 128)
    WGRAD_FAST_CASE_F32Z(5, 5, 16, 32, 8, 4, 8, 13)   // s3 input conv (128 -> 256)
    WGRAD_FAST_CASE_F32Z(3, 3, 32, 32, 8, 4, 8, 10)   // s3 nodes / output conv (256 -> 256)
    {   // user-chosen architectures (cnn_conv_fast_ext.hip)
      const int rc = gt_wgrad_fast_ext(a, stream);
      if (rc != -100) return rc;
    }
    return -100;
  }
  if (a->prec != 0) return -1;
  WGRAD_FAST_CASE(5, 5, 1, 3, 32, 8, 4, 1)      // s1 input conv (3 -> 20)
  WGRAD_FAST_CASE(3, 3, 3, 3, 32, 8, 4, 1)      // s1 nodes / output conv (20 -> 20)
  WGRAD_FAST_CASE(5, 5, 3, 7, 16, 16, 8, 2)     // s2 input conv (20 -> 50)
  WGRAD_FAST_CASE(3, 3, 7, 7, 16, 16, 8, 2)     // s2 nodes / output conv (50 -> 50)
  return -100;
}
#endif  // GT_KERNELS_ONLY

// ===========================================================================
// Fragment-major weight planes of the shape-specialised convs (ConvArgs::wfrag)
// ===========================================================================
// Entry e of a conv's reduction list -> its row-major chunk (kk * NCBI + cb), as the kernels order it
// (part-major for the stage-2 3x3 fp32 shape, S2Parts; kk-major otherwise); -1 past the list.
extern "C" int gt_conv_frag_order(int KH, int KW, int NCBI, int W, int prec, int* out, int n) {
  const int NCH = KH * KW * NCBI;
  const bool parts = prec == 1 && NCBI == 7 && W == 16 && KH == 3 && KW == 3;
  for (int e = 0; e < n; ++e) {
    int kk, cb;
    if (e >= NCH) { out[e] = -1; continue; }
    if (parts) {
      const int E0 = KH * KW * 4;
      if (e < E0) { kk = e >> 2; cb = e & 3; }
      else { const int e1 = e - E0; kk = e1 / 3; cb = 4 + e1 - kk * 3; }
    } else {
      kk = e / NCBI; cb = e - kk * NCBI;
    }
    out[e] = kk * NCBI + cb;
  }
  return (NCH + 3) / 4;
}

struct FragSeg {
  const float* w;        // fp32 master [Q][Cop][KH][KW][Cip] of the layer
  uint16_t* dst;         // [npl][Q][NT][NKS][64][8] bf16 planes
  const int* order;      // [NKS * 4]: row-major chunk of each entry in the conv's view, -1 = zero
  long ps;               // plane stride (elements)
  int Q, Cop, Cip, KH, KW;
  int NT, NKS, NCBIc;    // the conv's co tiles, k-steps, input chunks (layer Cip / 8, or Cop / 8 for dgrad)
  int dgrad;             // 1: the flipped / transposed kernel of the data gradient
  int npl;               // 3 (fp32: exact split) or 1 (bf16)
};

struct FragArgs {
  const FragSeg* segs;
  const int2* blocks;    // per block: (segment, first lane-item of Q x NT x NKS x 64)
};

__global__ void __launch_bounds__(256) conv_wfrag_kernel(FragArgs a) {
  const int2 blk = a.blocks[blockIdx.x];
  const FragSeg s = a.segs[blk.x];
  const long item = (long)blk.y + threadIdx.x;
  if (item >= (long)s.Q * s.NT * s.NKS * 64) return;
  const int lane = (int)(item & 63);
  long r = item >> 6;
  const int ks = (int)(r % s.NKS); r /= s.NKS;
  const int t = (int)(r % s.NT);
  const int q = (int)(r / s.NT);
  const int row = t * 16 + (lane & 15), e = ks * 4 + (lane >> 4);
  const int nat = s.order[e];
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = 0.f;
  if (nat >= 0) {
    const int kk = nat / s.NCBIc, cb = nat - kk * s.NCBIc;
    const int kh = kk / s.KW, kw = kk - kh * s.KW;
    if (!s.dgrad && row < s.Cop) {
      const float* src = s.w + ((((long)q * s.Cop + row) * s.KH + kh) * s.KW + kw) * s.Cip + cb * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = src[j];
    } else if (s.dgrad && row < s.Cip) {
      // the data gradient's row = layer input channel, its chunk cb = layer output channels cb*8.., flipped taps
      const int khl = s.KH - 1 - kh, kwl = s.KW - 1 - kw;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        v[j] = s.w[((((long)q * s.Cop + cb * 8 + j) * s.KH + khl) * s.KW + kwl) * s.Cip + row];
    }
  }
  uint16_t* d = s.dst + item * 8;
  if (s.npl == 1) {
    *reinterpret_cast<uint4*>(d) = pack8(v);
    return;
  }
  uint4 p0, p1, p2;
  split8(v, p0, p1, p2);
  *reinterpret_cast<uint4*>(d) = p0;
  *reinterpret_cast<uint4*>(d + s.ps) = p1;
  *reinterpret_cast<uint4*>(d + 2 * s.ps) = p2;
}

extern "C" int gt_conv_wfrag(const void* av, int nblocks, hipStream_t stream) {
  if (nblocks < 1) return 0;
  hipLaunchKernelGGL(conv_wfrag_kernel, dim3(nblocks), dim3(256), 0, stream, *static_cast<const FragArgs*>(av));
  return (int)hipGetLastError();
}

extern "C" size_t gt_sizeof_frag_seg() { return sizeof(FragSeg); }
