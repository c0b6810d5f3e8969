// Shape-specialised implicit-GEMM convolution (forward and data-gradient)
// for the layer shapes of a Genetic-CNN search space on MI355X (gfx950).
//
// Why: the generic conv_fwd_kernel (cnn_conv.hip) computes every address at
// run time and walks dependent global round trips per workgroup; on the
// population-batched launches (Q = candidates x folds groups) PMC counters
// showed ~680 VALU instructions and 55 % of wave time in s_waitcnt per 28
// MFMAs. Here the geometry (kernel KHxKW, input chunks NCBI = Cin/8, image
// width W, tile rows TH, output 16-channel tiles NT) is a template, so:
//   * the input patch ((TH+KH-1) x (W+KW-1) x Cin, zero halo) is staged into
//     LDS with ALL of a thread's global loads issued before its first LDS
//     store (compile-time trip count, mul-shift index math), the DAG's N-ary
//     Add and the batch gather fused in;
//   * weights (MFMA A operand, 16 B per lane) stream from global / L2 straight
//     into registers, prefetched 4 k-steps ahead -- no LDS, no barriers in the
//     k loop; all four waves of a workgroup read the same rows (L1 hits);
//   * the B operand (pixels) is one ds_read_b128 per 16-pixel group and
//     k-step at  lane base + per-k-step chunk offset (LDS table, one add)
//     + compile-time group offset (instruction immediate);
//   * a wave owns CT (<= 2) output-channel tiles x PG pixel groups: 16 MFMA
//     (v_mfma_f32_16x16x32_bf16) per k-step for every 2 + PG LDS/global reads.
// Tile = TH*W = 256 pixels of one image of one group; workgroups are
// XCD-swizzled so the workgroups of one group share an XCD's L2 (weights).
// Epilogue = generic kernel's: bias + ReLU (forward) or per-group DAG
// fan-out (accumulate, ReLU mask) for the data gradient.

#include "cnn_args.h"

template <int KH, int KW, int NCBI, int W, int TH, int NT>
__global__ void __launch_bounds__(256) conv_fast_kernel(ConvArgs a) {
  constexpr int PH = TH + KH - 1, PW = W + KW - 1;
  constexpr int NP = PH * PW * NCBI;                // patch chunks (16 B)
  constexpr int NPT = (NP + 255) / 256;             // patch chunks per thread
  constexpr int NCH = KH * KW * NCBI;               // reduction chunks
  constexpr int NKS = (NCH + 3) / 4;                // k-steps (32 k each)
  constexpr int TP = TH * W;                        // tile pixels
  constexpr int NPG = TP / 16;                      // pixel groups
  constexpr int CT = NT >= 2 ? 2 : 1;               // co tiles per wave
  constexpr int WC = NT / CT;                       // waves along co
  constexpr int WP = 4 / WC;                        // waves along pixels
  constexpr int PG = NPG / WP;                      // pixel groups per wave
  constexpr int PF = NKS < 4 ? NKS : 4;             // weight prefetch depth (k-steps)
  static_assert(NPG % WP == 0 && NT % CT == 0 && WC * WP == 4, "tile shape");
  static_assert(W % 16 == 0 || 16 % W == 0, "pixel groups must tile image rows");

  __shared__ __attribute__((aligned(16))) uint4 patch[NP];
  __shared__ int coff[NKS * 4];

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, kq = lane >> 4, l16 = lane & 15;
  // XCD-aware order: hardware places consecutive workgroups on consecutive
  // XCDs; give each XCD a contiguous range of (group, image, band) tiles
  const int nbx = gridDim.x;
  const int total = nbx * gridDim.y;
  int lin = blockIdx.y * nbx + blockIdx.x;
  if ((total & 7) == 0) lin = (lin & 7) * (total >> 3) + (lin >> 3);
  const int by = lin / nbx, bx = lin - by * nbx;
  const int nband = (a.H + TH - 1) / TH;
  const int b = bx / nband;
  const int h0 = (bx - b * nband) * TH;
  const GroupRec gr = group_rec(a.gtab, by, a.n_in, a.n_out, a.acc_flags, a.out_mask);
  const int g = gr.g;
  const long img = (long)a.H * W * NCBI * 8;

  // ---- weights: first PF k-steps in flight before the patch ---------------
  const int wco = (wave % WC) * CT;                 // first co tile of this wave
  const int pgw = (wave / WC) * PG;                 // first pixel group of this wave
  const uint16_t* wrow[CT];
  bool wok[CT];
#pragma unroll
  for (int t = 0; t < CT; ++t) {
    const int co = (wco + t) * 16 + l16;
    wok[t] = co < a.Coutp;
    wrow[t] = a.w + ((long)g * a.Coutp + (wok[t] ? co : 0)) * (NCH * 8);
  }
  uint4 areg[PF][CT];
  auto load_a = [&](int s, uint4* dst) {
    const int c = s * 4 + kq;
#pragma unroll
    for (int t = 0; t < CT; ++t)
      dst[t] = (wok[t] && c < NCH) ? *reinterpret_cast<const uint4*>(wrow[t] + c * 8) : make_uint4(0, 0, 0, 0);
  };
#pragma unroll
  for (int s = 0; s < PF; ++s) load_a(s, areg[s]);

  // ---- patch: summed inputs (or gathered dataset image), zero halo --------
  const uint16_t* src[GT_MAXSLOT];
  int n_src = 0;
#pragma unroll
  for (int k = 0; k < GT_MAXSLOT; ++k)
    if ((gr.in_mask >> k) & 1) src[n_src++] = a.in[k] + ((long)g * a.B + b) * img;
  if (a.gather) {
    const long id = a.gather[((long)a.st->cur_step * a.G + g) * a.B + b];
    src[0] = a.in[0] + id * img;
    n_src = 1;
  }
  long poff[NPT];
  bool pok[NPT];
#pragma unroll
  for (int j = 0; j < NPT; ++j) {
    const int i = tid + 256 * j;
    const int cb = i % NCBI, pix = i / NCBI;
    const int pr = pix / PW, pc = pix % PW;
    const int hh = h0 - KH / 2 + pr, ww = pc - KW / 2;
    pok[j] = i < NP && hh >= 0 && hh < a.H && ww >= 0 && ww < W;
    poff[j] = ((long)hh * W + ww) * (NCBI * 8) + cb * 8;
  }
  if (n_src == 1) {
    uint4 v[NPT];
#pragma unroll
    for (int j = 0; j < NPT; ++j)
      v[j] = pok[j] ? *reinterpret_cast<const uint4*>(src[0] + poff[j]) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < NPT; ++j)
      if (tid + 256 * j < NP) patch[tid + 256 * j] = v[j];
  } else {
#pragma unroll
    for (int j = 0; j < NPT; ++j) {
      if (tid + 256 * j >= NP) continue;
      float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, t8[8];
      if (pok[j]) {
        for (int k = 0; k < n_src; ++k) {
          unpack8(*reinterpret_cast<const uint4*>(src[k] + poff[j]), t8);
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[e] += t8[e];
        }
      }
      patch[tid + 256 * j] = pack8(acc);
    }
  }
  // chunk c -> patch offset of its (kh, kw, cb) relative to the output pixel
  for (int c = tid; c < NKS * 4; c += 256) {
    const int kk = c / NCBI, cb = c % NCBI;
    coff[c] = c < NCH ? ((kk / KW) * PW + (kk % KW)) * NCBI + cb : 0;
  }
  // bias of this lane's output channels (forward only)
  float bias_v[CT][4];
#pragma unroll
  for (int t = 0; t < CT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int co = (wco + t) * 16 + kq * 4 + i;
      bias_v[t][i] = (a.bias && co < a.Coutp) ? a.bias[(long)g * a.Coutp + co] : 0.f;
    }
  __syncthreads();

  // ---- MFMA main loop ------------------------------------------------------
  // lane's pixel within a group: (l16 / W) rows down, l16 % W across (W >= 16: same row)
  const int lbase = ((l16 / W) * PW + (l16 % W)) * NCBI;
  int gbase;
  {
    const int p = pgw * 16;
    gbase = ((p / W) * PW + (p % W)) * NCBI;
  }
  f32x4_t acc[CT][PG];
#pragma unroll
  for (int t = 0; t < CT; ++t)
#pragma unroll
    for (int h = 0; h < PG; ++h) acc[t][h] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < NKS; ++s) {
    const uint4* pb = patch + lbase + gbase + coff[s * 4 + kq];
    uint4 bfr[PG];
#pragma unroll
    for (int h = 0; h < PG; ++h) {
      const int p = h * 16;                        // relative to the wave's first group
      bfr[h] = pb[((p / W) * PW + (p % W)) * NCBI];
    }
    uint4 acur[CT];
#pragma unroll
    for (int t = 0; t < CT; ++t) acur[t] = areg[s % PF][t];
    if (s + PF < NKS) load_a(s + PF, areg[s % PF]);
#pragma unroll
    for (int t = 0; t < CT; ++t)
#pragma unroll
      for (int h = 0; h < PG; ++h) acc[t][h] = mfma16(acur[t], bfr[h], acc[t][h]);
  }

  // ---- epilogue --------------------------------------------------------------
#pragma unroll
  for (int h = 0; h < PG; ++h) {
    const int p = (pgw + h) * 16 + l16;
    const int y = h0 + p / W, x = p % W;
    if (y >= a.H) continue;
    const long obase = ((((long)g * a.B + b) * a.H + y) * W + x) * a.Coutp;
#pragma unroll
    for (int t = 0; t < CT; ++t) {
      const int co0 = (wco + t) * 16 + kq * 4;
      if (co0 >= a.Coutp) continue;
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float xv = acc[t][h][i] + bias_v[t][i];
        if (a.relu) xv = fmaxf(xv, 0.f);
        v[i] = xv;
      }
      for (int k = 0; k < GT_MAXSLOT; ++k) {
        if (!((gr.out_mask >> k) & 1)) continue;
        uint2* dst = reinterpret_cast<uint2*>(a.out[k] + obase + co0);
        float sum[4] = {v[0], v[1], v[2], v[3]};
        if ((gr.out_mask >> (8 + k)) & 1) {
          const uint2 old = *dst;
          sum[0] += __uint_as_float(old.x << 16); sum[1] += __uint_as_float(old.x & 0xffff0000u);
          sum[2] += __uint_as_float(old.y << 16); sum[3] += __uint_as_float(old.y & 0xffff0000u);
        }
        if ((gr.out_mask >> (16 + k)) & 1) {
          const uint2 m = *reinterpret_cast<const uint2*>(a.out_mask[k] + obase + co0);
          const uint32_t mw[4] = {m.x & 0xffffu, m.x >> 16, m.y & 0xffffu, m.y >> 16};
#pragma unroll
          for (int i = 0; i < 4; ++i) sum[i] = (mw[i] != 0u && mw[i] < 0x8000u) ? sum[i] : 0.f;
        }
        *dst = pack4(sum);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// dispatch: (KH, KW, Cinp, W, Coutp-tiles) -> instantiation; -100 = no match
// (the caller then uses the generic kernel)
// ---------------------------------------------------------------------------

#define CONV_FAST_CASE(KH_, KW_, NCBI_, W_, TH_, NT_)                                                   \
  if (a->KH == KH_ && a->KW == KW_ && a->Cinp == NCBI_ * 8 && a->W == W_ && nt == NT_ && a->H % TH_ == 0) { \
    dim3 grid(a->B * (a->H / TH_), a->ngroups);                                                         \
    hipLaunchKernelGGL((conv_fast_kernel<KH_, KW_, NCBI_, W_, TH_, NT_>), grid, dim3(256), 0, stream, *a); \
    return (int)hipGetLastError();                                                                      \
  }

extern "C" int gt_conv_fast(const ConvArgs* a, hipStream_t stream) {
  if (a->mask) return -100;                  // staged ReLU mask: generic kernel only
  const int nt = (a->Coutp + 15) / 16;
  // Genetic-CNN CIFAR-shaped S=(3,5) space, kernels (20, 50), 5x5 stage convs
  CONV_FAST_CASE(5, 5, 1, 32, 8, 2)          // s1 input conv (3 -> 20)
  CONV_FAST_CASE(3, 3, 3, 32, 8, 2)          // s1 nodes / output conv, and their dgrad (20 -> 20)
  CONV_FAST_CASE(5, 5, 3, 16, 16, 4)         // s2 input conv (20 -> 50)
  CONV_FAST_CASE(3, 3, 7, 16, 16, 4)         // s2 nodes / output conv, and their dgrad (50 -> 50)
  CONV_FAST_CASE(5, 5, 7, 16, 16, 2)         // s2 input conv dgrad (50 -> 20)
  return -100;
}
