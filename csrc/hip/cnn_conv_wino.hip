// Winograd F(2x2, 3x3) fp32 convolution (forward and data gradient) for the
// 3x3 / stride-1 / 'same' layers of a Genetic-CNN search space on MI355X
// (gfx950): the DAG node convs and the stage output convs, whose direct
// implicit GEMM (cnn_conv_fast.hip) took half the fp32 population step at
// 32-34 % MFMA busy.
//
// Algorithm (Lavin & Gray, "Fast Algorithms for Convolutional Neural
// Networks", 2016): every 2x2 output tile y of a channel is
//   y = A^T [ sum_ci (G g G^T) (.) (B^T d B) ] A
// over the tile's 4x4 input patch d, so the 36 multiplies per tile and
// channel pair of the direct conv become 16: per transform index xi (4x4)
// one GEMM  M[xi][co][tile] = sum_ci U[xi][co][ci] V[xi][ci][tile].
// On the matrix cores that is 2x fewer v_mfma_f32_16x16x32_bf16 for the
// stage-2 shape (the reduction is ci only: 56 -> 64 padded, vs 63 -> 64
// chunks of (kh, kw, ci) for the direct conv). fp32 precision as everywhere
// (common.h): U and V are fp32 values split exactly into three bf16 planes,
// six MFMA terms per product; the transforms themselves run in fp32 (B^T
// and A^T are +-1 adds, G has 1/2 factors), so the error is fp32-level
// (tests/test_hip_wino.py: fp64 oracle next to torch fp32).
//
// Data flow of one workgroup (group g, image b, band of TH output rows =
// TH/2 x W/2 tiles):
//   1. the input patch ((TH+2) x (W+2) x Cin, zero halo; the DAG's N-ary Add
//      and the batch gather fused as in cnn_conv_fast.hip) is staged into
//      LDS as fp32 -- one plane, 4 bytes per value instead of three bf16
//      planes (6 bytes);
//   2. per xi (16 phases, one barrier each): every thread owns one (tile,
//      8-channel chunk) item and computes V[xi] of it from the row transform
//      T = B^T d of its xi-row (8 patch reads per xi-row, kept in registers),
//      splits it and writes the three planes into a double-buffered LDS
//      V tile; in the same phase every wave runs the MFMAs of the previous
//      xi on the other buffer (B = V from LDS, conflict-free ds_read_b128:
//      16 consecutive tiles per 8-channel chunk) with A = U fragments
//      streamed from global / L2 into registers one xi ahead;
//   3. each xi's 16x16 accumulator is folded into the 2x2 output tile right
//      away (A^T M A is +-1 adds, fixed xi order: the summation order of
//      every output is independent of the tile height and of the groups in
//      the launch -- batch invariance holds);
//   4. register epilogue: bias + ReLU (forward), the zero-padded-image
//      zeros, the DAG fan-out (write / accumulate / ReLU mask per slot), and
//      the fused 2x2 max-pool, which is lane-local here (a lane holds a whole
//      2x2 output tile) -- or the fused un-pool of a pool's gradient.
//
// The transformed weights U (and the U of the flipped, transposed kernel the
// data gradient convolves with) are written by gt_wino_wtrans from the fp32
// master weights once per optimizer step: planes [3][G][16][R][K] bf16,
// R = output channels padded to 16, K = input channels padded to 32, stored
// fragment-major (each 16 x 32 MFMA A fragment one contiguous KB in lane
// order; cnn_kernels.wino_unpack gives the logical layout).

#include <algorithm>

#include "cnn_args.h"

// B^T (input transform) rows: row i has two +-1 entries, at columns wbt_a(i) and wbt_b(i)
//   i = 0: d0 - d2   i = 1: d1 + d2   i = 2: d2 - d1   i = 3: d1 - d3
__host__ __device__ constexpr int wbt_a(int i) { return i == 0 ? 0 : 1; }
__host__ __device__ constexpr int wbt_b(int i) { return i == 3 ? 3 : 2; }
__host__ __device__ constexpr bool wbt_na(int i) { return i == 2; }              // entry a is -1
__host__ __device__ constexpr bool wbt_nb(int i) { return i == 0 || i == 3; }    // entry b is -1
// A^T (output transform) [r][i]: r = 0: (1, 1, 1, 0); r = 1: (0, 1, -1, -1)
__host__ __device__ constexpr int wat(int r, int i) { return r == 0 ? (i < 3 ? 1 : 0) : (i == 0 ? 0 : (i == 1 ? 1 : -1)); }

__device__ __forceinline__ float wbt_row(int i, float da, float db) {
  // d[a] * (+-1) + d[b] * (+-1), exact sign handling (no multiplies)
  const float x = wbt_na(i) ? -da : da;
  return wbt_nb(i) ? x - db : x + db;
}

template <int NCBI, int NT, int W, int TH>
struct WinoCfg {
  static constexpr int PH = TH + 2, PW = W + 2;
  static constexpr int NP = PH * PW * NCBI;          // patch chunks (8 fp32 each)
  static constexpr int TW = W / 2, NTL = (TH / 2) * TW, NTG = NTL / 16;   // tiles, 16-tile groups
  static constexpr int NKS = (NCBI + 3) / 4, NKC = NKS * 4;              // k-steps, chunk slots
  static constexpr int NVI = NTL * NKC;               // V items (tile, chunk slot) per xi
  static constexpr int NWV = 4, NTH = NWV * 64;
  static constexpr int WC = NT < NWV ? NT : NWV;      // waves along co
  static constexpr int WP = NWV / WC;                 // waves along tile groups
  static constexpr int CT = NT / WC, PGW = NTG / WP;  // co tiles / tile groups per wave
  static constexpr int NIT = (NVI + NTH - 1) / NTH;   // V items per thread
  // patch, two V buffers, 3 x 64 dummy rows (branch-free stores of threads without an item)
  static size_t lds() { return (size_t)NP * 32 + (size_t)2 * 3 * NKC * NTL * 16 + 3 * 64 * 16; }
};

template <int NCBI, int NT, int W, int TH>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
conv_wino_kernel(ConvArgs a) {
  using C = WinoCfg<NCBI, NT, W, TH>;
  constexpr int NTH = C::NTH, PW = C::PW, NP = C::NP, TW = C::TW, NTL = C::NTL;
  constexpr int NKS = C::NKS, NKC = C::NKC, NVI = C::NVI, NIT = C::NIT;
  constexpr int WC = C::WC, CT = C::CT, PGW = C::PGW;
  constexpr int R = NT * 16, K = NKC * 8;            // U rows / columns
  constexpr int NPT = (NP + NTH - 1) / NTH;           // patch chunks per thread
  static_assert(W % 2 == 0 && TH % 2 == 0 && NTL % 16 == 0, "whole 16-tile groups");
  static_assert(NT % WC == 0 && C::NTG % C::WP == 0, "tile split");

  extern __shared__ __attribute__((aligned(16))) uint4 smem[];
  float4* patch = reinterpret_cast<float4*>(smem);               // [NP][2] float4
  uint4* vbuf = smem + NP * 2;                                    // [2 buf][3 planes][NKC][NTL]

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, kq = lane >> 4, l16 = lane & 15;
  // XCD-aware order (as cnn_conv_fast.hip): each XCD gets a contiguous range of (group, image, band)
  const int nbx = gridDim.x, total = nbx * gridDim.y;
  int lin = blockIdx.y * nbx + blockIdx.x;
  if ((total & 7) == 0) lin = (lin & 7) * (total >> 3) + (lin >> 3);
  const int by = lin / nbx, bx = lin - by * nbx;
  const int nband = a.H / TH;
  const int b = bx / nband, h0 = (bx - b * nband) * TH;
  const GroupRec gr = group_rec(a.gtab, by, a.n_in, a.n_out, a.acc_flags, a.out_mask);
  const int g = gr.g;
  const long img = (long)a.H * W * NCBI * 8;
  if (a.dbg & 64) return;                              // (dbg bit 64, diagnostics only: empty workgroup)

  // ---- U fragments (A operand): lane = row l16 of co tile, 8 k of chunk slot ks*4 + kq -------------
  // buffer loads: one descriptor over the group's planes (wave-uniform base), the lane's constant
  // byte offset in voffset, (xi, k-step, plane) as the scalar offset -- no 64-bit address math per load
  const int wco = (wave % WC) * CT;                    // first co tile of this wave
  const int tgw = (wave / WC) * PGW;                   // first tile group of this wave
  const int gu = __builtin_amdgcn_readfirstlane(g);
  const __amdgpu_buffer_rsrc_t ursrc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.w + (long)gu * 16 * R * K), (short)0, (int)(((2 * a.wps) + 16L * R * K) * 2), 0x00020000);
  // fragment-major U (gt_wino_wtrans): the 16 rows x 32 k of one (xi, co tile, k-step, plane) are ONE
  // contiguous KB in lane order, so a wave's fragment load fills 8 whole 128-byte lines (row-major U
  // used half of 16 lines per load: the L1 line rate, not the MFMAs, paced the first build)
  const int uoff = lane * 16 + wco * NKS * 1024;
  const int ups2 = __builtin_amdgcn_readfirstlane((int)(a.wps * 2));
  uint4 areg[2][NKS][CT][3];
  auto load_a = [&](int x, uint4 (*dst)[CT][3]) {
    if (a.dbg & 16) x = 0;                             // (dbg bit 16, diagnostics only: every xi reads xi 0's U)
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
          const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(
              ursrc, uoff + (ct * NKS + ks) * 1024, p * ups2 + x * R * K * 2, 0);
          dst[ks][ct][p] = make_uint4(v.x, v.y, v.z, v.w);
        }
  };
  load_a(0, areg[0]);

  // ---- patch (fp32): summed DAG inputs or the gathered dataset image, zero halo ---------------------
  const long gimg = ((long)g * a.B + b) * img;
  const int n_src = a.gather ? 1 : __builtin_popcount(gr.in_mask);
  const float* src0 = a.gather ? static_cast<const float*>(a.in[0]) + a.gather[((long)a.st->cur_step * a.G + g) * a.B + b] * img
                               : static_cast<const float*>(a.in[__builtin_ctz(gr.in_mask | 0x100) & 7]) + gimg;
  {
    long poff[NPT];
    bool pok[NPT];
#pragma unroll
    for (int j = 0; j < NPT; ++j) {
      const int i = tid + NTH * j;
      const int cb = i % NCBI, pix = i / NCBI;
      const int pr = pix / PW, pc = pix % PW;
      const int hh = h0 - 1 + pr, ww = pc - 1;
      pok[j] = i < NP && hh >= 0 && hh < a.H && ww >= 0 && ww < W;
      poff[j] = ((long)hh * W + ww) * (NCBI * 8) + cb * 8;
    }
    constexpr int JB = NPT < 5 ? NPT : 5;
#pragma unroll
    for (int j0 = 0; j0 < NPT; j0 += JB) {
      float acc8[JB][8];
#pragma unroll
      for (int j = 0; j < JB; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc8[j][e] = 0.f;
      if (a.dbg & 32) {                              // (dbg bit 32, diagnostics only: no patch loads)
      } else if (n_src == 1) {
#pragma unroll
        for (int j = 0; j < JB; ++j)
          if (j0 + j < NPT && pok[j0 + j]) load8f(src0 + poff[j0 + j], acc8[j]);
      } else {
        // DAG inputs two at a time, summed in increasing slot order (bit-identical to the direct kernels)
        int m = gr.in_mask & 0xff;
        while (m) {
          const int k0 = __builtin_ctz(m);
          m &= m - 1;
          const bool two = m != 0;
          const int k1 = two ? __builtin_ctz(m) : k0;
          if (two) m &= m - 1;
          const float* s0 = static_cast<const float*>(a.in[k0]) + gimg;
          const float* s1 = static_cast<const float*>(a.in[k1]) + gimg;
          float t0[JB][8], t1[JB][8];
#pragma unroll
          for (int j = 0; j < JB; ++j) {
#pragma unroll
            for (int e = 0; e < 8; ++e) t0[j][e] = t1[j][e] = 0.f;
            if (j0 + j < NPT && pok[j0 + j]) {
              load8f(s0 + poff[j0 + j], t0[j]);
              if (two) load8f(s1 + poff[j0 + j], t1[j]);
            }
          }
#pragma unroll
          for (int j = 0; j < JB; ++j)
#pragma unroll
            for (int e = 0; e < 8; ++e) acc8[j][e] += t0[j][e];
          if (two) {
#pragma unroll
            for (int j = 0; j < JB; ++j)
#pragma unroll
              for (int e = 0; e < 8; ++e) acc8[j][e] += t1[j][e];
          }
        }
      }
#pragma unroll
      for (int j = 0; j < JB; ++j) {
        const int i = tid + NTH * (j0 + j);
        if (j0 + j >= NPT || i >= NP) continue;
        patch[2 * i] = make_float4(acc8[j][0], acc8[j][1], acc8[j][2], acc8[j][3]);
        patch[2 * i + 1] = make_float4(acc8[j][4], acc8[j][5], acc8[j][6], acc8[j][7]);
      }
    }
  }
  // chunk slots beyond the real input chunks are zero in both V buffers (written once)
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int i = tid + NTH * it;
    if (i < NVI && i / NTL >= NCBI)
#pragma unroll
      for (int q = 0; q < 6; ++q) vbuf[(q * NKC + i / NTL) * NTL + i % NTL] = make_uint4(0, 0, 0, 0);
  }
  load_a(1, areg[1]);
  __syncthreads();
  if (a.xsum && n_src > 1) {
    // the summed input of this band (patch interior) for the layer's wgrad: the exact fp32 sum
    float* xo = static_cast<float*>(a.xsum) + gimg + (long)h0 * W * NCBI * 8;
    for (int i = tid; i < TH * W * NCBI; i += NTH) {
      const int cb = i % NCBI, pix = i / NCBI;
      const int r = pix / W, c = pix % W;
      const int pi = ((r + 1) * PW + c + 1) * NCBI + cb;
      *reinterpret_cast<float4*>(xo + (long)i * 8) = patch[2 * pi];
      *reinterpret_cast<float4*>(xo + (long)i * 8 + 4) = patch[2 * pi + 1];
    }
  }

  // ---- V items of this thread: (tile vt, chunk slot vc), row transform T = B^T d of the current xi-row --
  // Branch-free (a branch around the split keeps hipcc from interleaving it with the MFMAs): threads
  // without a real item (chunk slots past the input channels, or past the item count) compute on a
  // clamped item and store into a dummy LDS row
  uint4* vdummy = vbuf + 2 * 3 * NKC * NTL;            // [3][64] scratch rows
  float T[NIT][4][8];
  auto row_transform = [&](int i) {
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int v = min(tid + NTH * it, NVI - 1);
      const int vc = min(v / NTL, NCBI - 1), vt = v % NTL;
      const int ty = vt / TW, tx = vt % TW;
      const float4* pa = patch + 2 * (((2 * ty + wbt_a(i)) * PW + 2 * tx) * NCBI + vc);
      const float4* pb = patch + 2 * (((2 * ty + wbt_b(i)) * PW + 2 * tx) * NCBI + vc);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float4 a0 = pa[2 * c * NCBI], a1 = pa[2 * c * NCBI + 1];
        const float4 b0 = pb[2 * c * NCBI], b1 = pb[2 * c * NCBI + 1];
        const float da[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
        const float db[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) T[it][c][e] = wbt_row(i, da[e], db[e]);
      }
    }
  };
  uint4* vdst[NIT];
  int vpl[NIT];                                        // plane stride of the item's destination (uint4)
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int v = tid + NTH * it;
    const bool real = v < NVI && v / NTL < NCBI;
    vdst[it] = real ? vbuf + (v / NTL) * NTL + v % NTL : vdummy + lane;
    vpl[it] = real ? NKC * NTL : 64;
  }
  auto make_v = [&](int j, int buf) {
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      float f[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = wbt_row(j, T[it][wbt_a(j)][e], T[it][wbt_b(j)][e]);
      uint4 p0, p1, p2;
      split8(f, p0, p1, p2);
      uint4* dst = vdst[it] + (vpl[it] == 64 ? 0 : buf * 3 * NKC * NTL);
      dst[0] = p0;
      dst[vpl[it]] = p1;
      dst[2 * vpl[it]] = p2;
    }
  };

  // ---- main loop over the 16 transform indices ----------------------------------------------------
  float Y[CT][PGW][4][4];                              // [co tile][tile group][2x2 pixel][4 channels]
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int h = 0; h < PGW; ++h)
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e) Y[ct][h][q][e] = 0.f;
  // output transform of one xi, folded into the 2x2 tile: Y[r][c] += A^T[r][i] A^T[c][j] M
  auto fold = [&](int x, const f32x4_t (&M)[CT][PGW]) {
    const int i = x >> 2, j = x & 3;
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int sgn = wat(r, i) * wat(c, j);
        if (sgn == 0) continue;
#pragma unroll
        for (int ct = 0; ct < CT; ++ct)
#pragma unroll
          for (int h = 0; h < PGW; ++h)
#pragma unroll
            for (int e = 0; e < 4; ++e) Y[ct][h][r * 2 + c][e] += sgn > 0 ? M[ct][h][e] : -M[ct][h][e];
      }
  };

  row_transform(0);
  make_v(0, 0);
  __syncthreads();
  if (a.dbg & 128) return;                             // (dbg bit 128, diagnostics only: prologue only)
  f32x4_t Mprev[CT][PGW];
#pragma unroll
  for (int x = 0; x < 16; ++x) {
    const int buf = x & 1;
    // B fragments of this xi (its V was written before the last barrier)
    uint4 bfr[NKS][PGW][3];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
      for (int h = 0; h < PGW; ++h)
#pragma unroll
        for (int p = 0; p < 3; ++p)
          bfr[ks][h][p] = vbuf[((buf * 3 + p) * NKC + ks * 4 + kq) * NTL + (tgw + h) * 16 + l16];
    // V of the next xi into the other buffer (its last reader, xi - 1, finished before the barrier)
    if (x + 1 < 16 && !(a.dbg & 4)) {            // (dbg bit 4, diagnostics only: no V compute)
      if (((x + 1) & 3) == 0) row_transform((x + 1) >> 2);
      make_v((x + 1) & 3, buf ^ 1);
    }
    // the previous xi's accumulators, folded now: their MFMAs have long completed (no hazard stall)
    if (x > 0) fold(x - 1, Mprev);
    // the MFMAs of this xi: six split terms per k-step
    f32x4_t M[CT][PGW];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
      for (int h = 0; h < PGW; ++h) M[ct][h] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    if (!(a.dbg & 1))                              // (dbg bit 1, diagnostics only: no MFMA)
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
#pragma unroll
        for (int h = 0; h < PGW; ++h) M[ct][h] = mfma_np<3>(areg[buf][ks][ct], bfr[ks][h], M[ct][h]);
    // U of xi + 2 into the register slot this xi used
    if (x + 2 < 16) load_a(x + 2, areg[buf]);
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
      for (int h = 0; h < PGW; ++h) Mprev[ct][h] = M[ct][h];
    if (x + 1 < 16 && !(a.dbg & 8)) __syncthreads();   // (dbg bit 8, diagnostics only: no barrier)
  }
  fold(15, Mprev);

  // ---- epilogue: lane = 4 channels (kq*4..) of the 2x2 output tile (tgw + h) * 16 + l16 ------------
  if (a.dbg & 2) return;
  const int COP = a.Coutp;
  const long n = (long)g * a.B + b;
  const bool pool = a.pool_y && ((gr.out_mask >> 24) & 1);
  const bool unpool = (gr.out_mask >> 25) & 1;
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const int co0 = (wco + ct) * 16 + kq * 4;
    if (co0 >= COP) continue;                          // whole float4 inside the padded channel row
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (a.bias) {
      const float4 q = *reinterpret_cast<const float4*>(a.bias + (long)g * COP + co0);
      bv[0] = q.x; bv[1] = q.y; bv[2] = q.z; bv[3] = q.w;
    }
#pragma unroll
    for (int h = 0; h < PGW; ++h) {
      const int t = (tgw + h) * 16 + l16;
      const int ty = t / TW, tx = t % TW;
      float val[4][4];
      long off[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int hh = h0 + 2 * ty + (q >> 1), ww = 2 * tx + (q & 1);
        off[q] = ((n * a.H + hh) * W + ww) * COP + co0;
        const bool pad0 = a.Hr > 0 && !unpool && (hh >= a.Hr || ww >= a.Wr);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = Y[ct][h][q][e] + bv[e];
          if (a.relu) v = fmaxf(v, 0.f);
          val[q][e] = pad0 ? 0.f : v;
        }
      }
      if (unpool) {
        // the output is a pool's gradient: scatter each value to the forward's argmax cell (if > 0)
        float* dst = static_cast<float*>((a.unpool_sel && a.unpool_sel[g]) ? a.unpool_x1 : a.pool_y);
        const int H2 = 2 * a.H, W2 = 2 * W;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t mk = *reinterpret_cast<const uint32_t*>(a.pool_mask + off[q]);
          const int hh = h0 + 2 * ty + (q >> 1), ww = 2 * tx + (q & 1);
#pragma unroll
          for (int me = 0; me < 4; ++me) {
            float o[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const uint32_t bb = (mk >> (8 * e)) & 0xffu;
              o[e] = ((int)(bb & 3u) == me && (bb & 4u)) ? val[q][e] : 0.f;
            }
            *reinterpret_cast<float4*>(dst + ((n * H2 + 2 * hh + (me >> 1)) * W2 + 2 * ww + (me & 1)) * COP + co0) =
                make_float4(o[0], o[1], o[2], o[3]);
          }
        }
      } else {
        for (int k = 0; k < GT_MAXSLOT; ++k) {
          if (!((gr.out_mask >> k) & 1)) continue;
          float* dst = static_cast<float*>(a.out[k]);
          float o[4][4];
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int e = 0; e < 4; ++e) o[q][e] = val[q][e];
          if ((gr.out_mask >> (8 + k)) & 1) {                // accumulate into the slot
            float4 s[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) s[q] = *reinterpret_cast<const float4*>(dst + off[q]);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              o[q][0] += s[q].x; o[q][1] += s[q].y; o[q][2] += s[q].z; o[q][3] += s[q].w;
            }
          }
          if ((gr.out_mask >> (16 + k)) & 1) {               // ReLU mask of the slot's activation
            const float* mp = static_cast<const float*>(a.out_mask[k]);
            float4 s[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) s[q] = *reinterpret_cast<const float4*>(mp + off[q]);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              o[q][0] = s[q].x > 0.f ? o[q][0] : 0.f; o[q][1] = s[q].y > 0.f ? o[q][1] : 0.f;
              o[q][2] = s[q].z > 0.f ? o[q][2] : 0.f; o[q][3] = s[q].w > 0.f ? o[q][3] : 0.f;
            }
          }
#pragma unroll
          for (int q = 0; q < 4; ++q)
            *reinterpret_cast<float4*>(dst + off[q]) = make_float4(o[q][0], o[q][1], o[q][2], o[q][3]);
        }
      }
      if (pool) {
        // 2x2 max-pool + argmax mask of the lane's own tile (pool_fwd_kernel's rule: first strict
        // maximum over (0,0), (0,1), (1,0), (1,1); bit 2 = maximum > 0) from the values as stored
        float m[4];
        uint32_t mk = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float mm = val[0][e];
          int arg = 0;
#pragma unroll
          for (int q = 1; q < 4; ++q)
            if (val[q][e] > mm) { mm = val[q][e]; arg = q; }
          m[e] = mm;
          mk |= (uint32_t)(arg | (mm > 0.f ? 4 : 0)) << (8 * e);
        }
        const long o = ((n * (a.H >> 1) + (h0 >> 1) + ty) * (W >> 1) + tx) * COP + co0;
        *reinterpret_cast<float4*>(static_cast<float*>(a.pool_y) + o) = make_float4(m[0], m[1], m[2], m[3]);
        if (a.pool_mask) *reinterpret_cast<uint32_t*>(a.pool_mask + o) = mk;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// weight transform: U = G g G^T per (group, co, ci) from the fp32 master
// ---------------------------------------------------------------------------

struct WinoWSeg {
  const float* w;       // fp32 master [Q][Cop][3][3][Cip]
  uint16_t* u;          // bf16 planes [3][Q][16][R][K]
  long ups;             // plane stride (elements)
  int Q, Cop, Cip;
  int R, K;             // forward: rows = co (R >= Cop), columns = ci (K >= Cip); data gradient: swapped
  int dgrad;            // 1: the flipped, transposed kernel the data gradient convolves with
  int pad;
};

struct WinoWArgs {
  const WinoWSeg* segs;
  const int2* blocks;   // per block: (segment, first element of Q x R x K)
};

// G = [[1, 0, 0], [1/2, 1/2, 1/2], [1/2, -1/2, 1/2], [0, 0, 1]]: row i of G v
__device__ __forceinline__ float wino_g(int i, float v0, float v1, float v2) {
  if (i == 0) return v0;
  if (i == 3) return v2;
  return i == 1 ? 0.5f * ((v0 + v2) + v1) : 0.5f * ((v0 + v2) - v1);
}

__global__ void __launch_bounds__(256) wino_wtrans_kernel(WinoWArgs a) {
  const int2 blk = a.blocks[blockIdx.x];
  const WinoWSeg s = a.segs[blk.x];
  const long e = (long)blk.y + threadIdx.x;
  const long per = (long)s.R * s.K;
  if (e >= (long)s.Q * per) return;
  const int q = (int)(e / per);
  const int rem = (int)(e - (long)q * per);
  const int row = rem / s.K, col = rem - row * s.K;
  const int co = s.dgrad ? col : row, ci = s.dgrad ? row : col;
  float gk[3][3];
  const bool ok = co < s.Cop && ci < s.Cip;
#pragma unroll
  for (int kh = 0; kh < 3; ++kh)
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int sh = s.dgrad ? 2 - kh : kh, sw = s.dgrad ? 2 - kw : kw;
      gk[kh][kw] = ok ? s.w[(((long)q * s.Cop + co) * 9 + sh * 3 + sw) * s.Cip + ci] : 0.f;
    }
  float t[4][3];                                       // G g
#pragma unroll
  for (int kw = 0; kw < 3; ++kw)
#pragma unroll
    for (int i = 0; i < 4; ++i) t[i][kw] = wino_g(i, gk[0][kw], gk[1][kw], gk[2][kw]);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float u = wino_g(j, t[i][0], t[i][1], t[i][2]);   // (G g G^T)[i][j]
      const uint16_t h0 = f2bf(u);
      const float r1 = u - bf2f(h0);
      const uint16_t h1 = f2bf(r1);
      const uint16_t h2 = f2bf(r1 - bf2f(h1));
      // fragment-major: [q][xi][row / 16][col / 32][lane = (col % 32) / 8 * 16 + row % 16][col % 8]
      const long o = (((((long)q * 16 + i * 4 + j) * (s.R >> 4) + (row >> 4)) * (s.K >> 5) + (col >> 5)) * 64 +
                      ((col & 31) >> 3) * 16 + (row & 15)) * 8 + (col & 7);
      s.u[o] = h0;
      s.u[s.ups + o] = h1;
      s.u[2 * s.ups + o] = h2;
    }
}

// ---------------------------------------------------------------------------
// dispatch
// ---------------------------------------------------------------------------

template <typename F>
static void wino_lds_limit(F* fn, size_t bytes) {
  if (bytes > 65536)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

#define WINO_LAUNCH(NCBI_, NT_, W_, TH_)                                                               \
  {                                                                                                   \
    if (probe) return 1000 + TH_;                                                                     \
    dim3 grid(a->B * (a->H / TH_), a->ngroups);                                                       \
    const size_t lds = WinoCfg<NCBI_, NT_, W_, TH_>::lds();                                           \
    auto* fn = conv_wino_kernel<NCBI_, NT_, W_, TH_>;                                                 \
    wino_lds_limit(fn, lds);                                                                          \
    hipLaunchKernelGGL(fn, grid, dim3(256), lds, stream, *a);                                         \
    return (int)hipGetLastError();                                                                    \
  }

// below ~300 workgroups (small launches: few groups) the half-height tile doubles the grid; every
// output's summation order is the same for any tile height (bit-identical)
static int g_wino_smallq_wg = 300;

extern "C" int gt_conv_wino(const ConvArgs* a, hipStream_t stream, int probe) {
  if (!a->wino) return -100;
  if (a->prec != 1 || a->KH != 3 || a->KW != 3 || a->mask || a->Cinp % 8 || a->Coutp % 8) return -101;
  const int NCBI = a->Cinp / 8, NT = (a->Coutp + 15) / 16;
  const bool small = (long)a->ngroups * a->B * (a->H / 8) < g_wino_smallq_wg;
  // S=(3,5) kernels (20, 50): stage 2 (56 -> 56 channels at 16 x 16). Stage 1 (24 -> 24 at 32 x 32) stays
  // on the direct kernel: K = 24 leaves a quarter of the one k-step empty and the Winograd build ran
  // 20-25 % slower there (profiles/r6/wino_bench_r6.txt)
  if (NCBI == 7 && NT == 4 && a->W == 16 && a->H % 8 == 0) {
    if (small) WINO_LAUNCH(7, 4, 16, 4)
    WINO_LAUNCH(7, 4, 16, 8)
  }
  return -101;       // wino set for a shape without an instantiation: never fall back onto U planes
}

// U layout (rows, columns) the kernel expects for these channel counts, or 0 when no Winograd
// instantiation runs them: rows = Coutp rounded up to 16, columns = Cinp rounded up to 32
extern "C" int gt_conv_wino_supported(int Cinp, int Coutp, int H, int W) {
  const int NCBI = Cinp / 8, NT = (Coutp + 15) / 16;
  if (Cinp % 8 || Coutp % 8) return 0;
  if (NCBI == 7 && NT == 4 && W == 16 && H % 8 == 0) return 1;
  return 0;
}

extern "C" int gt_wino_wtrans(const void* av, int nblocks, hipStream_t stream) {
  const WinoWArgs* a = static_cast<const WinoWArgs*>(av);
  if (nblocks < 1) return 0;
  hipLaunchKernelGGL(wino_wtrans_kernel, dim3(nblocks), dim3(256), 0, stream, *a);
  return (int)hipGetLastError();
}

extern "C" size_t gt_sizeof_wino_wseg() { return sizeof(WinoWSeg); }
