// Genetic-CNN convolution kernels for MI355X (gfx950), NHWC bf16, channels
// padded to a multiple of 8 so one 16-byte access = 8 channels.
//
// conv_fwd  (K1 + K2 of SURVEY.md §2.4): implicit GEMM on
//   v_mfma_f32_16x16x32_bf16. One workgroup = 4 waves = TH full output rows
//   (<= 64 pixels) of one image of one fold, all output channels of a
//   64-channel block. The input patch (TH+KH-1 rows x W+KW-1 cols x Cin) is
//   staged ONCE into LDS, with the Genetic-CNN DAG's N-ary Add fused into the
//   staging (sum of up to 4 producer tensors, fp32 then bf16), an optional
//   ReLU-mask multiply (dgrad: dz = dy * (y > 0)) and an optional batch gather
//   (first layer reads dataset images through the epoch's index table, so no
//   separate gather kernel and no host->device batch copy).
//   MFMA operands: A = weights [co][k] (16-B global loads, L2-resident),
//   B = patch pixels (ds_read_b128). Epilogue: bias + ReLU, 8-byte stores of
//   4 consecutive channels, optional accumulate into up to 4 outputs (DAG
//   gradient fan-out without an add kernel).
//   The same kernel is the data-gradient (K2): stride-1 'same' dgrad is a
//   'same' conv of dz with the flipped, transposed weights W'.
//
// conv_wgrad (K3): dW[co][kh][kw][ci] = sum_pix dz[pix][co] * x[pix+(kh,kw)][ci]
//   as a split-K GEMM: each workgroup owns a 64(co) x 64(kh,kw,ci) block and
//   a pixel range; per 32-pixel K-step the dz tile and the im2col tile are
//   staged TRANSPOSED into LDS so both MFMA operands are ds_read_b128 rows.
//   Partial sums go to a [S][G][Coutp][K] fp32 workspace that the Adam kernel
//   reduces in a fixed order (deterministic, no float atomics).
//
// pool2x2 fwd/bwd (K4): vectorised 8-channel max-pool and its scatter.

#include <algorithm>

#include "common.h"

struct ConvArgs {
  const uint16_t* in[4];     // summed inputs [G][B][H][W][Cinp]
  const uint16_t* mask;      // optional: staged value *= (mask > 0), same shape as in
  const int64_t* gather;     // optional: image table [steps][G][B]; in[0] is then the dataset
  const StepState* st;       // cur_step for the gather table
  uint16_t* out[4];          // [G][B][H][W][Coutp]
  const uint16_t* out_mask[4];  // optional per output: final value *= (out_mask > 0) (dz of a ReLU layer)
  const uint16_t* w;         // [G][Coutp][KH][KW][Cinp] bf16
  const float* bias;         // [G][Coutp] or null
  int n_in, n_out, acc_flags, relu;
  int G, B, H, W, Cinp, Coutp, KH, KW, TH;
};

#define CF_KB 16                 // weight K-block: 16 chunks of 8 = 128 k
#define CF_WLD (CF_KB * 8 + 8)    // LDS row stride of a weight block (272 B: conflict-free b128 reads)

#ifndef CF_WPE
#define CF_WPE 5   // minimum waves per SIMD the register allocator must allow
#endif

template <int PXG>   // 16-pixel groups per wave (tile = 64 * PXG pixels)
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PXG == 4 ? 3 : CF_WPE))) conv_fwd_kernel(ConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int nth = (a.H + a.TH - 1) / a.TH;
  const int b = blockIdx.x / nth;
  const int h0 = (blockIdx.x % nth) * a.TH;
  const int g = blockIdx.y;
  const int co_blk = blockIdx.z * 64;
  const int ph = a.KH >> 1, pw = a.KW >> 1;
  const int PH = a.TH + a.KH - 1, PW = a.W + a.KW - 1;
  const int ncb = a.Cinp >> 3;
  const long img = (long)a.H * a.W * a.Cinp;
  const int total = PH * PW * ncb;
  const int nchunks = a.KH * a.KW * ncb;
  const int Kdim = a.KH * a.KW * a.Cinp;
  // LDS carve: [weight blocks: nbuf x wrows x CF_WLD][patch][chunk offset table].
  // Only as many weight rows / buffers as this layer needs (occupancy).
  const int nkb = (nchunks + CF_KB - 1) / CF_KB;
  const int nbuf = nkb > 1 ? 2 : 1;
  const int wrows = ((min(64, a.Coutp) + 15) >> 4) << 4;
  const size_t wbytes = (size_t)nbuf * wrows * CF_WLD * 2;
  uint16_t* wbuf = reinterpret_cast<uint16_t*>(smem);
  uint4* patch = reinterpret_cast<uint4*>(smem + wbytes);
  int* coff = reinterpret_cast<int*>(smem + wbytes + (size_t)total * 16);
  const uint16_t* wg = a.w + (long)g * a.Coutp * Kdim;

  // weight-block staging role: row = tid >> 2 (up to 64 rows), 8 chunks per thread
  const int wr = tid >> 2, wq = (tid & 3) * (CF_KB / 4);
  const bool wrow_live = wr < wrows;
  const bool wrow_ok = co_blk + wr < a.Coutp;
  const uint16_t* wsrc = wg + (long)(co_blk + wr) * Kdim;
  uint4 wreg[CF_KB / 4];
  auto load_wblock = [&](int kb) {
#pragma unroll
    for (int j = 0; j < CF_KB / 4; ++j) {
      const int c = kb * CF_KB + wq + j;
      wreg[j] = (wrow_ok && c < nchunks) ? *reinterpret_cast<const uint4*>(wsrc + c * 8) : make_uint4(0, 0, 0, 0);
    }
  };
  auto store_wblock = [&](int buf) {
    if (!wrow_live) return;
    uint16_t* dst = wbuf + buf * wrows * CF_WLD + wr * CF_WLD + wq * 8;
#pragma unroll
    for (int j = 0; j < CF_KB / 4; ++j) *reinterpret_cast<uint4*>(dst + j * 8) = wreg[j];
  };
  load_wblock(0);

  // ---- stage the summed / masked input patch -------------------------------
  const uint16_t* src[4];
  for (int k = 0; k < a.n_in; ++k) src[k] = a.in[k] + ((long)g * a.B + b) * img;
  if (a.gather) {
    const long id = a.gather[((long)a.st->cur_step * a.G + g) * a.B + b];
    src[0] = a.in[0] + id * img;
  }
  const uint16_t* msrc = a.mask ? a.mask + ((long)g * a.B + b) * img : nullptr;
  const FastDiv div_ncb(ncb), div_pw(PW);
  for (int i = tid; i < total; i += 256) {
    uint32_t pix, cbu, pr, pc;
    div_ncb.divmod((uint32_t)i, pix, cbu);
    div_pw.divmod(pix, pr, pc);
    const int cb = (int)cbu;
    const int hh = h0 - ph + (int)pr, ww = (int)pc - pw;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (hh >= 0 && hh < a.H && ww >= 0 && ww < a.W) {
      const long off = ((long)hh * a.W + ww) * a.Cinp + cb * 8;
      if (a.n_in == 1 && !msrc) {
        v = *reinterpret_cast<const uint4*>(src[0] + off);
      } else {
        float acc[8], t[8];
        unpack8(*reinterpret_cast<const uint4*>(src[0] + off), acc);
        for (int k = 1; k < a.n_in; ++k) {
          unpack8(*reinterpret_cast<const uint4*>(src[k] + off), t);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] += t[j];
        }
        if (msrc) {
          unpack8(*reinterpret_cast<const uint4*>(msrc + off), t);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] = t[j] > 0.f ? acc[j] : 0.f;
        }
        v = pack8(acc);
      }
    }
    patch[i] = v;
  }
  {
    const FastDiv div_kw(a.KW);
    for (int c = tid; c < nchunks + 4; c += 256) {
      if (c < nchunks) {
        uint32_t kk, cb, kh, kw;
        div_ncb.divmod((uint32_t)c, kk, cb);
        div_kw.divmod(kk, kh, kw);
        coff[c] = ((int)kh * PW + (int)kw) * ncb + (int)cb;
      } else {
        coff[c] = -1;
      }
    }
  }
  store_wblock(0);
  __syncthreads();

  // ---- MFMA main loop: each wave = 32 pixels (2 B fragments) x all co tiles --
  const int wave = tid >> 6, lane = tid & 63;
  const int kq = lane >> 4, l16 = lane & 15;
  const int npx = a.TH * a.W;
  int pbase[PXG];
  bool pvalid[PXG];
  int pyy[PXG], pxx[PXG];
#pragma unroll
  for (int h = 0; h < PXG; ++h) {
    const int pl = wave * 16 * PXG + h * 16 + l16;
    pyy[h] = pl / a.W; pxx[h] = pl % a.W;
    pvalid[h] = (pl < npx) && (h0 + pyy[h] < a.H);
    pbase[h] = (pyy[h] * PW + pxx[h]) * ncb;
  }
  const int nco = min(64, a.Coutp - co_blk);
  const int NT = (nco + 15) >> 4;
  f32x4_t acc[PXG][4];
#pragma unroll
  for (int h = 0; h < PXG; ++h)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[h][t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  for (int kb = 0; kb < nkb; ++kb) {
    const bool more = kb + 1 < nkb;
    if (more) load_wblock(kb + 1);
    const uint16_t* wcur = wbuf + (kb & 1) * wrows * CF_WLD;
#pragma unroll
    for (int kk = 0; kk < CF_KB / 4; ++kk) {
      const int c = kb * CF_KB + kk * 4 + kq;
      if (kb * CF_KB + kk * 4 >= nchunks) break;
      const int co_off = coff[c];
      uint4 bfr[PXG];
#pragma unroll
      for (int h = 0; h < PXG; ++h)
        bfr[h] = (co_off >= 0 && pvalid[h]) ? patch[pbase[h] + co_off] : make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (t < NT) {
          const uint4 af = *reinterpret_cast<const uint4*>(wcur + (t * 16 + l16) * CF_WLD + (kk * 4 + kq) * 8);
#pragma unroll
          for (int h = 0; h < PXG; ++h) acc[h][t] = mfma16(af, bfr[h], acc[h][t]);
        }
      }
    }
    if (more) store_wblock((kb + 1) & 1);
    __syncthreads();
  }

  // ---- epilogue: bias + relu, 4 channels per lane ---------------------------
#pragma unroll
  for (int h = 0; h < PXG; ++h) {
    if (!pvalid[h]) continue;
    const long obase = ((((long)g * a.B + b) * a.H + (h0 + pyy[h])) * a.W + pxx[h]) * a.Coutp;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (t >= NT) continue;
      const int co0 = co_blk + t * 16 + kq * 4;
      if (co0 >= a.Coutp) continue;
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float x = acc[h][t][i];
        if (a.bias) x += a.bias[(long)g * a.Coutp + co0 + i];
        if (a.relu) x = fmaxf(x, 0.f);
        v[i] = x;
      }
      for (int k = 0; k < a.n_out; ++k) {
        uint2* dst = reinterpret_cast<uint2*>(a.out[k] + obase + co0);
        float sum[4] = {v[0], v[1], v[2], v[3]};
        if ((a.acc_flags >> k) & 1) {
          const uint2 old = *dst;
          sum[0] += __uint_as_float(old.x << 16); sum[1] += __uint_as_float(old.x & 0xffff0000u);
          sum[2] += __uint_as_float(old.y << 16); sum[3] += __uint_as_float(old.y & 0xffff0000u);
        }
        if (a.out_mask[k]) {
          const uint2 m = *reinterpret_cast<const uint2*>(a.out_mask[k] + obase + co0);
          // bf16 > 0  <=>  sign bit clear and not +0
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
// conv_fwd, LDS-DMA variant (single-input, unmasked layers: most of the DAG)
// ---------------------------------------------------------------------------
// The register-staged kernel above is latency-bound: a workgroup walks a chain
// of dependent global round trips (patch slots, then weight block k+1 behind
// block k, then bias), and only ~1-5 workgroups per CU exist to hide them.
// Here every byte reaches LDS through global_load_lds_dwordx4 (no VGPR
// destination), so the whole patch and the first two weight blocks are in
// flight at once and the workgroup waits for ONE latency before its MFMAs.
//   * LDS images are lane-linear (a wave-instruction writes 1 KiB
//     contiguously); weight rows are 256 B unpadded and XOR-swizzled through
//     the SOURCE address (chunk c of row r lands at slot c ^ (r & 15)), so the
//     16 rows an A-fragment read touches hit 16 different bank groups.
//   * Padding pixels / rows / chunks read a 16-byte zero line.
//   * Weight blocks > 1 stream through a 2-deep ring with counted vmcnt waits
//     and raw s_barrier (a __syncthreads() would drain the prefetch).

__device__ __attribute__((aligned(16))) uint4 g_zero16[4];

typedef __attribute__((address_space(1))) const void gvoid_t;
typedef __attribute__((address_space(3))) void lvoid_t;

__device__ __forceinline__ void glds16(const void* src, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((gvoid_t*)src, (lvoid_t*)lds_wave_base, 16, 0, 0);
}

// wait until at most n (0..4) LDS-DMA / vector loads of this wave are outstanding
__device__ __forceinline__ void vm_wait(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
  }
}

__device__ __forceinline__ void raw_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

// Weight-ring depth: as many 16-chunk blocks as the LDS share of one workgroup
// allows when the grid needs ceil(nwg / 256) workgroups resident per CU (the
// s2 / deep layers launch only ~1-2 workgroups per CU, so they can keep every
// block -- or most of them -- resident and issue all weight DMAs at once).
__host__ __device__ inline int conv_glds_nbuf(int nkb, int wblk, int fixed_bytes, long nwg) {
  long per_cu = (nwg + 255) / 256;
  if (per_cu < 1) per_cu = 1;
  if (per_cu > 8) per_cu = 8;
  const long budget = 160L * 1024 / per_cu - 1024 - fixed_bytes;
  long nb = budget / wblk;
  if (nb > nkb) nb = nkb;
  if (nb < 2) nb = nkb < 2 ? nkb : 2;
  return (int)nb;
}

__device__ __forceinline__ unsigned long long rt_stamp() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
  return t;
}

// STAMP (diagnostic build only): per workgroup realtime stamps (100 MHz) at
// entry / operands staged / MFMAs done / exit -> stamps[wg][4].
template <int PXG, bool STAMP = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PXG == 4 ? 3 : CF_WPE)))
conv_fwd_glds_kernel(ConvArgs a, unsigned long long* stamps = nullptr) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const long wg_lin = ((long)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
  if (STAMP && threadIdx.x == 0) stamps[wg_lin * 4 + 0] = rt_stamp();
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int nth = (a.H + a.TH - 1) / a.TH;
  const int b = blockIdx.x / nth;
  const int h0 = (blockIdx.x % nth) * a.TH;
  const int g = blockIdx.y;
  const int co_blk = blockIdx.z * 64;
  const int ph = a.KH >> 1, pw = a.KW >> 1;
  const int PW = a.W + a.KW - 1;
  const int ncb = a.Cinp >> 3;
  const long img = (long)a.H * a.W * a.Cinp;
  const int total = (a.TH + a.KH - 1) * PW * ncb;
  const int totalr = (total + 255) & ~255;
  const int nchunks = a.KH * a.KW * ncb;
  const int Kdim = a.KH * a.KW * a.Cinp;
  const int nkb = (nchunks + CF_KB - 1) / CF_KB;
  const int nco = min(64, a.Coutp - co_blk);
  const int wrows = ((nco + 15) >> 4) << 4;
  const int wcnt = wrows >> 4;                 // glds per wave per weight block
  const int wblk = wrows * 256;                // bytes of one block image
  const int fixed = totalr * 16 + 4 * (nchunks + 4);
  const int NB = conv_glds_nbuf(nkb, (((min(64, a.Coutp) + 15) >> 4) << 4) * 256, fixed,
                                (long)gridDim.x * gridDim.y * gridDim.z);
  const int wstride = (((min(64, a.Coutp) + 15) >> 4) << 4) * 256;   // buffer pitch (host LDS size uses it)
  char* wbuf = smem;
  uint4* patch = reinterpret_cast<uint4*>(smem + (size_t)NB * wstride);
  int* coff = reinterpret_cast<int*>(smem + (size_t)NB * wstride + (size_t)totalr * 16);
  const uint16_t* wg = a.w + ((long)g * a.Coutp + co_blk) * Kdim;
  const void* zero = g_zero16;

  auto issue_wblock = [&](int kb, int buf) {
    for (int q0 = wave * 64; q0 < wrows * 16; q0 += 256) {
      const int q = q0 + lane, r = q >> 4, c = kb * CF_KB + ((q & 15) ^ (r & 15));
      const void* src = (r < nco && c < nchunks) ? (const void*)(wg + (long)r * Kdim + c * 8) : zero;
      glds16(src, wbuf + buf * wstride + q0 * 16);
    }
  };
  // dependent scalar loads first: a plain load issued while DMAs fly makes the
  // compiler drain them (vmcnt(0)) at its first use
  const uint16_t* src0 = a.in[0] + ((long)g * a.B + b) * img;
  if (a.gather) {
    const long id = a.gather[((long)a.st->cur_step * a.G + g) * a.B + b];
    src0 = a.in[0] + id * img;
  }
  const int kq = lane >> 4, l16 = lane & 15;
  const int NT = (nco + 15) >> 4;
  float bias_v[4][4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int co = co_blk + t * 16 + kq * 4 + i;
      bias_v[t][i] = (a.bias && t < NT && co < a.Coutp) ? a.bias[(long)g * a.Coutp + co] : 0.f;
    }
  issue_wblock(0, 0);
  {
    const FastDiv div_ncb(ncb), div_pw(PW);
    for (int q0 = wave * 64; q0 < total; q0 += 256) {
      const int q = q0 + lane;
      uint32_t pix, cbu, pr, pc;
      div_ncb.divmod((uint32_t)q, pix, cbu);
      div_pw.divmod(pix, pr, pc);
      const int hh = h0 - ph + (int)pr, ww = (int)pc - pw;
      const bool ok = q < total && hh >= 0 && hh < a.H && ww >= 0 && ww < a.W;
      const void* src = ok ? (const void*)(src0 + ((long)hh * a.W + ww) * a.Cinp + (int)cbu * 8) : zero;
      glds16(src, reinterpret_cast<char*>(patch) + q0 * 16);
    }
  }
  for (int kb = 1; kb < NB; ++kb) issue_wblock(kb, kb);
  {
    const FastDiv div_ncb(ncb), div_kw(a.KW);
    for (int c = tid; c < nchunks + 4; c += 256) {
      if (c < nchunks) {
        uint32_t kk, cb, kh, kw;
        div_ncb.divmod((uint32_t)c, kk, cb);
        div_kw.divmod(kk, kh, kw);
        coff[c] = ((int)kh * PW + (int)kw) * ncb + (int)cb;
      } else {
        coff[c] = -1;
      }
    }
  }
  // Everything staged so far lands before the first MFMA: hipcc waits
  // vmcnt(0) before any LDS read that may alias an in-flight LDS-DMA anyway.
  vm_wait(0);
  raw_barrier();
  if (STAMP && threadIdx.x == 0) stamps[wg_lin * 4 + 1] = rt_stamp();

  const int npx = a.TH * a.W;
  int pbase[PXG];
  bool pvalid[PXG];
  int pyy[PXG], pxx[PXG];
#pragma unroll
  for (int h = 0; h < PXG; ++h) {
    const int pl = wave * 16 * PXG + h * 16 + l16;
    pyy[h] = pl / a.W; pxx[h] = pl % a.W;
    pvalid[h] = (pl < npx) && (h0 + pyy[h] < a.H);
    pbase[h] = (pyy[h] * PW + pxx[h]) * ncb;
  }
  f32x4_t acc[PXG][4];
#pragma unroll
  for (int h = 0; h < PXG; ++h)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[h][t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  for (int kb = 0; kb < nkb; ++kb) {
    const char* wcur = wbuf + (kb % NB) * wstride;
#pragma unroll
    for (int kk = 0; kk < CF_KB / 4; ++kk) {
      const int cl = kk * 4 + kq;
      if (kb * CF_KB + kk * 4 >= nchunks) break;
      const int co_off = coff[kb * CF_KB + cl];
      uint4 bfr[PXG];
#pragma unroll
      for (int h = 0; h < PXG; ++h)
        bfr[h] = (co_off >= 0 && pvalid[h]) ? patch[pbase[h] + co_off] : make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (t < NT) {
          const uint4 af = *reinterpret_cast<const uint4*>(wcur + (t * 16 + l16) * 256 + ((cl ^ l16) << 4));
#pragma unroll
          for (int h = 0; h < PXG; ++h) acc[h][t] = mfma16(af, bfr[h], acc[h][t]);
        }
      }
    }
    if (kb + NB < nkb) {                   // ring refill (layers whose weights do not fit)
      raw_barrier();                       // every wave is done with buffer kb % NB
      issue_wblock(kb + NB, kb % NB);
      vm_wait(wcnt);                       // block kb+1 landed, kb+NB may fly
      raw_barrier();
    }
  }
  if (STAMP && threadIdx.x == 0) stamps[wg_lin * 4 + 2] = rt_stamp();

  // ---- epilogue (as the register-staged kernel) ------------------------------
#pragma unroll
  for (int h = 0; h < PXG; ++h) {
    if (!pvalid[h]) continue;
    const long obase = ((((long)g * a.B + b) * a.H + (h0 + pyy[h])) * a.W + pxx[h]) * a.Coutp;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (t >= NT) continue;
      const int co0 = co_blk + t * 16 + kq * 4;
      if (co0 >= a.Coutp) continue;
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float x = acc[h][t][i] + bias_v[t][i];
        if (a.relu) x = fmaxf(x, 0.f);
        v[i] = x;
      }
      for (int k = 0; k < a.n_out; ++k) {
        uint2* dst = reinterpret_cast<uint2*>(a.out[k] + obase + co0);
        float sum[4] = {v[0], v[1], v[2], v[3]};
        if ((a.acc_flags >> k) & 1) {
          const uint2 old = *dst;
          sum[0] += __uint_as_float(old.x << 16); sum[1] += __uint_as_float(old.x & 0xffff0000u);
          sum[2] += __uint_as_float(old.y << 16); sum[3] += __uint_as_float(old.y & 0xffff0000u);
        }
        if (a.out_mask[k]) {
          const uint2 m = *reinterpret_cast<const uint2*>(a.out_mask[k] + obase + co0);
          const uint32_t mw[4] = {m.x & 0xffffu, m.x >> 16, m.y & 0xffffu, m.y >> 16};
#pragma unroll
          for (int i = 0; i < 4; ++i) sum[i] = (mw[i] != 0u && mw[i] < 0x8000u) ? sum[i] : 0.f;
        }
        *dst = pack4(sum);
      }
    }
  }
  if (STAMP) {
    __syncthreads();
    if (threadIdx.x == 0) stamps[wg_lin * 4 + 3] = rt_stamp();
  }
}

// ---------------------------------------------------------------------------
// conv_fwd, persistent LDS-DMA variant (single-input layers whose weights fit)
// ---------------------------------------------------------------------------
// Stamps of the one-tile kernels show every workgroup of a launch moving in
// lock-step through three bursts -- all operands staged (~4 us, the whole
// grid's loads at once), MFMAs (LDS-bound), stores -- with the memory system
// idle during the MFMAs and vice versa, and every workgroup re-reading the
// fold's weights from L2 (more bytes than the patches for 3x3 layers).
// Here a workgroup keeps ALL of its fold's weight blocks resident, walks a
// strided list of output tiles, and DMAs tile i+1's patch into the second
// patch buffer while it runs tile i's MFMAs and stores.
//   The DMA of the next patch is issued by inline asm: hipcc does not model it,
//   so it does not put vmcnt(0) in front of every LDS read of the current tile
//   (which it does for the builtin); the kernel waits for it by hand
//   (vmcnt(0) + barrier at the end of each tile). A plain load that hipcc does
//   track can only over-wait (counters retire in order), never under-wait.

__device__ __forceinline__ void glds16_asm(const void* src, const void* lds_wave_base) {
  const uint32_t l = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lvoid_t*)lds_wave_base);
  uint32_t keep;   // m0 is reserved by the compiler: save / restore it around the DMA
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(l) : "memory");
}

#define CP_MAXT 64   // tiles per workgroup (gather ids cached in LDS)

template <int PXG>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PXG == 4 ? 3 : CF_WPE)))
conv_fwd_pers_kernel(ConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int nth = (a.H + a.TH - 1) / a.TH;
  const int ntile = a.B * nth;
  const int g = blockIdx.y;
  const int co_blk = blockIdx.z * 64;
  const int ph = a.KH >> 1, pw = a.KW >> 1;
  const int PW = a.W + a.KW - 1;
  const int ncb = a.Cinp >> 3;
  const long img = (long)a.H * a.W * a.Cinp;
  const int total = (a.TH + a.KH - 1) * PW * ncb;
  const int totalr = (total + 255) & ~255;
  const int nchunks = a.KH * a.KW * ncb;
  const int Kdim = a.KH * a.KW * a.Cinp;
  const int nkb = (nchunks + CF_KB - 1) / CF_KB;
  const int nco = min(64, a.Coutp - co_blk);
  const int wrows = ((nco + 15) >> 4) << 4;
  const int wstride = (((min(64, a.Coutp) + 15) >> 4) << 4) * 256;
  char* wbuf = smem;
  char* pbuf = smem + (size_t)nkb * wstride;                          // 2 x totalr x 16 B
  int* coff = reinterpret_cast<int*>(pbuf + (size_t)2 * totalr * 16);
  long* gid = reinterpret_cast<long*>(coff + ((nchunks + 4 + 1) & ~1));
  float* sbias = reinterpret_cast<float*>(gid + CP_MAXT);              // [64]
  const uint16_t* wg = a.w + ((long)g * a.Coutp + co_blk) * Kdim;
  const uint16_t* in_fold = a.in[0] + (long)g * a.B * img;
  const void* zero = g_zero16;
  const int t0 = blockIdx.x, tstep = gridDim.x;
  const int my_tiles = t0 < ntile ? (ntile - 1 - t0) / tstep + 1 : 0;

  // gather ids of every tile this workgroup will stage (plain loads, waited below)
  if (a.gather) {
    for (int i = tid; i < my_tiles; i += 256) {
      const int b = (t0 + i * tstep) / nth;
      gid[i] = a.gather[((long)a.st->cur_step * a.G + g) * a.B + b];
    }
  }
  const int kq = lane >> 4, l16 = lane & 15;
  const int NT = (nco + 15) >> 4;
  // bias lives in LDS: an epilogue use of a register loaded from global memory
  // would make hipcc wait vmcnt(0), i.e. for the next tile's patch DMA
  if (tid < 64) sbias[tid] = (a.bias && tid < nco) ? a.bias[(long)g * a.Coutp + co_blk + tid] : 0.f;
  __syncthreads();   // gid / sbias visible (and the plain loads above retired)

  const FastDiv div_ncb(ncb), div_pw(PW);
  auto issue_patch = [&](int i, int buf) {          // tile t0 + i*tstep -> patch buffer buf
    const int t = t0 + i * tstep;
    const int b = t / nth, h0 = (t % nth) * a.TH;
    const uint16_t* src0 = a.gather ? a.in[0] + gid[i] * img : in_fold + (long)b * img;
    char* dst = pbuf + (size_t)buf * totalr * 16;
    for (int q0 = wave * 64; q0 < total; q0 += 256) {
      const int q = q0 + lane;
      uint32_t pix, cbu, pr, pc;
      div_ncb.divmod((uint32_t)q, pix, cbu);
      div_pw.divmod(pix, pr, pc);
      const int hh = h0 - ph + (int)pr, ww = (int)pc - pw;
      const bool ok = q < total && hh >= 0 && hh < a.H && ww >= 0 && ww < a.W;
      glds16_asm(ok ? (const void*)(src0 + ((long)hh * a.W + ww) * a.Cinp + (int)cbu * 8) : zero, dst + q0 * 16);
    }
  };
  // all weight blocks (resident for the whole launch)
  for (int kb = 0; kb < nkb; ++kb) {
    for (int q0 = wave * 64; q0 < wrows * 16; q0 += 256) {
      const int q = q0 + lane, r = q >> 4, c = kb * CF_KB + ((q & 15) ^ (r & 15));
      const void* src = (r < nco && c < nchunks) ? (const void*)(wg + (long)r * Kdim + c * 8) : zero;
      glds16_asm(src, wbuf + (size_t)kb * wstride + q0 * 16);
    }
  }
  if (my_tiles > 0) issue_patch(0, 0);
  {
    const FastDiv div_kw(a.KW);
    for (int c = tid; c < nchunks + 4; c += 256) {
      if (c < nchunks) {
        uint32_t kk, cb, kh, kw;
        div_ncb.divmod((uint32_t)c, kk, cb);
        div_kw.divmod(kk, kh, kw);
        coff[c] = ((int)kh * PW + (int)kw) * ncb + (int)cb;
      } else {
        coff[c] = -1;
      }
    }
  }
  vm_wait(0);
  raw_barrier();

  const int npx = a.TH * a.W;
  int pbase[PXG], pyy[PXG], pxx[PXG];
  bool pin[PXG];
#pragma unroll
  for (int h = 0; h < PXG; ++h) {
    const int pl = wave * 16 * PXG + h * 16 + l16;
    pyy[h] = pl / a.W; pxx[h] = pl % a.W;
    pin[h] = pl < npx;
    pbase[h] = (pyy[h] * PW + pxx[h]) * ncb;
  }

  for (int i = 0; i < my_tiles; ++i) {
    if (i + 1 < my_tiles) issue_patch(i + 1, (i + 1) & 1);
    const int t = t0 + i * tstep;
    const int b = t / nth, h0 = (t % nth) * a.TH;
    const uint4* patch = reinterpret_cast<const uint4*>(pbuf + (size_t)(i & 1) * totalr * 16);
    bool pvalid[PXG];
#pragma unroll
    for (int h = 0; h < PXG; ++h) pvalid[h] = pin[h] && (h0 + pyy[h] < a.H);
    f32x4_t acc[PXG][4];
#pragma unroll
    for (int h = 0; h < PXG; ++h)
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) acc[h][tt] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    for (int kb = 0; kb < nkb; ++kb) {
      const char* wcur = wbuf + (size_t)kb * wstride;
#pragma unroll
      for (int kk = 0; kk < CF_KB / 4; ++kk) {
        const int cl = kk * 4 + kq;
        if (kb * CF_KB + kk * 4 >= nchunks) break;
        const int co_off = coff[kb * CF_KB + cl];
        uint4 bfr[PXG];
#pragma unroll
        for (int h = 0; h < PXG; ++h)
          bfr[h] = (co_off >= 0 && pvalid[h]) ? patch[pbase[h] + co_off] : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int tt = 0; tt < 4; ++tt) {
          if (tt < NT) {
            const uint4 af = *reinterpret_cast<const uint4*>(wcur + (tt * 16 + l16) * 256 + ((cl ^ l16) << 4));
#pragma unroll
            for (int h = 0; h < PXG; ++h) acc[h][tt] = mfma16(af, bfr[h], acc[h][tt]);
          }
        }
      }
    }
#pragma unroll
    for (int h = 0; h < PXG; ++h) {
      if (!pvalid[h]) continue;
      const long obase = ((((long)g * a.B + b) * a.H + (h0 + pyy[h])) * a.W + pxx[h]) * a.Coutp;
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) {
        if (tt >= NT) continue;
        const int co0 = co_blk + tt * 16 + kq * 4;
        if (co0 >= a.Coutp) continue;
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float x = acc[h][tt][j] + sbias[tt * 16 + kq * 4 + j];
          if (a.relu) x = fmaxf(x, 0.f);
          v[j] = x;
        }
        for (int k = 0; k < a.n_out; ++k) {
          uint2* dst = reinterpret_cast<uint2*>(a.out[k] + obase + co0);
          float sum[4] = {v[0], v[1], v[2], v[3]};
          if ((a.acc_flags >> k) & 1) {
            const uint2 old = *dst;
            sum[0] += __uint_as_float(old.x << 16); sum[1] += __uint_as_float(old.x & 0xffff0000u);
            sum[2] += __uint_as_float(old.y << 16); sum[3] += __uint_as_float(old.y & 0xffff0000u);
          }
          if (a.out_mask[k]) {
            const uint2 m = *reinterpret_cast<const uint2*>(a.out_mask[k] + obase + co0);
            const uint32_t mw[4] = {m.x & 0xffffu, m.x >> 16, m.y & 0xffffu, m.y >> 16};
#pragma unroll
            for (int j = 0; j < 4; ++j) sum[j] = (mw[j] != 0u && mw[j] < 0x8000u) ? sum[j] : 0.f;
          }
          *dst = pack4(sum);
        }
      }
    }
    vm_wait(0);        // next patch landed (this wave's part) ...
    raw_barrier();     // ... everyone's, and nobody still reads the buffer the next DMA overwrites
  }
}

// ---------------------------------------------------------------------------
// weight gradient (split-K, deterministic partials)
// ---------------------------------------------------------------------------

struct WgradArgs {
  const uint16_t* in[4];     // summed inputs of the layer [G][B][H][W][Cinp]
  const int64_t* gather;     // optional dataset gather (first layer)
  const StepState* st;
  const uint16_t* dz;        // ReLU-masked grad of the layer output [G][B][H][W][Coutp]
  float* part_w;             // [S][G][Coutp][Kdim]
  float* part_b;             // [S][G][Coutp]
  int n_in;
  int G, B, H, W, Cinp, Coutp, KH, KW, S, pps;  // pps = pixels per split (multiple of 64)
};

#define WG_LD 72   // LDS row stride (elements) of the [32 pixel][64] tiles (144 B: 16-B aligned rows)
#define WG_TILE (64 * WG_LD)   // 64 pixels per K-step

typedef __attribute__((ext_vector_type(4))) short short4_t;

// Two ds_read_b64_tr_b16 give a lane the 8 k-values (pixels 8g..8g+7 of the
// K-step) of column (col0 + lane&15) of a row-major [pixel][col] LDS tile:
// exactly the 16x16x32 MFMA operand layout (k = 8*(lane>>4) + j).
__device__ __forceinline__ uint4 tr_frag(const uint16_t* tile, int col0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  typedef __attribute__((address_space(3))) short4_t lds_s4;
  const uint16_t* r0 = tile + (8 * g + q) * WG_LD + col0 + 4 * p;
  const uint16_t* r1 = r0 + 4 * WG_LD;
  const short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(r0));
  const short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(r1));
  typedef __attribute__((ext_vector_type(8))) short short8_t;
  const short8_t v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(uint4, v);
}

// Coalesced staging of one 64-pixel K-step (pixels p0 .. p0+63 of one fold,
// consecutive in memory because the fold's images are contiguous):
//   dz tile  [64 px][64 co] : slot i -> (pixel i / ncc, co chunk i % ncc): a wave
//                             reads one contiguous run of dy / ymask bytes;
//   im2col   [64 px][64 col]: slot i -> (col chunk i / 64 (wave-uniform), pixel
//                             i % 64 = lane): a wave reads 64 consecutive
//                             pixels at one (kh, kw, cb) shift.
struct WgSlots {
  uint4 dz[2], xs[2];
};

__global__ void __launch_bounds__(256) conv_wgrad_kernel(WgradArgs a) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[4 * WG_TILE];   // 2 buffers x (dz, im2col)
  const int tid = threadIdx.x;
  const int nb = blockIdx.x;
  const int s = blockIdx.y;
  const int mblocks = (a.Coutp + 63) / 64;
  const int g = blockIdx.z / mblocks;
  const int co_blk = (blockIdx.z % mblocks) * 64;
  const int Kdim = a.KH * a.KW * a.Cinp;
  const int ncb = a.Cinp >> 3;
  const long HW = (long)a.H * a.W;
  const long npix = (long)a.B * HW;
  const long p_begin = (long)s * a.pps;
  const long p_end = (p_begin + a.pps < npix) ? p_begin + a.pps : npix;
  const int ncc = min(8, (a.Coutp - co_blk) >> 3);          // dz chunks per pixel in this co block
  const int ndz = 64 * ncc;                                   // dz slots per K-step (<= 512)
  const int wave = tid >> 6, lane = tid & 63, kq = lane >> 4, l16 = lane & 15;
  const FastDiv div_ncc(ncc), div_hw((uint32_t)HW), div_w(a.W), div_ncb(ncb), div_kw(a.KW);

  // im2col roles: this thread stages column chunks (wave, wave + 4) of the block
  // column chunk Kdim/8 is the bias chunk: a column of ones, so dW and db come
  // out of the same MFMAs (db[co] = sum_pix dz[pix][co] * 1)
  int c_kh[2], c_kw[2], c_cb[2];
  bool c_ok[2], c_one[2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int col = nb * 64 + (wave + 4 * r) * 8;
    c_ok[r] = col < Kdim;
    c_one[r] = (col == Kdim) && (a.part_b != nullptr);
    uint32_t kk = 0, cb = 0, kh = 0, kw = 0;
    if (c_ok[r]) { div_ncb.divmod((uint32_t)(col >> 3), kk, cb); div_kw.divmod(kk, kh, kw); }
    c_kh[r] = (int)kh - (a.KH >> 1); c_kw[r] = (int)kw - (a.KW >> 1); c_cb[r] = (int)cb;
  }
  const uint16_t* fold_in[4];
  for (int k = 0; k < a.n_in; ++k) fold_in[k] = a.in[k] + (long)g * a.B * HW * a.Cinp;
  const long fold_out = (long)g * npix * a.Coutp;

  const int MT = (min(64, a.Coutp - co_blk) + 15) >> 4;
  const bool wave_live = nb * 64 + wave * 16 <= Kdim;
  f32x4_t acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  WgSlots sl;
  auto load_step = [&](long p0) {
    // dz (masked by the layer's own ReLU output)
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int i = tid + 256 * r;
      sl.dz[r] = make_uint4(0, 0, 0, 0);
      if (i < ndz) {
        uint32_t px, cc;
        div_ncc.divmod((uint32_t)i, px, cc);
        const long p = p0 + px;
        if (p < p_end) sl.dz[r] = *reinterpret_cast<const uint4*>(a.dz + fold_out + p * a.Coutp + co_blk + cc * 8);
      }
    }
    // im2col: lane = pixel
    const long p = p0 + lane;
    uint32_t bq = 0, rem = 0, hq = 0, wq = 0;
    if (p < p_end) { div_hw.divmod((uint32_t)p, bq, rem); div_w.divmod(rem, hq, wq); }
    const uint16_t* gimg = nullptr;
    if (a.gather && p < p_end)
      gimg = a.in[0] + a.gather[((long)a.st->cur_step * a.G + g) * a.B + bq] * HW * a.Cinp;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      sl.xs[r] = make_uint4(0, 0, 0, 0);
      if (c_one[r] && p < p_end) sl.xs[r].x = 0x3f80u;          // bf16 1.0 in element 0
      const int ih = (int)hq + c_kh[r], iw = (int)wq + c_kw[r];
      if (p < p_end && c_ok[r] && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W) {
        const long pix_off = ((long)ih * a.W + iw) * a.Cinp + c_cb[r] * 8;
        if (gimg) {
          sl.xs[r] = *reinterpret_cast<const uint4*>(gimg + pix_off);
        } else if (a.n_in == 1) {
          sl.xs[r] = *reinterpret_cast<const uint4*>(fold_in[0] + (long)bq * HW * a.Cinp + pix_off);
        } else {
          float xsum[8] = {0, 0, 0, 0, 0, 0, 0, 0}, t[8];
          for (int k = 0; k < a.n_in; ++k) {
            unpack8(*reinterpret_cast<const uint4*>(fold_in[k] + (long)bq * HW * a.Cinp + pix_off), t);
#pragma unroll
            for (int j = 0; j < 8; ++j) xsum[j] += t[j];
          }
          sl.xs[r] = pack8(xsum);
        }
      }
    }
  };
  auto store_step = [&](int bf) {
    uint16_t* dzT = lds + bf * 2 * WG_TILE;
    uint16_t* colT = dzT + WG_TILE;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int i = tid + 256 * r;
      if (i < ndz) {
        uint32_t px, cc;
        div_ncc.divmod((uint32_t)i, px, cc);
        *reinterpret_cast<uint4*>(&dzT[px * WG_LD + cc * 8]) = sl.dz[r];
      }
      *reinterpret_cast<uint4*>(&colT[lane * WG_LD + (wave + 4 * r) * 8]) = sl.xs[r];
    }
  };
  // dz columns beyond this block's channels must read as zero
  if (ncc < 8) {
    for (int i = tid; i < 2 * 64 * (8 - ncc); i += 256) {
      const int bf = i / (64 * (8 - ncc)), rem = i % (64 * (8 - ncc));
      const int px = rem / (8 - ncc), cc = ncc + rem % (8 - ncc);
      *reinterpret_cast<uint4*>(&lds[bf * 2 * WG_TILE + px * WG_LD + cc * 8]) = make_uint4(0, 0, 0, 0);
    }
  }
  load_step(p_begin);
  store_step(0);
  __syncthreads();
  int buf = 0;
  for (long p0 = p_begin; p0 < p_end; p0 += 64) {
    const bool more = p0 + 64 < p_end;
    if (more) load_step(p0 + 64);
    const uint16_t* dzT = lds + buf * 2 * WG_TILE;
    const uint16_t* colT = dzT + WG_TILE;
    if (wave_live) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint4 bfrag = tr_frag(colT + h * 32 * WG_LD, wave * 16, lane);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          if (t < MT) {
            const uint4 afrag = tr_frag(dzT + h * 32 * WG_LD, t * 16, lane);
            acc[t] = mfma16(afrag, bfrag, acc[t]);
          }
        }
      }
    }
    if (more) store_step(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }

  const int col = nb * 64 + wave * 16 + l16;
  if (col < Kdim) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (t >= MT) continue;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int co = co_blk + t * 16 + kq * 4 + i;
        if (co < a.Coutp) a.part_w[(((long)s * a.G + g) * a.Coutp + co) * Kdim + col] = acc[t][i];
      }
    }
  } else if (col == Kdim && a.part_b) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (t >= MT) continue;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int co = co_blk + t * 16 + kq * 4 + i;
        if (co < a.Coutp) a.part_b[((long)s * a.G + g) * a.Coutp + co] = acc[t][i];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// 2x2/2 max-pool (floor) and its backward scatter
// ---------------------------------------------------------------------------

__global__ void pool_fwd_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y, int NB, int H, int W,
                                int Cp) {
  const int Ho = H >> 1, Wo = W >> 1, ncb = Cp >> 3;
  const long total = (long)NB * Ho * Wo * ncb;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int cb = (int)(i % ncb);
    long r = i / ncb;
    const int wo = (int)(r % Wo); r /= Wo;
    const int ho = (int)(r % Ho);
    const long n = r / Ho;
    const uint16_t* base = x + ((n * H + 2 * ho) * W + 2 * wo) * Cp + cb * 8;
    float m[8], t[8];
    unpack8(*reinterpret_cast<const uint4*>(base), m);
    const long offs[3] = {(long)Cp, (long)W * Cp, (long)W * Cp + Cp};
    for (int q = 0; q < 3; ++q) {
      unpack8(*reinterpret_cast<const uint4*>(base + offs[q]), t);
#pragma unroll
      for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], t[j]);
    }
    *reinterpret_cast<uint4*>(y + ((n * Ho + ho) * Wo + wo) * Cp + cb * 8) = pack8(m);
  }
}

// dx[pixel] = dy[pool cell] if pixel is the cell's first maximum else 0
__global__ void pool_bwd_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ dy,
                                uint16_t* __restrict__ dx, int NB, int H, int W, int Cp, int relu_mask) {
  const int Ho = H >> 1, Wo = W >> 1, ncb = Cp >> 3;
  const long total = (long)NB * H * W * ncb;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int cb = (int)(i % ncb);
    long r = i / ncb;
    const int w = (int)(r % W); r /= W;
    const int h = (int)(r % H);
    const long n = r / H;
    float out[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int ho = h >> 1, wo = w >> 1;
    if (ho < Ho && wo < Wo) {
      const uint16_t* base = x + ((n * H + 2 * ho) * W + 2 * wo) * Cp + cb * 8;
      float v[4][8];
      unpack8(*reinterpret_cast<const uint4*>(base), v[0]);
      unpack8(*reinterpret_cast<const uint4*>(base + Cp), v[1]);
      unpack8(*reinterpret_cast<const uint4*>(base + (long)W * Cp), v[2]);
      unpack8(*reinterpret_cast<const uint4*>(base + (long)W * Cp + Cp), v[3]);
      float g[8];
      unpack8(*reinterpret_cast<const uint4*>(dy + ((n * Ho + ho) * Wo + wo) * Cp + cb * 8), g);
      const int me = (h & 1) * 2 + (w & 1);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        int arg = 0;
        float m = v[0][j];
        for (int q = 1; q < 4; ++q) if (v[q][j] > m) { m = v[q][j]; arg = q; }
        out[j] = (arg == me && (!relu_mask || m > 0.f)) ? g[j] : 0.f;
      }
    }
    *reinterpret_cast<uint4*>(dx + ((n * H + h) * W + w) * Cp + cb * 8) = pack8(out);
  }
}

// ---------------------------------------------------------------------------
// host launchers (C ABI; stream = the caller's current hipStream_t)
// ---------------------------------------------------------------------------

extern "C" {

static int g_conv_mode = 0;   // single-input layers: 1 persistent / one-tile LDS-DMA, 2 one-tile LDS-DMA only, 0 register-staged (fastest measured: profiles/conv_modes.txt)
static unsigned long long* g_conv_stamps = nullptr;   // diagnostic: stamped LDS-DMA kernel
static int g_conv_wgs = 512;   // persistent conv: target workgroups per launch

int gt_conv_set_wgs(int n) {
  const int old = g_conv_wgs;
  if (n > 0) g_conv_wgs = n;
  return old;
}

int gt_conv_set_stamps(void* p) {
  g_conv_stamps = reinterpret_cast<unsigned long long*>(p);
  return 0;
}

int gt_conv_set_mode(int mode) {
  const int old = g_conv_mode;
  g_conv_mode = mode;
  return old;
}

int gt_conv_fwd(const ConvArgs* a, hipStream_t stream) {
  if (a->Cinp % 8 || a->Coutp % 8 || a->n_in < 1 || a->n_in > 4 || a->n_out < 1 || a->n_out > 4) return -1;
  if (a->TH * a->W > 256 || a->TH < 1) return -2;
  const int nth = (a->H + a->TH - 1) / a->TH;
  const size_t total = (size_t)(a->TH + a->KH - 1) * (a->W + a->KW - 1) * (a->Cinp / 8);
  const int nchunks = a->KH * a->KW * (a->Cinp / 8);
  const int nkb = (nchunks + CF_KB - 1) / CF_KB;
  const int wrows = ((std::min(64, a->Coutp) + 15) / 16) * 16;
  const size_t lds = (size_t)(nkb > 1 ? 2 : 1) * wrows * CF_WLD * 2 + total * 16 + 4 * ((size_t)nchunks + 4);
  if (lds > 160 * 1024) return -3;
  dim3 grid(a->B * nth, a->G, (a->Coutp + 63) / 64);
  if (g_conv_mode == 1 && a->n_in == 1 && !a->mask && !g_conv_stamps) {
    // persistent kernel when every weight block + 2 patch buffers fit a 2-per-CU share
    const size_t totalr = (total + 255) / 256 * 256;
    const size_t lds_p = (size_t)nkb * wrows * 256 + 2 * totalr * 16 + 4 * ((size_t)nchunks + 6) + 8 * CP_MAXT + 256;
    const int ntile = a->B * nth;
    const int per_fold = a->G * ((a->Coutp + 63) / 64);
    int nwg = (g_conv_wgs + per_fold - 1) / per_fold;
    if (nwg > ntile) nwg = ntile;
    if (nwg < (ntile + CP_MAXT - 1) / CP_MAXT) nwg = (ntile + CP_MAXT - 1) / CP_MAXT;
    if (lds_p <= 80 * 1024 && ntile >= 2 * nwg) {
      dim3 pg(nwg, a->G, (a->Coutp + 63) / 64);
      if (a->TH * a->W > 64)
        hipLaunchKernelGGL(conv_fwd_pers_kernel<2>, pg, dim3(256), lds_p, stream, *a);
      else
        hipLaunchKernelGGL(conv_fwd_pers_kernel<1>, pg, dim3(256), lds_p, stream, *a);
      return (int)hipGetLastError();
    }
  }
  if (g_conv_mode >= 1 && a->n_in == 1 && !a->mask) {
    const size_t totalr = (total + 255) / 256 * 256;
    const int fixed = (int)(totalr * 16 + 4 * ((size_t)nchunks + 4));
    const int NB = conv_glds_nbuf(nkb, wrows * 256, fixed, (long)grid.x * grid.y * grid.z);
    const size_t lds2 = (size_t)NB * wrows * 256 + fixed;
    if (lds2 > 160 * 1024) return -3;
    if (g_conv_stamps) {
      if (a->TH * a->W > 64)
        hipLaunchKernelGGL((conv_fwd_glds_kernel<2, true>), grid, dim3(256), lds2, stream, *a, g_conv_stamps);
      else
        hipLaunchKernelGGL((conv_fwd_glds_kernel<1, true>), grid, dim3(256), lds2, stream, *a, g_conv_stamps);
      return (int)hipGetLastError();
    }
    if (a->TH * a->W > 128)
      hipLaunchKernelGGL(conv_fwd_glds_kernel<4>, grid, dim3(256), lds2, stream, *a);
    else if (a->TH * a->W > 64)
      hipLaunchKernelGGL(conv_fwd_glds_kernel<2>, grid, dim3(256), lds2, stream, *a);
    else
      hipLaunchKernelGGL(conv_fwd_glds_kernel<1>, grid, dim3(256), lds2, stream, *a);
    return (int)hipGetLastError();
  }
  if (a->TH * a->W > 128)
    hipLaunchKernelGGL(conv_fwd_kernel<4>, grid, dim3(256), lds, stream, *a);
  else if (a->TH * a->W > 64)
    hipLaunchKernelGGL(conv_fwd_kernel<2>, grid, dim3(256), lds, stream, *a);
  else
    hipLaunchKernelGGL(conv_fwd_kernel<1>, grid, dim3(256), lds, stream, *a);
  return (int)hipGetLastError();
}

int gt_conv_wgrad(const WgradArgs* a, hipStream_t stream) {
  if (a->Cinp % 8 || a->Coutp % 8 || a->pps % 64 || a->n_in < 1 || a->n_in > 4) return -1;
  const int Kdim = a->KH * a->KW * a->Cinp;
  dim3 grid((Kdim + (a->part_b ? 8 : 0) + 63) / 64, a->S, a->G * ((a->Coutp + 63) / 64));
  hipLaunchKernelGGL(conv_wgrad_kernel, grid, dim3(256), 0, stream, *a);
  return (int)hipGetLastError();
}

int gt_pool_fwd(const uint16_t* x, uint16_t* y, int NB, int H, int W, int Cp, hipStream_t stream) {
  const long total = (long)NB * (H / 2) * (W / 2) * (Cp / 8);
  const int blocks = (int)std::min<long>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(pool_fwd_kernel, dim3(blocks), dim3(256), 0, stream, x, y, NB, H, W, Cp);
  return (int)hipGetLastError();
}

int gt_pool_bwd(const uint16_t* x, const uint16_t* dy, uint16_t* dx, int NB, int H, int W, int Cp, int relu_mask,
                hipStream_t stream) {
  const long total = (long)NB * H * W * (Cp / 8);
  const int blocks = (int)std::min<long>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(pool_bwd_kernel, dim3(blocks), dim3(256), 0, stream, x, dy, dx, NB, H, W, Cp,
                     relu_mask);
  return (int)hipGetLastError();
}

size_t gt_sizeof_conv_args() { return sizeof(ConvArgs); }
size_t gt_sizeof_wgrad_args() { return sizeof(WgradArgs); }

}  // extern "C"
