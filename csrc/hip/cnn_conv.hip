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

#include "cnn_args.h"

#define CF_KB 16                 // weight K-block: 16 chunks of 8 = 128 k
#define CF_WLD (CF_KB * 8 + 8)    // LDS row stride of a weight block (272 B: conflict-free b128 reads)

#ifndef CF_WPE
#define CF_WPE 5   // minimum waves per SIMD the register allocator must allow
#endif

template <int PXG, int PREC>   // 16-pixel groups per wave (tile = 64 * PXG pixels); precision (cnn_args.h)
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PREC ? 2 : (PXG == 4 ? 3 : CF_WPE))))
conv_fwd_kernel(ConvArgs a) {
  typedef typename ActT<PREC>::T AT;
  constexpr int NPL = PREC ? GT_NPL_F32 : 1;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  // tile = NI whole images (small images: the launcher passes TH = NI * H so
  // the weights staged per workgroup serve up to 256 pixels) or TH rows of one
  const int NI = a.TH > a.H ? a.TH / a.H : 1;
  const int THr = a.TH > a.H ? a.H : a.TH;            // rows per image in the tile
  const int nth = (a.H + THr - 1) / THr;
  const int b0 = (blockIdx.x / nth) * NI;
  const int h0 = (blockIdx.x % nth) * THr;
  const GroupRec gr = group_rec(a.gtab, blockIdx.y, a.n_in, a.n_out, a.acc_flags, a.out_mask);
  const int g = gr.g;
  const int co_blk = blockIdx.z * 64;
  const int ph = a.KH >> 1, pw = a.KW >> 1;
  const int PH = THr + a.KH - 1, PW = a.W + a.KW - 1;
  const int ncb_all = a.Cinp >> 3;
  // channel blocks: the patch holds ncb input chunks at a time (wide fp32
  // layers whose whole patch does not fit in LDS); accumulators persist
  const int ncb = a.cbb > 0 && a.cbb < ncb_all ? a.cbb : ncb_all;
  const int ncblk = (ncb_all + ncb - 1) / ncb;
  const long img = (long)a.H * a.W * a.Cinp;
  const int pimg = PH * PW * ncb;                       // patch chunks per image
  const int total = NI * pimg;                          // patch chunks per plane
  const int nchunks = a.KH * a.KW * ncb;                // k chunks per channel block
  const int Kdim = a.KH * a.KW * a.Cinp;
  // LDS carve: [weight blocks: NPL x nbuf x wrows x CF_WLD][patch: NPL x total][chunk offset table].
  // Only as many weight rows / buffers as this layer needs (occupancy).
  const int nkb = (nchunks + CF_KB - 1) / CF_KB;
  const int nbuf = nkb > 1 || ncblk > 1 ? 2 : 1;
  const int wrows = ((min(64, a.Coutp) + 15) >> 4) << 4;
  const int wplane = nbuf * wrows * CF_WLD;             // elements per weight plane
  const size_t wbytes = (size_t)NPL * wplane * 2;
  uint16_t* wbuf = reinterpret_cast<uint16_t*>(smem);
  uint4* patch = reinterpret_cast<uint4*>(smem + wbytes);
  int* coff = reinterpret_cast<int*>(smem + wbytes + (size_t)NPL * total * 16);
  const uint16_t* wg = a.w + (long)g * a.Coutp * Kdim;

  // weight-block staging role: row = tid >> 2 (up to 64 rows), 4 chunks per thread and plane
  const int wr = tid >> 2, wq = (tid & 3) * (CF_KB / 4);
  const bool wrow_live = wr < wrows;
  const bool wrow_ok = co_blk + wr < a.Coutp;
  const uint16_t* wsrc = wg + (long)(co_blk + wr) * Kdim;
  uint4 wreg[NPL][CF_KB / 4];
  const FastDiv div_ncb(ncb);
  auto load_wblock = [&](int kb, int cb0) {
#pragma unroll
    for (int q = 0; q < NPL; ++q)
#pragma unroll
      for (int j = 0; j < CF_KB / 4; ++j) {
        const int c = kb * CF_KB + wq + j;
        // block-local chunk (kh, kw, cb) -> the weight row's chunk (kh, kw, cb0 + cb)
        uint32_t kk, cb;
        div_ncb.divmod((uint32_t)c, kk, cb);
        const int cg = (int)kk * ncb_all + cb0 + (int)cb;
        wreg[q][j] = (wrow_ok && c < nchunks && cb0 + (int)cb < ncb_all)
                         ? *reinterpret_cast<const uint4*>(wsrc + q * a.wps + (long)cg * 8)
                         : make_uint4(0, 0, 0, 0);
      }
  };
  auto store_wblock = [&](int buf) {
    if (!wrow_live) return;
#pragma unroll
    for (int q = 0; q < NPL; ++q) {
      uint16_t* dst = wbuf + q * wplane + buf * wrows * CF_WLD + wr * CF_WLD + wq * 8;
#pragma unroll
      for (int j = 0; j < CF_KB / 4; ++j) *reinterpret_cast<uint4*>(dst + j * 8) = wreg[q][j];
    }
  };
  const int n_src = a.gather ? 1 : __builtin_popcount(gr.in_mask);
  const FastDiv div_pw(PW), div_pimg(pimg);
  const int wave = tid >> 6, lane = tid & 63;
  const int kq = lane >> 4, l16 = lane & 15;
  const int ipx = THr * a.W;                            // tile pixels per image
  int pbase[PXG];
  bool pvalid[PXG];
  int pyy[PXG], pxx[PXG], pim[PXG];
#pragma unroll
  for (int h = 0; h < PXG; ++h) {
    const int pl = wave * 16 * PXG + h * 16 + l16;
    pim[h] = pl / ipx;
    const int pp = pl - pim[h] * ipx;
    pyy[h] = pp / a.W; pxx[h] = pp % a.W;
    pvalid[h] = (pl < NI * ipx) && (h0 + pyy[h] < a.H) && (b0 + pim[h] < a.B);
    pbase[h] = pim[h] * pimg + (pyy[h] * PW + pxx[h]) * ncb;
  }
  const int nco = min(64, a.Coutp - co_blk);
  const int NT = (nco + 15) >> 4;
  f32x4_t acc[PXG][4];
#pragma unroll
  for (int h = 0; h < PXG; ++h)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[h][t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
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

  for (int blk = 0; blk < ncblk; ++blk) {
  const int cb0 = blk * ncb;
  load_wblock(0, cb0);

  // ---- stage the summed / masked input patch of every image ----------------
  for (int i = tid; i < total; i += 256) {
    uint32_t im, r, pix, cbu, pr, pc;
    div_pimg.divmod((uint32_t)i, im, r);
    div_ncb.divmod(r, pix, cbu);
    div_pw.divmod(pix, pr, pc);
    const int cb = cb0 + (int)cbu, b = b0 + (int)im;
    const int hh = h0 - ph + (int)pr, ww = (int)pc - pw;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    uint4 v = make_uint4(0, 0, 0, 0);
    bool raw = false;                                   // prec 0 single source: v holds the bf16 chunk as is
    if (b < a.B && hh >= 0 && hh < a.H && ww >= 0 && ww < a.W && cb < ncb_all) {
      const long off = ((long)hh * a.W + ww) * a.Cinp + cb * 8;
      const long ioff = ((long)g * a.B + b) * img;
      const AT* msrc = a.mask ? static_cast<const AT*>(a.mask) + ioff : nullptr;
      if (a.gather) {
        const AT* src = static_cast<const AT*>(a.in[0]) + a.gather[((long)a.st->cur_step * a.G + g) * a.B + b] * img + off;
        if (PREC) ld_chunk(src, acc); else { v = *reinterpret_cast<const uint4*>(src); raw = true; }
      } else if (n_src == 1 && !msrc) {
        const AT* src = static_cast<const AT*>(a.in[__builtin_ctz(gr.in_mask | 0x100) & 7]) + ioff + off;
        if (PREC) ld_chunk(src, acc); else { v = *reinterpret_cast<const uint4*>(src); raw = true; }
      } else {
        float t[8];
        for (int k = 0; k < GT_MAXSLOT; ++k) {
          if (!((gr.in_mask >> k) & 1)) continue;
          ld_chunk(static_cast<const AT*>(a.in[k]) + ioff + off, t);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] += t[j];
        }
        if (msrc) {
          ld_chunk(msrc + off, t);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] = t[j] > 0.f ? acc[j] : 0.f;
        }
      }
    }
    if (PREC) {
      split8(acc, patch[i], patch[total + i], patch[2 * total + i]);
    } else {
      patch[i] = raw ? v : pack8(acc);
    }
  }
  if (a.xsum && n_src > 1) {
    // the summed input of this tile (patch interiors) for the layer's wgrad
    __syncthreads();
    const int per = THr * a.W * ncb;
    for (int i = tid; i < NI * per; i += 256) {
      const int im = i / per, q = i - im * per;
      const int cb = q % ncb, pix = q / ncb;
      const int r = pix / a.W, cc = pix % a.W;
      if (b0 + im < a.B && h0 + r < a.H && cb0 + cb < ncb_all) {
        AT* xo = static_cast<AT*>(a.xsum) + ((long)g * a.B + b0 + im) * img +
                 (((long)h0 * a.W + pix) * ncb_all + cb0 + cb) * 8;
        const int pi = im * pimg + ((r + ph) * PW + cc + pw) * ncb + cb;
        if (PREC) {
          float f[8];
          join8(patch[pi], patch[total + pi], patch[2 * total + pi], f);
          st_chunk(xo, f);
        } else {
          *reinterpret_cast<uint4*>(xo) = patch[pi];
        }
      }
    }
  }
  store_wblock(0);
  __syncthreads();

  // ---- MFMA main loop: each wave = 16*PXG pixels x all co tiles --------------
  for (int kb = 0; kb < nkb; ++kb) {
    const bool more = kb + 1 < nkb;
    if (more) load_wblock(kb + 1, cb0);
    const uint16_t* wcur = wbuf + (kb & 1) * wrows * CF_WLD;
#pragma unroll
    for (int kk = 0; kk < CF_KB / 4; ++kk) {
      const int c = kb * CF_KB + kk * 4 + kq;
      if (kb * CF_KB + kk * 4 >= nchunks) break;
      const int co_off = coff[c];
      uint4 bfr[PXG][NPL];
#pragma unroll
      for (int h = 0; h < PXG; ++h)
#pragma unroll
        for (int q = 0; q < NPL; ++q)
          bfr[h][q] = (co_off >= 0 && pvalid[h]) ? patch[q * total + pbase[h] + co_off] : make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (t < NT) {
          uint4 af[NPL];
#pragma unroll
          for (int q = 0; q < NPL; ++q)
            af[q] = *reinterpret_cast<const uint4*>(wcur + q * wplane + (t * 16 + l16) * CF_WLD + (kk * 4 + kq) * 8);
#pragma unroll
          for (int h = 0; h < PXG; ++h) acc[h][t] = mfma_np<NPL>(af, bfr[h], acc[h][t]);
        }
      }
    }
    if (more) store_wblock((kb + 1) & 1);
    __syncthreads();
  }
  }  // channel blocks

  // ---- epilogue: bias + relu, 4 channels per lane ---------------------------
#pragma unroll
  for (int h = 0; h < PXG; ++h) {
    if (!pvalid[h]) continue;
    const long obase = ((((long)g * a.B + b0 + pim[h]) * a.H + (h0 + pyy[h])) * a.W + pxx[h]) * a.Coutp;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      if (t >= NT) continue;
      const int co0 = co_blk + t * 16 + kq * 4;
      if (co0 >= a.Coutp) continue;
      float v[4];
      // zero-padded image (ConvArgs::Hr / Wr): exact zeros outside the real rows / columns
      const bool pad0 = a.Hr > 0 && (h0 + pyy[h] >= a.Hr || pxx[h] >= a.Wr);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float x = acc[h][t][i];
        if (a.bias) x += a.bias[(long)g * a.Coutp + co0 + i];
        if (a.relu) x = fmaxf(x, 0.f);
        v[i] = pad0 ? 0.f : x;
      }
      for (int k = 0; k < GT_MAXSLOT; ++k) {
        if (!((gr.out_mask >> k) & 1)) continue;
        AT* dst = static_cast<AT*>(a.out[k]) + obase + co0;
        float sum[4] = {v[0], v[1], v[2], v[3]};
        float o[4];
        if ((gr.out_mask >> (8 + k)) & 1) {
          if (PREC) { const float4 q = *reinterpret_cast<const float4*>(dst); o[0] = q.x; o[1] = q.y; o[2] = q.z; o[3] = q.w; }
          else { const uint2 q = *reinterpret_cast<const uint2*>(dst);
                 o[0] = __uint_as_float(q.x << 16); o[1] = __uint_as_float(q.x & 0xffff0000u);
                 o[2] = __uint_as_float(q.y << 16); o[3] = __uint_as_float(q.y & 0xffff0000u); }
#pragma unroll
          for (int i = 0; i < 4; ++i) sum[i] += o[i];
        }
        if ((gr.out_mask >> (16 + k)) & 1) {
          const AT* msrc = static_cast<const AT*>(a.out_mask[k]) + obase + co0;
          if (PREC) { const float4 q = *reinterpret_cast<const float4*>(msrc); o[0] = q.x; o[1] = q.y; o[2] = q.z; o[3] = q.w; }
          else { const uint2 q = *reinterpret_cast<const uint2*>(msrc);
                 o[0] = __uint_as_float(q.x << 16); o[1] = __uint_as_float(q.x & 0xffff0000u);
                 o[2] = __uint_as_float(q.y << 16); o[3] = __uint_as_float(q.y & 0xffff0000u); }
#pragma unroll
          for (int i = 0; i < 4; ++i) sum[i] = o[i] > 0.f ? sum[i] : 0.f;
        }
        if (PREC) *reinterpret_cast<float4*>(dst) = make_float4(sum[0], sum[1], sum[2], sum[3]);
        else *reinterpret_cast<uint2*>(dst) = pack4(sum);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// weight gradient (split-K, deterministic partials)
// ---------------------------------------------------------------------------

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
// PREC 1: the chunks are fp32, staged as three exact bf16 planes per tile.
template <int PREC>
__global__ void __launch_bounds__(256) conv_wgrad_kernel(WgradArgs a) {
  typedef typename ActT<PREC>::T AT;
  constexpr int NPL = PREC ? GT_NPL_F32 : 1;
  __shared__ __attribute__((aligned(16))) uint16_t lds[2 * 2 * NPL * WG_TILE];   // 2 buffers x (dz, im2col) x planes
  const int tid = threadIdx.x;
  const int nb = blockIdx.x;
  const int s = blockIdx.y;
  const int mblocks = (a.Coutp + 63) / 64;
  const GroupRec gr = group_rec(a.gtab, blockIdx.z / mblocks, a.n_in, 0, 0, nullptr);
  const int g = gr.g;
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
  auto tile = [&](int bf, int which, int q) { return lds + ((bf * 2 + which) * NPL + q) * WG_TILE; };

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
  const AT* fold_in[GT_MAXSLOT];
  int n_src = 0;
  for (int k = 0; k < GT_MAXSLOT; ++k)
    if ((gr.in_mask >> k) & 1) fold_in[n_src++] = static_cast<const AT*>(a.in[k]) + (long)g * a.B * HW * a.Cinp;
  const long fold_out = (long)g * npix * a.Coutp;
  const AT* dzp = static_cast<const AT*>(a.dz);

  const int MT = (min(64, a.Coutp - co_blk) + 15) >> 4;
  const bool wave_live = nb * 64 + wave * 16 <= Kdim;
  f32x4_t acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  float dzf[2][8], xsf[2][8];
  auto load_step = [&](long p0) {
    // dz (masked by the layer's own ReLU output)
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int i = tid + 256 * r;
#pragma unroll
      for (int e = 0; e < 8; ++e) dzf[r][e] = 0.f;
      if (i < ndz) {
        uint32_t px, cc;
        div_ncc.divmod((uint32_t)i, px, cc);
        const long p = p0 + px;
        if (p < p_end) ld_chunk(dzp + fold_out + p * a.Coutp + co_blk + cc * 8, dzf[r]);
      }
    }
    // im2col: lane = pixel
    const long p = p0 + lane;
    uint32_t bq = 0, rem = 0, hq = 0, wq = 0;
    if (p < p_end) { div_hw.divmod((uint32_t)p, bq, rem); div_w.divmod(rem, hq, wq); }
    const AT* gimg = nullptr;
    if (a.gather && p < p_end)
      gimg = static_cast<const AT*>(a.in[0]) + a.gather[((long)a.st->cur_step * a.G + g) * a.B + bq] * HW * a.Cinp;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
#pragma unroll
      for (int e = 0; e < 8; ++e) xsf[r][e] = 0.f;
      if (c_one[r] && p < p_end) xsf[r][0] = 1.f;              // 1.0 in element 0 (exact in every plane split)
      const int ih = (int)hq + c_kh[r], iw = (int)wq + c_kw[r];
      if (p < p_end && c_ok[r] && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W) {
        const long pix_off = ((long)ih * a.W + iw) * a.Cinp + c_cb[r] * 8;
        if (gimg) {
          ld_chunk(gimg + pix_off, xsf[r]);
        } else {
          float t[8];
          for (int k = 0; k < n_src; ++k) {
            ld_chunk(fold_in[k] + (long)bq * HW * a.Cinp + pix_off, t);
#pragma unroll
            for (int j = 0; j < 8; ++j) xsf[r][j] += t[j];
          }
        }
      }
    }
  };
  auto put = [&](uint16_t* t0, int off, const float* f) {
    if (PREC) {
      uint4 p0, p1, p2;
      split8(f, p0, p1, p2);
      *reinterpret_cast<uint4*>(t0 + off) = p0;
      *reinterpret_cast<uint4*>(t0 + WG_TILE + off) = p1;
      *reinterpret_cast<uint4*>(t0 + 2 * WG_TILE + off) = p2;
    } else {
      *reinterpret_cast<uint4*>(t0 + off) = pack8(f);
    }
  };
  auto store_step = [&](int bf) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int i = tid + 256 * r;
      if (i < ndz) {
        uint32_t px, cc;
        div_ncc.divmod((uint32_t)i, px, cc);
        put(tile(bf, 0, 0), px * WG_LD + cc * 8, dzf[r]);
      }
      put(tile(bf, 1, 0), lane * WG_LD + (wave + 4 * r) * 8, xsf[r]);
    }
  };
  // dz columns beyond this block's channels must read as zero
  if (ncc < 8) {
    for (int i = tid; i < 2 * NPL * 64 * (8 - ncc); i += 256) {
      const int per = 64 * (8 - ncc);
      const int bq = i / per, rem = i % per;          // bq = buffer * NPL + plane
      const int px = rem / (8 - ncc), cc = ncc + rem % (8 - ncc);
      *reinterpret_cast<uint4*>(tile(bq / NPL, 0, bq % NPL) + px * WG_LD + cc * 8) = make_uint4(0, 0, 0, 0);
    }
  }
  load_step(p_begin);
  store_step(0);
  __syncthreads();
  int buf = 0;
  for (long p0 = p_begin; p0 < p_end; p0 += 64) {
    const bool more = p0 + 64 < p_end;
    if (more) load_step(p0 + 64);
    if (wave_live) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        uint4 bfrag[NPL];
#pragma unroll
        for (int q = 0; q < NPL; ++q) bfrag[q] = tr_frag(tile(buf, 1, q) + h * 32 * WG_LD, wave * 16, lane);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          if (t < MT) {
            uint4 afrag[NPL];
#pragma unroll
            for (int q = 0; q < NPL; ++q) afrag[q] = tr_frag(tile(buf, 0, q) + h * 32 * WG_LD, t * 16, lane);
            acc[t] = mfma_np<NPL>(afrag, bfrag, acc[t]);
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
// 2x2/2 max-pool (floor) and its backward scatter. Per group the source slot
// is x0 or x1 (sel[g]): a stage without a DAG pools its input conv, a stage
// with one pools its output conv. AT = bf16 (uint16_t) or fp32 storage.
// ---------------------------------------------------------------------------

template <typename AT>
__global__ void pool_fwd_kernel(const AT* __restrict__ x0, const AT* __restrict__ x1,
                                const int* __restrict__ sel, AT* __restrict__ y, int NB, int B, int H, int W,
                                int Cp, uint8_t* __restrict__ mask) {
  const int Ho = H >> 1, Wo = W >> 1, ncb = Cp >> 3;
  const uint32_t total = (uint32_t)NB * Ho * Wo * ncb;       // < 2^31 (host-checked): 32-bit index math
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int cb = (int)(i % ncb);
    uint32_t r = i / ncb;
    const int wo = (int)(r % Wo); r /= Wo;
    const int ho = (int)(r % Ho);
    const long n = r / Ho;
    const AT* x = (sel && sel[n / B]) ? x1 : x0;
    const AT* base = x + ((n * H + 2 * ho) * W + 2 * wo) * Cp + cb * 8;
    float m[8], t[8];
    int arg[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    ld_chunk(base, m);
    const long offs[3] = {(long)Cp, (long)W * Cp, (long)W * Cp + Cp};
    for (int q = 0; q < 3; ++q) {
      ld_chunk(base + offs[q], t);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (t[j] > m[j]) { m[j] = t[j]; arg[j] = q + 1; }      // first strict maximum, as pool_bwd_kernel
    }
    const long o = ((n * Ho + ho) * Wo + wo) * Cp + cb * 8;
    st_chunk(y + o, m);
    if (mask) {
      // per channel: bits 0-1 = which of the 4 cell pixels holds the maximum, bit 2 = maximum > 0
      uint32_t lo = 0, hi = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) lo |= (uint32_t)(arg[j] | (m[j] > 0.f ? 4 : 0)) << (8 * j);
#pragma unroll
      for (int j = 0; j < 4; ++j) hi |= (uint32_t)(arg[4 + j] | (m[4 + j] > 0.f ? 4 : 0)) << (8 * j);
      *reinterpret_cast<uint2*>(mask + o) = make_uint2(lo, hi);
    }
  }
}

// dx[pixel] = dy[pool cell] if pixel is the cell's first maximum (and, with
// relu_mask, the maximum is > 0) else 0; dx / x slot chosen per group by sel
template <typename AT>
__global__ void pool_bwd_kernel(const AT* __restrict__ x0, const AT* __restrict__ x1,
                                const int* __restrict__ sel, const AT* __restrict__ dy,
                                AT* __restrict__ dx0, AT* __restrict__ dx1, int NB, int B, int H, int W,
                                int Cp, int relu_mask) {
  const int Ho = H >> 1, Wo = W >> 1, ncb = Cp >> 3;
  const uint32_t total = (uint32_t)NB * H * W * ncb;         // < 2^31 (host-checked): 32-bit index math
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int cb = (int)(i % ncb);
    uint32_t r = i / ncb;
    const int w = (int)(r % W); r /= W;
    const int h = (int)(r % H);
    const long n = r / H;
    const bool s1 = sel && sel[n / B];
    const AT* x = s1 ? x1 : x0;
    AT* dx = s1 ? dx1 : dx0;
    float out[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int ho = h >> 1, wo = w >> 1;
    if (ho < Ho && wo < Wo) {
      const AT* base = x + ((n * H + 2 * ho) * W + 2 * wo) * Cp + cb * 8;
      float v[4][8];
      ld_chunk(base, v[0]);
      ld_chunk(base + Cp, v[1]);
      ld_chunk(base + (long)W * Cp, v[2]);
      ld_chunk(base + (long)W * Cp + Cp, v[3]);
      float g[8];
      ld_chunk(dy + ((n * Ho + ho) * Wo + wo) * Cp + cb * 8, g);
      const int me = (h & 1) * 2 + (w & 1);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        int arg = 0;
        float m = v[0][j];
        for (int q = 1; q < 4; ++q) if (v[q][j] > m) { m = v[q][j]; arg = q; }
        out[j] = (arg == me && (!relu_mask || m > 0.f)) ? g[j] : 0.f;
      }
    }
    st_chunk(dx + ((n * H + h) * W + w) * Cp + cb * 8, out);
  }
}

// Backward scatter from the forward's argmax mask (1 byte per pooled channel
// instead of re-reading the 4 cell inputs: the pool_bwd traffic drops from
// x + dy + dx to mask + dy + dx). Same first-maximum rule, so dx is identical
// to pool_bwd_kernel's.
template <typename AT>
__global__ void pool_bwd_mask_kernel(const uint8_t* __restrict__ mask, const int* __restrict__ sel,
                                     const AT* __restrict__ dy, AT* __restrict__ dx0,
                                     AT* __restrict__ dx1, int NB, int B, int H, int W, int Cp, int relu_mask) {
  const int Ho = H >> 1, Wo = W >> 1, ncb = Cp >> 3;
  const uint32_t total = (uint32_t)NB * H * W * ncb;         // < 2^31 (host-checked): 32-bit index math
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int cb = (int)(i % ncb);
    uint32_t r = i / ncb;
    const int w = (int)(r % W); r /= W;
    const int h = (int)(r % H);
    const long n = r / H;
    AT* dx = (sel && sel[n / B]) ? dx1 : dx0;
    float out[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int ho = h >> 1, wo = w >> 1;
    if (ho < Ho && wo < Wo) {
      const long o = ((n * Ho + ho) * Wo + wo) * Cp + cb * 8;
      const uint2 mk = *reinterpret_cast<const uint2*>(mask + o);
      float g[8];
      ld_chunk(dy + o, g);
      const uint32_t me = (uint32_t)((h & 1) * 2 + (w & 1));
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t b = ((j < 4 ? mk.x : mk.y) >> (8 * (j & 3))) & 0xffu;
        out[j] = ((b & 3u) == me && (!relu_mask || (b & 4u))) ? g[j] : 0.f;
      }
    }
    st_chunk(dx + ((n * H + h) * W + w) * Cp + cb * 8, out);
  }
}

// ---------------------------------------------------------------------------
// host launchers (C ABI; stream = the caller's current hipStream_t)
// ---------------------------------------------------------------------------

extern "C" int gt_conv_fast(const ConvArgs* a, hipStream_t stream);
extern "C" int gt_wgrad_fast(const WgradArgs* a, hipStream_t stream);

static int g_conv_fast = 1;   // shape-specialised kernels (cnn_conv_fast.hip) where one matches
static int g_conv_imgs = 2;   // max whole small images per generic-conv workgroup (2: measured best, deep space)

template <typename F>
static void set_lds_limit(F* fn, size_t bytes) {
  if (bytes > 65536) (void)hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)bytes);
}

template <int PREC>
static int conv_fwd_generic(const ConvArgs* a, hipStream_t stream) {
  constexpr int NPL = PREC ? GT_NPL_F32 : 1;
  const int nchunks = a->KH * a->KW * (a->Cinp / 8);
  const int nkb = (nchunks + CF_KB - 1) / CF_KB;
  const int wrows = ((std::min(64, a->Coutp) + 15) / 16) * 16;
  auto lds_of = [&](int ni, int th) {
    const size_t total = (size_t)ni * (th + a->KH - 1) * (a->W + a->KW - 1) * (a->Cinp / 8);
    return (size_t)NPL * ((size_t)(nkb > 1 ? 2 : 1) * wrows * CF_WLD * 2 + total * 16) + 4 * ((size_t)nchunks + 4);
  };
  // small images: several whole images per workgroup (up to 256 pixels), so
  // one staged weight block serves 4x the pixels (8x8 stages: weight traffic
  // per image was 6x the patch's)
  int ni = 1;
  if (a->TH == a->H && 2 * a->H * a->W <= 256) {
    ni = std::min(g_conv_imgs, 256 / (a->H * a->W));
    while (ni > 1 && lds_of(ni, a->H) > 160 * 1024) --ni;
  }
  ConvArgs t = *a;
  t.cbb = 0;
  // fp32 planes triple the patch: shrink the row band to >= 128-pixel tiles,
  // then stage the input channels block by block
  while (ni == 1 && lds_of(1, t.TH) > 160 * 1024 && t.TH > 1 && (t.TH / 2) * a->W >= 128) t.TH = (t.TH + 1) / 2;
  if (lds_of(ni, t.TH) > 160 * 1024) {
    ni = 1;
    t.TH = a->TH;
    const int ncb = a->Cinp / 8;
    for (int cbb : {16, 8, 4, 2, 1}) {
      if (cbb >= ncb) continue;
      const size_t w = (size_t)NPL * 2 * wrows * CF_WLD * 2;
      const size_t p = (size_t)NPL * (t.TH + a->KH - 1) * (a->W + a->KW - 1) * cbb * 16;
      if (w + p + 4 * ((size_t)a->KH * a->KW * cbb + 4) <= 160 * 1024) { t.cbb = cbb; break; }
    }
    if (!t.cbb) return -3;
  }
  if (ni > 1) t.TH = ni * a->H;                      // kernel: TH > H = ni whole images per tile
  const int nth = ni > 1 ? 1 : (a->H + t.TH - 1) / t.TH;
  const int tile = ni > 1 ? ni * a->H * a->W : t.TH * a->W;
  size_t lds = lds_of(ni, ni > 1 ? a->H : t.TH);
  if (t.cbb) lds = (size_t)NPL * (2 * wrows * CF_WLD * 2 + (size_t)(t.TH + a->KH - 1) * (a->W + a->KW - 1) * t.cbb * 16) +
                   4 * ((size_t)a->KH * a->KW * t.cbb + 4);
  dim3 grid(((a->B + ni - 1) / ni) * nth, a->ngroups, (a->Coutp + 63) / 64);
  if (tile > 128) {
    set_lds_limit(conv_fwd_kernel<4, PREC>, lds);
    hipLaunchKernelGGL((conv_fwd_kernel<4, PREC>), grid, dim3(256), lds, stream, t);
  } else if (tile > 64) {
    set_lds_limit(conv_fwd_kernel<2, PREC>, lds);
    hipLaunchKernelGGL((conv_fwd_kernel<2, PREC>), grid, dim3(256), lds, stream, t);
  } else {
    set_lds_limit(conv_fwd_kernel<1, PREC>, lds);
    hipLaunchKernelGGL((conv_fwd_kernel<1, PREC>), grid, dim3(256), lds, stream, t);
  }
  return (int)hipGetLastError();
}

extern "C" {

int gt_conv_set_imgs(int n) {
  const int old = g_conv_imgs;
  g_conv_imgs = n < 1 ? 1 : n;
  return old;
}

int gt_conv_set_fast(int on) {
  const int old = g_conv_fast;
  g_conv_fast = on;
  return old;
}

int gt_conv_wino(const ConvArgs* a, hipStream_t stream, int probe);

int gt_conv_fwd(const ConvArgs* a, hipStream_t stream) {
  if (a->wino) return gt_conv_wino(a, stream, 0);   // transformed weight planes: Winograd kernels only
  if (a->Cinp % 8 || a->Coutp % 8) return -1;
  if (a->prec != 0 && a->prec != 1) return -1;
  if (g_conv_fast && a->ngroups >= 1) {
    const int rc = gt_conv_fast(a, stream);
    if (rc != -100) return rc;
  }
  if (a->wfrag) return -102;                 // fragment-major planes: shape-specialised kernels only
  if (a->pool_y) return -60;                 // fused pool / un-pool: shape-specialised kernels only (gt_conv_fast_probe)
  if (!a->gtab && (a->n_in < 1 || a->n_in > GT_MAXSLOT || a->n_out < 1 || a->n_out > GT_MAXSLOT)) return -1;
  if (a->TH * a->W > 256 || a->TH < 1 || a->TH > a->H) return -2;
  if (a->ngroups < 1) return 0;
  return a->prec ? conv_fwd_generic<1>(a, stream) : conv_fwd_generic<0>(a, stream);
}

int gt_conv_wgrad(const WgradArgs* a, hipStream_t stream) {
  if (a->Cinp % 8 || a->Coutp % 8 || a->pps % 64) return -1;
  if (a->prec != 0 && a->prec != 1) return -1;
  if (!a->gtab && (a->n_in < 1 || a->n_in > GT_MAXSLOT)) return -1;
  if (a->ngroups < 1) return 0;
  if (g_conv_fast) {
    const int rc = gt_wgrad_fast(a, stream);
    if (rc != -100) return rc;
  }
  const int Kdim = a->KH * a->KW * a->Cinp;
  dim3 grid((Kdim + (a->part_b ? 8 : 0) + 63) / 64, a->S, a->ngroups * ((a->Coutp + 63) / 64));
  if (a->prec)
    hipLaunchKernelGGL(conv_wgrad_kernel<1>, grid, dim3(256), 0, stream, *a);
  else
    hipLaunchKernelGGL(conv_wgrad_kernel<0>, grid, dim3(256), 0, stream, *a);
  return (int)hipGetLastError();
}

// pool launchers: prec 0 = bf16 tensors, 1 = fp32
#define POOL_GRID(total) dim3((int)std::min<long>(((total) + 255) / 256, 16384))

int gt_pool_fwd(const void* x0, const void* x1, const int* sel, void* y, int NB, int B, int H, int W, int Cp,
                int prec, hipStream_t stream) {
  const long total = (long)NB * (H / 2) * (W / 2) * (Cp / 8);
  if ((long)NB * H * W * (Cp / 8) >= (1L << 31)) return -4;
  if (prec)
    hipLaunchKernelGGL(pool_fwd_kernel<float>, POOL_GRID(total), dim3(256), 0, stream, (const float*)x0,
                       (const float*)x1, sel, (float*)y, NB, B, H, W, Cp, (uint8_t*)nullptr);
  else
    hipLaunchKernelGGL(pool_fwd_kernel<uint16_t>, POOL_GRID(total), dim3(256), 0, stream, (const uint16_t*)x0,
                       (const uint16_t*)x1, sel, (uint16_t*)y, NB, B, H, W, Cp, (uint8_t*)nullptr);
  return (int)hipGetLastError();
}

// training forward: also writes the argmax mask [NB][H/2][W/2][Cp] (uint8) for gt_pool_bwd_mask
int gt_pool_fwd_mask(const void* x0, const void* x1, const int* sel, void* y, int NB, int B, int H, int W, int Cp,
                     uint8_t* mask, int prec, hipStream_t stream) {
  const long total = (long)NB * (H / 2) * (W / 2) * (Cp / 8);
  if ((long)NB * H * W * (Cp / 8) >= (1L << 31)) return -4;
  if (Cp % 8 || mask == nullptr) return -1;
  if (prec)
    hipLaunchKernelGGL(pool_fwd_kernel<float>, POOL_GRID(total), dim3(256), 0, stream, (const float*)x0,
                       (const float*)x1, sel, (float*)y, NB, B, H, W, Cp, mask);
  else
    hipLaunchKernelGGL(pool_fwd_kernel<uint16_t>, POOL_GRID(total), dim3(256), 0, stream, (const uint16_t*)x0,
                       (const uint16_t*)x1, sel, (uint16_t*)y, NB, B, H, W, Cp, mask);
  return (int)hipGetLastError();
}

int gt_pool_bwd_mask(const uint8_t* mask, const int* sel, const void* dy, void* dx0, void* dx1, int NB, int B,
                     int H, int W, int Cp, int relu_mask, int prec, hipStream_t stream) {
  const long total = (long)NB * H * W * (Cp / 8);
  if (total >= (1L << 31)) return -4;
  if (Cp % 8 || mask == nullptr) return -1;
  if (prec)
    hipLaunchKernelGGL(pool_bwd_mask_kernel<float>, POOL_GRID(total), dim3(256), 0, stream, mask, sel,
                       (const float*)dy, (float*)dx0, (float*)dx1, NB, B, H, W, Cp, relu_mask);
  else
    hipLaunchKernelGGL(pool_bwd_mask_kernel<uint16_t>, POOL_GRID(total), dim3(256), 0, stream, mask, sel,
                       (const uint16_t*)dy, (uint16_t*)dx0, (uint16_t*)dx1, NB, B, H, W, Cp, relu_mask);
  return (int)hipGetLastError();
}

int gt_pool_bwd(const void* x0, const void* x1, const int* sel, const void* dy, void* dx0, void* dx1, int NB, int B,
                int H, int W, int Cp, int relu_mask, int prec, hipStream_t stream) {
  const long total = (long)NB * H * W * (Cp / 8);
  if (total >= (1L << 31)) return -4;
  if (prec)
    hipLaunchKernelGGL(pool_bwd_kernel<float>, POOL_GRID(total), dim3(256), 0, stream, (const float*)x0,
                       (const float*)x1, sel, (const float*)dy, (float*)dx0, (float*)dx1, NB, B, H, W, Cp, relu_mask);
  else
    hipLaunchKernelGGL(pool_bwd_kernel<uint16_t>, POOL_GRID(total), dim3(256), 0, stream, (const uint16_t*)x0,
                       (const uint16_t*)x1, sel, (const uint16_t*)dy, (uint16_t*)dx0, (uint16_t*)dx1, NB, B, H, W,
                       Cp, relu_mask);
  return (int)hipGetLastError();
}

size_t gt_sizeof_conv_args() { return sizeof(ConvArgs); }
size_t gt_sizeof_wgrad_args() { return sizeof(WgradArgs); }

}  // extern "C"
