// Shape-specialised fp32 / bf16 conv and weight-gradient KERNEL TEMPLATES (device code), shared by the
// dispatch translation units cnn_conv_fast.hip (the S=(3,5) / deep / wide search-space shapes) and
// cnn_conv_fast_ext.hip (user-chosen architectures: 32/64-channel stages, 3x3 stage-input kernels),
// which compile in parallel. Moved verbatim from cnn_conv_fast.hip (round 6).
#pragma once
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

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "cnn_args.h"

// Rejected variants are recorded in profiles/ and were removed from the source (round 5): branch-free
// staging selects (conv_stage_select_ab_r3.txt), register-computed / register-held patch offsets and deeper
// weight prefetch (conv_f32_regoff_pf_ab_r4.txt, conv_f32_kreg_ab_r4.txt), the unpipelined fp32 loop, the
// round-3 two-team "duo" and persistent kernels and the round-5 fixed-role "pipe" kernel
// (conv_f32_duo_ab_r3.txt, conv_f32_persistent_ab_r2.txt, r5/conv_f32_sched_pipe_ab_r5.txt).

// a value the compiler cannot see through (nor hoist computations on it out of a loop)
__device__ __forceinline__ int opaque_i(int x) {
  asm volatile("" : "+v"(x));
  return x;
}

// The stage-2 3x3 fp32 shape (7 input chunks, 16 wide) reduces its chunks PART-MAJOR -- (kh, kw, cb)
// for cb 0-3, then for cb 4-6 -- in every kernel that runs it (so the small-launch tiles stay
// bit-identical to the 8-row one): +2.6 % per population step over the kk-major order
// (profiles/conv_s2_parts_split_ab_r4.txt; a two-part staging kernel built on it and a bank-paired order
// were slower, same file and conv_s2_bank_order_ab_r4.txt).
template <int KH, int KW, int NCBI, int W, int PREC>
struct S2Parts {
  static constexpr bool on = PREC == 1 && NCBI == 7 && W == 16 && KH == 3 && KW == 3;
  static constexpr int e0 = KH * KW * 4;     // chunk-list entries of part 0 (every tap x chunks 0-3)
};

// LDS bytes of one launch: the patch (NPL bf16 planes) or the output tile
// (fp32, or bf16 for prec-0 forward launches -- measured 7-9 % faster: more
// workgroups per CU), whichever is larger
template <int KH, int KW, int NCBI, int W, int TH, int NT, int NCO, int PREC>
struct FastCfg {
  static constexpr int NPL = PREC ? GT_NPL_F32 : 1;
  static constexpr int PW = W + KW - 1;
  static constexpr int NP = (TH + KH - 1) * PW * NCBI;
  // LDS pixel stride of the patch in 16-byte chunks: odd (an even stride -- 8, 16, 32 chunks of
  // the wide deep space -- put every lane of a ds_read_b128 pass on the same banks: 8-16 way
  // conflicts, PMC LDSbc 0.7-0.86 on those launches); the S=(3,5) / (20,50,100) strides are odd already
  static constexpr int NCBP = NCBI + ((NCBI & 1) ? 0 : 1);
  // PAIR layout (fp32 shapes with >= 2 input chunks): chunk PAIRS (cb 2j, 2j+1) of every pixel side by side,
  // pixel stride 2 chunks, one pair-plane of PP2 chunks per j. A ds_read_b128 lane group holds 8 pixels of k
  // entry kq and 8 of kq+1; when those entries are chunks of opposite parity (cb, cb+1 of one tap: every
  // k-step of the part-major stage-2 order, most of the kk-major ones) the 16 addresses fall on 16 different
  // 16-byte bank quads (2 x pixel is even, the chunk parity adds 0 / 1). With the pixel-major odd stride
  // NCBP, seven of the eight lane pairs met on one quad: every patch read took 2 LDS passes (PMC LDSbc
  // 0.47 on the stage-2 conv, profiles/r5/pmc_step_fp32_p5_final_r5.txt). PP2 mod 8 is picked per chunk count
  // for the fewest read, then write, conflicts (tools/lds_patch_sim.py models every lane group of the reads
  // and the staging writes).
  static constexpr int NPIX = (TH + KH - 1) * PW;
  static constexpr int PPR = (S2Parts<KH, KW, NCBI, W, PREC>::on || NCBI == 3) ? 5 : (NCBI % 2 == 0) ? (NCBI == 4 ? 4 : 2) : 6;
  static constexpr int PP2 = 2 * NPIX + ((PPR - (2 * NPIX) % 8) + 8) % 8;
  static constexpr int TP = TH * W;
  static constexpr int OROW = NT * 16 + 4;          // fp32 tile row (floats; conflict-free float4 writes)
  static constexpr int OROWB = NT * 16 + 8;         // bf16 tile row (elements; conflict-free 8-byte writes)
  static constexpr int NPL_ = PREC ? GT_NPL_F32 : 1;
  static constexpr long OTILE = (long)TP * OROW * 4;
  static constexpr long LDS_PM = (long)NPIX * NCBP * 16 * NPL_ > OTILE ? (long)NPIX * NCBP * 16 * NPL_ : OTILE;
  static constexpr long LDS_PR = (long)((NCBI + 1) / 2) * PP2 * 16 * NPL_ > OTILE ? (long)((NCBI + 1) / 2) * PP2 * 16 * NPL_ : OTILE;
  static constexpr long LDS_CU = 160 * 1024;
  // only where the patch's LDS does not cost a workgroup per CU: the s1 3x3 tile (3 -> 2 workgroups per CU by
  // LDS) ran 7-14 % slower per launch in the pair layout, the stage-2 tiles 0.5-1.5 % faster, the population
  // step -0.8 % with this rule (profiles/r6/conv_patch_pair_r6.txt)
  static constexpr bool PAIR = PREC == 1 && NCBI >= 2 && LDS_CU / LDS_PR >= LDS_CU / LDS_PM;
  static constexpr int PXS = PAIR ? 2 : NCBP;       // LDS pixel stride (chunks)
  static constexpr int NPP = PAIR ? ((NCBI + 1) / 2) * PP2 : NPIX * NCBP;
  // LDS chunk offset of chunk cb within a pixel
  __host__ __device__ static constexpr int cbo(int cb) { return PAIR ? (cb >> 1) * PP2 + (cb & 1) : cb; }
  static size_t lds(bool fwd) {
    const size_t p = (size_t)NPP * 16 * NPL;
    const size_t o = (fwd && !PREC) ? (size_t)TP * OROWB * 2 : (size_t)TP * OROW * 4;
    return p > o ? p : o;
  }
};

// occupancy targets (measured, profiles/conv_occupancy.txt): 4 waves / SIMD
// (<= 128 registers) for 32-channel output tiles, 3 for the 5x5 64-channel
// tile; the 3x3 56-channel-input tile spills at 3 and keeps 2
// tile; NWV = 8 waves per workgroup: half the pixels per wave (fewer
// registers, 4 waves / SIMD) for the same 256-pixel tile. PREC 1 (fp32
// tensors, six-term split MFMA): three operand planes per fragment, LDS-bound
// at 2-3 workgroups per CU -> 2 waves / SIMD.
// Fused 2x2 max-pool of a forward tile (K4): TH x W output pixels in LDS
// (ld(pixel, chunk, f) reads 8 channels) -> pooled chunks + the argmax mask
// of pool_fwd_kernel (cnn_conv.hip: first strict maximum over (0,0), (0,1),
// (1,0), (1,1); bit 2 = maximum > 0), from the values exactly as stored.
template <int TH, int W, int NCO, int NTH, int PREC, typename LD>
__device__ __forceinline__ void fused_pool(const ConvArgs& a, LD ld, int g, int b, int h0, int tid) {
  typedef typename ActT<PREC>::T AT;
  constexpr int WO = W / 2, NPP = (TH / 2) * WO * NCO;
  static_assert(TH % 2 == 0 && W % 2 == 0, "pooled tiles need even rows / columns");
  const int Ho = a.H >> 1;
  const long n = (long)g * a.B + b;
  for (int i = tid; i < NPP; i += NTH) {
    const int cb = i % NCO, pp = i / NCO, pr = pp / WO, pc = pp - pr * WO;
    const int p0 = 2 * pr * W + 2 * pc;
    float m[8], t[8];
    int arg[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    ld(p0, cb, m);
    const int offs[3] = {1, W, W + 1};
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      ld(p0 + offs[q], cb, t);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (t[j] > m[j]) { m[j] = t[j]; arg[j] = q + 1; }
    }
    const long o = ((n * Ho + (h0 >> 1) + pr) * WO + pc) * (NCO * 8) + cb * 8;
    st_chunk(static_cast<AT*>(a.pool_y) + o, m);
    if (a.pool_mask) {
      uint32_t lo = 0, hi = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) lo |= (uint32_t)(arg[j] | (m[j] > 0.f ? 4 : 0)) << (8 * j);
#pragma unroll
      for (int j = 0; j < 4; ++j) hi |= (uint32_t)(arg[4 + j] | (m[4 + j] > 0.f ? 4 : 0)) << (8 * j);
      *reinterpret_cast<uint2*>(a.pool_mask + o) = make_uint2(lo, hi);
    }
  }
}

// Fused pool backward (K4): a data-gradient launch whose output is a pool's
// gradient scatters it straight to the pool source's gradient (2H x 2W):
// each chunk of 8 channels to the 4 cell pixels, the value at the forward's
// argmax when the maximum was > 0 (pool_bwd_mask_kernel's rule), else 0.
// The pooled gradient itself is never stored.
template <typename AT>
__device__ __forceinline__ void unpool_chunk(const ConvArgs& a, int g, long n, int h, int w, int cb, const float* v) {
  const int Cp = a.Coutp, H2 = 2 * a.H, W2 = 2 * a.W;
  const long o = ((n * a.H + h) * a.W + w) * Cp + cb * 8;
  const uint2 mk = *reinterpret_cast<const uint2*>(a.pool_mask + o);
  AT* dst = static_cast<AT*>((a.unpool_sel && a.unpool_sel[g]) ? a.unpool_x1 : a.pool_y);
#pragma unroll
  for (int me = 0; me < 4; ++me) {
    float out[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t b = ((j < 4 ? mk.x : mk.y) >> (8 * (j & 3))) & 0xffu;
      out[j] = ((int)(b & 3u) == me && (b & 4u)) ? v[j] : 0.f;
    }
    st_chunk(dst + ((n * H2 + 2 * h + (me >> 1)) * W2 + 2 * w + (me & 1)) * Cp + cb * 8, out);
  }
}

// PK (prec 1, shapes where every wave owns all NT co tiles): the last
// output-channel tile holds <= 4 real channels (20 = 16 + 4, 100 = 96 + 4),
// so 12+ of its 16 MFMA rows would multiply zero weights. Its rows carry the
// three weight planes of those channels instead (row 4c + p = plane p of
// channel 16 (NT-1) + c, row 4c + 3 = 0): three MFMAs (one per patch plane,
// one accumulator) give every row a_p (b0 + b1 + b2), and the epilogue sums
// the plane rows of a channel -- all nine split terms in 3 MFMAs instead of
// six terms in 6.
// forward declaration: the register-direct fp32 epilogue (defined below)
template <int CT, int PG, int PK, int W, int NCO, bool POOLABLE>
__device__ __forceinline__ void f32_epi_regs(const ConvArgs& a, const GroupRec& gr, int b, int h0,
                                             const f32x4_t (&acc)[CT][PG], int wco, int pgw, int lane);

// RE (fp32 only): 1 = register-direct epilogue (f32_epi_regs), 0 = through the LDS output tile
// CTX > 0 forces the co tiles per wave (1: waves split the co tiles, more pixel groups each)
// SCH (fp32): 1 = the unrolled k loop as an ENFORCED software pipeline (sched_barrier between the patch
// reads of k-step s+1, the MFMAs of k-step s and the weight loads of k-step s+2, a 3-slot weight ring).
// hipcc's own schedule sinks every prefetch next to its first use; that is hidden where two MFMA waves
// share a SIMD (neutral on the 2-tile shapes, slower on stage 1) but not on the one-co-tile-per-wave
// s2 input-conv data gradient (-13 %): r5/conv_f32_sched_pipe_ab_r5.txt
template <int KH, int KW, int NCBI, int W, int TH, int NT, int NCO, int NWV = 4, int PREC = 0, int PK = 0, int RE = 0,
          int CTX = 0, int SCH = 0>
__global__ void __launch_bounds__(NWV * 64)
__attribute__((amdgpu_waves_per_eu(PREC ? 2 : (NWV == 8 ? 4 : (NT >= 4 ? (NCBI >= 7 ? 2 : 3) : 4)))))
conv_fast_kernel(ConvArgs a) {
  typedef typename ActT<PREC>::T AT;
  constexpr int NPL = PREC ? GT_NPL_F32 : 1;
  constexpr int NTH = NWV * 64;                     // threads
  constexpr int PH = TH + KH - 1, PW = W + KW - 1;
  constexpr int NP = PH * PW * NCBI;                // patch chunks (8 channels) per plane
  using FCL = FastCfg<KH, KW, NCBI, W, TH, NT, NCO, PREC>;
  constexpr int NCBP = FCL::NCBP;                   // LDS chunks per patch pixel (pixel-major layout)
  constexpr int PXS = FCL::PXS;                     // LDS pixel stride (chunks)
  constexpr int NPP = FCL::NPP;                     // LDS plane stride (chunks)
  // staged chunk i (pixel i / NCBI, chunk i % NCBI) -> its LDS slot
  auto pslot = [&](int i) {
    if constexpr (NCBP == NCBI && !FCL::PAIR) return i;
    else return (i / NCBI) * PXS + FCL::cbo(i % NCBI);
  };
  constexpr int NPT = (NP + NTH - 1) / NTH;             // patch chunks per thread
  constexpr int NCH = KH * KW * NCBI;               // reduction chunks
  constexpr int NKS = (NCH + 3) / 4;                // k-steps (32 k each)
  // reduction order: entry e of the chunk list -> (kk = kh * KW + kw, cb); part-major for the
  // stage-2 3x3 fp32 shape (S2Parts), else kk-major
  constexpr bool PARTS = S2Parts<KH, KW, NCBI, W, PREC>::on;
  auto ent = [&](int e, int& kk, int& cb) {
    if constexpr (PARTS) {
      constexpr int E0 = S2Parts<KH, KW, NCBI, W, PREC>::e0;
      if (e < E0) { kk = e >> 2; cb = e & 3; }
      else { const int e1 = e - E0; kk = e1 / 3; cb = 4 + e1 - kk * 3; }
    } else {
      kk = e / NCBI; cb = e - kk * NCBI;
    }
  };
  constexpr int TP = TH * W;                        // tile pixels
  constexpr int NPG = TP / 16;                      // pixel groups
  // co tiles per wave (odd NT: one per wave; packed last tile: all NT, so every wave carries the same work)
  constexpr int CT = CTX ? CTX : PK ? NT : ((NT >= 2 && NT % 2 == 0) ? 2 : 1);
  constexpr int WC = NT / CT;                       // waves along co
  constexpr int WP = NWV / WC;                        // waves along pixels
  constexpr int PG = NPG / WP;                      // pixel groups per wave
  // weight prefetch depth (k-steps; 3 planes each in prec 1). The S=(3,5) stage-2 tiles with one co tile per
  // wave hold 3 k-steps of weights (12 VGPRs each): -0.6 % per population step, 2 and 4 neither
  // (r5/conv_s2n_ct1_ab_r5.txt)
  constexpr int PFM = PREC ? ((CTX == 1 && !SCH && NWV == 4 && NCBI <= 7) ? 3 : 2) : 4;
  constexpr int PF = NKS < PFM ? NKS : PFM;
  // fp32 enforced pipeline (SCH): the weights of k-step s+PF load into the ring slot k-step s-1 used, so
  // no load waits for an MFMA still reading its registers
  constexpr bool SCHED = SCH && PREC != 0 && NKS <= 64;
  constexpr int RA = SCHED ? PF + 1 : PF;
  static_assert(NPG % WP == 0 && NT % CT == 0 && WC * WP == NWV, "tile shape");
  static_assert(!PK || (PREC == 1 && WC == 1), "packed last tile: fp32, every wave owns all co tiles");
  static_assert(W % 16 == 0 || 16 % W == 0, "pixel groups must tile image rows");

  using FC = FastCfg<KH, KW, NCBI, W, TH, NT, NCO, PREC>;
  constexpr int OROW = FC::OROW, OROWB = FC::OROWB;
  extern __shared__ __attribute__((aligned(16))) uint4 smem[];   // patch planes, then the output tile
  uint4* patch = smem;
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
  // weight planes: row-major [Q][Coutp][KH][KW][Cinp] (a.wfrag = 0), or FRAGMENT-MAJOR [Q][NT][NKS][64 lanes][8]
  // (a.wfrag = 1, written by gt_conv_wfrag: the 16 rows x 32 k of one (co tile, k-step) are one contiguous KB
  // in lane order, so a wave's 16-byte-per-lane load fills 8 whole 128-byte lines instead of touching 16 half
  // used ones -- 6-16 % per launch, profiles/r6/conv_wfrag_r6.txt). wrow: the lane's row base; per k-step the
  // offset is the entry's chunk (row-major) or s * 512 (fragment-major)
  const uint16_t* wrow[CT];
  bool wok[CT];
#pragma unroll
  for (int t = 0; t < CT; ++t) {
    if (PK && t == CT - 1) {                        // packed tile: row l16 = (channel l16/4, plane l16%4)
      const int co = (wco + t) * 16 + (l16 >> 2), pl = l16 & 3;
      wok[t] = pl < 3 && co < a.cout_real;
      wrow[t] = a.wfrag ? a.w + (((long)g * NT + wco + t) * NKS * 64 + kq * 16 + (l16 >> 2)) * 8 + (wok[t] ? pl : 0) * a.wps
                        : a.w + ((long)g * (NCO * 8) + (wok[t] ? co : 0)) * (NCH * 8) + (wok[t] ? pl : 0) * a.wps;
      continue;
    }
    const int co = (wco + t) * 16 + l16;
    wok[t] = co < NCO * 8;
    wrow[t] = a.wfrag ? a.w + (((long)g * NT + wco + t) * NKS * 64 + lane) * 8
                      : a.w + ((long)g * (NCO * 8) + (wok[t] ? co : 0)) * (NCH * 8);
  }
  uint4 areg[RA][CT][NPL];
  auto load_a = [&](int s, uint4 (*dst)[NPL]) {
    // (dbg bit 8, diagnostics only: every k-step re-reads k-step 0's weights -- L1-resident operands)
    const int e = ((a.dbg & 8) ? 0 : s * 4) + kq;
    int c = e;                                      // the entry's chunk in the weight row (kk * NCBI + cb)
    if constexpr (PARTS) {
      int kk, cb;
      ent(e, kk, cb);
      c = kk * NCBI + cb;
    }
    const bool fr = a.wfrag != 0;
#pragma unroll
    for (int t = 0; t < CT; ++t) {
      // fragment-major planes hold exact zeros in padded rows and entries past the chunk list
      const bool ok = fr ? (!(PK && t == CT - 1) || wok[t]) : (wok[t] && e < NCH);
      const long off = fr ? (long)((a.dbg & 8) ? 0 : s) * 512 : (long)c * 8;
#pragma unroll
      for (int p = 0; p < ((PK && t == CT - 1) ? 1 : NPL); ++p)
        dst[t][p] = *reinterpret_cast<const uint4*>(ok ? (const void*)(wrow[t] + p * a.wps + off) : (const void*)gt_zero8);
    }
  };
  // one k-step of tile t: the six-term product, or the packed tile's three MFMAs
  auto mma = [&](int t, const uint4* af, const uint4* bf, f32x4_t c) {
    if (PK && t == CT - 1) {
      c = mfma16(af[0], bf[2], c);
      c = mfma16(af[0], bf[1], c);
      return mfma16(af[0], bf[0], c);
    }
    return mfma_np<NPL>(af, bf, c);
  };

  // ---- patch: summed inputs (or gathered dataset image), zero halo --------
  const long gimg = ((long)g * a.B + b) * img;
  const int n_src = a.gather ? 1 : __builtin_popcount(gr.in_mask);
  const AT* src0 = a.gather ? static_cast<const AT*>(a.in[0]) + a.gather[((long)a.st->cur_step * a.G + g) * a.B + b] * img
                            : static_cast<const AT*>(a.in[__builtin_ctz(gr.in_mask | 0x100) & 7]) + gimg;
  long poff[NPT];
  bool pok[NPT];
#pragma unroll
  for (int j = 0; j < NPT; ++j) {
    const int i = tid + NTH * j;
    const int cb = i % NCBI, pix = i / NCBI;
    const int pr = pix / PW, pc = pix % PW;
    const int hh = h0 - KH / 2 + pr, ww = pc - KW / 2;
    pok[j] = i < NP && hh >= 0 && hh < a.H && ww >= 0 && ww < W;
    poff[j] = ((long)hh * W + ww) * (NCBI * 8) + cb * 8;
  }
  if (a.dbg & 4) {
#pragma unroll
    for (int j = 0; j < NPT; ++j)
#pragma unroll
      for (int p = 0; p < NPL; ++p)
        if (tid + NTH * j < NP) patch[p * NPP + pslot(tid + NTH * j)] = make_uint4(0, 0, 0, 0);
  } else if (!PREC && n_src == 1) {
    uint4 v[NPT];
#pragma unroll
    for (int j = 0; j < NPT; ++j)
      v[j] = *reinterpret_cast<const uint4*>(pok[j] ? (const void*)(src0 + poff[j]) : (const void*)gt_zero8);
#pragma unroll
    for (int j = 0; j < NPT; ++j)
      if (tid + NTH * j < NP) patch[pslot(tid + NTH * j)] = v[j];
  } else {
    // chunks in batches of JB with the batch's loads in flight; N-ary DAG
    // input summed in fp32 (prec 0: one rounding to bf16 at the end; prec 1:
    // exact split of the fp32 sum into the three planes)
    constexpr int JB = NPT < 5 ? NPT : 5;
#pragma unroll
    for (int j0 = 0; j0 < NPT; j0 += JB) {
      float acc8[JB][8];
#pragma unroll
      for (int j = 0; j < JB; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc8[j][e] = 0.f;
      if (n_src == 1) {
#pragma unroll
        for (int j = 0; j < JB; ++j)
          if (j0 + j < NPT && pok[j0 + j]) ld_chunk(src0 + poff[j0 + j], acc8[j]);
      } else {
        // DAG inputs two at a time: both inputs' chunk loads are in flight before either is
        // summed (one input at a time waited a global round trip per input). Still summed in
        // increasing slot order: bit-identical.
        int m = gr.in_mask & 0xff;
        while (m) {
          const int k0 = __builtin_ctz(m);
          m &= m - 1;
          const bool two = m != 0;
          const int k1 = two ? __builtin_ctz(m) : k0;
          if (two) m &= m - 1;
          const AT* s0 = static_cast<const AT*>(a.in[k0]) + gimg;
          const AT* s1 = static_cast<const AT*>(a.in[k1]) + gimg;
          float t0[JB][8], t1[JB][8];
#pragma unroll
          for (int j = 0; j < JB; ++j) {
#pragma unroll
            for (int e = 0; e < 8; ++e) t0[j][e] = t1[j][e] = 0.f;
            if (j0 + j < NPT && pok[j0 + j]) {
              ld_chunk(s0 + poff[j0 + j], t0[j]);
              if (two) ld_chunk(s1 + poff[j0 + j], t1[j]);
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
        if (PREC) {
          uint4 p0, p1, p2;
          split8(acc8[j], p0, p1, p2);
          patch[pslot(i)] = p0;
          patch[NPP + pslot(i)] = p1;
          patch[2 * NPP + pslot(i)] = p2;
        } else {
          patch[pslot(i)] = pack8(acc8[j]);
        }
      }
    }
  }
  if (a.xsum && n_src > 1) {
    // the summed input of this band (interior of the patch) for the layer's wgrad
    __syncthreads();
    AT* xo = static_cast<AT*>(a.xsum) + ((long)g * a.B + b) * img + (long)h0 * W * NCBI * 8;
    for (int i = tid; i < TH * W * NCBI; i += NTH) {
      const int cb = i % NCBI, pix = i / NCBI;
      const int r = pix / W, c = pix % W;
      if (h0 + r >= a.H) continue;
      const int pi = ((r + KH / 2) * PW + c + KW / 2) * PXS + FCL::cbo(cb);
      if (PREC) {
        float f[8];
        join8(patch[pi], patch[NPP + pi], patch[2 * NPP + pi], f);   // exact: the fp32 sum
        st_chunk(xo + (long)i * 8, f);
      } else {
        *reinterpret_cast<uint4*>(xo + (long)i * 8) = patch[pi];
      }
    }
  }
  // chunk c -> patch offset of its (kh, kw, cb) relative to the output pixel
  for (int c = tid; c < NKS * 4; c += NTH) {
    int kk, cb;
    ent(c, kk, cb);
    coff[c] = c < NCH ? ((kk / KW) * PW + (kk % KW)) * PXS + FCL::cbo(cb) : 0;
  }
  // first PF k-steps of weights in flight before the barrier (after the patch
  // staging: its registers are dead by now -- lower peak register pressure)
#pragma unroll
  for (int s = 0; s < PF; ++s) load_a(s, areg[s]);
  // bias of this lane's output channels (forward only)
  float bias_v[CT][4];
#pragma unroll
  for (int t = 0; t < CT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int co = (PK && t == CT - 1) ? (i == 0 ? (wco + t) * 16 + kq : NCO * 8) : (wco + t) * 16 + kq * 4 + i;
      bias_v[t][i] = (a.bias && co < NCO * 8) ? a.bias[(long)g * (NCO * 8) + co] : 0.f;
    }
  __syncthreads();

  // ---- MFMA main loop ------------------------------------------------------
  // lane's pixel within a group: (l16 / W) rows down, l16 % W across (W >= 16: same row)
  const int lbase = ((l16 / W) * PW + (l16 % W)) * PXS;
  int gbase;
  {
    const int p = pgw * 16;
    gbase = ((p / W) * PW + (p % W)) * PXS;
  }
  f32x4_t acc[CT][PG];
#pragma unroll
  for (int t = 0; t < CT; ++t)
#pragma unroll
    for (int h = 0; h < PG; ++h) acc[t][h] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  // chunk c of the reduction -> patch offset of its (kh, kw, cb) (the coff table, computed in registers)
  auto koff = [&](int s) {
    const int c = s * 4 + kq;
    int kk, cb;
    ent(c, kk, cb);
    return c < NCH ? ((kk / KW) * PW + (kk % KW)) * PXS + FCL::cbo(cb) : 0;
  };
  // the patch fragments of k-step s: the offset from the LDS table, or (pipelined loop) computed in
  // registers so no table read drains lgkmcnt in the middle of the MFMA stream
  auto load_b = [&](int s, uint4 (*dst)[NPL]) {
    const uint4* pb = patch + lbase + gbase + (SCHED ? koff(s) : coff[s * 4 + kq]);
#pragma unroll
    for (int h = 0; h < PG; ++h) {
      const int p = h * 16;                        // relative to the wave's first group
#pragma unroll
      for (int q = 0; q < NPL; ++q) dst[h][q] = pb[q * NPP + ((p / W) * PW + (p % W)) * PXS];
    }
  };
  if (!(a.dbg & 1)) {
    if constexpr (PREC != 0 && NKS > 64) {
      // long reductions (wide layers: 72-100 k-steps): a runtime loop over k-step PAIRS, so the
      // register sets stay compile-time indexed (a fully unrolled loop this long is not unrolled
      // by hipcc and its dynamically indexed operand arrays went to scratch); the prefetches are
      // unconditional (clamped k-step: the tail re-reads the last one)
      static_assert(PF == 2, "k-step pairs need a 2-deep weight prefetch");
      uint4 bfr[2][PG][NPL];
      load_b(0, bfr[0]);
      auto kstep = [&](int s, auto par) {
        constexpr int P = decltype(par)::value;
        load_b(min(s + 1, NKS - 1), bfr[P ^ 1]);
#pragma unroll
        for (int t = 0; t < CT; ++t)
#pragma unroll
          for (int h = 0; h < PG; ++h) acc[t][h] = mma(t, areg[P][t], bfr[P][h], acc[t][h]);
        load_a(min(s + PF, NKS - 1), areg[P]);
      };
      for (int s = 0; s < NKS; s += 2) {
        kstep(s, std::integral_constant<int, 0>());
        if (s + 1 < NKS) kstep(s + 1, std::integral_constant<int, 1>());
      }
    } else if constexpr (SCHED) {
      // fp32, unrolled k loop as an explicit software pipeline. Left alone, hipcc sinks every prefetch
      // next to its first use (round-4 ISA: a k-step's weight loads were waited on 2-4 MFMAs after they
      // issued, its patch reads right before the MFMAs), so both waves of a SIMD stall on L2 / LDS
      // latency in the middle of the MFMA stream. Per k-step s, fenced by sched_barrier:
      //   1. LDS reads of k-step s+1's patch fragments (double buffer; offsets held in registers)
      //   2. the 6 x CT x PG MFMAs of k-step s
      //   3. global loads of k-step s+PF's weights into the ring slot k-step s-1 used
      // The MFMA order (and so every accumulator's summation order) is the unpipelined loop's.
      uint4 bfr[2][PG][NPL];
      load_b(0, bfr[0]);
#pragma unroll
      for (int s = 0; s < NKS; ++s) {
        if (s + 1 < NKS) load_b(s + 1, bfr[(s + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < CT; ++t)
#pragma unroll
          for (int h = 0; h < PG; ++h) acc[t][h] = mma(t, areg[s % RA][t], bfr[s & 1][h], acc[t][h]);
        __builtin_amdgcn_sched_barrier(0);
        if (s + PF < NKS) load_a(s + PF, areg[(s + PF) % RA]);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else if constexpr (PREC != 0) {
      // fp32: the next k-step's patch fragments are read while this step's 6 x CT x PG
      // MFMAs run (the unpipelined loop waited for its LDS reads before every k-step)
      uint4 bfr[2][PG][NPL];
      load_b(0, bfr[0]);
#pragma unroll
      for (int s = 0; s < NKS; ++s) {
        if (s + 1 < NKS) load_b(s + 1, bfr[(s + 1) & 1]);
#pragma unroll
        for (int t = 0; t < CT; ++t)
#pragma unroll
          for (int h = 0; h < PG; ++h) acc[t][h] = mma(t, areg[s % PF][t], bfr[s & 1][h], acc[t][h]);
        if (s + PF < NKS) load_a(s + PF, areg[s % PF]);
      }
    } else {
      // bf16
#pragma unroll
      for (int s = 0; s < NKS; ++s) {
        uint4 bfr[PG][NPL];
        load_b(s, bfr);
#pragma unroll
        for (int t = 0; t < CT; ++t)
#pragma unroll
          for (int h = 0; h < PG; ++h) acc[t][h] = mma(t, areg[s % PF][t], bfr[h], acc[t][h]);
        if (s + PF < NKS) load_a(s + PF, areg[s % PF]);
      }
    }
  }

  if constexpr (RE != 0 && PREC != 0 && W % 16 == 0) {
    // register-direct: no LDS round trip, no barrier (and the pool from lane shuffles)
    constexpr bool PL = TH % 2 == 0 && PG % (2 * (W / 16)) == 0;
    f32_epi_regs<CT, PG, PK, W, NCO, PL>(a, gr, b, h0, acc, wco, pgw, lane);
    return;
  }
  // ---- epilogue: accumulators -> tile in LDS -> 16-byte row stores ---------
  // (a lane holds 4 channels of one pixel per tile: 8-byte scattered stores
  // are store-issue bound; through LDS every store is a contiguous chunk of
  // the band, which is one contiguous range of the NHWC output)
  if (a.epi_bf16 && !PREC) {
    // forward launches: values rounded once to bf16 in an LDS tile, copied out
    // as contiguous 16-byte chunks of the band (one contiguous NHWC range)
    __syncthreads();                                 // everyone is done with the patch
    uint16_t* ot = reinterpret_cast<uint16_t*>(smem);
#pragma unroll
    for (int t = 0; t < CT; ++t) {
      const int co0 = (wco + t) * 16 + kq * 4;
#pragma unroll
      for (int h = 0; h < PG; ++h) {
        const int p = (pgw + h) * 16 + l16;
        const bool pad0 = a.Hr > 0 && (h0 + p / W >= a.Hr || p % W >= a.Wr);   // zero-padded image
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          v[i] = acc[t][h][i] + bias_v[t][i];
          if (a.relu) v[i] = fmaxf(v[i], 0.f);
          if (pad0) v[i] = 0.f;
        }
        *reinterpret_cast<uint2*>(ot + p * OROWB + co0) = pack4(v);
      }
    }
    __syncthreads();
    const long obase = (((long)g * a.B + b) * a.H + h0) * W * (NCO * 8);
    if (!(a.dbg & 2))
#pragma unroll
    for (int j = 0; j < (TP * NCO + NTH - 1) / NTH; ++j) {
      const int i = tid + NTH * j;
      if (i >= TP * NCO) break;
      const int p = i / NCO, cb = i - p * NCO;
      const uint4 val = *reinterpret_cast<const uint4*>(ot + p * OROWB + cb * 8);
#pragma unroll
      for (int k = 0; k < GT_MAXSLOT; ++k)
        if ((gr.out_mask >> k) & 1) *reinterpret_cast<uint4*>(static_cast<uint16_t*>(a.out[k]) + obase + (long)i * 8) = val;
    }
    if constexpr (TH % 2 == 0)
      if (a.pool_y && ((gr.out_mask >> 24) & 1))
        fused_pool<TH, W, NCO, NTH, 0>(
            a, [&](int p, int cb, float* f) { unpack8(*reinterpret_cast<const uint4*>(ot + p * OROWB + cb * 8), f); },
            g, b, h0, tid);
    return;
  }
  // fp32 tile in LDS, then one contiguous chunk per thread and slot: plain
  // store (forward), or the data gradient's DAG fan-out (several output
  // slots, accumulate, ReLU masks) as a read-modify-write
  __syncthreads();                                   // everyone is done with the patch
  float* otile = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int t = 0; t < CT; ++t) {
    const int co0 = (wco + t) * 16 + kq * 4;
#pragma unroll
    for (int h = 0; h < PG; ++h) {
      const int p = (pgw + h) * 16 + l16;
      const bool pad0 = a.Hr > 0 && (h0 + p / W >= a.Hr || p % W >= a.Wr);   // zero-padded image
      if (PK && t == CT - 1) {
        // channel (wco + t) * 16 + kq = sum of its three plane rows; the tile's other columns are 0
        float s0 = acc[t][h][0] + acc[t][h][1] + acc[t][h][2] + bias_v[t][0];
        if (a.relu) s0 = fmaxf(s0, 0.f);
        if (pad0) s0 = 0.f;
        float* orow = otile + p * OROW + (wco + t) * 16;
        orow[kq] = s0;
        orow[4 + kq] = 0.f;
        orow[8 + kq] = 0.f;
        orow[12 + kq] = 0.f;
        continue;
      }
      float4 v;
      v.x = acc[t][h][0] + bias_v[t][0];
      v.y = acc[t][h][1] + bias_v[t][1];
      v.z = acc[t][h][2] + bias_v[t][2];
      v.w = acc[t][h][3] + bias_v[t][3];
      if (a.relu) { v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f); }
      if (pad0) v = make_float4(0.f, 0.f, 0.f, 0.f);
      *reinterpret_cast<float4*>(otile + p * OROW + co0) = v;
    }
  }
  __syncthreads();
  if (a.dbg & 2) return;
  const long obase = (((long)g * a.B + b) * a.H + h0) * W * (NCO * 8);
#pragma unroll
  for (int j = 0; j < (TP * NCO + NTH - 1) / NTH; ++j) {
    const int i = tid + NTH * j;
    if (i >= TP * NCO) break;
    const int p = i / NCO, cb = i - p * NCO;
    const float4 lo = *reinterpret_cast<const float4*>(otile + p * OROW + cb * 8);
    const float4 hi = *reinterpret_cast<const float4*>(otile + p * OROW + cb * 8 + 4);
    const float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    const long off = obase + (long)i * 8;
    if ((gr.out_mask >> 25) & 1) {          // the output is a pool's gradient: un-pool it (slot 0)
      unpool_chunk<AT>(a, g, (long)g * a.B + b, h0 + p / W, p % W, cb, v);
      continue;
    }
    for (int k = 0; k < GT_MAXSLOT; ++k) {
      if (!((gr.out_mask >> k) & 1)) continue;
      AT* dst = static_cast<AT*>(a.out[k]) + off;
      float sum[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) sum[e] = v[e];
      if ((gr.out_mask >> (8 + k)) & 1) {
        float o[8];
        ld_chunk(dst, o);
#pragma unroll
        for (int e = 0; e < 8; ++e) sum[e] += o[e];
      }
      if ((gr.out_mask >> (16 + k)) & 1) {
        float m[8];
        ld_chunk(static_cast<const AT*>(a.out_mask[k]) + off, m);
#pragma unroll
        for (int e = 0; e < 8; ++e) sum[e] = m[e] > 0.f ? sum[e] : 0.f;
      }
      st_chunk(dst, sum);
    }
  }
  if constexpr (TH % 2 == 0)
    if (a.pool_y && ((gr.out_mask >> 24) & 1))
      fused_pool<TH, W, NCO, NTH, PREC>(
          a, [&](int p, int cb, float* f) { load8f(otile + p * OROW + cb * 8, f); }, g, b, h0, tid);
}

// Register-direct fp32 epilogue of one output tile of the tile kernel: lane = 4 channels of pixel (pgw + h) * 16 + l16; bias / ReLU;
// plain store, or the data gradient's DAG fan-out (accumulate, ReLU mask, up to
// 8 slots) with every global load of a slot's read-modify-write issued before
// its first use; the fused un-pool; the fused 2x2 max-pool + argmax mask from
// lane shuffles and the paired pixel-group register (a wave's pixel groups
// cover whole row pairs). Bit-identical to the LDS-tile epilogue.
template <int CT, int PG, int PK, int W, int NCO, bool POOLABLE>
__device__ __forceinline__ void f32_epi_regs(const ConvArgs& a, const GroupRec& gr, int b, int h0,
                                             const f32x4_t (&acc)[CT][PG], int wco, int pgw, int lane) {
  constexpr int COP = NCO * 8, RG = W / 16;
  const int kq = lane >> 4, l16 = lane & 15;
  const long oimg = (long)a.H * W * COP;

  if (a.dbg & 2) return;
  const int g = gr.g;
  const long n = (long)g * a.B + b;
  const long obase = n * oimg + (long)h0 * W * COP;
  const bool pool = a.pool_y && ((gr.out_mask >> 24) & 1);
  const bool unpool = (gr.out_mask >> 25) & 1;
  float val[CT][PG][4];
  bool cok[CT];
#pragma unroll
  for (int t = 0; t < CT; ++t) {
    const bool pkt = PK && t == CT - 1;
    const int co0 = (wco + t) * 16 + kq * 4;
    cok[t] = co0 < COP;                                  // whole float4 inside the padded row
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (a.bias) {
      if (pkt) {
        const int co = (wco + t) * 16 + kq;
        bv[0] = co < COP ? a.bias[(long)g * COP + co] : 0.f;
      } else if (co0 < COP) {
        const float4 q = *reinterpret_cast<const float4*>(a.bias + (long)g * COP + co0);
        bv[0] = q.x; bv[1] = q.y; bv[2] = q.z; bv[3] = q.w;
      }
    }
#pragma unroll
    for (int h = 0; h < PG; ++h) {
      if (pkt) {
        // channel (wco+t)*16 + kq (its three plane rows summed) -> lane kq == 0 gathers channels +0..+3
        float s0 = acc[t][h][0] + acc[t][h][1] + acc[t][h][2] + bv[0];
        if (a.relu) s0 = fmaxf(s0, 0.f);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float o = __shfl(s0, l16 + 16 * i, 64);
          val[t][h][i] = kq == 0 ? o : 0.f;
        }
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float v = acc[t][h][i] + bv[i];
          if (a.relu) v = fmaxf(v, 0.f);
          val[t][h][i] = v;
        }
      }
    }
  }
  if (a.Hr > 0 && !unpool) {
    // zero-padded image (ConvArgs::Hr / Wr): exact zeros outside the real rows / columns
#pragma unroll
    for (int h = 0; h < PG; ++h) {
      const int p = (pgw + h) * 16 + l16;
      if (h0 + p / W >= a.Hr || p % W >= a.Wr) {
#pragma unroll
        for (int t = 0; t < CT; ++t)
#pragma unroll
          for (int i = 0; i < 4; ++i) val[t][h][i] = 0.f;
      }
    }
  }
  auto off_of = [&](int t, int h) {
    return obase + (long)((pgw + h) * 16 + l16) * COP + (wco + t) * 16 + kq * 4;
  };
  if (unpool) {
    // the output is a pool's gradient: scatter each value to the forward's argmax cell (if > 0)
    uint32_t mk[CT][PG];
#pragma unroll
    for (int t = 0; t < CT; ++t)
#pragma unroll
      for (int h = 0; h < PG; ++h)
        mk[t][h] = *reinterpret_cast<const uint32_t*>(a.pool_mask + (cok[t] ? off_of(t, h) : 0));
    float* dst = static_cast<float*>((a.unpool_sel && a.unpool_sel[g]) ? a.unpool_x1 : a.pool_y);
    const int H2 = 2 * a.H, W2 = 2 * W;
#pragma unroll
    for (int t = 0; t < CT; ++t) {
      if (!cok[t]) continue;
#pragma unroll
      for (int h = 0; h < PG; ++h) {
        const int p = (pgw + h) * 16 + l16;
        const int hh = h0 + p / W, ww = p % W;
#pragma unroll
        for (int me = 0; me < 4; ++me) {
          float o[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const uint32_t bb = (mk[t][h] >> (8 * i)) & 0xffu;
            o[i] = ((int)(bb & 3u) == me && (bb & 4u)) ? val[t][h][i] : 0.f;
          }
          *reinterpret_cast<float4*>(dst + ((n * H2 + 2 * hh + (me >> 1)) * W2 + 2 * ww + (me & 1)) * COP +
                                     (wco + t) * 16 + kq * 4) = make_float4(o[0], o[1], o[2], o[3]);
        }
      }
    }
  } else {
    for (int k = 0; k < GT_MAXSLOT; ++k) {
      if (!((gr.out_mask >> k) & 1)) continue;
      float* dst = static_cast<float*>(a.out[k]);
      float o[CT][PG][4];
#pragma unroll
      for (int t = 0; t < CT; ++t)
#pragma unroll
        for (int h = 0; h < PG; ++h)
#pragma unroll
          for (int i = 0; i < 4; ++i) o[t][h][i] = val[t][h][i];
      if ((gr.out_mask >> (8 + k)) & 1) {              // accumulate into the slot
        float4 q[CT][PG];
#pragma unroll
        for (int t = 0; t < CT; ++t)
#pragma unroll
          for (int h = 0; h < PG; ++h) q[t][h] = *reinterpret_cast<const float4*>(dst + (cok[t] ? off_of(t, h) : 0));
#pragma unroll
        for (int t = 0; t < CT; ++t)
#pragma unroll
          for (int h = 0; h < PG; ++h) {
            o[t][h][0] += q[t][h].x; o[t][h][1] += q[t][h].y; o[t][h][2] += q[t][h].z; o[t][h][3] += q[t][h].w;
          }
      }
      if ((gr.out_mask >> (16 + k)) & 1) {             // ReLU mask of the slot's activation
        const float* mp = static_cast<const float*>(a.out_mask[k]);
        float4 q[CT][PG];
#pragma unroll
        for (int t = 0; t < CT; ++t)
#pragma unroll
          for (int h = 0; h < PG; ++h) q[t][h] = *reinterpret_cast<const float4*>(mp + (cok[t] ? off_of(t, h) : 0));
#pragma unroll
        for (int t = 0; t < CT; ++t)
#pragma unroll
          for (int h = 0; h < PG; ++h) {
            o[t][h][0] = q[t][h].x > 0.f ? o[t][h][0] : 0.f; o[t][h][1] = q[t][h].y > 0.f ? o[t][h][1] : 0.f;
            o[t][h][2] = q[t][h].z > 0.f ? o[t][h][2] : 0.f; o[t][h][3] = q[t][h].w > 0.f ? o[t][h][3] : 0.f;
          }
      }
#pragma unroll
      for (int t = 0; t < CT; ++t) {
        if (!cok[t]) continue;
#pragma unroll
        for (int h = 0; h < PG; ++h)
          *reinterpret_cast<float4*>(dst + off_of(t, h)) = make_float4(o[t][h][0], o[t][h][1], o[t][h][2], o[t][h][3]);
      }
    }
  }
  if constexpr (POOLABLE) {
    if (pool) {
      // 2x2 max-pool + argmax mask (pool_fwd_kernel's rule: first strict maximum over
      // (0,0), (0,1), (1,0), (1,1); bit 2 = maximum > 0) of the values as stored
      const int Ho = a.H >> 1, Wo = W >> 1;
#pragma unroll
      for (int t = 0; t < CT; ++t) {
#pragma unroll
        for (int h = 0; h < PG; ++h) {
          if ((h / RG) % 2) continue;                     // top row of each row pair
          float m[4];
          uint32_t mk = 0;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float v00 = val[t][h][i], v10 = val[t][h + RG][i];
            const float v01 = __shfl(v00, lane + 1, 64), v11 = __shfl(v10, lane + 1, 64);
            float mm = v00;
            int arg = 0;
            if (v01 > mm) { mm = v01; arg = 1; }
            if (v10 > mm) { mm = v10; arg = 2; }
            if (v11 > mm) { mm = v11; arg = 3; }
            m[i] = mm;
            mk |= (uint32_t)(arg | (mm > 0.f ? 4 : 0)) << (8 * i);
          }
          if ((l16 & 1) || !cok[t]) continue;
          const int p = (pgw + h) * 16 + l16;
          const int pr = (h0 + p / W) >> 1, pc = (p % W) >> 1;
          const long o = ((n * Ho + pr) * Wo + pc) * COP + (wco + t) * 16 + kq * 4;
          *reinterpret_cast<float4*>(static_cast<float*>(a.pool_y) + o) = make_float4(m[0], m[1], m[2], m[3]);
          if (a.pool_mask) *reinterpret_cast<uint32_t*>(a.pool_mask + o) = mk;
        }
      }
    }
  }
}


// ===========================================================================
// Weight gradient, shape-specialised:
//   dW[co][kh][kw][ci] (+ db[co]) = sum_px dz[px][co] * x[px + (kh, kw)][ci]
// One workgroup = one group x one split (a contiguous range of R-row image
// bands) and owns the WHOLE dW of the layer in registers: wave w accumulates
// k-column tiles w, w+4, ... for every output-channel tile. Per band, the
// dz rows and the zero-haloed input rows (DAG inputs summed, batch gather for
// the first layer) are staged into LDS with all loads in flight; each 32-pixel
// K-step then reads both MFMA operands with ds_read_b64_tr_b16 (A = dz^T,
// B = shifted input) at per-lane addresses fixed for the whole kernel plus
// compile-time K-step offsets -- no index math in the loop. The bias gradient
// is an extra "ones" column. The workgroup writes one fp32 partial
// [S][G][Coutp][Kdim] (+ [S][G][Coutp]) that Adam reduces in fixed order.
// ===========================================================================

typedef __attribute__((ext_vector_type(4))) short wf_short4_t;
typedef __attribute__((ext_vector_type(8))) short wf_short8_t;

__device__ __forceinline__ uint4 tr_pair(const char* lo_addr, const char* hi_addr) {
  typedef __attribute__((address_space(3))) wf_short4_t lds_s4;
  const wf_short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(lo_addr));
  const wf_short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(hi_addr));
  const wf_short8_t v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(uint4, v);
}

__device__ __attribute__((aligned(16))) uint4 wf_zero16[1];

typedef __attribute__((address_space(3))) void wf_lvoid_t;

// one 16-byte chunk per lane into LDS at wave base + 16 * lane. Inline asm so
// hipcc does not see an LDS write it would fence every later LDS read behind
// (it waits vmcnt(0) before any ds_read that may alias an in-flight builtin
// DMA): the kernel waits for its DMAs explicitly (vmcnt(0) + barrier) before
// reading the buffer they fill. m0 is saved / restored around the DMA.
__device__ __forceinline__ void wf_glds16(const void* src, const void* lds_wave_base) {
  const uint32_t l = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(wf_lvoid_t*)lds_wave_base);
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(src), "s"(l) : "memory");
}

// NB = LDS band buffers: 2 overlaps band i+1's DMA with band i's MFMAs; 1
// halves the LDS so more workgroups share a CU
template <int KH, int KW, int NCBI, int NCBO, int W, int R, int NW, int NB>
__global__ void __launch_bounds__(NW * 64) wgrad_fast_kernel(WgradArgs a) {
  constexpr int NT_ = NW * 64;                     // threads
  constexpr int PW = W + KW - 1, PR = R + KH - 1;
  constexpr int NCH = KH * KW * NCBI;              // weight chunks (8 input channels each)
  constexpr int NKT = (NCH + 1 + 1) / 2;           // 16-column tiles incl. the bias chunk
  constexpr int MT = (NCBO * 8 + 15) / 16;         // output-channel tiles
  constexpr int TPW = (NKT + NW - 1) / NW;         // k-column tiles per wave
  constexpr int KS = R * W / 32;                   // K-steps per band
  constexpr int XCH = PR * PW * NCBI;              // staged input chunks per band
  constexpr int DCH = R * W * NCBO;                // staged dz chunks per band
  constexpr int XT = (XCH + NT_ - 1) / NT_, DT = (DCH + NT_ - 1) / NT_;
  constexpr int XCR = (XCH + 63) / 64 * 64, DCR = (DCH + 63) / 64 * 64;   // wave-granular LDS images
  constexpr int XROW = NCBI * 16, DROW = NCBO * 16;   // LDS bytes per pixel
  static_assert(R * W % 32 == 0 && (W == 16 || W == 32), "bands must be whole 32-pixel K-steps");

  // two band buffers (DMA of band i+1 overlaps the MFMAs of band i); whole
  // NT_-chunk rows so every DMA wave-instruction has a full 1 KiB target
  __shared__ __attribute__((aligned(16))) uint4 xs[NB][XCR];
  __shared__ __attribute__((aligned(16))) uint4 ds[NB][DCR];

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int s = blockIdx.x;
  const GroupRec gr = group_rec(a.gtab, blockIdx.y, a.n_in, 0, 0, nullptr);
  const int g = gr.g;
  const int nbi = a.H / R;                                     // bands per image
  const int bps = a.pps / (R * W);                             // bands per split
  const int band0 = s * bps;
  const int band1 = min(band0 + bps, a.B * nbi);
  const long img_in = (long)a.H * W * NCBI * 8, img_out = (long)a.H * W * NCBO * 8;
  const int first_in = __builtin_ctz(gr.in_mask | 0x100);
  const bool single = __builtin_popcount(gr.in_mask) == 1 || a.gather;
  const long fold_off = (long)g * a.B * img_in;

  auto issue = [&](int band, int buf) {
    const int b = band / nbi, h0 = (band - b * nbi) * R;
    const uint16_t* src0 = a.gather ? static_cast<const uint16_t*>(a.in[0]) +
                                          a.gather[((long)a.st->cur_step * a.G + g) * a.B + b] * img_in
                                    : static_cast<const uint16_t*>(a.in[first_in & 7]) + fold_off + (long)b * img_in;
#pragma unroll
    for (int j = 0; j < XT; ++j) {
      const int i = tid + NT_ * j;
      const int cb = i % NCBI, pix = i / NCBI;
      const int hh = h0 - KH / 2 + pix / PW, ww = pix % PW - KW / 2;
      const bool ok = i < XCH && hh >= 0 && hh < a.H && ww >= 0 && ww < W;
      const long off = ((long)hh * W + ww) * (NCBI * 8) + cb * 8;
      if (single) {
        if (NT_ * j + 64 * wave < XCR)          // wave-uniform: whole 1 KiB targets only
          wf_glds16(ok ? (const void*)(src0 + off) : (const void*)wf_zero16, &xs[buf][NT_ * j + 64 * wave]);
      } else if (i < XCH) {
        // N-ary DAG input: sum in fp32 through registers
        float sum[8] = {0, 0, 0, 0, 0, 0, 0, 0}, t8[8];
        if (ok) {
#pragma unroll
          for (int k = 0; k < GT_MAXSLOT; ++k) {
            if (!((gr.in_mask >> k) & 1)) continue;
            unpack8(*reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(a.in[k]) + fold_off +
                                                    (long)b * img_in + off), t8);
#pragma unroll
            for (int e = 0; e < 8; ++e) sum[e] += t8[e];
          }
        }
        xs[buf][i] = pack8(sum);
      }
    }
    const char* dsrc = reinterpret_cast<const char*>(static_cast<const uint16_t*>(a.dz) + (long)g * a.B * img_out +
                                                     (long)b * img_out + (long)h0 * W * NCBO * 8);
#pragma unroll
    for (int j = 0; j < DT; ++j) {
      const int i = tid + NT_ * j;
      if (NT_ * j + 64 * wave < DCR)
        wf_glds16(i < DCH ? (const void*)(dsrc + (long)i * 16) : (const void*)wf_zero16, &ds[buf][NT_ * j + 64 * wave]);
    }
  };

  // ---- per-lane operand addresses (fixed for the whole kernel) -------------
  const int gq = lane >> 4, q = (lane >> 2) & 3, p = lane & 3, l16 = lane & 15;
  const int px0 = 8 * gq + q;                                  // lane's first K row (pixel of a K-step)
  const int prow = px0 / W, pcol = px0 % W;                    // its position inside the band
  const int xlane = (prow * PW + pcol) * XROW;
  const int dlane = px0 * DROW + p * 8;
  int xoff[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    const int n = wave + NW * t;
    int c = 2 * n + (p >> 1);
    if (c >= NCH) c = 0;                                       // bias / padding columns: any valid row
    const int kk = c / NCBI, cb = c % NCBI;
    xoff[t] = xlane + ((kk / KW) * PW + (kk % KW)) * XROW + cb * 16 + (p & 1) * 8;
  }
  const bool ones_lane = l16 == (NCH & 1) * 8;                 // the bias column inside its tile

  f32x4_t acc[MT][TPW];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int t = 0; t < TPW; ++t) acc[m][t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  if (band0 < band1) issue(band0, 0);
  int cur = 0;
  for (int band = band0; band < band1; ++band, cur ^= (NB - 1)) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();                      // band landed everywhere; buffer cur^1 no longer read
    if (NB == 2 && band + 1 < band1) issue(band + 1, cur ^ 1);
    const char* xb = reinterpret_cast<const char*>(xs[cur]);
    const char* db = reinterpret_cast<const char*>(ds[cur]) + dlane;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int xrow_off = ((ks * 32) / W) * PW * XROW;        // compile-time after unrolling
      uint4 afr[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const char* d0 = db + ks * 32 * DROW + m * 32;
        afr[m] = tr_pair(d0, d0 + 4 * DROW);
      }
#pragma unroll
      for (int t = 0; t < TPW; ++t) {
        const int n = wave + NW * t;
        if (n >= NKT) continue;
        const char* x0 = xb + xrow_off + xoff[t];
        uint4 bfr = tr_pair(x0, x0 + 4 * XROW);
        if (n == NCH / 2 && ones_lane) bfr = make_uint4(0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u);
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[m][t] = mfma16(afr[m], bfr, acc[m][t]);
      }
    }
    if (NB == 1 && band + 1 < band1) {
      __syncthreads();                    // every wave is done reading the single buffer
      issue(band + 1, 0);
    }
  }

  // ---- partial out: lane holds rows 4*kq..+3 (co) of column l16 (k col) ------
  const int kq = lane >> 4;
  constexpr int Kdim = NCH * 8;
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    const int n = wave + NW * t;
    if (n >= NKT) continue;
    const int col = n * 16 + l16;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int co = m * 16 + kq * 4 + i;
        if (co >= a.Coutp) continue;
        if (col < Kdim)
          a.part_w[(((long)s * a.G + g) * a.Coutp + co) * Kdim + col] = acc[m][t][i];
        else if (col == Kdim && a.part_b)
          a.part_b[((long)s * a.G + g) * a.Coutp + co] = acc[m][t][i];
      }
  }
}

// ---------------------------------------------------------------------------
// fp32 tensors (prec 1): the same workgroup shape, but the band is staged
// through registers -- each 32-byte fp32 chunk is loaded (DAG inputs summed),
// split exactly into three bf16 planes (common.h split8) and written to
// plane-major LDS images that the same ds_read_b64_tr_b16 operand reads walk;
// every (dz tile, input tile) pair is then the six-term split product. The
// next band's global loads are issued before the current band's MFMAs and
// written to LDS after them (async-STAGE split).
// ---------------------------------------------------------------------------
//
// PK: the last output-channel tile has <= 4 real channels (conv_fast_kernel's
// packed tile, on the M side): a per-band LDS block holds, per pixel, the
// three dz planes of those channels at row 4c + p, and that tile costs three
// MFMAs per column tile and K-step (one per input plane) instead of six.
// NZ > 1 (wide layers: 104 x 936 weights do not fit one workgroup's
// registers): grid.z splits the k-column tiles into NZ slices, each workgroup
// stages the same bands and owns its slice; the co tiles are then walked in
// the outer loop (one dz fragment set live at a time).
template <int KH, int KW, int NCBI, int NCBO, int W, int R, int NW, int NB, int PK = 0, int NZ = 1>
__global__ void __launch_bounds__(NW * 64) wgrad_fast_f32_kernel(WgradArgs a) {
  constexpr int NPL = GT_NPL_F32;
  constexpr int NT_ = NW * 64;                     // threads
  constexpr int PW = W + KW - 1, PR = R + KH - 1;
  constexpr int NCH = KH * KW * NCBI;              // weight chunks (8 input channels each)
  constexpr int NKT = (NCH + 1 + 1) / 2;           // 16-column tiles incl. the bias chunk
  constexpr int MT = (NCBO * 8 + 15) / 16;         // output-channel tiles
  constexpr int TPW = ((NKT + NZ - 1) / NZ + NW - 1) / NW;   // k-column tiles per wave (in its slice)
  constexpr int KS = R * W / 32;                   // K-steps per band
  constexpr int XCH = PR * PW * NCBI;              // staged input chunks per band (per plane)
  constexpr int DCH = R * W * NCBO;                // staged dz chunks per band (per plane)
  constexpr int XT = (XCH + NT_ - 1) / NT_, DT = (DCH + NT_ - 1) / NT_;
  // LDS pixel strides in 16-byte chunks, odd: an even stride (8 / 16 / 32 chunks, the wide deep
  // space) put the 8 pixels of a ds_read_b64_tr_b16 pass on the same banks (PMC LDSbc 0.7-0.8)
  // (kept unpadded when the padded double buffers would not fit the 160 KB of LDS)
  constexpr int NCBIP0 = NCBI + ((NCBI & 1) ? 0 : 1), NCBOP0 = NCBO + ((NCBO & 1) ? 0 : 1);
  constexpr bool PADOK = (long)NB * NPL * (PR * PW * NCBIP0 + R * W * NCBOP0) * 16 + (long)NB * R * W * 32 <= 160 * 1024;
  constexpr int NCBIP = PADOK ? NCBIP0 : NCBI, NCBOP = PADOK ? NCBOP0 : NCBO;
  constexpr int XCHL = PR * PW * NCBIP, DCHL = R * W * NCBOP;   // LDS chunks per band (per plane)
  constexpr int XROW = NCBIP * 16, DROW = NCBOP * 16;   // LDS bytes per pixel (one plane)
  auto xslot = [&](int i) {
    if constexpr (NCBIP == NCBI) return i;
    else return (i / NCBI) * NCBIP + i % NCBI;
  };
  auto dslot = [&](int i) {
    if constexpr (NCBOP == NCBO) return i;
    else return (i / NCBO) * NCBOP + i % NCBO;
  };
  constexpr bool MOUT = NZ > 1;                    // co tiles in the outer loop
  static_assert(R * W % 32 == 0 && (W == 8 || W == 16 || W == 32), "bands must be whole 32-pixel K-steps");

  __shared__ __attribute__((aligned(16))) uint4 xs[NB][NPL][XCHL];
  __shared__ __attribute__((aligned(16))) uint4 ds[NB][NPL][DCHL];
  constexpr int PKC = 2 * (MT - 1);                // dz chunk holding the packed tile's channels
  constexpr int PKR = PK ? R * W : 1;
  __shared__ __attribute__((aligned(16))) uint4 dpk[NB][PKR][2];   // packed plane rows per pixel (PK)
  static_assert(!PK || PKC < NCBO, "packed tile inside the staged dz chunks");

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int s = blockIdx.x;
  const int nz0 = NZ > 1 ? (int)blockIdx.z * NW * TPW : 0;       // first column tile of this slice
  const GroupRec gr = group_rec(a.gtab, blockIdx.y, a.n_in, 0, 0, nullptr);
  const int g = gr.g;
  const int nbi = a.H / R;                                     // bands per image
  const int bps = a.pps / (R * W);                             // bands per split
  const int band0 = s * bps;
  const int band1 = min(band0 + bps, a.B * nbi);
  const long img_in = (long)a.H * W * NCBI * 8, img_out = (long)a.H * W * NCBO * 8;
  const long fold_off = (long)g * a.B * img_in;
  const int n_src = a.gather ? 1 : __builtin_popcount(gr.in_mask);
  const float* in0 = static_cast<const float*>(a.in[__builtin_ctz(gr.in_mask | 0x100) & 7]);

  float xr[XT][8], dr[DT][8];
  auto load = [&](int band) {
    const int b = band / nbi, h0 = (band - b * nbi) * R;
    const long boff = fold_off + (long)b * img_in;
    const float* src0 = a.gather ? static_cast<const float*>(a.in[0]) +
                                       a.gather[((long)a.st->cur_step * a.G + g) * a.B + b] * img_in
                                 : in0 + boff;
#pragma unroll
    for (int j = 0; j < XT; ++j) {
      const int i = tid + NT_ * j;
      const int cb = i % NCBI, pix = i / NCBI;
      const int hh = h0 - KH / 2 + pix / PW, ww = pix % PW - KW / 2;
      const bool ok = i < XCH && hh >= 0 && hh < a.H && ww >= 0 && ww < W;
      const long off = ((long)hh * W + ww) * (NCBI * 8) + cb * 8;
      // unconditional loads (zero chunk for the halo): see conv_fast_kernel's staging
      if (n_src == 1) {
#pragma unroll
        for (int e = 0; e < 8; ++e) xr[j][e] = 0.f;
        if (ok) load8f(src0 + off, xr[j]);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) xr[j][e] = 0.f;
        for (int k = 0; k < GT_MAXSLOT; ++k) {
          if (!((gr.in_mask >> k) & 1)) continue;
          float t8[8];
          load8f_or0(static_cast<const float*>(a.in[k]) + boff + off, ok, t8);
#pragma unroll
          for (int e = 0; e < 8; ++e) xr[j][e] += t8[e];
        }
      }
    }
    const float* dsrc = static_cast<const float*>(a.dz) + (long)g * a.B * img_out + (long)b * img_out +
                        (long)h0 * W * NCBO * 8;
#pragma unroll
    for (int j = 0; j < DT; ++j) {
      const int i = tid + NT_ * j;
      if (i < DCH) load8f(dsrc + (long)i * 8, dr[j]);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < XT; ++j) {
      const int i = tid + NT_ * j;
      if (i < XCH) split8(xr[j], xs[buf][0][xslot(i)], xs[buf][1][xslot(i)], xs[buf][2][xslot(i)]);
    }
#pragma unroll
    for (int j = 0; j < DT; ++j) {
      const int i = tid + NT_ * j;
      if (i >= DCH) continue;
      uint4 q0, q1, q2;
      split8(dr[j], q0, q1, q2);
      ds[buf][0][dslot(i)] = q0;
      ds[buf][1][dslot(i)] = q1;
      ds[buf][2][dslot(i)] = q2;
      if (PK && i % NCBO == PKC) {
        // channels 16 (MT-1) + c, c < 4: plane p at element 4c + p (element 4c + 3 = 0)
        const int creal = a.cout_real - 16 * (MT - 1);
        uint32_t w[8];
        const uint32_t h0[4] = {q0.x & 0xffffu, q0.x >> 16, q0.y & 0xffffu, q0.y >> 16};
        const uint32_t h1[4] = {q1.x & 0xffffu, q1.x >> 16, q1.y & 0xffffu, q1.y >> 16};
        const uint32_t h2[4] = {q2.x & 0xffffu, q2.x >> 16, q2.y & 0xffffu, q2.y >> 16};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          w[2 * c] = c < creal ? (h0[c] | (h1[c] << 16)) : 0u;
          w[2 * c + 1] = c < creal ? h2[c] : 0u;
        }
        const int px = i / NCBO;
        dpk[buf][px][0] = make_uint4(w[0], w[1], w[2], w[3]);
        dpk[buf][px][1] = make_uint4(w[4], w[5], w[6], w[7]);
      }
    }
  };

  // ---- per-lane operand addresses (fixed for the whole kernel) -------------
  const int gq = lane >> 4, q = (lane >> 2) & 3, p = lane & 3, l16 = lane & 15;
  const int px0 = 8 * gq + q;                                  // lane's first K row (pixel of a K-step)
  const int prow = px0 / W, pcol = px0 % W;                    // its position inside the band
  const int xlane = (prow * PW + pcol) * XROW;
  const int dlane = px0 * DROW + p * 8;
  int xoff[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    const int n = nz0 + wave + NW * t;
    int c = 2 * n + (p >> 1);
    if (c >= NCH) c = 0;                                       // bias / padding columns: any valid row
    const int kk = c / NCBI, cb = c % NCBI;
    xoff[t] = xlane + ((kk / KW) * PW + (kk % KW)) * XROW + cb * 16 + (p & 1) * 8;
  }
  const bool ones_lane = l16 == (NCH & 1) * 8;                 // the bias column inside its tile

  f32x4_t acc[MT][TPW];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int t = 0; t < TPW; ++t) acc[m][t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  // Two buffers: the two halves of the workgroup (waves w and w + NW/2 share a SIMD) take
  // opposite orders inside a band -- the first half multiplies, then stages the next band; the
  // second half stages first (from registers loaded one band earlier), then multiplies -- so on
  // every SIMD one wave's split + LDS stores run beside the other wave's MFMAs instead of all
  // waves staging while the matrix pipe idles. Same per-wave MFMA order: bit-identical.
  const bool early = NB == 2 && wave >= NW / 2;
  if (band0 < band1) {
    load(band0);
    store(0);
    if (early && band0 + 1 < band1) load(band0 + 1);
  }
  int cur = 0;
  for (int band = band0; band < band1; ++band, cur ^= (NB - 1)) {
    __syncthreads();                      // band `cur` staged everywhere; the other buffer no longer read
    const bool more = band + 1 < band1;
    if (early) {
      if (more) {
        store(cur ^ 1);                   // band + 1, loaded during the previous band
        if (band + 2 < band1) load(band + 2);
      }
    } else if (more) {
      load(band + 1);                     // global loads in flight during the MFMAs
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int xrow_off = ((ks * 32) / W) * PW * XROW;        // compile-time after unrolling
      // dz^T fragments of co tile m (three planes, or the packed plane rows)
      auto load_at = [&](int m, uint4* af) {
        if (PK && m == MT - 1) {
          const char* d0 = reinterpret_cast<const char*>(dpk[cur]) + px0 * 32 + p * 8 + ks * 32 * 32;
          af[0] = tr_pair(d0, d0 + 4 * 32);
          return;
        }
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl) {
          const char* d0 = reinterpret_cast<const char*>(ds[cur][pl]) + dlane + ks * 32 * DROW + m * 32;
          af[pl] = tr_pair(d0, d0 + 4 * DROW);
        }
      };
      // the im2col fragments of column tile t
      auto load_bt = [&](int t, uint4* bfr) {
        const int n = nz0 + wave + NW * t;
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl) {
          const char* x0 = reinterpret_cast<const char*>(xs[cur][pl]) + xrow_off + xoff[t];
          bfr[pl] = tr_pair(x0, x0 + 4 * XROW);
        }
        if (n == NCH / 2 && ones_lane) {                       // exact 1.0 = (1, 0, 0)
          bfr[0] = make_uint4(0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u);
          bfr[1] = bfr[2] = make_uint4(0, 0, 0, 0);
        }
      };
      auto mma = [&](int m, const uint4* af, const uint4* bf, f32x4_t c) {
        if (PK && m == MT - 1) {
          c = mfma16(af[0], bf[2], c);
          c = mfma16(af[0], bf[1], c);
          return mfma16(af[0], bf[0], c);
        }
        return mfma_np<NPL>(af, bf, c);
      };
      if constexpr (MOUT) {
        // all of this wave's column fragments live; co tiles streamed (next one read during the MFMAs)
        uint4 bfr[TPW][NPL];
#pragma unroll
        for (int t = 0; t < TPW; ++t) load_bt(t, bfr[t]);
        uint4 af[2][NPL];
        load_at(0, af[0]);
#pragma unroll
        for (int m = 0; m < MT; ++m) {
          if (m + 1 < MT) load_at(m + 1, af[(m + 1) & 1]);
#pragma unroll
          for (int t = 0; t < TPW; ++t)
            if (nz0 + wave + NW * t < NKT) acc[m][t] = mma(m, af[m & 1], bfr[t], acc[m][t]);
        }
      } else {
        uint4 afr[MT][NPL];
#pragma unroll
        for (int m = 0; m < MT; ++m) load_at(m, afr[m]);
        // the next column tile's im2col fragments are read while this tile's MFMAs run
        uint4 bfr[2][NPL];
        load_bt(0, bfr[0]);
#pragma unroll
        for (int t = 0; t < TPW; ++t) {
          const int n = wave + NW * t;
          if (t + 1 < TPW) load_bt(t + 1, bfr[(t + 1) & 1]);
          if (n >= NKT) continue;
#pragma unroll
          for (int m = 0; m < MT; ++m) acc[m][t] = mma(m, afr[m], bfr[t & 1], acc[m][t]);
        }
      }
    }
    if (more && !early) {
      if (NB == 1) __syncthreads();       // every wave is done reading the single buffer
      store(cur ^ (NB - 1));
    }
  }

  // ---- partial out: lane holds rows 4*kq..+3 (co) of column l16 (k col) ------
  const int kq = lane >> 4;
  constexpr int Kdim = NCH * 8;
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    const int n = nz0 + wave + NW * t;
    if (n >= NKT) continue;
    const int col = n * 16 + l16;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        // packed tile: row 4kq + p = plane p of channel 16 (MT-1) + kq; its sum is that channel's value
        const bool pkm = PK && m == MT - 1;
        const int co = pkm ? m * 16 + kq + 4 * i : m * 16 + kq * 4 + i;
        const float v = pkm ? (i == 0 ? acc[m][t][0] + acc[m][t][1] + acc[m][t][2] : 0.f) : acc[m][t][i];
        if (co >= a.Coutp) continue;
        if (col < Kdim)
          a.part_w[(((long)s * a.G + g) * a.Coutp + co) * Kdim + col] = v;
        else if (col == Kdim && a.part_b)
          a.part_b[((long)s * a.G + g) * a.Coutp + co] = v;
      }
  }
}

// Split-K reduction of a wgrad launch's partials, launched right after it on
// the weight-gradient stream: split 0 <- sum over splits in split order
// (adam_segments' order, so the update is bit-identical); the optimizer at the
// end of the step then reads one gradient instead of S partials. Grid
// (chunks of 4 elements per thread, launch groups).
