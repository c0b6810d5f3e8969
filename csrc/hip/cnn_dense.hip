// Genetic-CNN head + optimizer kernels for MI355X (gfx950).
//
// step_begin   : advances the captured step's device state (batch row, Adam t,
//                bias-corrected lr_t) -- keeps the whole step graph-replayable.
// dense_fwd    : K7  h = dropout(relu(x W1 + b1)): split-K over feature ranges
//                straight from the fp32 master W1 (exact bf16 planes staged in
//                LDS, v_mfma_f32_16x16x32_bf16), the ranges summed in order by
//                a second launch that runs the epilogue; dropout keyed by
//                hash(seed, fold, global step, row, unit) (deterministic).
// head         : K9  logits = h W2 + b2, softmax, loss gradient (bce_compat =
//                Keras softmax + binary_crossentropy with eps clipping, or ce),
//                dh -> dH = dh * scale * (h > 0), dW2, db2, db1 -- one
//                workgroup per fold, everything through LDS.
// dense_dgrad  : K8  dX = dH W1^T from the master W1: fp32 on the f32-input
//                MFMA (exact products), bf16 mode on the bf16 MFMA.
// dense_wgrad_adam : K8+K10 fused: dW1 = X^T dH (K = batch, VALU) immediately
//                applied by Adam to the fp32 master/m/v -- the gradient of the
//                largest tensor (90 % of all parameters) never touches HBM.
// adam_segments: K10 multi-tensor Adam over every other parameter; reduces
//                the conv wgrad split-K partials in fixed order, writes bf16
//                copies (and the flipped/transposed dgrad copy of conv weights).
// eval_head    : per-sample loss / binary-accuracy / categorical-accuracy.

#include <algorithm>
#include <cstdlib>

#include "common.h"

#define HEAD_MAXC_FWD 16
#define ADAM_B1 0.9f
#define ADAM_B2 0.999f
#define ADAM_EPS 1e-7f
#define CLIP_EPS 1e-7f
#define GT_DGRAD_BUF 2     // dense_dgrad_stream2_kernel: k-steps in flight per wave (4: 3 % slower, profiles/dense_dgrad_buf_ab_r4.txt)
#define GT_ADAM_UNROLL 1   // adam_segments_kernel tiled path: elements per thread whose loads issue together (4: neutral, profiles/adam_unroll_ab_r4.txt)
// (dense_wgrad_adam_kernel with the optimizer-state loads hoisted above the row branches was 1.67x slower:
// profiles/dense_wadam_hoist_ab_r3.txt; removed)

__global__ void step_begin_kernel(StepState* s) {
  s->cur_step = s->step_ctr;
  s->step_ctr += 1;
  s->global_step += 1;
  const float t = s->t + 1.0f;
  s->t = t;
  s->lr_t = s->opt == 1 ? s->lr : s->lr * sqrtf(1.0f - powf(ADAM_B2, t)) / (1.0f - powf(ADAM_B1, t));
}

// ---------------------------------------------------------------------------
struct DenseFwdArgs {
  const void* x;           // [G][B][Fp] (pooled features, NHWC flatten), bf16 or fp32 (prec)
  const void* wt;          // transposed copy of W1 [G][Up][Fp]: bf16 (prec 0), fp32 (prec 1: split on the fly)
  const float* bias;       // [G][Up]
  void* out;               // [G][B][Up] bf16 or fp32
  const float* w2;         // [G][Up][C] fp32: dense2 weights (fused partial logits)
  float* plog;             // [G][Up/16][B][C] partial logits of this 16-unit tile (fixed-order sum later)
  const StepState* st;
  const int* fold_ids;     // [G]
  const unsigned* seeds;   // [G] per-group dropout keys (population jobs) or null -> seed
  int G, B, Fp, Up;
  float drop_p;
  int train;
  unsigned seed;
  int C;
  int prec;                // 0: bf16 tensors, bf16 MFMA; 1: fp32 tensors, split-fp32 MFMA (common.h)
  long wps;                // unused (kept for the ABI)
  int row_off;             // data parallelism (X5): this rank's first row of the full batch (dropout keys)
  // split-K forward (dense_fwd_sk_kernel): W1 read from the fp32 master [G][Fp][Up] itself, KS
  // feature splits per output tile, partial tiles in `part` (summed in range order by dense_fwd_skred_kernel)
  const float* w1;
  float* part;             // [G][ceil(B/32)][Up/64][KS][4][2][64] f32x4 range partials
  int* cnt;                // unused, 0 (ABI: the round-4 last-workgroup reduction's arrival counters)
  int ks;
};

// bias + ReLU + dropout of one 16-unit x 32-row tile (D[row = unit][col =
// batch row], two 16-row MFMA tiles), the activation store and the tile's
// partial logits (plog tile index `utile`)
template <int PREC>
__device__ __forceinline__ void dense_fwd_epilogue(const DenseFwdArgs& a, int g, int u_t, int b0,
                                                   const f32x4_t (&acc)[2], int lane, int utile) {
  typedef typename ActT<PREC>::T AT;
  const int kq = lane >> 4, l16 = lane & 15;
  // D[row = unit][col = batch row]
  const int u0 = u_t + kq * 4;
  const bool uok = u0 < a.Up;
  const float keep_scale = 1.0f / (1.0f - a.drop_p);
  const uint32_t thr = (uint32_t)(a.drop_p * 4294967296.0);
  const int gstep = a.st ? a.st->global_step : 0;
  const uint32_t fid = a.fold_ids ? (uint32_t)a.fold_ids[g] : (uint32_t)g;
  const uint32_t seed = a.seeds ? a.seeds[g] : a.seed;
  const int C = a.C;
  const float* w2 = a.w2 + ((long)g * a.Up + u0) * C;
  // this lane's dense2 rows, all loads in flight at once (a load per class under
  // a `c < C` branch waited for each one in turn)
  float w2v[4][HEAD_MAXC_FWD];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int c = 0; c < HEAD_MAXC_FWD; ++c)
      w2v[i][c] = (a.plog != nullptr && uok) ? w2[i * C + min(c, C - 1)] : 0.f;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = b0 + h * 16 + l16;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (uok && row < a.B) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float z = acc[h][i] + a.bias[(long)g * a.Up + u0 + i];
        z = fmaxf(z, 0.f);
        if (a.train && a.drop_p > 0.f) {
          const uint32_t r = hash4(seed ^ (fid * 0x632be5abU), (uint32_t)gstep, (uint32_t)(row + a.row_off),
                                   (uint32_t)(u0 + i));
          z = (r >= thr) ? z * keep_scale : 0.f;
        }
        v[i] = PREC ? z : bf2f(f2bf(z));      // the head sees exactly the stored activation
      }
      AT* dst = static_cast<AT*>(a.out) + ((long)g * a.B + row) * a.Up + u0;
      if (PREC) *reinterpret_cast<float4*>(dst) = make_float4(v[0], v[1], v[2], v[3]);
      else *reinterpret_cast<uint2*>(dst) = pack4(v);
    }
    if (a.plog == nullptr) continue;
    // partial logits of this 16-unit tile: 4 units per lane, reduced over the 4 lane groups
    float pl[HEAD_MAXC_FWD];
#pragma unroll
    for (int c = 0; c < HEAD_MAXC_FWD; ++c) {
      float t = 0.f;
      if (c < C && uok) {
#pragma unroll
        for (int i = 0; i < 4; ++i) t += v[i] * w2v[i][c];
      }
      t += __shfl_xor(t, 16);
      t += __shfl_xor(t, 32);
      pl[c] = t;
    }
    if (kq == 0 && row < a.B) {
      float* dst = a.plog + (((long)g * (a.Up / 16) + utile) * a.B + row) * C;
      for (int c = 0; c < C; ++c) dst[c] = pl[c];
    }
  }
}

// raw loads of 8 consecutive values (zero chunk when !ok: no branch around a load)
template <typename T>
__device__ __forceinline__ void ld8_raw(const T* p, bool ok, float* f) {
  if constexpr (sizeof(T) == 4) {
    load8f(ok ? reinterpret_cast<const float*>(p) : gt_zero8, f);
  } else {
    const uint4 v = *reinterpret_cast<const uint4*>(ok ? reinterpret_cast<const void*>(p)
                                                       : reinterpret_cast<const void*>(gt_zero8));
    unpack8(v, f);
  }
}

template <int PREC>
__device__ __forceinline__ void planes8(const float* f, uint4* q) {
  if (PREC) split8(f, q[0], q[1], q[2]);
  else q[0] = pack8(f);
}

// linear workgroup id -> (x, z) with the workgroups of one z on as few XCDs as
// possible (hardware deals consecutive ids round-robin over the 8 XCDs)
__device__ __forceinline__ void xcd_tile(int& bx, int& bz) {
  const int nbx = gridDim.x, total = nbx * gridDim.z;
  int lin = blockIdx.z * nbx + blockIdx.x;
  if ((total & 7) == 0) lin = (lin & 7) * (total >> 3) + (lin >> 3);
  bz = lin / nbx;
  bx = lin - bz * nbx;
}

// plane q (0..2) of the exact split of p (q = 0: the bf16 rounding)
__device__ __forceinline__ void split3(float p, uint16_t* h) {
  h[0] = f2bf(p);
  const float r1 = p - bf2f(h[0]);
  h[1] = f2bf(r1);
  h[2] = f2bf(r1 - bf2f(h[1]));
}

// Split-K forward (the default): one workgroup = 4 unit tiles (64 units) x 32
// rows x ONE of KS contiguous ranges of the feature k-steps, so a launch is
// (Up/64) x KS x G workgroups instead of (Up/64) x G -- the streaming kernel
// ran 8 workgroups per group, 16 at 2 groups and 200 at 25 (latency-bound at
// every population size, each wave walking 25 of the 100 k-steps). W1 comes
// from the fp32 master [G][Fp][Up] (the transposed copy the optimizer used to
// write every step is gone): per k-step the workgroup stages the [32 f][64 u]
// W1 tile (16-byte loads along u) and the [32 rows][32 f] activation tile
// into LDS as exact bf16 planes, and each wave reads its unit tile's A operand
// with ds_read_b64_tr_b16 (transposing reads: k = feature runs down the rows
// of the natural layout). Wave w owns unit tile w over the whole range; the
// KS range partials go to `part` and dense_fwd_skred_kernel sums them in
// range order and runs the bias / ReLU / dropout / partial-logit epilogue.
// Every sum has a fixed order: deterministic, and independent of how many
// groups share the launch (KS is a per-shape constant).
#define DSK_WLD 72            // W1 tile row stride (bf16): 64 units + 8 (16-byte aligned rows)
#define DSK_XLD 40            // activation tile row stride (bf16): 32 features + 8
typedef __attribute__((ext_vector_type(4))) short dsk_short4;

__device__ __forceinline__ uint4 dsk_tr_frag(const uint16_t* tile, int col0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  typedef __attribute__((address_space(3))) dsk_short4 lds_s4;
  const uint16_t* r0 = tile + (8 * g + q) * DSK_WLD + col0 + 4 * p;
  const uint16_t* r1 = r0 + 4 * DSK_WLD;
  const dsk_short4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(r0));
  const dsk_short4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(r1));
  typedef __attribute__((ext_vector_type(8))) short short8_t;
  return __builtin_bit_cast(uint4, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

template <int PREC>
__global__ void __launch_bounds__(256) dense_fwd_sk_kernel(DenseFwdArgs a) {
  constexpr int NPL = PREC ? GT_NPL_F32 : 1;
  typedef typename ActT<PREC>::T AT;
  __shared__ __attribute__((aligned(16))) uint16_t wl[2][NPL][32 * DSK_WLD];
  __shared__ __attribute__((aligned(16))) uint16_t xl[2][NPL][32 * DSK_XLD];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, kq = lane >> 4, l16 = lane & 15;
  int bx, g;
  xcd_tile(bx, g);
  const int KS = a.ks, nut = a.Up / 64, nby = gridDim.y;
  const int ut = bx / KS, s = bx - ut * KS;
  const int u_t = ut * 64;
  const int b0 = blockIdx.y * 32;
  const int nks = (a.Fp + 31) >> 5;                         // k-steps of 32 features
  const int per = (nks + KS - 1) / KS;
  const int j0 = s * per, j1 = min(nks, j0 + per);
  // staging lanes: W1 row f = tid / 8 of the k-step, units u_t + 8 (tid % 8) .. +7;
  // activations row b0 + tid / 8, features 4 (tid % 8) .. +3
  const int wf = tid >> 3, wu = (tid & 7) * 8;
  const float* w1 = a.w1 + (long)g * a.Fp * a.Up + u_t + wu;
  const int xr = b0 + (tid >> 3), xf = (tid & 7) * 4;
  const bool xok = xr < a.B;
  const AT* xg = static_cast<const AT*>(a.x) + ((long)g * a.B + (xok ? xr : 0)) * a.Fp + xf;
  float rw[8], rx[4];
  auto load = [&](int j) {
    const int f = 32 * j + wf;
    const bool ok = j < j1 && f < a.Fp;
    const float* src = ok ? w1 + (long)f * a.Up : gt_zero8;
    const float4 q0 = *reinterpret_cast<const float4*>(src);
    const float4 q1 = *reinterpret_cast<const float4*>(src + (ok ? 4 : 0));
    rw[0] = q0.x; rw[1] = q0.y; rw[2] = q0.z; rw[3] = q0.w;
    rw[4] = q1.x; rw[5] = q1.y; rw[6] = q1.z; rw[7] = q1.w;
    const int fx = 32 * j + xf;
    const bool okx = j < j1 && xok && fx < a.Fp;            // Fp % 8 == 0: a 4-run never straddles the end
    if constexpr (PREC != 0) {
      const float4 v = *reinterpret_cast<const float4*>(okx ? reinterpret_cast<const float*>(xg + 32 * j) : gt_zero8);
      rx[0] = v.x; rx[1] = v.y; rx[2] = v.z; rx[3] = v.w;
    } else {
      const uint2 v = *reinterpret_cast<const uint2*>(okx ? reinterpret_cast<const void*>(xg + 32 * j)
                                                          : reinterpret_cast<const void*>(gt_zero8));
      rx[0] = __uint_as_float(v.x << 16); rx[1] = __uint_as_float(v.x & 0xffff0000u);
      rx[2] = __uint_as_float(v.y << 16); rx[3] = __uint_as_float(v.y & 0xffff0000u);
    }
  };
  auto stage = [&](int buf) {
    uint4 wp[NPL];
    planes8<PREC>(rw, wp);
#pragma unroll
    for (int p = 0; p < NPL; ++p) *reinterpret_cast<uint4*>(&wl[buf][p][wf * DSK_WLD + wu]) = wp[p];
    if constexpr (PREC != 0) {
      uint16_t h[4][3];
#pragma unroll
      for (int i = 0; i < 4; ++i) split3(rx[i], h[i]);
#pragma unroll
      for (int p = 0; p < NPL; ++p)
        *reinterpret_cast<uint2*>(&xl[buf][p][(tid >> 3) * DSK_XLD + xf]) =
            make_uint2(h[0][p] | ((uint32_t)h[1][p] << 16), h[2][p] | ((uint32_t)h[3][p] << 16));
    } else {
      *reinterpret_cast<uint2*>(&xl[buf][0][(tid >> 3) * DSK_XLD + xf]) = pack4(rx);
    }
  };
  f32x4_t acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  load(j0);
  for (int j = j0; j < j1; ++j) {
    const int buf = (j - j0) & 1;
    stage(buf);
    __syncthreads();                    // buf complete; the other buffer's readers are done (previous step)
    load(j + 1);                        // next k-step's raw values in flight during the MFMAs
    uint4 af[NPL], b0f[NPL], b1f[NPL];
#pragma unroll
    for (int p = 0; p < NPL; ++p) {
      af[p] = dsk_tr_frag(wl[buf][p], wave * 16, lane);
      b0f[p] = *reinterpret_cast<const uint4*>(&xl[buf][p][l16 * DSK_XLD + kq * 8]);
      b1f[p] = *reinterpret_cast<const uint4*>(&xl[buf][p][(16 + l16) * DSK_XLD + kq * 8]);
    }
    acc[0] = mfma_np<NPL>(af, b0f, acc[0]);
    acc[1] = mfma_np<NPL>(af, b1f, acc[1]);
  }
  if (KS > 1) {                        // range partial; dense_fwd_skred_kernel sums the ranges
    const long tile = ((long)g * nby + blockIdx.y) * nut + ut;
    f32x4_t* pt = reinterpret_cast<f32x4_t*>(a.part) + (((tile * KS + s) * 4 + wave) * 2) * 64 + lane;
    pt[0] = acc[0];
    pt[64] = acc[1];
    return;
  }
  f32x4_t r2[2] = {acc[0], acc[1]};
  dense_fwd_epilogue<PREC>(a, g, u_t + wave * 16, b0, r2, lane, u_t / 16 + wave);
}

// the KS range partials of a split-K forward tile summed in range order (a
// launch of its own: visibility of the partials comes with the kernel
// boundary -- a last-arriving-workgroup protocol needed a device-scope L2
// write-back per workgroup and ran 10x slower), then the epilogue.
// Grid (Up/64, ceil(B/32), G), wave w = unit tile w.
template <int PREC>
__global__ void __launch_bounds__(256) dense_fwd_skred_kernel(DenseFwdArgs a) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  int ut, g;
  xcd_tile(ut, g);
  const int KS = a.ks, nut = a.Up / 64, nby = gridDim.y;
  const long tile = ((long)g * nby + blockIdx.y) * nut + ut;
  const f32x4_t* pt = reinterpret_cast<const f32x4_t*>(a.part) + ((tile * KS * 4 + wave) * 2) * 64 + lane;
  f32x4_t v[2][16];
  f32x4_t r2[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  for (int q0 = 0; q0 < KS; q0 += 16) {      // all loads of a batch in flight, then the ordered sum
    const int n = min(16, KS - q0);
#pragma unroll
    for (int q = 0; q < 16; ++q)
      if (q < n) { v[0][q] = pt[(long)(q0 + q) * 4 * 2 * 64]; v[1][q] = pt[(long)(q0 + q) * 4 * 2 * 64 + 64]; }
#pragma unroll
    for (int q = 0; q < 16; ++q)
      if (q < n) { r2[0] += v[0][q]; r2[1] += v[1][q]; }
  }
  dense_fwd_epilogue<PREC>(a, g, ut * 64 + wave * 16, blockIdx.y * 32, r2, lane, ut * 4 + wave);
}


// ---------------------------------------------------------------------------
struct HeadArgs {
  const void* h;           // [G][B][Up] (post-dropout activations), bf16 or fp32 (prec)
  const float* w2;         // [G][Up][C] fp32 master
  const float* b2;         // [G][C]
  const int64_t* labels;   // [N]
  const int64_t* gather;   // [steps][G][B] sample ids
  const StepState* st;
  float* dH;               // [G][B][Up] fp32 (pre-activation grad)
  float* gw2;              // [G][Up][C]
  float* gb2;              // [G][C]
  float* gb1;              // [G][Up]
  float* eval_out;         // eval mode: [G][B][3] (loss, binary-correct, categorical-correct)
  float* dz;               // [G][B][C] logits gradient workspace
  const float* plog;       // [G][Up/16][B][C] partial logits from dense_fwd
  int G, B, Up, C;
  int loss_ce;             // 0 = bce_compat, 1 = ce
  float drop_scale;        // 1/(1-p)
  int eval;
  int prec;
  const int* valid;        // [steps][G] real rows of each training batch (Keras short batch) or null = B
  const int* valid_norm;   // X5: [steps][G] real rows of the FULL batch (loss mean over all ranks' rows) or null
  uint16_t* dHp;           // optional [NPL][G][B][Up] bf16 planes of dH (prec 1: the exact 3-way split; prec 0:
                           // the bf16 rounding), written once here so dense_dgrad does not re-split per wave
};

#define HEAD_MAXB 64
#define HEAD_MAXC 16

// (1) one 64-lane wave per (fold, sample): lane t loads the partial logits of
//     dense_fwd tile t, a shuffle tree sums them (fixed order), lane 0 adds b2
//     and does softmax -> loss gradient dz (train) or per-sample loss /
//     accuracies (eval).
__global__ void __launch_bounds__(64) head_fwd_kernel(HeadArgs a) {
  const int idx = blockIdx.x, lane = threadIdx.x;
  const int g = idx / a.B, b = idx % a.B;
  const int C = a.C, nt = a.Up / 16;
  // the label chain (step -> sample id -> label: three dependent loads) issued first, so it runs
  // beside the partial-logit loads instead of after the reduction
  const int step = a.st ? a.st->cur_step : 0;
  const long sid = a.gather[((long)step * a.G + g) * a.B + b];
  const int y = (int)a.labels[sid];
  float acc[HEAD_MAXC];
  const float* pl = a.plog + ((long)g * nt * a.B + b) * C;
#pragma unroll
  for (int c = 0; c < HEAD_MAXC; ++c) acc[c] = 0.f;
  // every class load of a tile issued at once (clamped index, masked add): a load under a
  // `c < C` branch made the wave wait for each one in turn (21-41 us per launch for ~10 KB)
  for (int t = lane; t < nt; t += 64) {
    float v[HEAD_MAXC];
#pragma unroll
    for (int c = 0; c < HEAD_MAXC; ++c) v[c] = pl[(long)t * a.B * C + min(c, C - 1)];
#pragma unroll
    for (int c = 0; c < HEAD_MAXC; ++c) acc[c] += c < C ? v[c] : 0.f;
  }
#pragma unroll
  for (int c = 0; c < HEAD_MAXC; ++c) {
    if (c < C) {
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) acc[c] += __shfl_xor(acc[c], o);
    }
  }
  if (lane != 0) return;
  float logit[HEAD_MAXC];
  for (int c = 0; c < C; ++c) logit[c] = acc[c] + a.b2[(long)g * C + c];
  float p[HEAD_MAXC];
  float mx = -INFINITY;
  for (int c = 0; c < C; ++c) mx = fmaxf(mx, logit[c]);
  float z = 0.f;
  for (int c = 0; c < C; ++c) { p[c] = expf(logit[c] - mx); z += p[c]; }
  int arg = 0;
  float loss = 0.f, binc = 0.f;
  for (int c = 0; c < C; ++c) {
    p[c] /= z;
    if (p[c] > p[arg]) arg = c;
    const float yc = (c == y) ? 1.f : 0.f;
    binc += (rintf(p[c]) == yc) ? 1.f : 0.f;
    if (!a.loss_ce) {
      const float pc = fminf(fmaxf(p[c], CLIP_EPS), 1.f - CLIP_EPS);
      loss += -(yc * logf(pc) + (1.f - yc) * logf(1.f - pc)) / C;
    }
  }
  if (a.loss_ce) loss = -logf(fmaxf(p[y], 1e-30f));
  if (a.eval) {
    float* e = a.eval_out + ((long)g * a.B + b) * 3;
    e[0] = loss; e[1] = binc; e[2] = (arg == y) ? 1.f : 0.f;
    return;
  }
  float* dz = a.dz + ((long)g * a.B + b) * C;
  // mean over the batch's real rows; padding rows of a short batch: zero weight
  const int nv = a.valid ? a.valid[(long)step * a.G + g] : a.B;
  const int nn = a.valid_norm ? a.valid_norm[(long)step * a.G + g] : nv;
  const float inv_b = (b < nv && nn > 0) ? 1.0f / nn : 0.f;
  if (a.loss_ce) {
    for (int c = 0; c < C; ++c) dz[c] = (p[c] - ((c == y) ? 1.f : 0.f)) * inv_b;
  } else {
    // dL/dp_c = (pc - y)/(pc(1-pc)) / C inside the clip range, 0 where clipped
    float dp[HEAD_MAXC], s = 0.f;
    for (int c = 0; c < C; ++c) {
      const float yc = (c == y) ? 1.f : 0.f;
      const bool inside = p[c] >= CLIP_EPS && p[c] <= 1.f - CLIP_EPS;
      const float pc = fminf(fmaxf(p[c], CLIP_EPS), 1.f - CLIP_EPS);
      dp[c] = inside ? (pc - yc) / (pc * (1.f - pc)) / C : 0.f;
      s += p[c] * dp[c];
    }
    for (int c = 0; c < C; ++c) dz[c] = p[c] * (dp[c] - s) * inv_b;
  }
}

// (2) grid (ceil(Up/64), G): per 64-unit slice, dH = (dz W2^T) * scale * (h > 0),
//     gb1 = sum_b dH, gW2 = h^T dz; block 0 also gb2 = sum_b dz.
__global__ void __launch_bounds__(256) head_bwd_kernel(HeadArgs a) {
  __shared__ float dzs[HEAD_MAXB * HEAD_MAXC];
  __shared__ float w2s[64 * HEAD_MAXC];
  __shared__ float hsl[HEAD_MAXB][65];
  __shared__ float colsum[4][64];
  const int g = blockIdx.y, u0 = blockIdx.x * 64, tid = threadIdx.x;
  const int B = a.B, Up = a.Up, C = a.C;
  const float* dz = a.dz + (long)g * B * C;
  for (int i = tid; i < B * C; i += 256) dzs[i] = dz[i];
  for (int i = tid; i < 64 * C; i += 256) {
    const int u = u0 + i / C;
    w2s[i] = (u < Up) ? a.w2[((long)g * Up + u0) * C + i] : 0.f;
  }
  for (int i = tid; i < B * 64; i += 256) {
    const int b = i >> 6, j = i & 63;
    const long hi = ((long)g * B + b) * Up + u0 + j;
    hsl[b][j] = (u0 + j < Up) ? (a.prec ? static_cast<const float*>(a.h)[hi] : bf2f(static_cast<const uint16_t*>(a.h)[hi]))
                              : 0.f;
  }
  __syncthreads();
  // dH and gb1: thread = (unit j, row quarter)
  {
    const int j = tid & 63, q = tid >> 6;
    float sb = 0.f;
    for (int b = q; b < B; b += 4) {
      float s = 0.f;
      for (int c = 0; c < C; ++c) s += dzs[b * C + c] * w2s[j * C + c];
      const float d = hsl[b][j] > 0.f ? s * a.drop_scale : 0.f;
      if (u0 + j < Up) {
        const long o = ((long)g * B + b) * Up + u0 + j;
        a.dH[o] = d;
        if (a.dHp) {
          if (a.prec) {
            uint16_t hq[3];
            split3(d, hq);
            const long ps = (long)a.G * B * Up;
            a.dHp[o] = hq[0]; a.dHp[ps + o] = hq[1]; a.dHp[2 * ps + o] = hq[2];
          } else {
            a.dHp[o] = f2bf(d);
          }
        }
      }
      sb += d;
    }
    colsum[q][j] = sb;
  }
  // gW2 slice
  for (int o = tid; o < 64 * C; o += 256) {
    const int j = o / C, c = o % C;
    if (u0 + j >= Up) continue;
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += hsl[b][j] * dzs[b * C + c];
    a.gw2[((long)g * Up + u0) * C + o] = s;
  }
  __syncthreads();
  if (tid < 64 && u0 + tid < Up)
    a.gb1[(long)g * Up + u0 + tid] = colsum[0][tid] + colsum[1][tid] + colsum[2][tid] + colsum[3][tid];
  if (blockIdx.x == 0 && tid < C) {
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += dzs[b * C + tid];
    a.gb2[(long)g * C + tid] = s;
  }
}

// ---------------------------------------------------------------------------
struct DenseDgradArgs {
  const float* dH;     // [G][B][Up]
  const void* wt;      // transposed copy of W1 [G][Up][Fp] (the values dense_fwd multiplied by): bf16 / fp32 (prec)
  void* dx;            // [G][B][Fp] bf16 or fp32 (prec)
  int G, B, Fp, Up;
  int prec;
  long wps;            // unused (kept for the ABI)
  // fused pool backward (K4): dx is the last pool's gradient; with a mask the
  // kernel scatters it to the pool source's gradient [G][B][Hs][Ws][Cp]
  // instead (slot 1 for groups with sel[g] = 1), pool_bwd_mask_kernel's rule
  const uint8_t* unpool_mask;   // [G*B][Hs/2][Ws/2][Cp] argmax mask of the forward, or null
  void* unpool_x0;
  void* unpool_x1;
  const int* unpool_sel;        // [G]
  int Hs, Ws, Cp;
  const float* w1;              // fp32 master W1 [G][Fp][Up]: streaming kernel (null: the copy + LDS transpose)
  const uint16_t* dHp;          // optional: head_bwd's bf16 planes of dH [NPL][G][B][Up] -> dense_dgrad_stream2
};

// dx (or, with an unpool mask, the fused pool backward) of one 16-feature x
// 32-row tile: D[row = feature][col = batch row]
template <int PREC>
__device__ __forceinline__ void dense_dgrad_epilogue(const DenseDgradArgs& a, int g, int f_t, int b0,
                                                     const f32x4_t (&acc)[2], int lane) {
  typedef typename ActT<PREC>::T AT;
  const int kq = lane >> 4, l16 = lane & 15;
  const int fo = f_t + kq * 4;
  if (fo >= a.Fp) return;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = b0 + h * 16 + l16;
    if (row >= a.B) continue;
    float v[4] = {acc[h][0], acc[h][1], acc[h][2], acc[h][3]};
    if (a.unpool_mask) {
      // features fo .. fo+3 = channels c0 .. c0+3 of pooled pixel (ho, wo)
      const long n = (long)g * a.B + row;
      const int pix = fo / a.Cp, c0 = fo - pix * a.Cp, wo_n = a.Ws >> 1;
      const int ho = pix / wo_n, wo = pix - ho * wo_n;
      const uint32_t mk = *reinterpret_cast<const uint32_t*>(a.unpool_mask + n * a.Fp + fo);
      AT* src = static_cast<AT*>((a.unpool_sel && a.unpool_sel[g]) ? a.unpool_x1 : a.unpool_x0);
#pragma unroll
      for (int me = 0; me < 4; ++me) {
        float o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t bb = (mk >> (8 * j)) & 0xffu;
          o[j] = ((int)(bb & 3u) == me && (bb & 4u)) ? v[j] : 0.f;
        }
        AT* d = src + ((n * a.Hs + 2 * ho + (me >> 1)) * a.Ws + 2 * wo + (me & 1)) * a.Cp + c0;
        if (PREC) *reinterpret_cast<float4*>(d) = make_float4(o[0], o[1], o[2], o[3]);
        else *reinterpret_cast<uint2*>(d) = pack4(o);
      }
      continue;
    }
    AT* dst = static_cast<AT*>(a.dx) + ((long)g * a.B + row) * a.Fp + fo;
    if (PREC) *reinterpret_cast<float4*>(dst) = make_float4(v[0], v[1], v[2], v[3]);
    else *reinterpret_cast<uint2*>(dst) = pack4(v);
  }
}

// Data gradient, bf16 mode (fp32: dense_dgrad_f32_kernel below): dX = dH W1^T with A = the fp32 master
// W1 [G][Fp][Up] itself (8 consecutive units of a feature row = one 32-byte load, rounded to bf16 in
// registers -- no transposed copy, no LDS, no barrier in the k loop); every wave carries TWO 16-feature
// tiles and takes dH as the bf16 plane head_bwd stored once. Grid (Fp/128, ceil(B/32), G), XCD-grouped.
// (The round-2 copy-based kernels and the streaming v1 kernel were removed in round 5.)
template <int PREC>
__global__ void __launch_bounds__(256) dense_dgrad_stream2_kernel(DenseDgradArgs a) {
  constexpr int NPL = PREC ? GT_NPL_F32 : 1;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, kq = lane >> 4, l16 = lane & 15;
  int bx, g;
  xcd_tile(bx, g);
  const int f_t = bx * 128 + wave * 32;
  const int b0 = blockIdx.y * 32;
  const float* wrow[2];
  bool fok[2];
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const int fa = f_t + 16 * m + l16;
    fok[m] = fa < a.Fp;
    wrow[m] = a.w1 + ((long)g * a.Fp + (fok[m] ? fa : 0)) * a.Up;
  }
  const long ps = (long)a.G * a.B * a.Up;               // plane stride of dHp
  const int br[2] = {b0 + l16, b0 + 16 + l16};
  const uint16_t* hp[2];
  bool bok[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    bok[h] = br[h] < a.B;
    hp[h] = a.dHp + ((long)g * a.B + (bok[h] ? br[h] : 0)) * a.Up;
  }
  const int nchunks = a.Up >> 3;
  const int nks = (nchunks + 3) >> 2;
  f32x4_t acc[2][2];
#pragma unroll
  for (int m = 0; m < 2; ++m) acc[m][0] = acc[m][1] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  constexpr int NBUF = GT_DGRAD_BUF;                   // k-steps in flight per wave (grid-limited occupancy:
                                                        // ~2.7 waves per SIMD, so registers are free)
  float rw[NBUF][2][8];
  uint4 rh[NBUF][2][NPL];
  const uint4* zero4 = reinterpret_cast<const uint4*>(gt_zero8);
  auto load = [&](int j, int buf) {
    const int c = 4 * j + kq;
    const bool cok = c < nchunks;
#pragma unroll
    for (int m = 0; m < 2; ++m) ld8_raw(wrow[m] + c * 8, cok && fok[m], rw[buf][m]);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int p = 0; p < NPL; ++p)
        rh[buf][h][p] = *((cok && bok[h]) ? reinterpret_cast<const uint4*>(hp[h] + p * ps + c * 8) : zero4);
  };
  auto step = [&](int buf) {
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      uint4 af[NPL];
      planes8<PREC>(rw[buf][m], af);
      acc[m][0] = mfma_np<NPL>(af, rh[buf][0], acc[m][0]);
      acc[m][1] = mfma_np<NPL>(af, rh[buf][1], acc[m][1]);
    }
  };
  // (unconditional loads, ordered: see dense_fwd_stream_kernel)
#pragma unroll
  for (int t = 0; t < NBUF; ++t) {
    load(t, t);
    __builtin_amdgcn_sched_barrier(0);
  }
  const int nks2 = (nks + 1) & ~1;      // the k-steps NBUF 2 runs (an odd count ends on a zero-loaded step)
  for (int j = 0; j < nks; j += NBUF) {
#pragma unroll
    for (int t = 0; t < NBUF; ++t) {
      // the same k-steps in the same order at any NBUF (bit-identical dx)
      if (j + t < nks2) step(t);
      __builtin_amdgcn_sched_barrier(0);
      load(j + NBUF + t, t);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int m = 0; m < 2; ++m) dense_dgrad_epilogue<PREC>(a, g, f_t + 16 * m, b0, acc[m], lane);
}


// ---------------------------------------------------------------------------
// fp32 data gradient on the fp32-input MFMA (v_mfma_f32_16x16x4_f32: exact f32 products, f32 accumulate;
// 1/16 of the bf16 rate, which at batch 32 is about the HBM rate of streaming W1). W1 is read once from
// the fp32 master with coalesced 16-byte loads -- no bf16 planes, no split VALU: 67.5-68.9 vs 73-74 us
// for dense_dgrad_stream2 at 25 groups, and exact products. (The same scheme for the forward -- A = 4
// unit tiles per 16-byte W1 load, split-K ranges reduced in order -- ran 72-92 us against the split-K
// bf16x6 kernel's 59-63 at any prefetch depth, and was dropped: profiles/r5/dense_f32_mfma_ab_r5.txt.)
// Operand maps of 16x16x4 f32: A[i][k], B[k][j] with lane l -> i or j = l & 15, k = l >> 4; C lane l
// holds rows 4 (l >> 4) + r of column l & 15.
__device__ __forceinline__ f32x4_t mfma4f(float a, float b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Data gradient: grid (Fp/128, ceil(B/32), G), XCD-grouped; wave = two 16-feature tiles x 32 rows over all
// Up units. Per 32-unit block a lane loads 8 consecutive units of its W1 row (tile m: feature f_t + 16 m + l16)
// and of its dH row (b0 + 16 h + l16), two 16-byte loads each; k-step s multiplies unit u0 + 8 k + s.
// C layout = dense_dgrad_epilogue's (rows = features 4 kq + r, column = batch row).
__global__ void __launch_bounds__(256) dense_dgrad_f32_kernel(DenseDgradArgs a) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, kq = lane >> 4, l16 = lane & 15;
  int bx, g;
  xcd_tile(bx, g);
  const int f_t = bx * 128 + wave * 32;
  const int b0 = blockIdx.y * 32;
  const float* wrow[2];
#pragma unroll
  for (int m = 0; m < 2; ++m) wrow[m] = a.w1 + ((long)g * a.Fp + min(f_t + 16 * m + l16, a.Fp - 1)) * a.Up + 8 * kq;
  const float* hrow[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) hrow[h] = a.dH + ((long)g * a.B + min(b0 + 16 * h + l16, a.B - 1)) * a.Up + 8 * kq;
  f32x4_t acc[2][2];
#pragma unroll
  for (int m = 0; m < 2; ++m) acc[m][0] = acc[m][1] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  constexpr int NB = 2;                                     // 32-unit blocks in flight per wave (3, 4: slower)
  float4 wv[NB][2][2], hv[NB][2][2];                        // [buf][m or h][half]
  const int nblk = a.Up >> 5;
  auto load = [&](int j, int buf) {
    const int jj = min(j, nblk - 1);                        // past the end: re-read the last block, unused
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      wv[buf][m][0] = *reinterpret_cast<const float4*>(wrow[m] + 32 * jj);
      wv[buf][m][1] = *reinterpret_cast<const float4*>(wrow[m] + 32 * jj + 4);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      hv[buf][h][0] = *reinterpret_cast<const float4*>(hrow[h] + 32 * jj);
      hv[buf][h][1] = *reinterpret_cast<const float4*>(hrow[h] + 32 * jj + 4);
    }
  };
  auto step = [&](int buf) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float w0 = (&wv[buf][0][q >> 2].x)[q & 3], w1 = (&wv[buf][1][q >> 2].x)[q & 3];
      const float h0 = (&hv[buf][0][q >> 2].x)[q & 3], h1 = (&hv[buf][1][q >> 2].x)[q & 3];
      acc[0][0] = mfma4f(w0, h0, acc[0][0]);
      acc[0][1] = mfma4f(w0, h1, acc[0][1]);
      acc[1][0] = mfma4f(w1, h0, acc[1][0]);
      acc[1][1] = mfma4f(w1, h1, acc[1][1]);
    }
  };
#pragma unroll
  for (int i = 0; i < NB - 1; ++i) load(i, i);
  for (int j = 0; j < nblk; j += NB) {
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      if (j + q >= nblk) break;
      load(j + q + NB - 1, (q + NB - 1) % NB);
      step(q);
    }
  }
#pragma unroll
  for (int m = 0; m < 2; ++m) dense_dgrad_epilogue<1>(a, g, f_t + 16 * m, b0, acc[m], lane);
}

// ---------------------------------------------------------------------------
struct DenseWgradAdamArgs {
  const void* x;       // [G][B][Fp] bf16 or fp32 (prec)
  const float* dH;     // [G][B][Up]
  float* p; float* m; float* v;   // [G][Fp][Up]
  void* wt;            // unused (kept for the ABI: the transposed W1 copy of rounds 2-4)
  const StepState* st;
  int G, B, Fp, Up;
  int Cp, Cr, Ur;      // feature = pixel * Cp + channel; channels >= Cr and units >= Ur are padding
                       // (zero forever: skipped, 13 % of the layer's optimizer traffic)
  int prec;
  long wps;            // unused (kept for the ABI)
  float* gbuf;         // X5 data parallelism: [G][Fp][Up] gradient buffer
  int mode;            // 0: fused gradient + update; 1: gradient -> gbuf only (all-reduced next);
                       // 2: update from gbuf
};

// grid (Fp/16, G), 256 threads. Thread: unit quad q (4 units), rows fr, fr+2, ..., fr+14.
template <int PREC>
__global__ void __launch_bounds__(256) dense_wgrad_adam_kernel(DenseWgradAdamArgs a) {
  typedef typename ActT<PREC>::T AT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* xs = reinterpret_cast<float*>(smem);                       // [B][16]
  const int g = blockIdx.y, f0 = blockIdx.x * 16, tid = threadIdx.x;
  const AT* x = static_cast<const AT*>(a.x) + (long)g * a.B * a.Fp;
  for (int i = tid; i < a.B * 16; i += 256) {
    const int b = i >> 4, j = i & 15;
    float xv = 0.f;
    if (f0 + j < a.Fp) {
      if (PREC) xv = static_cast<const float*>(static_cast<const void*>(x))[(long)b * a.Fp + f0 + j];
      else xv = bf2f(static_cast<const uint16_t*>(static_cast<const void*>(x))[(long)b * a.Fp + f0 + j]);
    }
    xs[i] = xv;
  }
  __syncthreads();
  const float lr_t = a.st->lr_t;
  const float* dH = a.dH + (long)g * a.B * a.Up;
  const int nq = a.Ur > 0 ? (a.Ur + 3) >> 2 : a.Up >> 2;
  const int fr = tid >> 7;
  for (int q = tid & 127; q < nq; q += 128) {
    const int u0 = q * 4;
    float acc[8][4];
#pragma unroll
    for (int r = 0; r < 8; ++r) acc[r][0] = acc[r][1] = acc[r][2] = acc[r][3] = 0.f;
    if (a.mode == 2) {                                  // all-reduced gradient from gbuf
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int f = f0 + fr + 2 * r;
        if (f < a.Fp) {
          const float4 q4 = *reinterpret_cast<const float4*>(a.gbuf + ((long)g * a.Fp + f) * a.Up + u0);
          acc[r][0] = q4.x; acc[r][1] = q4.y; acc[r][2] = q4.z; acc[r][3] = q4.w;
        }
      }
    }
    for (int b = 0; a.mode != 2 && b < a.B; ++b) {
      const float4 d = *reinterpret_cast<const float4*>(dH + (long)b * a.Up + u0);
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const float xv = xs[b * 16 + fr + 2 * r];
        acc[r][0] += xv * d.x; acc[r][1] += xv * d.y; acc[r][2] += xv * d.z; acc[r][3] += xv * d.w;
      }
    }
    if (a.mode == 1) {                                  // gradient only (this rank's rows)
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int f = f0 + fr + 2 * r;
        if (f < a.Fp)
          *reinterpret_cast<float4*>(a.gbuf + ((long)g * a.Fp + f) * a.Up + u0) =
              make_float4(acc[r][0], acc[r][1], acc[r][2], acc[r][3]);
      }
      continue;
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int f = f0 + fr + 2 * r;
      if (f >= a.Fp) continue;
      if (a.Cp > 0 && f % a.Cp >= a.Cr) continue;     // padded channel: weights stay 0
      const long off = ((long)g * a.Fp + f) * a.Up + u0;
      float4 pp = *reinterpret_cast<float4*>(a.p + off);
      float4 mm = *reinterpret_cast<float4*>(a.m + off);
      float4 vv = *reinterpret_cast<float4*>(a.v + off);
      float* P = &pp.x; float* M = &mm.x; float* V = &vv.x;
#pragma unroll
      for (int i = 0; i < 4; ++i) P[i] = opt_update(a.st, P[i], acc[r][i], M[i], V[i], lr_t);
      *reinterpret_cast<float4*>(a.p + off) = pp;
      *reinterpret_cast<float4*>(a.m + off) = mm;
      *reinterpret_cast<float4*>(a.v + off) = vv;
    }
  }
}

// ---------------------------------------------------------------------------
struct AdamSeg {
  float* p; float* m; float* v;
  const float* g;        // gradient (or S split-K partials, stride gstride)
  uint16_t* bf;          // optional bf16 copy (same layout)
  uint16_t* bfT;         // optional flipped/transposed conv copy [G][Ci][KH][KW][Co]
  long n, gstride;
  int S, tG, tCo, tKH, tKW, tCi;
  int tiled;             // 1: blocks are (group, 64-column) tiles of a [Co][KH*KW*Ci] weight (Co <= 128)
  int npl;               // bf16 planes of bf / bfT: 1, or 3 (exact split of the fp32 master, prec 1)
  long pstride_bf, pstride_bfT;   // plane strides (elements)
};


#define ADAM_TK 64
#define ADAM_BLK 1024   // elements per block of an element-wise (untiled) segment

struct AdamArgs {
  const AdamSeg* segs;
  const int2* blocks;    // per block: (segment, element offset)
  const StepState* st;
};

__global__ void __launch_bounds__(256) adam_segments_kernel(AdamArgs a) {
  const int2 blk = a.blocks[blockIdx.x];
  const AdamSeg sg = a.segs[blk.x];
  const int npl = sg.npl > 1 ? GT_NPL_F32 : 1;
  if (sg.tiled) {
    // conv weight tile: Co rows x ADAM_TK reduction columns (row-contiguous
    // reads of p/m/v/partials), bf16 values staged in LDS, then the flipped /
    // transposed dgrad copy written as 16-byte runs along co -- one element per
    // thread scattered 2-byte stores over a 1-2 KB stride instead (every store
    // its own L2 transaction: the kernel's old bottleneck)
    __shared__ __attribute__((aligned(16))) uint16_t tile[GT_NPL_F32][ADAM_TK][128 + 8];
    // Co > 128 (wide nodes): the weight is cut into 128-row co bands, one
    // block per (group, band, column tile); bfT runs stay 16-byte aligned
    const int CoF = sg.tCo, Ci = sg.tCi, KH = sg.tKH, KW = sg.tKW;
    const int Kd = KH * KW * Ci;
    const int nkt = (Kd + ADAM_TK - 1) / ADAM_TK;
    const int ncot = (CoF + 127) >> 7;
    const int gb = blk.y / nkt, k0 = (blk.y - gb * nkt) * ADAM_TK;
    const int gg = gb / ncot, c0 = (gb - gg * ncot) << 7;
    const int Co = min(128, CoF - c0);
    const long base = ((long)gg * CoF + c0) * Kd;
    const float lr_t = a.st->lr_t;
    // GT_ADAM_UNROLL elements per thread: all their loads issue before the first
    // update (4 measured neutral: the kernel moves ~260 MB at 25 groups, 12 B of
    // every parameter's 24 written being the exact bf16 planes of the two copies)
    constexpr int U = GT_ADAM_UNROLL;
    for (int idx0 = threadIdx.x; idx0 < Co * ADAM_TK; idx0 += 256 * U) {
      float gr[U], mv[U], vv[U], pv[U];
      long iv[U];
      bool ok[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int idx = idx0 + 256 * u;
        const int co = idx / ADAM_TK, kk = idx % ADAM_TK, k = k0 + kk;
        ok[u] = idx < Co * ADAM_TK && k < Kd;
        iv[u] = base + (long)co * Kd + (ok[u] ? k : 0);
        gr[u] = 0.f; mv[u] = vv[u] = pv[u] = 0.f;
        if (ok[u]) {
          for (int s = 0; s < sg.S; ++s) gr[u] += sg.g[(long)s * sg.gstride + iv[u]];
          mv[u] = sg.m[iv[u]]; vv[u] = sg.v[iv[u]]; pv[u] = sg.p[iv[u]];
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (!ok[u]) continue;
        const int idx = idx0 + 256 * u;
        const int co = idx / ADAM_TK, kk = idx % ADAM_TK;
        const long i = iv[u];
        float m = mv[u], v = vv[u];
        const float p = opt_update(a.st, pv[u], gr[u], m, v, lr_t);
        sg.m[i] = m; sg.v[i] = v; sg.p[i] = p;
        uint16_t h[3];
        split3(p, h);
        for (int q = 0; q < npl; ++q) {
          if (sg.bf) sg.bf[q * sg.pstride_bf + i] = h[q];
          tile[q][kk][co] = h[q];
        }
      }
    }
    __syncthreads();
    const int nc8 = Co >> 3;
    for (int idx = threadIdx.x; idx < ADAM_TK * nc8; idx += 256) {
      const int kk = idx / nc8, c8 = idx - kk * nc8, k = k0 + kk;
      if (k >= Kd) continue;
      const int ci = k % Ci, r = k / Ci, kw = r % KW, kh = r / KW;
      const long o = ((((long)gg * Ci + ci) * KH + (KH - 1 - kh)) * KW + (KW - 1 - kw)) * CoF + c0 + c8 * 8;
      for (int q = 0; q < npl; ++q)
        *reinterpret_cast<uint4*>(sg.bfT + q * sg.pstride_bfT + o) = *reinterpret_cast<const uint4*>(&tile[q][kk][c8 * 8]);
    }
    return;
  }
  // element-wise segment: ADAM_BLK elements per block, 4 consecutive per thread with 16-byte loads and
  // stores of p / m / v / gradient partials when aligned (one 4-byte element per thread kept too few
  // bytes in flight: ~2 TB/s); the per-element arithmetic and the partial-sum order are unchanged
  const float lr_t = a.st->lr_t;
  const int i0 = blk.y;                             // segments are < 2^31 elements
  auto one = [&](int i, float gr, float p, float& m, float& v) {
    p = opt_update(a.st, p, gr, m, v, lr_t);
    uint16_t h[3];
    split3(p, h);
    if (sg.bf)
      for (int q = 0; q < npl; ++q) sg.bf[q * sg.pstride_bf + i] = h[q];
    if (sg.bfT) {
      // flipped / transposed dgrad copy: 32-bit index math (64-bit division is
      // a long software sequence on the GPU)
      uint32_t r = (uint32_t)i;
      const uint32_t ci = r % (uint32_t)sg.tCi; r /= (uint32_t)sg.tCi;
      const uint32_t kw = r % (uint32_t)sg.tKW; r /= (uint32_t)sg.tKW;
      const uint32_t kh = r % (uint32_t)sg.tKH; r /= (uint32_t)sg.tKH;
      const uint32_t co = r % (uint32_t)sg.tCo;
      const uint32_t gg = r / (uint32_t)sg.tCo;
      const long o = ((((long)gg * sg.tCi + ci) * sg.tKH + (sg.tKH - 1 - kh)) * sg.tKW + (sg.tKW - 1 - kw)) * sg.tCo + co;
      for (int q = 0; q < npl; ++q) sg.bfT[q * sg.pstride_bfT + o] = h[q];
    }
    return p;
  };
  const bool vec = ((reinterpret_cast<uintptr_t>(sg.p) | reinterpret_cast<uintptr_t>(sg.m) |
                     reinterpret_cast<uintptr_t>(sg.v) | reinterpret_cast<uintptr_t>(sg.g)) & 15) == 0 &&
                   (sg.gstride & 3) == 0 && (long)i0 + ADAM_BLK <= sg.n;
  if (vec) {
    const int i = i0 + 4 * (int)threadIdx.x;
    float4 gr = make_float4(0.f, 0.f, 0.f, 0.f);     // 0 + partial 0 + ...: the scalar path's order
    for (int s = 0; s < sg.S; ++s) {
      const float4 t = *reinterpret_cast<const float4*>(sg.g + (long)s * sg.gstride + i);
      gr.x += t.x; gr.y += t.y; gr.z += t.z; gr.w += t.w;
    }
    float4 m = *reinterpret_cast<const float4*>(sg.m + i), v = *reinterpret_cast<const float4*>(sg.v + i);
    float4 p = *reinterpret_cast<const float4*>(sg.p + i);
    p.x = one(i, gr.x, p.x, m.x, v.x);
    p.y = one(i + 1, gr.y, p.y, m.y, v.y);
    p.z = one(i + 2, gr.z, p.z, m.z, v.z);
    p.w = one(i + 3, gr.w, p.w, m.w, v.w);
    *reinterpret_cast<float4*>(sg.m + i) = m;
    *reinterpret_cast<float4*>(sg.v + i) = v;
    *reinterpret_cast<float4*>(sg.p + i) = p;
    return;
  }
  for (int e = 0; e < ADAM_BLK / 256; ++e) {
    const int i = i0 + e * 256 + (int)threadIdx.x;
    if (i >= sg.n) return;
    float gr = 0.f;
    for (int s = 0; s < sg.S; ++s) gr += sg.g[(long)s * sg.gstride + i];
    float m = sg.m[i], v = sg.v[i];
    const float p = one(i, gr, sg.p[i], m, v);
    sg.m[i] = m; sg.v[i] = v; sg.p[i] = p;
  }
}

extern "C" {

int gt_step_begin(StepState* s, hipStream_t stream) {
  hipLaunchKernelGGL(step_begin_kernel, dim3(1), dim3(1), 0, stream, s);
  return (int)hipGetLastError();
}

// feature ranges per output tile of the split-K forward: a per-shape constant (~12 k-steps of
// 32 features per range), never a function of the number of groups
int gt_dense_fwd_splits(int Fp) {
  const int nks = (Fp + 31) / 32;
  return std::max(1, std::min(16, nks / 12));
}

int gt_dense_fwd(const DenseFwdArgs* a, hipStream_t stream) {
  if (a->Fp % 8 || a->Up % 64 || a->C > HEAD_MAXC_FWD || (a->prec != 0 && a->prec != 1)) return -1;
  // W1 comes from the fp32 master only (the transposed copy of earlier rounds is gone)
  if (!a->w1 || a->ks < 1 || (a->ks > 1 && !a->part)) return -3;
  dim3 grid(a->Up / 64 * a->ks, (a->B + 31) / 32, a->G);
  if (a->prec) hipLaunchKernelGGL(dense_fwd_sk_kernel<1>, grid, dim3(256), 0, stream, *a);
  else hipLaunchKernelGGL(dense_fwd_sk_kernel<0>, grid, dim3(256), 0, stream, *a);
  if (a->ks > 1) {
    dim3 rgrid(a->Up / 64, (a->B + 31) / 32, a->G);
    if (a->prec) hipLaunchKernelGGL(dense_fwd_skred_kernel<1>, rgrid, dim3(256), 0, stream, *a);
    else hipLaunchKernelGGL(dense_fwd_skred_kernel<0>, rgrid, dim3(256), 0, stream, *a);
  }
  return (int)hipGetLastError();
}

int gt_head(const HeadArgs* a, hipStream_t stream) {
  if ((!a->eval && a->B > HEAD_MAXB) || a->C > HEAD_MAXC) return -1;    // the batch limit is head_bwd's LDS
  if (a->Up % 16) return -2;
  hipLaunchKernelGGL(head_fwd_kernel, dim3(a->G * a->B), dim3(64), 0, stream, *a);
  if (!a->eval) hipLaunchKernelGGL(head_bwd_kernel, dim3((a->Up + 63) / 64, a->G), dim3(256), 0, stream, *a);
  return (int)hipGetLastError();
}

int gt_dense_dgrad(const DenseDgradArgs* a, hipStream_t stream) {
  if (a->Fp % 64 && a->Fp % 8) return -1;
  if (a->unpool_mask && (a->Cp % 8 || a->Hs % 2 || a->Ws % 2 || (long)(a->Hs / 2) * (a->Ws / 2) * a->Cp != a->Fp))
    return -1;
  if (a->Up % 8) return -1;
  if (a->prec != 0 && a->prec != 1) return -1;
  if (!a->w1) return -3;                               // the fp32 master W1 (no transposed copy)
  dim3 grid((a->Fp + 127) / 128, (a->B + 31) / 32, a->G);
  if (a->prec == 1) {
    if (a->Up % 32) return -1;
    hipLaunchKernelGGL(dense_dgrad_f32_kernel, grid, dim3(256), 0, stream, *a);
  } else {
    if (!a->dHp) return -3;                            // head_bwd's bf16 dH
    hipLaunchKernelGGL(dense_dgrad_stream2_kernel<0>, grid, dim3(256), 0, stream, *a);
  }
  return (int)hipGetLastError();
}

int gt_dense_wgrad_adam(const DenseWgradAdamArgs* a, hipStream_t stream) {
  if (a->Up % 4 || (a->prec != 0 && a->prec != 1)) return -1;
  const size_t lds = sizeof(float) * (size_t)a->B * 16;
  if (lds > 160 * 1024) return -2;
  dim3 grid((a->Fp + 15) / 16, a->G);
  if (a->prec) {
    if (lds > 65536) (void)hipFuncSetAttribute(reinterpret_cast<const void*>(dense_wgrad_adam_kernel<1>),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(dense_wgrad_adam_kernel<1>, grid, dim3(256), lds, stream, *a);
  } else {
    hipLaunchKernelGGL(dense_wgrad_adam_kernel<0>, grid, dim3(256), lds, stream, *a);
  }
  return (int)hipGetLastError();
}

int gt_adam_segments(const AdamArgs* a, int nblocks, hipStream_t stream) {
  hipLaunchKernelGGL(adam_segments_kernel, dim3(nblocks), dim3(256), 0, stream, *a);
  return (int)hipGetLastError();
}

size_t gt_sizeof_adam_seg() { return sizeof(AdamSeg); }
int gt_adam_block_elems() { return ADAM_BLK; }
size_t gt_sizeof_dense_fwd_args() { return sizeof(DenseFwdArgs); }
size_t gt_sizeof_head_args() { return sizeof(HeadArgs); }
size_t gt_sizeof_dense_dgrad_args() { return sizeof(DenseDgradArgs); }
size_t gt_sizeof_dense_wgrad_args() { return sizeof(DenseWgradAdamArgs); }

}  // extern "C"
