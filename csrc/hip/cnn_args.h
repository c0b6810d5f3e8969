// Argument blocks of the Genetic-CNN convolution kernels (shared by the
// generic kernels in cnn_conv.hip and the shape-specialised ones in
// cnn_conv_fast.hip). Layouts must match gentun_amd/ops/cnn_kernels.py.
#pragma once
#include "common.h"

// Population batching: a launch covers the "groups" (candidate x fold
// replicas) listed in a group table. Activations / gradients live in SLOT
// tensors [Q][B][H][W][C] (Q = all groups of the job); a group's record says
// which slots it sums as input, which slots its output goes to, and for each
// output whether to accumulate and whether to apply the ReLU mask of that
// slot's activation (the DAG of every candidate is different, the launch is
// shared).  gtab == nullptr: legacy dense mode (group = blockIdx.y, inputs
// 0..n_in-1, outputs 0..n_out-1, acc_flags, masks where out_mask[k] != 0).
struct GroupRec {
  int g;          // group index into the slot tensors / weights
  int in_mask;    // bit k: in[k] is summed
  int out_mask;   // bits 0-7: outputs written, 8-15: accumulate, 16-23: apply out_mask[k] ReLU mask,
                  // 24: forward launch pools this group's output tile into pool_y / pool_mask (fused 2x2 max-pool),
                  // 25: data-gradient launch writing a pool's gradient un-pools it instead (fused pool backward)
  int pad;
};

#define GT_MAXSLOT 8

// Activation / gradient tensors are bf16 (prec 0) or fp32 (prec 1) -- void
// pointers here, typed by the kernel instantiation. Weights are always bf16
// PLANES: one plane in prec 0; in prec 1 the exact 3-way split of the fp32
// master (common.h split8), plane p at w + p * wps.
struct ConvArgs {
  const void* in[GT_MAXSLOT];       // input slot bases [Q][B][H][W][Cinp]
  const void* mask;                 // optional: staged value *= (mask > 0), same shape as in (legacy mode)
  const int64_t* gather;            // optional: image table [steps][Q][B]; in[0] is then the dataset
  const StepState* st;              // cur_step for the gather table
  void* out[GT_MAXSLOT];            // output slot bases [Q][B][H][W][Coutp]
  const void* out_mask[GT_MAXSLOT];  // per output slot: ReLU-mask source (that slot's activation)
  const uint16_t* w;                // [planes][Q][Coutp][KH][KW][Cinp] bf16
  const float* bias;                // [Q][Coutp] or null
  const GroupRec* gtab;             // [grid.y] or null
  int n_in, n_out, acc_flags, relu;
  int G, B, H, W, Cinp, Coutp, KH, KW, TH;   // G = Q (group count of the slot tensors)
  int ngroups;                      // launch groups (rows of gtab); legacy mode: G
  void* xsum;                       // optional [Q][B][H][W][Cinp]: groups summing >1 input slot write the sum
                                    // (the layer's wgrad then reads one tensor instead of re-summing)
  int dbg;                          // diagnostics only (0 in production): bit 0 skip MFMA, 1 skip stores, 2 skip loads
  int epi_bf16;                     // 1: forward launch (no accumulate / mask; prec 0 stages the output tile in
                                    //    bf16: same bits, half the LDS); 0: fp32 tile (exact accumulate)
  int prec;                         // 0: bf16 tensors, bf16 MFMA; 1: fp32 tensors, split-fp32 MFMA (common.h)
  long wps;                         // weight plane stride in elements (prec 1)
  int cbb;                          // generic kernel, set by its launcher: input chunks (8 channels) per channel
                                    // block (0: all at once). Wide fp32 layers stage the patch block by block.
  void* pool_y;                     // fused pool (groups with GroupRec bit 24): [Q][B][H/2][W/2][Coutp]
                                    // fused un-pool (bit 25): gradient of the pool source, slot 0 [Q][B][2H][2W][Coutp]
  uint8_t* pool_mask;               // argmax mask [Q*B][H/2][W/2][Coutp] (training forward) or null; un-pool: the
                                    // pooled layer's mask [Q*B][H][W][Coutp] (bit 2 = ReLU mask)
  void* unpool_x1;                  // un-pool: gradient of the pool source, slot 1 (groups with sel[g] = 1)
  const int* unpool_sel;            // un-pool: [Q] pool source per group (pop_schedule.pool_source)
  int cout_real;                    // real output channels (<= Coutp; 0 = unknown): prec-1 packed last co tile
  // real extent of a zero-padded ("virtual") image (0: not padded). A layer whose real H x W is stored
  // in a larger tensor (MNIST's 28 x 28 in 32 x 32, right / bottom padding, so every layer runs the 32 /
  // 16 / 8-wide shape-specialised kernels) writes exact zeros outside the real rows / columns from its
  // FORWARD epilogue; every other kernel then sees zeros there (the data gradient's ReLU / pool masks
  // zero the gradient, the dense W1 rows of padded pixels stay 0), so results equal the unpadded network
  int Hr, Wr;
  // 1: a 3x3 fp32 layer on the Winograd F(2x2, 3x3) kernels (cnn_conv_wino.hip); `w` then holds the
  // transformed weight planes [3][Q][16][R][K] written by gt_wino_wtrans, never the direct planes
  int wino;
  // 1: `w` holds FRAGMENT-MAJOR planes [planes][Q][NT][NKS][64][8] of the shape-specialised fp32 kernels
  // (gt_conv_wfrag, conv_fast_impl.h): each MFMA A fragment one contiguous KB in lane order
  int wfrag;
};

__device__ __forceinline__ GroupRec group_rec(const GroupRec* gtab, int y, int n_in, int n_out, int acc,
                                              const void* const* out_mask) {
  if (gtab) return gtab[y];
  GroupRec r;
  r.g = y;
  r.in_mask = (1 << n_in) - 1;
  int rm = 0;
  for (int k = 0; k < n_out; ++k)
    if (out_mask && out_mask[k]) rm |= 1 << k;
  r.out_mask = ((1 << n_out) - 1) | ((acc & 0xff) << 8) | (rm << 16);
  r.pad = 0;
  return r;
}

// Weight gradient (split-K, deterministic partials).
struct WgradArgs {
  const void* in[GT_MAXSLOT];       // input slots of the layer [Q][B][H][W][Cinp] (summed per group)
  const int64_t* gather;     // optional dataset gather (first layer)
  const StepState* st;
  const void* dz;            // ReLU-masked grad of the layer output [G][B][H][W][Coutp]
  float* part_w;             // [S][G][Coutp][Kdim]
  float* part_b;             // [S][G][Coutp]
  const GroupRec* gtab;      // [n_groups] or null (legacy: all G groups, inputs 0..n_in-1)
  int n_in;
  int G, B, H, W, Cinp, Coutp, KH, KW, S, pps;  // pps = pixels per split (multiple of 64)
  int ngroups;
  int prec;                  // 0: bf16 tensors; 1: fp32 tensors (split-fp32 MFMA)
  int cout_real;             // real output channels (<= Coutp; 0 = unknown): prec-1 packed last co tile
};

// "> 0" on a stored activation: bf16 bits (sign clear, not +0) or fp32
__device__ __forceinline__ bool pos_bits(uint32_t h) { return h != 0u && h < 0x8000u; }

