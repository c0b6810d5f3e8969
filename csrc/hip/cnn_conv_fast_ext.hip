// Shape-specialised conv / weight-gradient dispatch for user-chosen architectures (the reference lets the
// user pick kernels_per_layer and kernel_sizes, gentun/individuals.py:221-223): 32 / 64-channel stages
// (kernels (32, 64) -- padding them up to the wide (64, 128) shapes cost 4x the multiply-adds and ran slower
// than the generic kernels, profiles/r6/generality_r6.txt) and 3x3 stage-input convs, each tiled like its
// (20, 50) / 5x5 counterpart. Its own translation unit (compiled in parallel with cnn_conv_fast.hip); the
// switches (register epilogue, small-launch tiles, wgrad slices / band buffers) are cnn_conv_fast.hip's.
#include "conv_fast_host.h"

extern "C" int gt_conv_regepi_on();
extern "C" int gt_conv_smallq_th(const ConvArgs* a, int TH, int THMIN);
extern "C" int gt_wgrad_nb_force();
extern "C" int gt_wgrad_nz_of(const WgradArgs* a);

namespace {
int g_probe = 0;
int g_wgrad_nb = 0;
bool regepi_on() { return gt_conv_regepi_on() != 0; }
int smallq_th(const ConvArgs* a, int TH, int THMIN) { return gt_conv_smallq_th(a, TH, THMIN); }
int wgrad_nz(const WgradArgs* a) { return gt_wgrad_nz_of(a); }
}  // namespace

extern "C" int gt_conv_fast_ext(const ConvArgs* a, hipStream_t stream, int probe) {
  g_probe = probe;
  if (a->prec != 1) return -100;
  // 32 / 64-channel stages (kernels (32, 64): padding them to the wide (64, 128) shapes costs 4x the
  // multiply-adds and ran slower than the generic kernels, profiles/r6/generality_r6.txt), tiled like the
  // (20, 50) shapes
  if (CONV_FAST_MATCH(5, 5, 1, 32, 8, 2, 4) && smallq_th(a, 8, 4) == 4) CONV_FAST_LAUNCH(5, 5, 1, 32, 4, 2, 4, 2, 1)
  CONV_FAST_CASE_F32(5, 5, 1, 32, 8, 2, 4, 4)          // s1 input conv (3 -> 32)
  if (CONV_FAST_MATCH(3, 3, 1, 32, 8, 2, 4) && smallq_th(a, 8, 4) == 4) CONV_FAST_LAUNCH(3, 3, 1, 32, 4, 2, 4, 2, 1)
  CONV_FAST_CASE_F32(3, 3, 1, 32, 8, 2, 4, 4)          // s1 input conv 3x3 (3 -> 32)
  if (CONV_FAST_MATCH(3, 3, 4, 32, 8, 2, 4) && smallq_th(a, 8, 4) == 4) CONV_FAST_LAUNCH(3, 3, 4, 32, 4, 2, 4, 2, 1)
  CONV_FAST_CASE_F32(3, 3, 4, 32, 8, 2, 4, 4)          // s1 nodes / output conv and their dgrad (32 -> 32)
  if (CONV_FAST_MATCH(5, 5, 4, 16, 8, 4, 8)) {       // s2 input conv (32 -> 64)
    const int th = smallq_th(a, 8, 2);
    if (th == 4) CONV_FAST_LAUNCH(5, 5, 4, 16, 4, 4, 8, 4, 1)
    if (th == 2) CONV_FAST_LAUNCH_CT1(5, 5, 4, 16, 2, 4, 8, 4)
    CONV_FAST_LAUNCH_CT1S(5, 5, 4, 16, 8, 4, 8, 4, 0)
  }
  if (CONV_FAST_MATCH(3, 3, 4, 16, 8, 4, 8)) {       // s2 input conv 3x3 (32 -> 64)
    const int th = smallq_th(a, 8, 2);
    if (th == 4) CONV_FAST_LAUNCH(3, 3, 4, 16, 4, 4, 8, 4, 1)
    if (th == 2) CONV_FAST_LAUNCH_CT1(3, 3, 4, 16, 2, 4, 8, 4)
    CONV_FAST_LAUNCH_CT1S(3, 3, 4, 16, 8, 4, 8, 4, 0)
  }
  if (CONV_FAST_MATCH(3, 3, 8, 16, 8, 4, 8)) {       // s2 nodes / output conv and their dgrad (64 -> 64)
    const int th = smallq_th(a, 8, 2);
    if (th == 4) CONV_FAST_LAUNCH(3, 3, 8, 16, 4, 4, 8, 4, 1)
    if (th == 2) CONV_FAST_LAUNCH_CT1(3, 3, 8, 16, 2, 4, 8, 4)
    CONV_FAST_LAUNCH_CT1S(3, 3, 8, 16, 8, 4, 8, 4, 0)
  }
  if (CONV_FAST_MATCH(5, 5, 8, 16, 8, 2, 4)) {       // s2 input conv dgrad (64 -> 32)
    if (smallq_th(a, 8, 4) == 4) CONV_FAST_LAUNCH_CT1(5, 5, 8, 16, 4, 2, 4, 4)
    CONV_FAST_LAUNCH_CT1(5, 5, 8, 16, 8, 2, 4, 4)
  }
  if (CONV_FAST_MATCH(3, 3, 8, 16, 8, 2, 4)) {       // s2 input conv 3x3 dgrad (64 -> 32)
    if (smallq_th(a, 8, 4) == 4) CONV_FAST_LAUNCH_CT1(3, 3, 8, 16, 4, 2, 4, 4)
    CONV_FAST_LAUNCH_CT1(3, 3, 8, 16, 8, 2, 4, 4)
  }
  // 3x3 stage-input kernels (kernel_sizes ((3, 3), ...): a user choice, gentun/individuals.py:223), tiled
  // like their 5x5 counterparts above; the 3x3 node shapes are the same kernels already
  if (CONV_FAST_MATCH(3, 3, 1, 32, 8, 2, 3) && smallq_th(a, 8, 4) == 4) {      // s1 input conv 3x3
    if (pk_ok(a, 2)) CONV_FAST_LAUNCH_PK(3, 3, 1, 32, 4, 2, 3, 2, 1, 1)
    CONV_FAST_LAUNCH(3, 3, 1, 32, 4, 2, 3, 2, 1)
  }
  CONV_FAST_CASE_F32_PK(3, 3, 1, 32, 8, 2, 3, 4)      // s1 input conv 3x3 (3 -> 20)
  if (CONV_FAST_MATCH(3, 3, 3, 16, 8, 4, 7)) {       // s2 input conv 3x3 (20 -> 50)
    const int th = smallq_th(a, 8, 2);
    if (th == 4) CONV_FAST_LAUNCH(3, 3, 3, 16, 4, 4, 7, 4, 1)
    if (th == 2) CONV_FAST_LAUNCH_CT1(3, 3, 3, 16, 2, 4, 7, 4)
    CONV_FAST_LAUNCH_CT1S(3, 3, 3, 16, 8, 4, 7, 4, 0)
  }
  if (CONV_FAST_MATCH(3, 3, 7, 16, 8, 2, 3)) {       // s2 input conv 3x3 dgrad (50 -> 20)
    if (smallq_th(a, 8, 4) == 4) CONV_FAST_LAUNCH_CT1(3, 3, 7, 16, 4, 2, 3, 4)
    CONV_FAST_LAUNCH_CT1(3, 3, 7, 16, 8, 2, 3, 4)
  }
  CONV_FAST_CASE_F32_NARROW(3, 3, 7, 8, 8, 7, 13, 7)     // deep s3 input conv 3x3 (50 -> 100)
  CONV_FAST_CASE_F32_NARROW(3, 3, 13, 8, 8, 4, 7, 4)     // deep s3 input conv 3x3 dgrad (100 -> 50)
  CONV_FAST_CASE_F32_NARROW(3, 3, 1, 32, 8, 4, 8, 4)     // wide s1 input conv 3x3 (3 -> 64)
  if (CONV_FAST_MATCH(3, 3, 8, 16, 8, 8, 16)) CONV_FAST_LAUNCH_CT1S(3, 3, 8, 16, 8, 8, 16, 8, 0)   // wide s2 in 3x3
  CONV_FAST_CASE_F32_NARROW(3, 3, 16, 16, 4, 4, 8, 4)    // wide s2 input conv 3x3 dgrad (128 -> 64)
  CONV_FAST_CASE_F32_NARROW(3, 3, 16, 8, 8, 16, 32, 8)   // wide s3 input conv 3x3 (128 -> 256)
  CONV_FAST_CASE_F32_NARROW(3, 3, 32, 8, 4, 8, 16, 4)    // wide s3 input conv 3x3 dgrad (256 -> 128)
  return -100;
}

extern "C" int gt_wgrad_rows_ext(int KH, int KW, int Cinp, int Coutp, int H, int W, int prec) {
  if (prec != 1) return 0;
  // 32 / 64-channel stages
  if (KH == 5 && KW == 5 && Cinp == 8 && Coutp == 32 && W == 32 && H % 8 == 0) return 8;
  if (KH == 3 && KW == 3 && Cinp == 8 && Coutp == 32 && W == 32 && H % 8 == 0) return 8;
  if (KH == 3 && KW == 3 && Cinp == 32 && Coutp == 32 && W == 32 && H % 4 == 0) return 4;
  if (KH == 5 && KW == 5 && Cinp == 32 && Coutp == 64 && W == 16 && H % 4 == 0) return 4;
  if (KH == 3 && KW == 3 && Cinp == 32 && Coutp == 64 && W == 16 && H % 4 == 0) return 4;
  if (KH == 3 && KW == 3 && Cinp == 64 && Coutp == 64 && W == 16 && H % 4 == 0) return 4;
  // 3x3 stage-input kernels (bands as their 5x5 counterparts)
  if (KH == 3 && KW == 3 && Cinp == 8 && Coutp == 24 && W == 32 && H % 8 == 0) return 8;
  if (KH == 3 && KW == 3 && Cinp == 24 && Coutp == 56 && W == 16 && H % 4 == 0) return 4;
  if (KH == 3 && KW == 3 && Cinp == 56 && Coutp == 104 && W == 8 && H % 4 == 0) return 4;
  if (KH == 3 && KW == 3 && Cinp == 8 && Coutp == 64 && W == 32 && H % 4 == 0) return 4;
  if (KH == 3 && KW == 3 && Cinp == 64 && Coutp == 128 && W == 16 && H % 2 == 0) return 2;
  if (KH == 3 && KW == 3 && Cinp == 128 && Coutp == 256 && W == 8 && H % 4 == 0) return 4;
  return 0;
}

extern "C" int gt_wgrad_fast_ext(const WgradArgs* a, hipStream_t stream) {
  if (a->prec != 1) return -100;
  g_wgrad_nb = gt_wgrad_nb_force();
  // 32 / 64-channel stages
  WGRAD_FAST_CASE_F32(5, 5, 1, 4, 32, 8, 4, 1)      // s1 input conv (3 -> 32)
  WGRAD_FAST_CASE_F32(3, 3, 1, 4, 32, 8, 4, 1)      // s1 input conv 3x3 (3 -> 32)
  WGRAD_FAST_CASE_F32(3, 3, 4, 4, 32, 4, 4, 1)      // s1 nodes / output conv (32 -> 32)
  WGRAD_FAST_CASE_F32Z(5, 5, 4, 8, 16, 4, 8, 2)     // s2 input conv (32 -> 64)
  WGRAD_FAST_CASE_F32(3, 3, 4, 8, 16, 4, 8, 1)      // s2 input conv 3x3 (32 -> 64)
  WGRAD_FAST_CASE_F32(3, 3, 8, 8, 16, 4, 8, 1)      // s2 nodes / output conv (64 -> 64)
  // 3x3 stage-input kernels
  WGRAD_FAST_CASE_F32(3, 3, 1, 3, 32, 8, 4, 1)      // s1 input conv 3x3 (3 -> 20)
  WGRAD_FAST_CASE_F32(3, 3, 3, 7, 16, 4, 8, 1)      // s2 input conv 3x3 (20 -> 50)
  WGRAD_FAST_CASE_F32Z(3, 3, 7, 13, 8, 4, 8, 4)     // deep s3 input conv 3x3 (50 -> 100)
  WGRAD_FAST_CASE_F32(3, 3, 1, 8, 32, 4, 4, 1)      // wide s1 input conv 3x3 (3 -> 64)
  WGRAD_FAST_CASE_F32Z(3, 3, 8, 16, 16, 2, 8, 4)    // wide s2 input conv 3x3 (64 -> 128)
  WGRAD_FAST_CASE_F32Z(3, 3, 16, 32, 8, 4, 8, 5)    // wide s3 input conv 3x3 (128 -> 256)
  return -100;
}
