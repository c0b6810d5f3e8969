// Host-side dispatch helpers of the shape-specialised conv / wgrad kernels (conv_fast_impl.h), shared by
// cnn_conv_fast.hip and cnn_conv_fast_ext.hip. The launch macros expect, in the including translation
// unit: g_probe (probe mode: report the tile rows instead of launching), regepi_on(), smallq_th(),
// g_wgrad_nb and wgrad_nz().
#pragma once
#include "conv_fast_impl.h"

// dynamic LDS above 64 KiB: raise the per-function limit once (gfx950 has 160 KiB per CU)
template <typename F>
static void lds_limit(F* fn, size_t bytes) {
  if (bytes > 65536) (void)hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)bytes);
}

#define CONV_FAST_LAUNCH_PK(KH_, KW_, NCBI_, W_, TH_, NT_, NCO_, NWV_, PREC_, PK_)                        \
  {                                                                                                     \
    if (g_probe) return 1000 + TH_;                                                                     \
    dim3 grid(a->B * (a->H / TH_), a->ngroups);                                                         \
    const size_t lds = FastCfg<KH_, KW_, NCBI_, W_, TH_, NT_, NCO_, PREC_>::lds(a->epi_bf16 != 0);      \
    auto* fn = conv_fast_kernel<KH_, KW_, NCBI_, W_, TH_, NT_, NCO_, NWV_, PREC_, PK_>;                 \
    if (PREC_ == 1 && (W_ % 16) == 0 && regepi_on())                                                    \
      fn = conv_fast_kernel<KH_, KW_, NCBI_, W_, TH_, NT_, NCO_, NWV_, PREC_, PK_, 1>;                  \
    lds_limit(fn, lds);                                                                                 \
    hipLaunchKernelGGL(fn, grid, dim3(NWV_ * 64), lds, stream, *a);                                     \
    return (int)hipGetLastError();                                                                      \
  }
#define CONV_FAST_LAUNCH(KH_, KW_, NCBI_, W_, TH_, NT_, NCO_, NWV_, PREC_)                               \
  CONV_FAST_LAUNCH_PK(KH_, KW_, NCBI_, W_, TH_, NT_, NCO_, NWV_, PREC_, 0)

// one co tile per wave (CTX 1), fp32, register-direct epilogue
#define CONV_FAST_LAUNCH_CT1(KH_, KW_, NCBI_, W_, TH_, NT_, NCO_, NWV_) \
  CONV_FAST_LAUNCH_CT1S(KH_, KW_, NCBI_, W_, TH_, NT_, NCO_, NWV_, 1)
#define CONV_FAST_LAUNCH_CT1S(KH_, KW_, NCBI_, W_, TH_, NT_, NCO_, NWV_, SCH_)                            \
  {                                                                                                     \
    if (g_probe) return 1000 + TH_;                                                                     \
    dim3 grid(a->B * (a->H / TH_), a->ngroups);                                                         \
    const size_t lds = FastCfg<KH_, KW_, NCBI_, W_, TH_, NT_, NCO_, 1>::lds(a->epi_bf16 != 0);          \
    auto* fn = conv_fast_kernel<KH_, KW_, NCBI_, W_, TH_, NT_, NCO_, NWV_, 1, 0, 1, 1, SCH_>;           \
    lds_limit(fn, lds);                                                                                 \
    hipLaunchKernelGGL(fn, grid, dim3(NWV_ * 64), lds, stream, *a);                                     \
    return (int)hipGetLastError();                                                                      \
  }

// the packed last co tile applies: fp32, the real output channels leave <= 4 in the last 16-channel tile
static bool pk_ok(const ConvArgs* a, int nt) {
  const int last = a->cout_real - 16 * (nt - 1);
  return a->prec == 1 && a->cout_real > 0 && last >= 1 && last <= 4;
}

#define CONV_FAST_MATCH(KH_, KW_, NCBI_, W_, TH_, NT_, NCO_)                                             \
  (a->KH == KH_ && a->KW == KW_ && a->Cinp == NCBI_ * 8 && a->W == W_ && a->Coutp == NCO_ * 8 &&       \
   (NCO_ * 8 + 15) / 16 == NT_ && a->H % TH_ == 0)

#define CONV_FAST_CASE(KH_, KW_, NCBI_, W_, TH_, NT_, NCO_)                                              \
  if (CONV_FAST_MATCH(KH_, KW_, NCBI_, W_, TH_, NT_, NCO_)) CONV_FAST_LAUNCH(KH_, KW_, NCBI_, W_, TH_, NT_, NCO_, 4, 0)

// shapes with an 8-wave instantiation: `def_` waves unless overridden
#define CONV_FAST_CASE2(KH_, KW_, NCBI_, W_, TH_, NT_, NCO_, def_)                                       \
  if (CONV_FAST_MATCH(KH_, KW_, NCBI_, W_, TH_, NT_, NCO_)) {                                           \
    if ((g_conv_nwv ? g_conv_nwv : def_) == 8) CONV_FAST_LAUNCH(KH_, KW_, NCBI_, W_, TH_, NT_, NCO_, 8, 0) \
    CONV_FAST_LAUNCH(KH_, KW_, NCBI_, W_, TH_, NT_, NCO_, 4, 0)                                         \
  }

// odd tile counts (104 channels = 7 x 16): one co tile per wave, NT waves
#define CONV_FAST_CASE_NW(KH_, KW_, NCBI_, W_, TH_, NT_, NCO_, NWV_)                                      \
  if (CONV_FAST_MATCH(KH_, KW_, NCBI_, W_, TH_, NT_, NCO_)) CONV_FAST_LAUNCH(KH_, KW_, NCBI_, W_, TH_, NT_, NCO_, NWV_, 0)

#define CONV_FAST_CASE_F32(KH_, KW_, NCBI_, W_, TH_, NT_, NCO_, NWV_)                                     \
  if (CONV_FAST_MATCH(KH_, KW_, NCBI_, W_, TH_, NT_, NCO_)) {                                           \
    CONV_FAST_LAUNCH(KH_, KW_, NCBI_, W_, TH_, NT_, NCO_, NWV_, 1)                                      \
  }
// narrow images (W < 16: no persistent variant), and the wide deep-space shapes (tile kernel only)
#define CONV_FAST_CASE_F32_NARROW(KH_, KW_, NCBI_, W_, TH_, NT_, NCO_, NWV_)                              \
  if (CONV_FAST_MATCH(KH_, KW_, NCBI_, W_, TH_, NT_, NCO_)) CONV_FAST_LAUNCH(KH_, KW_, NCBI_, W_, TH_, NT_, NCO_, NWV_, 1)
// shapes whose every wave owns all NT co tiles: packed last tile when the real channels allow
#define CONV_FAST_CASE_F32_PK(KH_, KW_, NCBI_, W_, TH_, NT_, NCO_, NWV_)                                  \
  if (CONV_FAST_MATCH(KH_, KW_, NCBI_, W_, TH_, NT_, NCO_)) {                                           \
    if (pk_ok(a, NT_)) {                                                                                \
      CONV_FAST_LAUNCH_PK(KH_, KW_, NCBI_, W_, TH_, NT_, NCO_, NWV_, 1, 1)                              \
    }                                                                                                   \
    CONV_FAST_LAUNCH(KH_, KW_, NCBI_, W_, TH_, NT_, NCO_, NWV_, 1)                                      \
  }

#define WGRAD_FAST_CASE(KH_, KW_, NCBI_, NCBO_, W_, R_, NW_, NB_)                                         \
  if (a->KH == KH_ && a->KW == KW_ && a->Cinp == NCBI_ * 8 && a->Coutp == NCBO_ * 8 && a->W == W_ &&     \
      a->H % R_ == 0 && a->pps % (R_ * W_) == 0) {                                                        \
    dim3 grid(a->S, a->ngroups);                                                                         \
    if ((g_wgrad_nb ? g_wgrad_nb : NB_) == 1)                                                            \
      hipLaunchKernelGGL((wgrad_fast_kernel<KH_, KW_, NCBI_, NCBO_, W_, R_, NW_, 1>), grid, dim3(NW_ * 64), 0, stream, *a); \
    else                                                                                                 \
      hipLaunchKernelGGL((wgrad_fast_kernel<KH_, KW_, NCBI_, NCBO_, W_, R_, NW_, 2>), grid, dim3(NW_ * 64), 0, stream, *a); \
    return (int)hipGetLastError();                                                                       \
  }

#define WGRAD_F32_LAUNCH(KH_, KW_, NCBI_, NCBO_, W_, R_, NW_, NB_, PK_)                                   \
  hipLaunchKernelGGL((wgrad_fast_f32_kernel<KH_, KW_, NCBI_, NCBO_, W_, R_, NW_, NB_, PK_>), grid,           \
                     dim3(NW_ * 64), 0, stream, *a)
#define WGRAD_FAST_CASE_F32(KH_, KW_, NCBI_, NCBO_, W_, R_, NW_, NB_)                                     \
  if (a->KH == KH_ && a->KW == KW_ && a->Cinp == NCBI_ * 8 && a->Coutp == NCBO_ * 8 && a->W == W_ &&     \
      a->H % R_ == 0 && a->pps % (R_ * W_) == 0) {                                                        \
    const int nz_ = wgrad_nz(a);                                                                         \
    if (nz_ > 1) {                                                                                       \
      dim3 gz(a->S, a->ngroups, nz_);                                                                    \
      const bool pkz = wgrad_pk_ok(a, (NCBO_ * 8 + 15) / 16);                                            \
      if (nz_ == 2) {                                                                                    \
        /* the shape's band buffers (2 for the 16-wide stage: its 2 x S x G workgroups fit one per CU) */  \
        if (pkz) hipLaunchKernelGGL((wgrad_fast_f32_kernel<KH_, KW_, NCBI_, NCBO_, W_, R_, NW_, NB_, 1, 2>), gz, \
                                    dim3(NW_ * 64), 0, stream, *a);                                      \
        else hipLaunchKernelGGL((wgrad_fast_f32_kernel<KH_, KW_, NCBI_, NCBO_, W_, R_, NW_, NB_, 0, 2>), gz,     \
                                dim3(NW_ * 64), 0, stream, *a);                                          \
      } else if (nz_ == 8) {                                                                             \
        /* tiny launches (< 32 split x group blocks): 8 slices of 4-wave workgroups */                   \
        if (pkz) hipLaunchKernelGGL((wgrad_fast_f32_kernel<KH_, KW_, NCBI_, NCBO_, W_, R_, 4, 1, 1, 8>), gz, \
                                    dim3(256), 0, stream, *a);                                           \
        else hipLaunchKernelGGL((wgrad_fast_f32_kernel<KH_, KW_, NCBI_, NCBO_, W_, R_, 4, 1, 0, 8>), gz,     \
                                dim3(256), 0, stream, *a);                                               \
      } else {                                                                                           \
        if (pkz) hipLaunchKernelGGL((wgrad_fast_f32_kernel<KH_, KW_, NCBI_, NCBO_, W_, R_, NW_, 1, 1, 4>), gz, \
                                    dim3(NW_ * 64), 0, stream, *a);                                      \
        else hipLaunchKernelGGL((wgrad_fast_f32_kernel<KH_, KW_, NCBI_, NCBO_, W_, R_, NW_, 1, 0, 4>), gz,     \
                                dim3(NW_ * 64), 0, stream, *a);                                          \
      }                                                                                                  \
      return (int)hipGetLastError();                                                                     \
    }                                                                                                    \
    dim3 grid(a->S, a->ngroups);                                                                         \
    const bool pk = wgrad_pk_ok(a, (NCBO_ * 8 + 15) / 16);                                               \
    if ((g_wgrad_nb ? g_wgrad_nb : NB_) == 1) {                                                          \
      if (pk) WGRAD_F32_LAUNCH(KH_, KW_, NCBI_, NCBO_, W_, R_, NW_, 1, 1);                               \
      else WGRAD_F32_LAUNCH(KH_, KW_, NCBI_, NCBO_, W_, R_, NW_, 1, 0);                                  \
    } else {                                                                                             \
      if (pk) WGRAD_F32_LAUNCH(KH_, KW_, NCBI_, NCBO_, W_, R_, NW_, 2, 1);                               \
      else WGRAD_F32_LAUNCH(KH_, KW_, NCBI_, NCBO_, W_, R_, NW_, 2, 0);                                  \
    }                                                                                                    \
    return (int)hipGetLastError();                                                                       \
  }

// wide layers: NZ column slices per (split, group), single band buffer
#define WGRAD_FAST_CASE_F32Z(KH_, KW_, NCBI_, NCBO_, W_, R_, NW_, NZ_)                                    \
  if (a->KH == KH_ && a->KW == KW_ && a->Cinp == NCBI_ * 8 && a->Coutp == NCBO_ * 8 && a->W == W_ &&     \
      a->H % R_ == 0 && a->pps % (R_ * W_) == 0) {                                                        \
    dim3 grid(a->S, a->ngroups, NZ_);                                                                    \
    if (wgrad_pk_ok(a, (NCBO_ * 8 + 15) / 16))                                                           \
      hipLaunchKernelGGL((wgrad_fast_f32_kernel<KH_, KW_, NCBI_, NCBO_, W_, R_, NW_, 1, 1, NZ_>), grid,       \
                         dim3(NW_ * 64), 0, stream, *a);                                                 \
    else                                                                                                 \
      hipLaunchKernelGGL((wgrad_fast_f32_kernel<KH_, KW_, NCBI_, NCBO_, W_, R_, NW_, 1, 0, NZ_>), grid,       \
                         dim3(NW_ * 64), 0, stream, *a);                                                 \
    return (int)hipGetLastError();                                                                       \
  }

// packed last co tile of the fp32 wgrad
static bool wgrad_pk_ok(const WgradArgs* a, int mt) {
  const int last = a->cout_real - 16 * (mt - 1);
  return a->cout_real > 0 && last >= 1 && last <= 4;
}

