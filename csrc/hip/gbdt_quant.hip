// G1: on-device dataset quantisation for the GBDT GPU path (SURVEY.md §2.4;
// the reference builds an xgb.DMatrix per candidate, gentun/models/xgboost_models.py:32).
//
// Bit-identical to the CPU engine's quantize_column (csrc/gbdt/engine.cpp):
// NaN -> -inf, per feature either every distinct value is a bin (<= 256
// values) or 256 equal-count quantile cuts; bin = lower_bound(upper, v).
//   1. LDS-tiled transpose X[n][F] -> columns [F][n]
//   2. rocprim segmented radix sort of all F columns in one call
//   3. one workgroup per feature: distinct-value scan (ballot prefix sums,
//      stops after 257 values) or quantile cuts -> upper[F][256], nbins[F]
//   4. binary search per (row, feature) -> row-major bins [n][Fs] written
//      straight into the device bins cache (gbdt_cache.h) that the boosting
//      kernels read: the quantised dataset never crosses PCIe.

#include <hip/hip_runtime.h>

#include <cstring>

#include <rocprim/device/device_segmented_radix_sort.hpp>

#include <cmath>
#include <cstdint>
#include <vector>

#include "gbdt_cache.h"

namespace {

#define QHC(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { rc = -100 - (int)e_; goto done; } } while (0)

__device__ __forceinline__ float qt_clean(float v) { return isnan(v) ? -INFINITY : v; }

// 64x64 tiles, 256 threads: coalesced reads along features, coalesced writes along rows
__global__ void __launch_bounds__(256) qt_transpose(const float* __restrict__ X, int n, int F,
                                                    float* __restrict__ col) {
  __shared__ float t[64][65];
  const int r0 = blockIdx.x * 64, f0 = blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < 64; r += 4) {
    const int i = r0 + r, f = f0 + tx;
    if (i < n && f < F) t[r][tx] = qt_clean(X[(size_t)i * F + f]);
  }
  __syncthreads();
  for (int ff = ty; ff < 64; ff += 4) {
    const int f = f0 + ff, i = r0 + tx;
    if (i < n && f < F) col[(size_t)f * n + i] = t[tx][ff];
  }
}

// one workgroup (256 threads) per feature
__global__ void __launch_bounds__(256) qt_cuts(const float* __restrict__ sorted, int n,
                                               float* __restrict__ upper, int* __restrict__ nbins) {
  __shared__ float uq[257];
  __shared__ int wsum[4];
  const int f = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const float* s = sorted + (size_t)f * n;
  const unsigned long long below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  int cnt = 0;
  for (int base = 0; base < n && cnt <= 256; base += 256) {
    const int i = base + tid;
    bool flag = false;
    float v = 0.f;
    if (i < n) { v = s[i]; flag = (i == 0) || (v != s[i - 1]); }
    const unsigned long long m = __ballot(flag);
    if (lane == 0) wsum[wv] = __popcll(m);
    __syncthreads();
    int off = 0, tot = 0;
    for (int w = 0; w < 4; ++w) { off += (w < wv) ? wsum[w] : 0; tot += wsum[w]; }
    if (flag) {
      const int pos = cnt + off + __popcll(m & below);
      if (pos < 257) uq[pos] = v;
    }
    cnt += tot;
    __syncthreads();
  }
  float* up = upper + (size_t)f * 256;
  if (cnt <= 256) {
    for (int k = tid; k < cnt; k += 256) up[k] = uq[k];
    if (tid == 0) nbins[f] = cnt;
  } else if (tid == 0) {
    int nb = 0;
    for (int b = 1; b <= 256; ++b) {
      long long idx = (long long)((double)b * n / 256) - (b == 256 ? 1 : 0);
      if (idx > n - 1) idx = n - 1;
      const float v = s[idx];
      if (nb == 0 || v > up[nb - 1]) up[nb++] = v;
    }
    up[nb - 1] = s[n - 1];
    nbins[f] = nb;
  }
}

__global__ void __launch_bounds__(256) qt_bins(const float* __restrict__ X, int n, int F, int Fs,
                                               const float* __restrict__ upper, const int* __restrict__ nbins,
                                               uint8_t* __restrict__ bins) {
  const size_t total = (size_t)n * Fs;
  for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < total;
       idx += (size_t)gridDim.x * blockDim.x) {
    const int i = (int)(idx / Fs), f = (int)(idx - (size_t)i * Fs);
    int b = 0;
    if (f < F) {
      const float v = qt_clean(X[(size_t)i * F + f]);
      const float* up = upper + (size_t)f * 256;
      const int nb = nbins[f];
      int lo = 0, hi = nb;                    // first k with !(up[k] < v)
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (up[mid] < v) lo = mid + 1; else hi = mid;
      }
      b = lo >= nb ? nb - 1 : lo;
    }
    bins[idx] = (uint8_t)b;
  }
}

}  // namespace

extern "C" {

// Quantise X [n][F] (host, fp32) on the device into the bins cache under
// cache_key (row stride Fs >= F, Fs % 4 == 0, padding bins 0); nbins_out[F]
// receives the bins per feature. Returns 0 or < 0 on error.
int gbdt_quantize_hip(const float* X_h, int n, int F, int Fs, long long cache_key, int* nbins_out) {
  if (n <= 0 || F <= 0 || Fs < F || Fs % 4 || cache_key == 0) return -1;
  if ((long long)n * F >= (1ll << 31)) return -2;        // rocprim item count is an int
  std::lock_guard<std::mutex> lock(gbdt_cache::mu);
  int rc = 0;
  float *d_X = nullptr, *d_col = nullptr, *d_sorted = nullptr, *d_upper = nullptr;
  int *d_off = nullptr, *d_nb = nullptr;
  void* d_tmp = nullptr;
  size_t tmp_bytes = 0;
  const size_t nbytes = (size_t)n * Fs;
  std::vector<int> off(F + 1);
  for (int f = 0; f <= F; ++f) off[f] = f * n;
  QHC(hipMalloc(&d_X, sizeof(float) * (size_t)n * F));
  QHC(hipMalloc(&d_col, sizeof(float) * (size_t)n * F));
  QHC(hipMalloc(&d_sorted, sizeof(float) * (size_t)n * F));
  QHC(hipMalloc(&d_upper, sizeof(float) * (size_t)F * 256));
  QHC(hipMalloc(&d_off, sizeof(int) * (F + 1)));
  QHC(hipMalloc(&d_nb, sizeof(int) * F));
  QHC(hipMemcpy(d_X, X_h, sizeof(float) * (size_t)n * F, hipMemcpyHostToDevice));
  QHC(hipMemcpy(d_off, off.data(), sizeof(int) * (F + 1), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(qt_transpose, dim3((n + 63) / 64, (F + 63) / 64), dim3(256), 0, 0, d_X, n, F, d_col);
  QHC(rocprim::segmented_radix_sort_keys(nullptr, tmp_bytes, d_col, d_sorted, n * F, F, d_off, d_off + 1));
  QHC(hipMalloc(&d_tmp, tmp_bytes));
  QHC(rocprim::segmented_radix_sort_keys(d_tmp, tmp_bytes, d_col, d_sorted, n * F, F, d_off, d_off + 1));
  hipLaunchKernelGGL(qt_cuts, dim3(F), dim3(256), 0, 0, d_sorted, n, d_upper, d_nb);
  if (gbdt_cache::bins == nullptr || gbdt_cache::bytes != nbytes) {
    if (gbdt_cache::bins) (void)hipFree(gbdt_cache::bins);
    gbdt_cache::bins = nullptr; gbdt_cache::key = 0; gbdt_cache::bytes = 0;
    QHC(hipMalloc(&gbdt_cache::bins, nbytes));
    gbdt_cache::bytes = nbytes;
  }
  gbdt_cache::key = 0;                                    // invalid until the bins are written
  gbdt_cache::invalidate_derived();
  hipLaunchKernelGGL(qt_bins, dim3(2048), dim3(256), 0, 0, d_X, n, F, Fs, d_upper, d_nb, gbdt_cache::bins);
  QHC(hipGetLastError());
  QHC(hipMemcpy(nbins_out, d_nb, sizeof(int) * F, hipMemcpyDeviceToHost));
  gbdt_cache::key = cache_key;
done:
  for (void* p : {(void*)d_X, (void*)d_col, (void*)d_sorted, (void*)d_upper, (void*)d_off, (void*)d_nb, d_tmp})
    if (p) (void)hipFree(p);
  return rc;
}

// Copy the cached device bins back (tests); -7 if the key is not resident.
int gbdt_bins_hip_copy(long long cache_key, uint8_t* dst, size_t bytes) {
  std::lock_guard<std::mutex> lock(gbdt_cache::mu);
  if (cache_key == 0 || cache_key != gbdt_cache::key || bytes != gbdt_cache::bytes) return -7;
  return hipMemcpy(dst, gbdt_cache::bins, bytes, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -3;
}

}  // extern "C"
