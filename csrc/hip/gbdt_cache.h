// Device-resident quantised dataset shared by the GBDT GPU kernels
// (gbdt_hist.hip: k-fold boosting; gbdt_quant.hip: on-device quantisation).
// One entry per process, keyed by the caller's dataset key; every user holds
// the mutex for the whole call.
#pragma once
#include <cstddef>
#include <cstdint>
#include <mutex>

namespace gbdt_cache {
extern uint8_t* bins;      // row-major [n][Fs] uint8
extern long long key;      // 0 = empty
extern size_t bytes;
extern std::mutex mu;
void invalidate_derived();   // drop copies derived from bins (gbdt_hist.hip's feature-major copy); call with mu held
}  // namespace gbdt_cache
