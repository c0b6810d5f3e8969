// Glorot-uniform initialisation of a whole fold-batched parameter set in one
// launch (reference: Keras kernel initializers re-run per
// fold, gentun/models/keras_models.py:120-125).
//
// Every weight tensor is a segment [G][d0][d1][d2][d3] whose real extent
// [r0][r1][r2][r3] sits in the zero-padded layout the kernels use (channels
// padded to 8, dense units to 64). Element e of fold g draws
// U(-limit, limit) from Philox4x32-10 keyed by the fold's seed with counter
// (real linear index, segment tag), so values do not depend on the padding,
// on the launch shape, or on which other folds share the launch.

#include "common.h"

struct InitSeg {
  float* p;                 // [G][d0][d1][d2][d3]
  const uint64_t* seeds;    // [G] per-fold keys
  int d[4], r[4];
  int G, tag;
  float limit;
  int pad;
};

struct InitArgs {
  const InitSeg* segs;
  const int2* blocks;       // per block: (segment, element offset within the segment)
};

__global__ void __launch_bounds__(256) glorot_init_kernel(InitArgs a) {
  const int2 blk = a.blocks[blockIdx.x];
  const InitSeg sg = a.segs[blk.x];
  const long per = (long)sg.d[0] * sg.d[1] * sg.d[2] * sg.d[3];
  const long i = (long)blk.y + threadIdx.x;
  if (i >= per * sg.G) return;
  const int g = (int)(i / per);
  long rem = i - (long)g * per;
  const int i3 = (int)(rem % sg.d[3]); rem /= sg.d[3];
  const int i2 = (int)(rem % sg.d[2]); rem /= sg.d[2];
  const int i1 = (int)(rem % sg.d[1]);
  const int i0 = (int)(rem / sg.d[1]);
  float v = 0.f;
  if (i0 < sg.r[0] && i1 < sg.r[1] && i2 < sg.r[2] && i3 < sg.r[3]) {
    const uint64_t lin = (((uint64_t)i0 * sg.r[1] + i1) * sg.r[2] + i2) * sg.r[3] + i3;
    uint32_t c[4] = {(uint32_t)lin, (uint32_t)(lin >> 32), (uint32_t)sg.tag, 0x676c6f72u};
    const uint64_t key = sg.seeds[g];
    philox4x32_10(c, (uint32_t)key, (uint32_t)(key >> 32));
    const float u = (float)(c[0] >> 8) * (1.0f / 16777216.0f);      // [0, 1)
    v = (2.f * u - 1.f) * sg.limit;
  }
  sg.p[i] = v;
}

extern "C" {

size_t gt_sizeof_init_seg() { return sizeof(InitSeg); }

#ifndef GT_SRC_HASH
#define GT_SRC_HASH "unhashed"
#endif
// content hash of the sources this library was compiled from (tools/build_native.py)
const char* gt_build_hash() { return GT_SRC_HASH; }

int gt_glorot_init(const InitArgs* a, int nblocks, hipStream_t stream) {
  if (nblocks <= 0) return 0;
  hipLaunchKernelGGL(glorot_init_kernel, dim3(nblocks), dim3(256), 0, stream, *a);
  return (int)hipGetLastError();
}

// host reference of one draw (tests): same Philox stream as the kernel
float gt_glorot_ref(uint64_t key, uint64_t lin, int tag, float limit) {
  uint32_t c[4] = {(uint32_t)lin, (uint32_t)(lin >> 32), (uint32_t)tag, 0x676c6f72u};
  philox4x32_10(c, (uint32_t)key, (uint32_t)(key >> 32));
  const float u = (float)(c[0] >> 8) * (1.0f / 16777216.0f);
  return (2.f * u - 1.f) * limit;
}

}  // extern "C"
