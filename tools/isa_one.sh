#!/bin/bash
# Resource usage (VGPRs, spills, occupancy) and ISA of ONE kernel instantiation of cnn_conv_fast.hip,
# in seconds instead of the whole file's minutes:
#   bash tools/isa_one.sh 'conv_pipe_f32_kernel<3, 3, 7, 16, 8, 4, 7, 0>(ConvArgs, int)' [-DMACRO=V ...]
# -> /tmp/isa_one/one.s (+ the remarks on stdout)
set -e
cd "$(dirname "$0")/.."
inst=$1; shift
mkdir -p /tmp/isa_one
printf '#define GT_KERNELS_ONLY 1\n#include "cnn_conv_fast.hip"\ntemplate __global__ void %s;\n' "$inst" > /tmp/isa_one/one.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -munsafe-fp-atomics -I csrc/hip "$@" --cuda-device-only -S \
  -o /tmp/isa_one/one.s /tmp/isa_one/one.hip -Rpass-analysis=kernel-resource-usage 2>&1 |
  grep -E "Function Name|VGPRs:|AGPRs:|Spill|Scratch|Occupancy|LDS Size|error" | sed 's/.*remark: *//; s/ \[-Rpass.*//'
echo "mfma: $(grep -c v_mfma /tmp/isa_one/one.s)  scratch ops: $(grep -c scratch_ /tmp/isa_one/one.s)"
