#!/bin/bash
# Alternative build of the kernel library for same-box A/B runs (GENTUN_HIP_LIB=<path>):
#   bash tools/build_ab.sh NAME -DMACRO=VALUE ...   ->  gentun_amd/_native/ab/NAME.so
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p build/ab_$name gentun_amd/_native/ab
objs=()
for f in csrc/hip/*.hip; do
  o=build/ab_$name/$(basename $f).o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -DGT_SRC_HASH=\"ab\" "$@" -I csrc/hip -c -o $o $f &
  objs+=($o)
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o gentun_amd/_native/ab/$name.so "${objs[@]}"
echo gentun_amd/_native/ab/$name.so
