#!/bin/bash
# Alternative build of the kernel library for same-box A/B runs (GENTUN_HIP_LIB=<path>):
#   bash tools/build_ab.sh NAME -DMACRO=VALUE ...   ->  ab_libs/NAME.so
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p build/ab_$name ab_libs
objs=()
for f in csrc/hip/*.hip; do
  o=build/ab_$name/$(basename $f).o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -DGT_SRC_HASH=\"ab\" "$@" -I csrc/hip -c -o $o $f &
  objs+=($o)
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ab_libs/$name.so "${objs[@]}"
echo ab_libs/$name.so
