#!/bin/bash
# Alternative build of the kernel library for same-box A/B runs (GENTUN_HIP_LIB=<path>):
#   bash tools/build_ab.sh NAME -DMACRO=VALUE ...   ->  ab_libs/NAME.so
# ONLY=<basename> (e.g. ONLY=gbdt_hist) compiles just that source with the macros and links it with the
# in-tree build's objects of the others (build/obj_libgentun_hip, from tools/build_native.py).
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p build/ab_$name ab_libs
objs=()
for f in csrc/hip/*.hip; do
  b=$(basename $f)
  if [ -n "$ONLY" ] && [ "${b%.hip}" != "$ONLY" ]; then
    objs+=(build/obj_libgentun_hip/$b.o)
    continue
  fi
  o=build/ab_$name/$b.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -DGT_SRC_HASH=\"ab\" "$@" -I csrc/hip -c -o $o $f &
  objs+=($o)
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ab_libs/$name.so "${objs[@]}"
echo ab_libs/$name.so
