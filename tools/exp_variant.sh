#!/bin/bash
# Experiment build: the listed HIP sources (comma-separated, default
# dvcc_kernels.hip) rebuilt with extra -D flags and linked with the in-tree
# objects into exp_build/<name>/libdvcc.so (run with DVCC_LIB=...).
#   tools/exp_variant.sh <name> [src.hip,src2.hip] [-DFLAG ...]
# EXP_PATCH=<file.diff>: the sources are taken from a copy of csrc with that
# patch applied (measurement-only code kept out of the product's sources,
# e.g. tools/patches/lane_stamps.diff)
set -e
N=$1; shift
SRCS=dvcc_kernels.hip
if [ $# -gt 0 ] && [[ "$1" != -* ]]; then SRCS=$1; shift; fi
D=exp_build/$N
mkdir -p $D
B=deneva-plus_amd/build
objs=$(ls $B/*.o)
SRC=deneva-plus_amd/csrc
if [ -n "$EXP_PATCH" ]; then
  SRC=$D/src
  rm -rf $SRC && mkdir -p $SRC && cp deneva-plus_amd/csrc/* $SRC/
  patch -s -d $SRC -p3 < "$EXP_PATCH"
fi
for f in ${SRCS//,/ }; do
  o=$D/${f%.hip}.o
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I include -I $SRC "$@" \
      -c $SRC/$f -o $o
  objs=$(echo "$objs" | tr ' ' '\n' | grep -v "/${f%.hip}.o$")
  objs="$objs $o"
done
hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libdvcc.so $objs -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
