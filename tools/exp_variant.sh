#!/bin/bash
# Experiment build: the listed HIP sources (comma-separated, default
# dvcc_kernels.hip) rebuilt with extra -D flags and linked with the in-tree
# objects into exp_build/<name>/libdvcc.so (run with DVCC_LIB=...).
#   tools/exp_variant.sh <name> [src.hip,src2.hip] [-DFLAG ...]
set -e
N=$1; shift
SRCS=dvcc_kernels.hip
if [ $# -gt 0 ] && [[ "$1" != -* ]]; then SRCS=$1; shift; fi
D=exp_build/$N
mkdir -p $D
B=deneva-plus_amd/build
objs=$(ls $B/*.o)
for f in ${SRCS//,/ }; do
  o=$D/${f%.hip}.o
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I include -I deneva-plus_amd/csrc "$@" \
      -c deneva-plus_amd/csrc/$f -o $o
  objs=$(echo "$objs" | tr ' ' '\n' | grep -v "/${f%.hip}.o$")
  objs="$objs $o"
done
hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libdvcc.so $objs -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
