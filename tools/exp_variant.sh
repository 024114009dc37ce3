#!/bin/bash
# Experiment build: dvcc_kernels.hip with extra -D flags, linked with the
# in-tree objects into exp_build/<name>/libdvcc.so (run with DVCC_LIB=...).
#   tools/exp_variant.sh <name> [-DFLAG ...]
set -e
N=$1; shift
D=exp_build/$N
mkdir -p $D
B=deneva-plus_amd/build
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I include -I deneva-plus_amd/csrc "$@" \
    -c deneva-plus_amd/csrc/dvcc_kernels.hip -o $D/dvcc_kernels.o
objs=$(ls $B/*.o | grep -v dvcc_kernels.o)
hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libdvcc.so $D/dvcc_kernels.o $objs -L/opt/rocm/lib -lrccl \
    -Wl,-rpath,/opt/rocm/lib
