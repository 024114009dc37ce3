#!/bin/bash
# One-context A/B of experiment libraries (tools/exp_onectx.py), alternated:
#   tools/onectx_ab.sh <tag> <rounds> "<lib> <lib> ..." [steps] [lanes]
# <lib>: exp_build/<lib>/libdvcc.so, or "cur" for the in-tree build
set -e
OUT=gpurun_out/$1; N=$2; LIBS=$3; STEPS=${4:-30}; LN=${5:-1}
mkdir -p $OUT
for i in $(seq 1 $N); do
  for v in $LIBS; do
    lp=""; [ "$v" != cur ] && lp=$PWD/exp_build/$v/libdvcc.so
    DVCC_LIB=$lp timeout -k 10 300 python3 -u tools/exp_onectx.py $STEPS $LN > $OUT/$v$i.json 2> $OUT/$v$i.err
    echo "$v $(cat $OUT/$v$i.json)"
  done
done
