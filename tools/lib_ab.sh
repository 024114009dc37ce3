#!/bin/bash
# A/B of exp_build libraries on one bench command, alternated:
#   tools/lib_ab.sh <tag> <rounds> "<libA> <libB> ..." [bench args...]
set -e
OUT=gpurun_out/$1; N=$2; LIBS=$3; shift 3
mkdir -p $OUT
for i in $(seq 1 $N); do
  for v in $LIBS; do
    DVCC_LIB=$PWD/exp_build/$v/libdvcc.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-tpcc "$@" > $OUT/$v$i.json 2> $OUT/$v$i.err
    python3 -c "import json; d=json.loads(open('$OUT/$v$i.json').read().strip().splitlines()[-1]); print('$v', round(d['ms_per_step'],4), round(d['value']/1e6,2), round(d['stage_ms_mean']['ms_sort'],4), round(d['stage_ms_mean']['ms_total'],4))"
  done
done
