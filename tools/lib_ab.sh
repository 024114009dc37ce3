#!/bin/bash
# A/B of exp_build libraries / bench flags on one bench command, alternated:
#   tools/lib_ab.sh <tag> <rounds> "<var> <var> ..." [bench args...]
# a variant is <lib>[+flag,flag...]: <lib> an exp_build/<lib>/libdvcc.so, or
# "cur" for the in-tree build; the flags (comma-separated) go to that run only
set -e
OUT=gpurun_out/$1; N=$2; LIBS=$3; shift 3
mkdir -p $OUT
for i in $(seq 1 $N); do
  for v in $LIBS; do
    lib=${v%%+*}; extra=""
    [[ $v == *+* ]] && { extra=${v#*+}; extra=${extra//,/ }; }
    name=${v//[+,]/_}
    lp=""; [ "$lib" != cur ] && lp=$PWD/exp_build/$lib/libdvcc.so
    DVCC_LIB=$lp timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-tpcc --no-configs --detail-out $OUT/$name$i.detail.json "$@" $extra > $OUT/$name$i.json 2> $OUT/$name$i.err
    python3 -c "import json; d=json.load(open('$OUT/$name$i.detail.json')); print('$v', round(d['ms_per_step'],4), round(d['value']/1e6,2), round(d['stage_ms_mean']['ms_sort'],4), round(d['stage_ms_mean']['ms_total'],4), round(d['kernel_us_per_epoch'],1), [(k['kernel'], round(k['avg_us'],1)) for k in d['kernels'][:3] + [k for k in d['kernels'] if k['kernel'].startswith('k_exec')]])"
  done
done
