#!/bin/bash
# Config-D bench at several prefix sizes (dv_set_prefix), value and ms only.
#   tools/gpu_prefix_sweep.sh <tag> [K ...]
set -e
TAG=${1:-sweep}; shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
for K in ${@:--1 4096 8192 16384 32768}; do
  timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline --no-tpcc --prefix $K > $OUT/bench_$K.json 2> $OUT/bench_$K.err
  python3 -c "import json;d=json.loads(open('$OUT/bench_$K.json').read().strip().splitlines()[-1]);print('K=$K value %.4g ms %.4f rounds %.1f stages %s' % (d['value'], d['ms_per_step'], d['rounds_mean'], {k: round(v,4) for k,v in d['stage_ms_mean'].items()}))"
done
