#!/bin/bash
# k_probe duration (dispatch timestamps) and epoch time of the default bench,
# default library against exp_build variants given as names (safe variants only).
#   tools/probe_ab.sh <tag> [variant ...]
set -e
OUT=gpurun_out/$1; shift
mkdir -p $OUT
for v in default "$@" default "$@"; do
  L=""; [ $v != default ] && L="DVCC_LIB=$PWD/exp_build/$v/libdvcc.so"
  env $L timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-tpcc --steps 20 > $OUT/$v.json 2> $OUT/$v.err
  python3 -c "import json; d=json.loads(open('$OUT/$v.json').read().strip().splitlines()[-1]); print('$v', 'probe_us', round(d['roofline']['avg_launch_ms']*1e3,1), 'ms', round(d['ms_per_step'],4), 'stage', round(d['stage_ms_mean']['ms_total'],4))"
done
