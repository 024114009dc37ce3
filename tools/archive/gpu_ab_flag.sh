#!/bin/bash
# A/B of one bench option against the default on the same box, alternated:
#   tools/gpu_ab_flag.sh <tag> <rounds> "<option>" [bench args...]
set -e
OUT=gpurun_out/$1; N=$2; OPT=$3; shift 3
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for i in $(seq 1 $N); do
  for v in base opt; do
    X=""; [ $v = opt ] && X="$OPT"
    timeout -k 10 300 python -u bench.py --no-cpu-baseline $X "$@" > $OUT/$v$i.json 2> $OUT/$v$i.err
    python3 -c "
import json; d=json.loads(open('$OUT/$v$i.json').read().strip().splitlines()[-1])
t=d.get('tpcc',{}); w=t.get('window_10000',{})
print('$v$i', round(d['ms_per_step'],4), round(d['value']/1e6,2), 'kern', round(d.get('kernel_us_per_epoch',0),1),
      'tpcc', [round(t.get(c,{}).get('ms_per_epoch',0),4) for c in ('WAIT_DIE','CALVIN')],
      'win', [round(w.get(c,{}).get('ms_per_epoch',0),4) for c in ('WAIT_DIE','CALVIN')])"
  done
done
