#!/bin/bash
# A/B timing of the default bench under two environments, alternated:
#   tools/ab.sh <tag> "<env A>" "<env B>" [rounds] [bench args...]
set -e
OUT=gpurun_out/$1; A=$2; B=$3; N=${4:-3}; shift 4 || shift $#
mkdir -p $OUT
for i in $(seq 1 $N); do
  for v in A B; do
    E=$A; [ $v = B ] && E=$B
    env $E timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-tpcc --steps 20 "$@" > $OUT/$v$i.json 2> $OUT/$v$i.err
    python3 -c "import json,sys; d=json.loads(open('$OUT/$v$i.json').read().strip().splitlines()[-1]); print('$v', round(d['ms_per_step'],4), round(d['value']/1e6,2), round(d['stage_ms_mean']['ms_total'],4))"
  done
done
