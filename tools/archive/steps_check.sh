#!/bin/bash
# default bench line vs longer timed regions (the same build), per-step ms
set -e
OUT=gpurun_out/${1:-steps}; mkdir -p $OUT
for a in "--steps 10" "--steps 20" "--steps 10" "--steps 10 --warmup 4" "--steps 40" "--steps 10"; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-tpcc $a > $OUT/b.json 2> $OUT/b.err
  python3 -c "import json; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('$a', round(d['ms_per_step'],4), round(d['value']/1e6,2), d['distinct_epochs'] if 'distinct_epochs' in d else d['config']['distinct_epochs'])"
done
