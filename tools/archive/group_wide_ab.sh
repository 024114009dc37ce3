#!/bin/bash
# Epoch groups on one GPU (one-rank RCCL): group parity tests, then the bench
# with compact (4 B) against wide (8 B, --part-mode 4) batches, alternated.
#   tools/group_wide_ab.sh <tag> <rounds>
set -e
OUT=gpurun_out/$1; N=$2
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_partitioned.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "group" > $OUT/pytest_group.log 2>&1 || { tail -40 $OUT/pytest_group.log; exit 1; }
tail -2 $OUT/pytest_group.log
ARGS="--part1 --protocol group --steps 20 --no-cpu-baseline --no-tpcc --no-weak --mpr-sweep="
for i in $(seq 1 $N); do
  for v in compact wide; do
    X=""; [ $v = wide ] && X="--part-mode 4"
    timeout -k 10 300 python -u bench.py $ARGS $X > $OUT/$v$i.json 2> $OUT/$v$i.err
    python3 -c "import json; d=json.loads(open('$OUT/$v$i.json').read().strip().splitlines()[-1]); print('$v', round(d['ms_per_step'],4), round(d['value']/1e6,2))"
  done
done
