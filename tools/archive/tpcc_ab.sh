#!/bin/bash
# A/B of exp_build libraries on the TPC-C leg (10,000-txn window; TXNS=... for another size), alternated.
#   tools/tpcc_ab.sh <tag> <rounds> "<libA> <libB> ..."
set -e
OUT=gpurun_out/$1; N=$2; LIBS=$3
mkdir -p $OUT
for i in $(seq 1 $N); do
  for v in $LIBS; do
    DVCC_LIB=$PWD/exp_build/$v/libdvcc.so timeout -k 10 300 python -u bench.py --tpcc-only --tpcc-txns ${TXNS:-10000} --steps 50 --no-cpu-baseline > $OUT/t$v$i.json 2> $OUT/t$v$i.err
    python3 -c "import json; d=json.loads(open('$OUT/t$v$i.json').read().strip().splitlines()[-1])['tpcc']; print('$v', {k: round(d[k]['ms_per_epoch'],4) for k in ('WAIT_DIE','CALVIN')})"
  done
done
