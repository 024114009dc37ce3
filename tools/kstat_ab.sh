#!/bin/bash
# Per-kernel averages of exp_build libraries (rocprofv3 kernel stats of a
# short config-D bench each), for the kernels named.
#   tools/kstat_ab.sh <tag> "<libA> <libB> ..." "<kernel,kernel,...>"
set -e
OUT=gpurun_out/$1; LIBS=$2; KS=$3
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in $LIBS; do
  DVCC_LIB=$PWD/exp_build/$v/libdvcc.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/$v -o run \
      -- python3 bench.py --steps 10 --warmup 2 --epochs 2 --no-cpu-baseline --no-tpcc > $OUT/$v.json 2> $OUT/$v.err
  python3 - "$OUT/$v/run_kernel_stats.csv" "$KS" "$v" <<'PY'
import csv, sys
want = sys.argv[2].split(",")
rows = {r["Name"]: r for r in csv.DictReader(open(sys.argv[1]))}
print(sys.argv[3], " ".join(f"{k}={float(rows[k]['AverageNs'])/1000:.1f}" for k in want if k in rows))
PY
done
