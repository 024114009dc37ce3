#!/bin/bash
# experiment variants with per-kernel averages: tools/gpu_exp_k.sh <tag> <kernels,comma> <variant>...
set -e
T=gpurun_out/$1
K=$2
shift 2
mkdir -p $T
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for n in "$@"; do
  DVCC_LIB=$PWD/exp_build/$n/libdvcc.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -T -d $T/$n -o run \
      -- python3 bench.py --no-cpu-baseline --no-tpcc --steps 5 --warmup 2 --epochs 2 > $T/$n.json 2> $T/$n.err
  python3 - "$T/$n/run_kernel_stats.csv" "$K" "$n" <<'PY'
import csv, sys
rows = {r["Name"].split("(")[0].split("<")[0].split("::")[-1]: r for r in csv.DictReader(open(sys.argv[1]))}
print(sys.argv[3], {k: round(float(rows[k]["AverageNs"]) / 1e3, 1) for k in sys.argv[2].split(",") if k in rows})
PY
done
