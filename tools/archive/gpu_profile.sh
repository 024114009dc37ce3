#!/bin/bash
# rocprofv3 evidence for the bench line: kernel-trace stats, then separate
# PMC passes (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).
#   tools/gpu_profile.sh [tag] [extra bench args...]
set -e
TAG=${1:-r01}; shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
B="bench.py --steps 5 --warmup 2 --epochs 2 --no-cpu-baseline $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -T -d $OUT/kt -o run -- python3 $B \
    > $OUT/kt_bench.json 2> $OUT/kt.err
cat $OUT/kt_bench.json
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C -f csv -T -d $OUT/pmc_$C -o run -- python3 $B \
      > $OUT/pmc_$C.json 2> $OUT/pmc_$C.err
done
find $OUT -name '*.csv' | sort
