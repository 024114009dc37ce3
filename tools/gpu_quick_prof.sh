#!/bin/bash
# Quick kernel-time check of the config-D bench (no CPU baseline, no TPC-C).
#   tools/gpu_quick_prof.sh <tag>
set -e
OUT=gpurun_out/${1:-quick}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -T -d $OUT/kt -o run -- python3 bench.py --steps 5 --warmup 2 \
    --epochs 2 --no-cpu-baseline --no-tpcc > $OUT/kt_bench.json 2> $OUT/kt.err
timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline --no-tpcc > $OUT/bench.json 2> $OUT/bench.err
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('value',d['value'],'ms',d['ms_per_step'])"
head -12 $OUT/kt/run_kernel_stats.csv | cut -d, -f1-4
