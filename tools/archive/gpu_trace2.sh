#!/bin/bash
# Kernel traces of the config-D bench (N=1) and of its epoch-group leg on a
# one-rank communicator.   tools/gpu_trace2.sh <tag>
set -e
OUT=gpurun_out/${1:-trace}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -T -d $OUT/kt -o run -- python3 bench.py --steps 5 --warmup 2 \
    --epochs 2 --no-cpu-baseline --no-tpcc > $OUT/kt_bench.json 2> $OUT/kt.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -T -d $OUT/ktg -o run -- python3 bench.py --part1 --no-weak \
    --mpr-sweep "" --steps 5 --warmup 2 --epochs 2 --no-cpu-baseline --no-tpcc > $OUT/ktg_bench.json 2> $OUT/ktg.err
