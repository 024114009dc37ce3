#!/bin/bash
# Profiles for one tag: rocprofv3 kernel-trace summary of the config-D bench
# command (the line's roofline kernel), separate FETCH_SIZE / WRITE_SIZE passes
# reduced to per-launch traffic of k_round_pass, the same for the TPC-C leg,
# and the default bench line.
#   tools/gpu_prof.sh <tag>
set -e
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
B="bench.py --steps 5 --warmup 2 --epochs 2 --no-cpu-baseline --no-tpcc"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -T -d $OUT/kt -o run -- python3 $B \
    > $OUT/kt_bench.json 2> $OUT/kt.err
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C -f csv -T -d $OUT/pmc_$C -o run -- python3 $B \
      > $OUT/pmc_$C.json 2> $OUT/pmc_$C.err
done
python3 tools/pmc_summary.py $OUT/pmc_FETCH_SIZE/run_counter_collection.csv \
    $OUT/pmc_WRITE_SIZE/run_counter_collection.csv k_round_pass $OUT/pmc_round_pass.json \
    config=D cc=NO_WAIT n_gpus=1
mkdir -p profiles && cp $OUT/pmc_round_pass.json profiles/pmc_round_pass.json
T="bench.py --tpcc-only --steps 5 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -T -d $OUT/kt_tpcc -o run -- python3 $T \
    > $OUT/kt_tpcc.json 2> $OUT/kt_tpcc.err
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
