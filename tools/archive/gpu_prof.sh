#!/bin/bash
# Profiles for one tag: rocprofv3 kernel-trace summary of the config-D bench
# command, separate FETCH_SIZE / WRITE_SIZE passes reduced to per-launch
# traffic of the epoch's kernels (2 x FETCH_SIZE + WRITE_SIZE, the guide's
# gfx950 correction),
# the kernel trace of the TPC-C leg, and the default bench line.
#   tools/gpu_prof.sh <tag>
set -e
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
# (one context: per-kernel attribution and PMC; the two-lane timed path gets
# its own kernel trace below)
B="bench.py --steps 5 --warmup 2 --epochs 2 --no-cpu-baseline --no-tpcc --lanes 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -T -d $OUT/kt -o run -- python3 $B \
    > $OUT/kt_bench.json 2> $OUT/kt.err
KT=$(find $OUT/kt -name 'run_kernel_trace.csv' | head -1)
python3 tools/ktrace.py $KT --epoch 5 > $OUT/timeline.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -T -d $OUT/kt_lanes -o run -- python3 \
    bench.py --steps 5 --warmup 2 --epochs 2 --no-cpu-baseline --no-tpcc --lanes 2 > $OUT/kt_lanes.json 2> $OUT/kt_lanes.err
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C -f csv -T -d $OUT/pmc_$C -o run -- python3 $B \
      > $OUT/pmc_$C.json 2> $OUT/pmc_$C.err
done
SRC=$(python3 -c "import sys; sys.path.insert(0, 'deneva-plus_amd'); from dvcc import _lib; print(_lib.source_hash())")
python3 tools/pmc_summary.py $OUT/pmc_FETCH_SIZE/run_counter_collection.csv \
    $OUT/pmc_WRITE_SIZE/run_counter_collection.csv $OUT/pmc_config_d.json \
    k_probe,k_round_pass,k_round_settle,k_round_async,k_round_finalize,k_radix_hist,k_radix_scan,k_radix_scatter,k_bucket_sort,k_prefix_mark,k_kill,k_kill_count,k_kill_emit,k_sub_scatter_back,k_exec_txn,k_epoch_clear \
    config=D cc=NO_WAIT n_gpus=1 src_hash=$SRC
T="bench.py --tpcc-only --steps 5 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -T -d $OUT/kt_tpcc -o run -- python3 $T \
    > $OUT/kt_tpcc.json 2> $OUT/kt_tpcc.err
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
