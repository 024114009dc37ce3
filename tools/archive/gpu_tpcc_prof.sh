#!/bin/bash
# TPC-C (config E share) kernel evidence at the bench's epoch size and at the
# reference's 10,000-txn window: kernel-trace summaries of the --tpcc-only
# leg, then separate FETCH_SIZE / WRITE_SIZE passes reduced to per-launch
# traffic of k_tpcc_apply at the window.
#   tools/gpu_tpcc_prof.sh <tag>
set -e
TAG=${1:-tpcc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
SRC=$(python3 -c "import sys; sys.path.insert(0, 'deneva-plus_amd'); from dvcc import _lib; print(_lib.source_hash())")
for N in 65536 10000; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -T -d $OUT/kt_$N -o run -- python3 bench.py --tpcc-only \
      --tpcc-txns $N --steps 10 --warmup 2 --no-cpu-baseline > $OUT/kt_$N.json 2> $OUT/kt_$N.err
  python3 tools/ktrace.py $OUT/kt_$N/run_kernel_trace.csv --start k_tpcc_resolve > $OUT/timeline_$N.txt 2>&1 || true
done
B="bench.py --tpcc-only --tpcc-txns 10000 --steps 10 --warmup 2 --no-cpu-baseline"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C -f csv -T -d $OUT/pmc_$C -o run -- python3 $B \
      > $OUT/pmc_$C.json 2> $OUT/pmc_$C.err
done
python3 tools/pmc_summary.py $OUT/pmc_FETCH_SIZE/run_counter_collection.csv \
    $OUT/pmc_WRITE_SIZE/run_counter_collection.csv $OUT/pmc_tpcc.json \
    k_tpcc_apply,k_tpcc_oid,k_tpcc_resolve,k_probe,k_round_pass,k_round_async \
    config=E n_txn=10000 n_gpus=1 src_hash=$SRC
timeout -k 10 300 python -u bench.py --tpcc-only --steps 10 > $OUT/bench_tpcc.json 2> $OUT/bench_tpcc.err
cat $OUT/bench_tpcc.json
