#!/bin/bash
# Full GPU evidence for one tag: parity tests, smoke, the default bench line,
# a rocprofv3 kernel-trace summary of the same bench command, and separate
# FETCH_SIZE / WRITE_SIZE passes reduced to per-launch traffic of k_round_pass.
#   tools/gpu_round.sh <tag>
set -e
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
tail -4 $OUT/smoke.log
B="bench.py --steps 5 --warmup 2 --epochs 2 --no-cpu-baseline"
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
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
