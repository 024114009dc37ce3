#!/bin/bash
# TPC-C evidence: GPU parity tests, the bench line (with its TPC-C leg) and a
# rocprofv3 kernel-trace summary of the same bench command.
#   tools/gpu_tpcc.sh <tag>
set -e
TAG=${1:-tpcc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_tpcc_gpu.py -x -q --timeout 120 --timeout-method thread \
    > $OUT/pytest_tpcc.log 2>&1 || { tail -30 $OUT/pytest_tpcc.log; exit 1; }
tail -1 $OUT/pytest_tpcc.log
timeout -k 10 300 python -u bench.py --steps 10 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'], json.dumps(d.get('tpcc')))"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -T -d $OUT/kt -o run -- python3 bench.py --steps 5 --warmup 2 \
    --epochs 2 --no-cpu-baseline > $OUT/kt_bench.json 2> $OUT/kt.err
head -30 $OUT/kt/run_kernel_stats.csv | cut -d, -f1-8
