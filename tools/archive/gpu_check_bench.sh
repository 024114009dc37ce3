#!/bin/bash
# GPU-box session: the GPU parity suite, smoke, then the default bench line.
#   tools/gpu_check_bench.sh <tag> [bench args...]
set -e
TAG=${1:-r03}; shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
tail -2 $OUT/smoke.log
timeout -k 10 400 python -u bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err
python3 tools/bench_brief.py $OUT/bench.json
