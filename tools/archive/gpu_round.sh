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
bash tools/gpu_prof.sh $TAG
