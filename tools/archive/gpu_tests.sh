#!/bin/bash
# GPU-box session: the GPU parity suite and the smoke entry point only.
#   tools/gpu_tests.sh [tag] [pytest selection...]   (run from the repo root under gpurun)
set -e
TAG=${1:-r02}
shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
SEL=${@:-tests}
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -v --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
cat $OUT/smoke.log
