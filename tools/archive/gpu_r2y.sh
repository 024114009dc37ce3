#!/bin/bash
# GPU suite, smoke, the default bench line and the N=1 partitioned legs.
#   tools/gpu_r2y.sh <tag>
set -e
TAG=${1:-r02_y}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-tpcc > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 200 python -u bench.py --part1 --no-weak --mpr-sweep "" --steps 10 > $OUT/group1.json 2> $OUT/group1.err
python3 - $OUT <<'PY'
import json, sys
for f in ("bench", "group1"):
    d = json.loads(open(f"{sys.argv[1]}/{f}.json").read().strip().splitlines()[-1])
    print(f, round(d["value"] / 1e6, 2), "M/s", round(d["ms_per_step"], 3), "ms", d["stage_ms_mean"], d.get("strong_scaling"))
PY
