# TPC-C legs and the headline, host profile (one box)
set -e
export PYTHONUNBUFFERED=1
T=${1:-r05_z}
O=gpurun_out/$T
mkdir -p $O
for rep in 1 2; do
  DVCC_HOST_PROF=1 timeout -k 10 300 python -u bench.py --tpcc-only --no-cpu-baseline > $O/t.$rep.json 2> $O/t.$rep.err || { tail -20 $O/t.$rep.err; exit 1; }
  python3 - $O/t.$rep.json <<'PY'
import json, sys
t = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])["tpcc"]
w = t.get("window_10000", {})
print("tpcc65k", {cc: round(t[cc]["ms_per_epoch"], 4) for cc in ("WAIT_DIE", "CALVIN") if cc in t},
      "window", {cc: round(w[cc]["ms_per_epoch"], 4) for cc in ("WAIT_DIE", "CALVIN") if cc in w})
PY
  grep "dvcc host" $O/t.$rep.err | tail -4
done
