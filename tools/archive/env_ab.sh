#!/bin/bash
# A/B of one environment switch on a bench command, alternated:
#   tools/env_ab.sh <tag> <rounds> <VAR=value> [bench args...]
# prints "<on|off> ms/step value(M)" per run, and the TPC-C legs when present
set -e
OUT=gpurun_out/$1; N=$2; KV=$3; shift 3
mkdir -p $OUT
for i in $(seq 1 $N); do
  for v in off on; do
    if [ $v == on ]; then E="env $KV"; else E=""; fi
    $E timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > $OUT/$v$i.json 2> $OUT/$v$i.err
    python3 - $OUT/$v$i.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
out = [sys.argv[2]]
if "value" in d:
    out += [round(d["ms_per_step"], 4), round(d["value"] / 1e6, 2)]
t = d.get("tpcc", {})
for size, leg in [("", t)] + [(k, v) for k, v in t.items() if k.startswith("window")]:
    for cc, x in leg.items():
        if isinstance(x, dict) and "ms_per_epoch" in x:
            out.append(f"{size or 'tpcc'}:{cc} {x['ms_per_epoch']:.4f}")
print(*out)
PY
  done
done
