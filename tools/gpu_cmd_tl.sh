set -e
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03_tl; mkdir -p $OUT
for L in 1 2 4 2 4; do
  timeout -k 10 300 python -u bench.py --steps 50 --warmup 5 --lanes $L --tpcc-only > $OUT/tpcc_l$L.json 2> $OUT/tpcc_l$L.err || { tail -20 $OUT/tpcc_l$L.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/tpcc_l$L.json').read().strip().splitlines()[-1])['tpcc']
print($L, {k: round(v['ms_per_epoch'],4) for k,v in d.items() if isinstance(v, dict) and 'ms_per_epoch' in v}, {k: round(v['ms_per_epoch'],4) for k,v in d['window_10000'].items() if isinstance(v, dict) and 'ms_per_epoch' in v})"
done
