set -e
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03_b50; mkdir -p $OUT
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { tail -20 $OUT/bench_driver.err; exit 1; }
for f in bench bench_driver; do python3 -c "
import json; d=json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1])
print('$f', d['steps'], round(d['ms_per_step'],4), round(d['value']/1e6,1), d['roofline']['kernel'], round(d['roofline']['frac'],4), d['roofline']['traffic'])
t=d['tpcc']; print({k: round(v['ms_per_epoch'],4) for k,v in t.items() if isinstance(v, dict) and 'ms_per_epoch' in v}, {k: round(v['ms_per_epoch'],4) for k,v in t['window_10000'].items() if isinstance(v, dict) and 'ms_per_epoch' in v})"; done
