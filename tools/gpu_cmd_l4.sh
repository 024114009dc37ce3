set -e
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03_l4; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_tpcc_gpu.py -k "lane or batch" > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
grep lanes $OUT/smoke.log
for L in 1 2 4; do
  timeout -k 10 300 python -u bench.py --steps 200 --warmup 10 --lanes $L --no-cpu-baseline --no-tpcc > $OUT/bench_l$L.json 2> $OUT/bench_l$L.err || { tail -20 $OUT/bench_l$L.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/bench_l$L.json').read().strip().splitlines()[-1]); print($L, d['ms_per_step'], d['value'])"
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -20 $OUT/bench_default.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/bench_default.json').read().strip().splitlines()[-1]); print('default', d['ms_per_step'], d['value'])
t=d['tpcc']; print({k: round(v['ms_per_epoch'],4) for k,v in t.items() if isinstance(v, dict) and 'ms_per_epoch' in v}, {k: round(v['ms_per_epoch'],4) for k,v in t['window_10000'].items() if isinstance(v, dict) and 'ms_per_epoch' in v})"
