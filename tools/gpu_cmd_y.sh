set -e
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03_y; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_tpcc_gpu.py -k "lane or batch" > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
for L in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 50 --warmup 5 --lanes $L --tpcc-only > $OUT/tpcc_l$L.json 2> $OUT/tpcc_l$L.err || { tail -20 $OUT/tpcc_l$L.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/tpcc_l$L.json').read().strip().splitlines()[-1])['tpcc']
print($L, {k: round(v['ms_per_epoch'],4) for k,v in d.items() if isinstance(v, dict) and 'ms_per_epoch' in v}, {w: {k: round(v['ms_per_epoch'],4) for k,v in d[w].items() if isinstance(v, dict) and 'ms_per_epoch' in v} for w in d if w.startswith('window')})"
done
