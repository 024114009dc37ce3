set -e
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03_r; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "lane or batch" > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 1; }
tail -3 $OUT/pytest.txt
for L in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --lanes $L --no-cpu-baseline --no-tpcc > $OUT/bench_l$L.json 2> $OUT/bench_l$L.err || { tail -20 $OUT/bench_l$L.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/bench_l$L.json').read().strip().splitlines()[-1]); print($L, d['ms_per_step'], d['value'])"
done
