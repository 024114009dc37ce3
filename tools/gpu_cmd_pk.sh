set -e
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03_pk; mkdir -p $OUT
for K in 16384 24576 32768 49152 65536 32768; do
  timeout -k 10 300 python -u bench.py --steps 150 --warmup 10 --prefix $K --no-cpu-baseline --no-tpcc > $OUT/bench_$K.json 2> $OUT/bench_$K.err || { tail -20 $OUT/bench_$K.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/bench_$K.json').read().strip().splitlines()[-1]); print($K, round(d['ms_per_step'],4), round(d['value']/1e6,1))"
done
