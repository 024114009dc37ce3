set -e
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03_p1; mkdir -p $OUT
for L in 1 4; do
timeout -k 10 600 python -u bench.py --part1 --steps 30 --warmup 3 --no-cpu-baseline --lanes $L --no-tpcc --mpr-sweep "" > $OUT/part1_l$L.json 2> $OUT/part1_l$L.err || { echo "rc=$?"; tail -30 $OUT/part1_l$L.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/part1_l$L.json').read().strip().splitlines()[-1])
print($L, {k: (v if not isinstance(v, dict) else {a: b for a, b in v.items() if not isinstance(b, (dict, list))}) for k, v in d.items() if k in ('n_gpus','value','ms_per_step','scaling','extra_legs_error')}, d['config'].get('decision_lanes'), d['config'].get('protocol')[:40])"
done
