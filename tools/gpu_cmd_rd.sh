set -e
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03_rd; mkdir -p $OUT
timeout -k 10 900 python -u bench.py --gpus 2 --ipc-rehearsal --steps 8 --warmup 2 --no-cpu-baseline > $OUT/rehearsal.json 2> $OUT/rehearsal.err || { echo "rc=$?"; tail -30 $OUT/rehearsal.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/rehearsal.json').read().strip().splitlines()[-1])
print({k: (v if not isinstance(v, dict) else {a: b for a, b in v.items() if not isinstance(b, (dict, list))}) for k, v in d.items() if k in ('n_gpus','value','ms_per_step','scaling','extra_legs_error')}, d['config'].get('decision_lanes'))"
timeout -k 10 600 python -u bench.py --part1 --steps 20 --warmup 3 --no-cpu-baseline --no-tpcc --mpr-sweep "" > $OUT/part1.json 2> $OUT/part1.err || { echo "rc=$?"; tail -30 $OUT/part1.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/part1.json').read().strip().splitlines()[-1])
print(d['ms_per_step'], d['value'], d['config'].get('decision_lanes'))"
