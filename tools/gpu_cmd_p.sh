set -e
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03_p; mkdir -p $OUT
timeout -k 10 600 python -u bench.py --gpus 2 --ipc-rehearsal --steps 3 --warmup 1 --no-cpu-baseline --no-weak --mpr-sweep 0.5 > $OUT/rehearsal2.json 2> $OUT/rehearsal2.err || { echo "rehearsal rc=$?"; tail -30 $OUT/rehearsal2.err; exit 1; }
python3 tools/bench_brief.py $OUT/rehearsal2.json | head -8
python3 -c "
import json; d=json.loads(open('$OUT/rehearsal2.json').read().strip().splitlines()[-1])
print({k: (v if not isinstance(v, dict) else {a: b for a, b in v.items() if not isinstance(b, (dict, list))}) for k, v in d.items() if k in ('n_gpus','value','ms_per_step','scaling','strong_scaling','mpr_sweep','tpcc_partitioned','extra_legs_error')})"
