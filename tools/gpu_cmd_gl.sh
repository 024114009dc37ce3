set -e
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03_gl; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_partitioned.py -k "ordered_lanes or epoch_group_batch" > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
for L in 1 4; do
timeout -k 10 600 python -u bench.py --gpus 2 --ipc-rehearsal --steps 8 --warmup 2 --no-cpu-baseline --lanes $L --no-tpcc > $OUT/rehearsal_l$L.json 2> $OUT/rehearsal_l$L.err || { echo "rehearsal rc=$?"; tail -30 $OUT/rehearsal_l$L.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/rehearsal_l$L.json').read().strip().splitlines()[-1])
print($L, {k: (v if not isinstance(v, dict) else {a: b for a, b in v.items() if not isinstance(b, (dict, list))}) for k, v in d.items() if k in ('n_gpus','value','ms_per_step','scaling','extra_legs_error')}, d['config'].get('decision_lanes'))"
done
