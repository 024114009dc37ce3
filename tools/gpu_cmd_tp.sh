set -e
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03_tp; mkdir -p $OUT
for PL in 1 4; do
timeout -k 10 900 python -u bench.py --gpus 2 --ipc-rehearsal --steps 8 --warmup 2 --no-cpu-baseline --no-weak --mpr-sweep "" --part-lanes $PL > $OUT/rehearsal_pl$PL.json 2> $OUT/rehearsal_pl$PL.err || { echo "rc=$?"; tail -30 $OUT/rehearsal_pl$PL.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/rehearsal_pl$PL.json').read().strip().splitlines()[-1])
t=d.get('tpcc_partitioned', {}); print($PL, d.get('extra_legs_error'), t.get('decision_lanes'), {k: round(v['ms_per_epoch'],3) for k,v in t.items() if isinstance(v, dict) and 'ms_per_epoch' in v})"
done
