set -e
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03_m; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_tpcc_gpu.py tests/test_partitioned.py tests/test_ipc.py tests/test_host_cpp.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/t1.log 2>&1 || { tail -40 $OUT/t1.log; exit 1; }
tail -2 $OUT/t1.log
timeout -k 10 300 python -u bench.py --tpcc-only --no-cpu-baseline > $OUT/tpcc.json 2> $OUT/tpcc.err
python3 -c "
import json; d=json.loads(open('$OUT/tpcc.json').read().strip().splitlines()[-1]); t=d.get('tpcc',d); w=t['window_10000']
print('65K', [round(t[c]['ms_per_epoch'],4) for c in ('WAIT_DIE','CALVIN')], 'win', [round(w[c]['ms_per_epoch'],4) for c in ('WAIT_DIE','CALVIN')])"
