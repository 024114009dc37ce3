set -e
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03_cl; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_carry.py > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
timeout -k 10 600 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-tpcc > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
c=d['closed_loop_retry']; print(round(c['ms_per_epoch'],4), round(c['committed_per_s']/1e6,2), {k: (round(v,4) if isinstance(v,float) else v) for k,v in c['lanes'].items() if k != 'note'})"
