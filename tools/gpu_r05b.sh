set -e
export PYTHONUNBUFFERED=1
T=${1:-r05_g}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_carry.py tests/test_golden.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { tail -40 gpurun_out/$T/pytest.log; exit 1; }
tail -2 gpurun_out/$T/pytest.log
bash tools/gpu.sh bench $T --steps 20 --warmup 5
python3 -c "import json; d=json.load(open('gpurun_out/$T/bench_detail.json')); print({k: (d[k]['ms_per_epoch'], d[k]['committed_per_s']) for k in ('config_b','config_c')}); t=d['tpcc']; print({k:(v['ms_per_epoch']) for k,v in t.items() if isinstance(v,dict) and 'ms_per_epoch' in v}, {k:{c:x['ms_per_epoch'] for c,x in v.items() if isinstance(x,dict)} for k,v in t.items() if k.startswith('window')})"
