set -e
export PYTHONUNBUFFERED=1
T=${1:-r05_l}
mkdir -p gpurun_out/$T
bash tools/gpu.sh tests $T
bash tools/gpu.sh bench $T --steps 20 --warmup 5
python3 -c "import json; d=json.load(open('gpurun_out/$T/bench_detail.json')); print({k: (d[k]['ms_per_epoch'], d[k]['committed_per_s']) for k in ('config_b','config_c')}); t=d['tpcc']; print({k:(v['ms_per_epoch']) for k,v in t.items() if isinstance(v,dict) and 'ms_per_epoch' in v}, {k:{c:x['ms_per_epoch'] for c,x in v.items() if isinstance(x,dict)} for k,v in t.items() if k.startswith('window')})"
