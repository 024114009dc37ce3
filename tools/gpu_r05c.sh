# epoch groups at one rank (--part1), A/B of exp_build/base against the in-tree library, alternated
set -e
export PYTHONUNBUFFERED=1
T=${1:-r05_ae}; N=${2:-3}
O=gpurun_out/$T
mkdir -p $O
for i in $(seq 1 $N); do
  for v in base cur; do
    lp=""; [ $v != cur ] && lp=$PWD/exp_build/$v/libdvcc.so
    DVCC_LIB=$lp timeout -k 10 300 python -u bench.py --part1 --no-cpu-baseline --no-tpcc --no-configs --steps 20 --warmup 5 \
        --detail-out $O/$v$i.detail.json > $O/$v$i.json 2> $O/$v$i.err || { tail -20 $O/$v$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$v$i.detail.json')); print('$v $i', round(d['ms_per_step'],4), [(k['kernel'], round(k['avg_us'],1)) for k in d['kernels'] if k['kernel'].startswith('k_group')])"
  done
done
