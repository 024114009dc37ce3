# headline with the last T epochs of a call on unmasked streams (experiment), alternated
set -e
export PYTHONUNBUFFERED=1
T=${1:-r05_ao}
O=gpurun_out/$T
mkdir -p $O
for i in 1 2 3; do
for X in 0 1 2; do
  if [ $X = 0 ]; then unset DVCC_EXP_TAIL_SPREAD; else export DVCC_EXP_TAIL_SPREAD=$X; fi
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-tpcc --no-configs --steps 20 --warmup 5 \
      --detail-out $O/x$X.$i.detail.json > $O/x$X.$i.json 2> $O/x$X.$i.err || { tail -20 $O/x$X.$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/x$X.$i.detail.json')); print('tail $X', d['ms_per_step'], d.get('async_tries'))"
done
done
