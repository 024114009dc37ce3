# epoch groups over ordered lanes at one rank (--part1): event order vs the order dropped (experiment: timing only)
set -e
export PYTHONUNBUFFERED=1
T=${1:-r05_ab}
O=gpurun_out/$T
mkdir -p $O
for rep in 1 2; do
for X in 0 1; do
  if [ $X = 1 ]; then export DVCC_EXP_NO_ORDER=1; else unset DVCC_EXP_NO_ORDER; fi
  timeout -k 10 300 python -u bench.py --part1 --no-cpu-baseline --no-tpcc --no-configs --steps 20 --warmup 5 \
      --detail-out $O/x$X.$rep.detail.json > $O/x$X.$rep.json 2> $O/x$X.$rep.err || { tail -20 $O/x$X.$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/x$X.$rep.detail.json')); print('no_order $X', d['ms_per_step'], d.get('config', {}).get('parallelism'))"
done
done
