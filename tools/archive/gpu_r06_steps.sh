#!/bin/bash
# the driver's 20-step headline against the 100-step steady state on one box, alternated
set -e
O=gpurun_out/r06_steps
mkdir -p $O
for i in 1 2; do
  for n in 20 100; do
    timeout -k 10 300 python -u bench.py --steps $n --warmup 5 --no-cpu-baseline --no-configs --no-tpcc \
        --detail-out $O/s$n.$i.detail.json > $O/s$n.$i.json 2> $O/s$n.$i.err
    python3 -c "import json; d=json.load(open('$O/s$n.$i.detail.json')); print($n, d['ms_per_step'])"
  done
done
