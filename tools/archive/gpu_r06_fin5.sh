#!/bin/bash
# round 6 final (deferred decider counters in): the whole GPU suite and smoke,
# the driver's bench line, rocprofv3 kernel stats and the PMC passes; then a
# 100-step --part1 A/B of the group path without / with the deferred read
set -e
bash tools/gpu.sh tests r06_fin5
bash tools/gpu.sh bench r06_fin5 --steps 20 --warmup 5
bash tools/gpu.sh prof r06_fin5 --steps 20 --warmup 5 --no-cpu-baseline --no-configs --no-tpcc
bash tools/gpu.sh pmc r06_fin5 k_round_async,k_probe_tb,k_kill,k_kill_emit,k_kill_count,k_bucket_sort,k_radix_scatter,k_radix_hist,k_radix_scan,k_round_pass,k_round_settle,k_exec_txn,k_prefix_mark,k_epoch_clear,k_sub_scatter_back,k_lane_wait,k_lane_post --steps 10 --warmup 3 --no-cpu-baseline --no-configs --no-tpcc
O=gpurun_out/r06_fin5/ab
mkdir -p $O
for i in 1 2; do
  for v in nodefer defer; do
    DVCC_LIB=$PWD/exp_build/$v/libdvcc.so timeout -k 10 240 python -u bench.py --part1 --steps 100 --warmup 5 \
        --no-cpu-baseline --no-configs --no-tpcc --no-tpcc-part --mpr-sweep= --no-weak \
        --detail-out $O/$v$i.detail.json > $O/$v$i.json 2> $O/$v$i.err
    python3 -c "import json; d=json.load(open('$O/$v$i.detail.json')); print('$v', d['ms_per_step'], d['kernel_us_per_epoch'])"
  done
done
