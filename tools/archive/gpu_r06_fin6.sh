#!/bin/bash
# round 6 final: the whole GPU suite and smoke, the driver's bench line, then
# rocprofv3 kernel stats and the FETCH_SIZE / WRITE_SIZE passes of the same
# bench for the roofline's traffic (tools/gpu.sh)
set -e
bash tools/gpu.sh tests r06_fin6
bash tools/gpu.sh bench r06_fin6 --steps 20 --warmup 5
bash tools/gpu.sh prof r06_fin6 --steps 20 --warmup 5 --no-cpu-baseline --no-configs --no-tpcc
bash tools/gpu.sh pmc r06_fin6 k_round_async,k_probe_tb,k_kill,k_kill_emit,k_kill_count,k_bucket_sort,k_radix_scatter,k_radix_hist,k_radix_scan,k_round_pass,k_round_settle,k_exec_txn,k_prefix_mark,k_epoch_clear,k_sub_scatter_back,k_lane_wait,k_lane_post --steps 10 --warmup 3 --no-cpu-baseline --no-configs --no-tpcc
