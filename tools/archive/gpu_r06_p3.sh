set -e
# group-path launch folding: the group / partitioned / IPC tests, then part1
bash tools/gpu.sh tests r06_p3 tests/test_partitioned.py tests/test_ipc.py tests/test_tpcc_gpu.py
A="--part1 --steps 40 --warmup 5 --no-cpu-baseline --no-configs --no-tpcc --no-tpcc-part --mpr-sweep= --no-weak"
bash tools/gpu.sh bench r06_p3 $A
cp gpurun_out/r06_p3/bench.json gpurun_out/r06_p3/part1_a.json
bash tools/gpu.sh bench r06_p3 $A
cp gpurun_out/r06_p3/bench.json gpurun_out/r06_p3/part1_b.json
