set -e
# deferred decider counters: the new asynchronous-decider group test first, then the group suites and part1
bash tools/gpu.sh tests r06_p5a tests/test_partitioned.py -k asynchronous_deciders
bash tools/gpu.sh tests r06_p5 tests/test_partitioned.py tests/test_ipc.py tests/test_tpcc_gpu.py
A="--part1 --steps 40 --warmup 5 --no-cpu-baseline --no-configs --no-tpcc --no-tpcc-part --mpr-sweep= --no-weak"
bash tools/gpu.sh bench r06_p5 $A
cp gpurun_out/r06_p5/bench.json gpurun_out/r06_p5/part1_a.json
bash tools/gpu.sh bench r06_p5 $A --steps 100
cp gpurun_out/r06_p5/bench.json gpurun_out/r06_p5/part1_b.json
