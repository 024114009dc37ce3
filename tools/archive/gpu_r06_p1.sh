set -e
A="--part1 --steps 40 --warmup 5 --no-cpu-baseline --no-configs --no-tpcc --no-tpcc-part --mpr-sweep= --no-weak"
bash tools/gpu.sh bench r06_p1 $A
cp gpurun_out/r06_p1/bench.json gpurun_out/r06_p1/part1_L4.json
cp gpurun_out/r06_p1/bench_detail.json gpurun_out/r06_p1/part1_L4.detail.json
bash tools/gpu.sh bench r06_p1 $A --group-lanes 1
cp gpurun_out/r06_p1/bench.json gpurun_out/r06_p1/part1_L1.json
cp gpurun_out/r06_p1/bench_detail.json gpurun_out/r06_p1/part1_L1.detail.json
bash tools/gpu.sh prof r06_p1 $A --group-lanes 1
