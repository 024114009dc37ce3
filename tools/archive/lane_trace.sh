set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r04_lt
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -T -d gpurun_out/r04_lt/kt -o run -- python3 bench.py --steps 40 --no-cpu-baseline --no-configs --no-tpcc > gpurun_out/r04_lt/b.json 2> gpurun_out/r04_lt/b.err
f=$(find gpurun_out/r04_lt/kt -name 'run_kernel_trace.csv' | head -1)
python3 tools/lane_gaps.py $f > gpurun_out/r04_lt/lane_gaps.txt
cat gpurun_out/r04_lt/lane_gaps.txt
