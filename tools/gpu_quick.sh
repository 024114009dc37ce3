set -e
TAG=${1:-r02}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { tail -40 gpurun_out/$TAG/pytest.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
cat gpurun_out/$TAG/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -T -d gpurun_out/$TAG/kt -o run -- python3 bench.py --steps 5 --warmup 2 --epochs 2 --no-cpu-baseline > gpurun_out/$TAG/kt_bench.json 2>gpurun_out/$TAG/kt.err
