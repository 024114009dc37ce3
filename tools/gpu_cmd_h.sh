set -e
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03_h; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
bash tools/gpu_ab_flag.sh r03_h 2 "--lsd-sort"
python3 tools/bench_brief.py $OUT/base2.json
