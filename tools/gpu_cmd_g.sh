set -e
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03_g; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "bucket or lsd_sort or sorts_past or prefix_kill or hand_scenario or ragged or randomized" > $OUT/t1.log 2>&1 || { tail -40 $OUT/t1.log; exit 1; }
tail -2 $OUT/t1.log
bash tools/gpu_ab_flag.sh r03_g 2 "--lsd-sort"
python3 tools/bench_brief.py $OUT/base2.json
