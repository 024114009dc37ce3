set -e
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03_i; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_tpcc_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "bucket or lsd_sort or sorts_past or prefix_kill or hand_scenario or ragged or randomized or config_e or small" > $OUT/t1.log 2>&1 || { tail -40 $OUT/t1.log; exit 1; }
tail -2 $OUT/t1.log
timeout -k 10 200 python -u tools/exp_rounds.py > $OUT/rounds.txt 2>&1; cat $OUT/rounds.txt
bash tools/gpu_ab_flag.sh r03_i 2 "--lsd-sort"
python3 tools/bench_brief.py $OUT/base2.json
python3 -c "import json; d=json.loads(open('$OUT/base2.json').read().strip().splitlines()[-1]); print(d['stage_sizes_mean'])"
