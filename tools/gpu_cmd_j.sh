set -e
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03_j; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_carry.py -m gpu -x -q --timeout 120 --timeout-method thread -k "prefix_kill or async or hand_scenario or ragged or randomized or many_rounds or medium or batch or carry" > $OUT/t1.log 2>&1 || { tail -40 $OUT/t1.log; exit 1; }
tail -2 $OUT/t1.log
bash tools/lib_ab.sh r03_j 3 "base new"
