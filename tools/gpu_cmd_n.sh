set -e
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03_n; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_carry.py tests/test_tpcc_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "prefix_kill or async or hand_scenario or ragged or randomized or many_rounds or medium or batch or carry or sorts_past or tpcc_epoch_parity or config_d" > $OUT/t1.log 2>&1 || { tail -40 $OUT/t1.log; exit 1; }
tail -2 $OUT/t1.log
bash tools/lib_ab.sh r03_n 2 "base new"
for f in base1 new1 base2 new2; do python3 -c "
import json; d=json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1])
k={r['kernel']:r for r in d['kernels']}
print('$f', round(d['kernel_us_per_epoch'],1), 'async', round(k['k_round_async']['avg_us'],1), 'ltail', round(k.get('k_round_ltail',{}).get('avg_us',0),1), 'rounds', d['rounds_mean'], 'yields', d['async_tries'])"; done
