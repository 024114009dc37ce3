set -e
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03_o; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_tpcc_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "bucket or lsd_sort or sorts_past or prefix_kill or hand_scenario or ragged or randomized or tpcc_epoch_parity or config_b or medium" > $OUT/t1.log 2>&1 || { tail -40 $OUT/t1.log; exit 1; }
tail -2 $OUT/t1.log
for i in 1 2; do for v in base new; do
  DVCC_LIB=$PWD/exp_build/$v/libdvcc.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --tpcc-txns 65536,10000 > $OUT/$v$i.json 2> $OUT/$v$i.err
  python3 -c "
import json; d=json.loads(open('$OUT/$v$i.json').read().strip().splitlines()[-1])
k={r['kernel']:r for r in d['kernels']}; t=d['tpcc']; w=t['window_10000']
print('$v$i', round(d['ms_per_step'],4), 'kern', round(d['kernel_us_per_epoch'],1), 'bucket', round(k['k_bucket_sort']['avg_us'],1), 'scatter', round(k['k_radix_scatter']['avg_us'],1), 'tpcc', [round(t[c]['ms_per_epoch'],4) for c in ('WAIT_DIE','CALVIN')], 'win', [round(w[c]['ms_per_epoch'],4) for c in ('WAIT_DIE','CALVIN')])"
done; done
