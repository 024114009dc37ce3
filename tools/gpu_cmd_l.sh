set -e
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03_l; mkdir -p $OUT
for v in bx0 bx1 bx2; do
  DVCC_LIB=$PWD/exp_build/$v/libdvcc.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-tpcc --steps 5 > $OUT/$v.json 2> $OUT/$v.err || true
  python3 -c "
import json; d=json.loads(open('$OUT/$v.json').read().strip().splitlines()[-1])
k={r['kernel']:r for r in d['kernels']}
print('$v', round(d['ms_per_step'],4), 'bucket', round(k['k_bucket_sort']['avg_us'],1))" || true
done
