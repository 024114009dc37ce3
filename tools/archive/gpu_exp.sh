set -e
# experiment variants: tools/gpu_exp.sh <tag> <variant>...  (exp_build/<variant>/libdvcc.so)
T=gpurun_out/$1
shift
mkdir -p $T
for n in "$@"; do
  DVCC_LIB=$PWD/exp_build/$n/libdvcc.so timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --no-tpcc --steps 10 > $T/$n.json 2> $T/$n.err
  python3 -c "import json,sys; d=json.load(open('$T/$n.json')); print('$n', round(d['ms_per_step'],4), d['stage_ms_mean'])"
done
