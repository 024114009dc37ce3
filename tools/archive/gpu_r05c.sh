# TPC-C legs, A/B of exp_build/base against the in-tree library: probe kernel time (rocprofv3 stats) and the legs
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${1:-r05_al}
O=gpurun_out/$T
mkdir -p $O
for v in base cur; do
  lp=""; [ $v != cur ] && lp=$PWD/exp_build/$v/libdvcc.so
  DVCC_LIB=$lp timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/kt_$v -o run -- python3 bench.py --tpcc-only --no-cpu-baseline \
      > $O/kt_$v.json 2> $O/kt_$v.err || { tail -20 $O/kt_$v.err; exit 1; }
  f=$(find $O/kt_$v -name 'run_kernel_stats.csv' | head -1)
  grep -E '"k_probe"|"k_round_async"|"k_tpcc_apply"' $f | cut -d, -f1-4 | sed "s/^/$v /"
  rm -f $(find $O/kt_$v -name 'run_kernel_trace.csv')
done
for i in 1 2 3; do
  for v in base cur; do
    lp=""; [ $v != cur ] && lp=$PWD/exp_build/$v/libdvcc.so
    DVCC_LIB=$lp timeout -k 10 300 python -u bench.py --tpcc-only --no-cpu-baseline > $O/t$v$i.json 2> $O/t$v$i.err || { tail -20 $O/t$v$i.err; exit 1; }
    python3 - $O/t$v$i.json $v <<'PY'
import json, sys
t = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])["tpcc"]
w = t.get("window_10000", {})
print(sys.argv[2], "tpcc65k", {cc: round(t[cc]["ms_per_epoch"], 4) for cc in ("WAIT_DIE", "CALVIN") if cc in t},
      "window", {cc: round(w[cc]["ms_per_epoch"], 4) for cc in ("WAIT_DIE", "CALVIN") if cc in w})
PY
  done
done
