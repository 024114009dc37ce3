# A/B of exp_build/base (HEAD) against the in-tree library, alternated on one
# box: the headline, the TPC-C legs (65,536 and the 10,000-txn window), config B
set -e
export PYTHONUNBUFFERED=1
T=${1:-r05_u}; N=${2:-3}
O=gpurun_out/$T
mkdir -p $O
for i in $(seq 1 $N); do
  for v in base cur; do
    lp=""; [ $v != cur ] && lp=$PWD/exp_build/$v/libdvcc.so
    DVCC_LIB=$lp timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-tpcc --detail-out $O/$v$i.detail.json \
        --steps 20 --warmup 5 > $O/$v$i.json 2> $O/$v$i.err || { tail -20 $O/$v$i.err; exit 1; }
    DVCC_LIB=$lp timeout -k 10 300 python -u bench.py --tpcc-only --no-cpu-baseline --detail-out $O/t$v$i.detail.json \
        > $O/t$v$i.json 2> $O/t$v$i.err || { tail -20 $O/t$v$i.err; exit 1; }
    python3 - $O $v $i <<'PY'
import json, sys
o, v, i = sys.argv[1:]
d = json.load(open(f"{o}/{v}{i}.detail.json"))
t = json.loads(open(f"{o}/t{v}{i}.json").read().strip().splitlines()[-1])
t = t.get("tpcc", t)
w = t.get("window_10000", {})
print(v, i, "D", round(d["ms_per_step"], 4), "B", round(d["config_b"]["ms_per_epoch"], 4),
      "C", round(d["config_c"].get("ms_per_epoch", 0), 4),
      "tpcc65k", {cc: round(t[cc]["ms_per_epoch"], 4) for cc in ("WAIT_DIE", "CALVIN") if cc in t},
      "window", {cc: round(w[cc]["ms_per_epoch"], 4) for cc in ("WAIT_DIE", "CALVIN") if cc in w})
PY
  done
done
