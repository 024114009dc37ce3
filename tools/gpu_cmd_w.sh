set -e
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03_w; mkdir -p $OUT
for V in "0 0" "1 0" "3 0" "0 1" "1 1" "0 2" "1 2"; do
set -- $V
DVCC_LANE_VARIANT=$1 DVCC_LANE_CUMASK=$2 DVCC_DEBUG_LANES=1 timeout -k 10 300 python -u tools/exp_lanes.py 30 > $OUT/v$1_$2.txt 2>&1 || { tail -20 $OUT/v$1_$2.txt; exit 1; }
echo "variant $1 cumask $2 halts $(grep -c 'lane halt' $OUT/v$1_$2.txt || true)"
grep "^lanes" $OUT/v$1_$2.txt
done
