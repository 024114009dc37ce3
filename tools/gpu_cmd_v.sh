set -e
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03_v; mkdir -p $OUT
for V in 0 1 2 3; do
DVCC_LANE_VARIANT=$V DVCC_DEBUG_LANES=1 timeout -k 10 300 python -u tools/exp_lanes.py 30 > $OUT/v$V.txt 2>&1 || { tail -20 $OUT/v$V.txt; exit 1; }
echo "variant $V halts $(grep -c 'lane halt' $OUT/v$V.txt || true)"
grep "^lanes" $OUT/v$V.txt
done
