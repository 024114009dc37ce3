set -e
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03_ht; mkdir -p $OUT
DVCC_LANE_HOSTT=1 EXP_NLANES=4 EXP_LSEQ=2,4,2,4 timeout -k 10 300 python -u tools/exp_lanes.py 60 > $OUT/lanes.txt 2>&1 || { tail -20 $OUT/lanes.txt; exit 1; }
grep -E "^lanes" $OUT/lanes.txt
grep "lanes host" $OUT/lanes.txt | tail -4
