set -e
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03_l8; mkdir -p $OUT
for G in 100 75; do
EXP_NLANES=8 EXP_LSEQ=1,2,4,6,8,4,8 DVCC_LANE_GPCT=$G timeout -k 10 300 python -u tools/exp_lanes.py 40 > $OUT/g$G.txt 2>&1 || { tail -20 $OUT/g$G.txt; exit 1; }
echo "gpct $G"; grep "^lanes" $OUT/g$G.txt
done
