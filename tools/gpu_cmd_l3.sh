set -e
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03_l3; mkdir -p $OUT
for G in 100 90 75 60; do
EXP_NLANES=4 EXP_LSEQ=2,3,4,3,4 DVCC_LANE_GPCT=$G timeout -k 10 300 python -u tools/exp_lanes.py 30 > $OUT/g$G.txt 2>&1 || { tail -20 $OUT/g$G.txt; exit 1; }
echo "gpct $G"; grep "^lanes" $OUT/g$G.txt
done
