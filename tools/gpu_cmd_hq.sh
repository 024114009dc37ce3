set -e
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03_hq; mkdir -p $OUT
for Q in 4 8 16; do
GPU_MAX_HW_QUEUES=$Q EXP_NLANES=8 EXP_LSEQ=1,2,4,8,4,8 DVCC_LANE_GPCT=75 timeout -k 10 300 python -u tools/exp_lanes.py 40 > $OUT/q$Q.txt 2>&1 || { tail -20 $OUT/q$Q.txt; exit 1; }
echo "hw queues $Q"; grep "^lanes" $OUT/q$Q.txt
done
