set -e
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03_mv; mkdir -p $OUT
for R in 1 2; do
for V in 0 1 2 3 4; do
DVCC_MASK_V=$V EXP_NLANES=4 EXP_LSEQ=4,2 timeout -k 10 300 python -u tools/exp_lanes.py 60 > $OUT/v$V.txt 2>&1 || { tail -20 $OUT/v$V.txt; exit 1; }
echo "mask $V: $(grep '^lanes' $OUT/v$V.txt | tr '\n' ' ')"
done
done
