set -e
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03_u; mkdir -p $OUT
DVCC_DEBUG_LANES=1 timeout -k 10 300 python -u tools/exp_lanes.py 20 > $OUT/lanes_torch.txt 2>&1 || { tail -20 $OUT/lanes_torch.txt; exit 1; }
grep -c "lane halt" $OUT/lanes_torch.txt || true
grep "lane halt" $OUT/lanes_torch.txt | head -20 || true
grep "^lanes" $OUT/lanes_torch.txt
