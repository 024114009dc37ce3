set -e
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03_t; mkdir -p $OUT
timeout -k 10 300 python -u tools/exp_lanes.py 20 > $OUT/lanes_torch.txt 2>&1 || { tail -20 $OUT/lanes_torch.txt; exit 1; }
grep lanes $OUT/lanes_torch.txt
timeout -k 10 300 python -u tools/exp_lanes.py 20 own > $OUT/lanes_own.txt 2>&1 || { tail -20 $OUT/lanes_own.txt; exit 1; }
grep lanes $OUT/lanes_own.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o kt -- python3 -u tools/exp_lanes.py 6 own > $OUT/prof.txt 2>&1 || { tail -20 $OUT/prof.txt; exit 1; }
find $OUT/kt -name "*.csv" | head
