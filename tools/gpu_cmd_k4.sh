set -e
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03_k4; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
EXP_NLANES=4 EXP_LSEQ=1,4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/kt -o run -- python3 -u tools/exp_lanes.py 40 > $OUT/lanes.txt 2>&1 || { tail -20 $OUT/lanes.txt; exit 1; }
grep "^lanes" $OUT/lanes.txt
python3 tools/kt_overlap.py $(find $OUT/kt -name 'run_kernel_trace.csv' | head -1) > $OUT/overlap.txt
cat $OUT/overlap.txt
