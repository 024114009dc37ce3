set -e
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03_k; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
B="bench.py --steps 5 --warmup 2 --epochs 2 --no-cpu-baseline --no-tpcc"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -T -d $OUT/kt -o run -- python3 $B > $OUT/kt_bench.json 2> $OUT/kt.err
KT=$(find $OUT/kt -name 'run_kernel_trace.csv' | head -1)
python3 tools/ktrace.py $KT --epoch 5 > $OUT/timeline.txt
sed -n '/epoch 5 timeline/,$p' $OUT/timeline.txt
