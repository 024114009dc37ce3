set -e
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r03_q; mkdir -p $OUT
timeout -k 10 300 python -u tools/exp_two_lanes.py 20 > $OUT/two_lanes.txt 2>&1 || { tail -20 $OUT/two_lanes.txt; exit 1; }
tail -3 $OUT/two_lanes.txt
bash tools/gpu_prefix_sweep.sh r03_ps 16384 24576 32768 49152 65536 32768
