set -e
export PYTHONUNBUFFERED=1
bash tools/lib_ab.sh r03_sl4 3 "sl8 sl20 sl48" --steps 100 --warmup 5 --lanes 4
bash tools/lib_ab.sh r03_sl1 2 "sl8 sl20 sl48" --steps 100 --warmup 5 --lanes 1
