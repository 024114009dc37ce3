set -e
export PYTHONUNBUFFERED=1
T=${1:-r05_f}
mkdir -p gpurun_out/$T
bash tools/gpu.sh tests $T
bash tools/lib_ab.sh $T 3 "nolist cur"
