set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r06_d
timeout -k 10 900 python -u -m pytest tests/test_carry.py -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r06_d/pytest_carry.log 2>&1 || { tail -40 gpurun_out/r06_d/pytest_carry.log; exit 1; }
tail -3 gpurun_out/r06_d/pytest_carry.log
bash tools/onectx_ab.sh r06_d 2 "cur asmall" 30 1
