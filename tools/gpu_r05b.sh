set -e
export PYTHONUNBUFFERED=1
T=${1:-r05_p}
mkdir -p gpurun_out/$T
timeout -k 10 1100 python -u -m pytest tests/test_partitioned.py tests/test_ipc.py -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { tail -60 gpurun_out/$T/pytest.log; exit 1; }
tail -3 gpurun_out/$T/pytest.log
