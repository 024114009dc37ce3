set -e
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_partitioned.py tests/test_tpcc_gpu.py > gpurun_out/pl_pytest.txt 2>&1 || { tail -40 gpurun_out/pl_pytest.txt; exit 1; }
tail -2 gpurun_out/pl_pytest.txt
