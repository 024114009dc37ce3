set -e
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "lanes_setup_error" > gpurun_out/le_pytest.txt 2>&1 || { tail -40 gpurun_out/le_pytest.txt; exit 1; }
tail -2 gpurun_out/le_pytest.txt
