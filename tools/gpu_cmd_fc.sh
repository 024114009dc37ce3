set -e
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "async or batch or lane" > gpurun_out/fc_pytest.txt 2>&1 || { tail -30 gpurun_out/fc_pytest.txt; exit 1; }
tail -1 gpurun_out/fc_pytest.txt
bash tools/lib_ab.sh r03_fc 3 "base fc" --steps 100 --warmup 5 --lanes 1
bash tools/lib_ab.sh r03_fc4 3 "base fc" --steps 100 --warmup 5 --lanes 4
