#!/bin/bash
# round 6 q: the list protocol in position-major order -- partitioned, TPC-C
# and IPC tests
set -e
O=gpurun_out/r06_q; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests/test_partitioned.py tests/test_tpcc_gpu.py tests/test_ipc.py -m gpu -x -v \
    --timeout 600 --timeout-method thread -k "position or engine_driver or part or ipc" > $O/pytest.log 2>&1 \
    || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
