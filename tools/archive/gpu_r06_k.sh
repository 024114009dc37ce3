#!/bin/bash
# round 6 k: lanes queue their first epochs from one host thread each --
# the lanes tests, the short-run A/B against DVCC_LANES_SERIAL, and the fused
# round 0's phase stamps
set -e
O=gpurun_out/r06_k; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_carry.py -m gpu -x -q --timeout 600 \
    --timeout-method thread -k "lanes or pipelined or graphs or fused" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
  DVCC_HOST_PROF=1 timeout -k 10 300 python3 -u tools/exp_hostbound.py 5 > $O/par$i.json 2> $O/par$i.err
  DVCC_LANES_SERIAL=1 DVCC_HOST_PROF=1 timeout -k 10 300 python3 -u tools/exp_hostbound.py 5 > $O/ser$i.json 2> $O/ser$i.err
done
cat $O/par*.json $O/ser*.json
DVCC_LIB=$PWD/exp_build/bstamps/libdvcc.so timeout -k 10 300 python3 -u tools/exp_bucket_stamps.py 20 > $O/bstamps.json
