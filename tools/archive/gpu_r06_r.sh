#!/bin/bash
# round 6 r: the carry copy streamed per block -- closed-loop tests, then A/B
# against the wave form (exp_build/cwave) on the closed loop
set -e
O=gpurun_out/r06_r; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_carry.py -m gpu -x -q --timeout 600 --timeout-method thread \
    > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2 3; do
  for v in cur cwave; do
    lp=""; [ $v != cur ] && lp=$PWD/exp_build/$v/libdvcc.so
    DVCC_LIB=$lp timeout -k 10 300 python3 -u tools/exp_closed_loop.py > $O/$v$i.json 2> $O/$v$i.err
    echo "$v $(cat $O/$v$i.json)"
  done
done
