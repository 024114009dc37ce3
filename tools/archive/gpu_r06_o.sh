#!/bin/bash
# round 6 o: idle-stream hand-over and cached epoch arrays -- lanes tests,
# the Python-vs-C timing probe, then the driver's bench arguments twice
set -e
O=gpurun_out/r06_o; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_carry.py -m gpu -x -q --timeout 600 \
    --timeout-method thread -k "lanes or pipelined or graphs or small_sorts" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
DVCC_PY_PROF=1 DVCC_HOST_PROF=1 timeout -k 10 300 python3 -u tools/exp_hostbound.py 5 > $O/hb.json 2> $O/hb.err
cat $O/hb.json; grep "dvcc" $O/hb.err
for i in 1 2; do
  timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-configs --no-tpcc > $O/bench$i.json 2> $O/bench$i.err
  python3 -c "import json; d=json.load(open('$O/bench$i.json')); print('bench', d['ms_per_step'], d['value'])"
done
