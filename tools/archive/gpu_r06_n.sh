#!/bin/bash
# round 6 n: the lanes wrapper's Python time against the C call's own
set -e
O=gpurun_out/r06_n; mkdir -p $O
DVCC_PY_PROF=1 DVCC_HOST_PROF=1 timeout -k 10 300 python3 -u tools/exp_hostbound.py 5 > $O/hb.json 2> $O/hb.err
cat $O/hb.json; grep "dvcc" $O/hb.err
