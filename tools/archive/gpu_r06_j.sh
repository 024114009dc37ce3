#!/bin/bash
# round 6 j: host cost of a launch (plain vs ext API, plain vs CU-masked
# stream) and the lanes wrapper's pieces
set -e
O=gpurun_out/r06_j; mkdir -p $O
timeout -k 10 120 tools/micro/launch_cost > $O/launch_cost.txt
cat $O/launch_cost.txt
DVCC_HOST_PROF=1 timeout -k 10 300 python3 -u tools/exp_hostbound.py 5 > $O/hostbound.json 2> $O/hostbound.err
cat $O/hostbound.json
