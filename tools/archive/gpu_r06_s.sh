#!/bin/bash
# round 6 s: register-staged chunk scans (radix / carry / owner) and the
# streamed carry copy -- the whole GPU suite, then one-context and closed-loop
# kernel times
set -e
O=gpurun_out/r06_s; mkdir -p $O
bash tools/gpu.sh tests r06_s
timeout -k 10 300 python3 -u tools/exp_onectx.py 30 1 > $O/onectx.json
cat $O/onectx.json
timeout -k 10 300 python3 -u tools/exp_closed_loop.py > $O/closed.json
cat $O/closed.json
