#!/bin/bash
# round 6 m: device-stamped timeline of a 20-epoch and a 100-epoch lanes call
set -e
O=gpurun_out/r06_m; mkdir -p $O
DVCC_LIB=$PWD/exp_build/lst/libdvcc.so timeout -k 10 300 python3 -u tools/exp_lane_stamps.py 20 4 > $O/lst20.json
DVCC_LIB=$PWD/exp_build/lst/libdvcc.so timeout -k 10 300 python3 -u tools/exp_lane_stamps.py 100 4 > $O/lst100.json
python3 -c "
import json
for f in ('lst20','lst100'):
    d=json.load(open('$O/'+f+'.json')); d.pop('timeline',None); print(f, json.dumps(d))
"
