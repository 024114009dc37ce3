#!/bin/bash
# round 6 i: is the driver's 20-step run host-bound?  (host time per epoch,
# launch calls, Python wrapper time); round 0 per bucket size class vs its pass
set -e
O=gpurun_out/r06_i; mkdir -p $O
DVCC_HOST_PROF=1 timeout -k 10 300 python3 -u tools/exp_hostbound.py 5 > $O/default.json 2> $O/default.err
DVCC_HOST_PROF=1 DVCC_NO_GRAPHS=1 timeout -k 10 300 python3 -u tools/exp_hostbound.py 5 > $O/nographs.json 2> $O/nographs.err
cat $O/*.json
bash tools/onectx_ab.sh r06_i 2 "cur nofuse" 30 1
