#!/bin/bash
# The N>1 bench path rehearsed on a one-GPU box: 2 ranks sharing the card
# (bench.py --ipc-rehearsal) -> gpurun_out/<tag>/rehearsal.json
set -e
OUT=gpurun_out/$1; shift
mkdir -p $OUT
timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29531 bench.py --gpus 2 --ipc-rehearsal "$@" > $OUT/rehearsal.json 2> $OUT/rehearsal.err \
    || { tail -30 $OUT/rehearsal.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$OUT/rehearsal.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['config']['sequence_order'])"
