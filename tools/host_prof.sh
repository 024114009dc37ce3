#!/bin/bash
# DVCC_HOST_PROF over the config-D headline (four lanes): the host's time per
# epoch queueing vs waiting for read-backs -> gpurun_out/<tag>/host_prof.txt
set -e
OUT=gpurun_out/$1; shift
mkdir -p $OUT
DVCC_HOST_PROF=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-configs --no-tpcc "$@" > $OUT/b.json 2> $OUT/b.err
grep "dvcc host" $OUT/b.err > $OUT/host_prof.txt || true
python3 tools/bench_brief.py $OUT/b.json | head -1
cat $OUT/host_prof.txt
