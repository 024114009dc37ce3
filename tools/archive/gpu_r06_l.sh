#!/bin/bash
# round 6 l: kernel-trace timeline of a 20-epoch lanes run (where a short run
# loses its time against the steady state), lanes started from one host thread
# each and one after the other
set -e
export TMPDIR=/tmp
O=gpurun_out/r06_l; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/kt -o run -- python3 tools/exp_hostbound.py 5 > $O/hb.json 2> $O/hb.err
f=$(find $O/kt -name 'run_kernel_trace.csv' | head -1)
python3 tools/lane_window.py $f --gap 100 > $O/window.txt
DVCC_LANES_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/kts -o run -- python3 tools/exp_hostbound.py 5 > $O/hbs.json 2> $O/hbs.err
f=$(find $O/kts -name 'run_kernel_trace.csv' | head -1)
python3 tools/lane_window.py $f --gap 100 > $O/window_serial.txt
cat $O/window.txt $O/window_serial.txt
