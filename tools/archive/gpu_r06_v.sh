#!/bin/bash
# round 6 v: k_kill_emit reads k_kill's skip bits instead of re-gathering the
# row state -- prefix/lanes/closed-loop tests, A/B, and FETCH_SIZE of both
set -e
export TMPDIR=/tmp
O=gpurun_out/r06_v; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_carry.py -m gpu -x -q --timeout 600 \
    --timeout-method thread -k "prefix or lanes or kill or closed or config_d or skip or longest or pipelined" \
    > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/onectx_ab.sh r06_v 3 "cur emitrs" 30 1
for v in cur emitrs; do
  lp=""; [ $v != cur ] && lp=$PWD/exp_build/$v/libdvcc.so
  DVCC_LIB=$lp timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/pmc_$v -o run -- python3 tools/exp_onectx.py 10 1 > $O/pmc_$v.json 2> $O/pmc_$v.err
  f=$(find $O/pmc_$v -name '*counter_collection.csv' | head -1)
  python3 -c "
import csv
v=[float(r['Counter_Value']) for r in csv.DictReader(open('$f')) if 'k_kill_emit' in r['Kernel_Name']]
print('$v k_kill_emit FETCH_SIZE KiB per launch', sum(v)/max(1,len(v)), len(v))"
done
