set -e
export PYTHONUNBUFFERED=1
T=${1:-r05_n}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests/test_tpcc_gpu.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { tail -40 gpurun_out/$T/pytest.log; exit 1; }
tail -1 gpurun_out/$T/pytest.log
for i in 1 2; do
DVCC_HOST_PROF=1 timeout -k 10 300 python bench.py --tpcc-only > gpurun_out/$T/tp$i.json 2> gpurun_out/$T/tp$i.err
python3 tools/bench_brief.py gpurun_out/$T/tp$i.json
grep "dvcc host" gpurun_out/$T/tp$i.err | grep -v "8 epochs" | grep "200 epochs"
done
for i in 1 2; do
for v in 0 1; do
  if [ $v = 1 ]; then export DVCC_PREFIX_GRAPHS=1; else unset DVCC_PREFIX_GRAPHS; fi
  DVCC_HOST_PROF=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-tpcc --no-configs --epochs 4 --steps 100 --detail-out gpurun_out/$T/pg$v.$i.json > gpurun_out/$T/pg$v.$i.line 2> gpurun_out/$T/pg$v.$i.err
  python3 -c "import json; d=json.load(open('gpurun_out/$T/pg$v.$i.json')); print('prefix graphs $v', round(d['ms_per_step'],4))"
  grep "dvcc host" gpurun_out/$T/pg$v.$i.err | sed -n 2,3p
done
done
