set -e
# cost of the engine's timing modes on the default bench workload
mkdir -p gpurun_out/tim
for m in full kernel off full kernel off; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 20 --timing $m > gpurun_out/tim/$m.json 2>gpurun_out/tim/$m.err
  python3 -c "import json; print('$m', json.load(open('gpurun_out/tim/$m.json'))['ms_per_step'])"
done
