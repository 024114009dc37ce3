set -e
T=gpurun_out/exp1
mkdir -p $T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $T/pytest.log 2>&1 || { tail -40 $T/pytest.log; exit 1; }
tail -1 $T/pytest.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $T/bench.json 2> $T/bench.err
head -c 600 $T/bench.json; echo
for n in base tick nolb nogather nodecide all; do
  DVCC_LIB=$PWD/exp_build/$n/libdvcc.so timeout -k 10 120 rocprofv3 --kernel-trace -f csv -T -d $T/$n -o run -- python3 tools/exp_pass.py > $T/$n.log 2>&1
  tail -1 $T/$n.log
done
