set -e
# per-variant k_round_pass durations of rounds 0-2 (tools/exp_pass.py under a
# kernel trace): tools/gpu_exp_pass.sh <tag> <variant>...  (exp_build/<variant>)
T=gpurun_out/$1
shift
mkdir -p $T
for n in "$@"; do
  DVCC_LIB=$PWD/exp_build/$n/libdvcc.so timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d $T/$n -o run -- python3 tools/exp_pass.py > $T/$n.log 2>&1
  python3 tools/pass_times.py $T/$n/run_kernel_trace.csv $n
done
