set -e
mkdir -p gpurun_out/r06_b
DVCC_LIB=$PWD/exp_build/stamps/libdvcc.so timeout -k 10 300 python3 -u tools/exp_stamps.py 30 > gpurun_out/r06_b/async_stamps.json 2> gpurun_out/r06_b/async_stamps.err
cat gpurun_out/r06_b/async_stamps.json
DVCC_LIB=$PWD/exp_build/bstamps/libdvcc.so timeout -k 10 300 python3 -u tools/exp_bucket_stamps.py 30 > gpurun_out/r06_b/bucket_stamps.json 2> gpurun_out/r06_b/bucket_stamps.err
cat gpurun_out/r06_b/bucket_stamps.json
