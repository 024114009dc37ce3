"""k_bucket_sort's per-bucket time: config D on one
context with the DVCC_BUCKET_STAMPS measurement build (tools/exp_variant.sh
bstamps dvcc_kernels.hip -DDVCC_BUCKET_STAMPS; run with
DVCC_LIB=exp_build/bstamps/libdvcc.so).  Thread 0 of every bucket's
workgroup stamps its start and end with the 100-MHz wall clock.  Prints one
JSON line: the launch's slowest bucket against the mean bucket, and the
buckets' time against their key counts."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deneva-plus_amd"))
import dvcc  # noqa: E402
from dvcc import _lib as L  # noqa: E402

rows, n_txn, epochs = 16_777_216, 1_048_576, int(sys.argv[1]) if len(sys.argv) > 1 else 20
gen = dvcc.YCSBQueryGenerator(rows, part_cnt=1, req_per_query=10, zipf_theta=0.9, txn_write_perc=1.0,
                              tup_write_perc=0.5, part_per_txn=1, strict_ppt=1, mpr=-1.0)
eps = [gen.gen(n_txn, dvcc.epoch_seed(0, e)) for e in range(3)]
deps = [dvcc.DeviceEpoch(e) for e in eps]
eng = dvcc.CCEngine("NO_WAIT", n_txn, n_txn * 10)
eng.set_stream(torch.cuda.current_stream().cuda_stream)
eng.load_ycsb_partition(rows)
d = torch.zeros(n_txn, dtype=torch.uint8, device="cuda")
lib = L.lib()
lib.dv_debug_bucket_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
buf = np.zeros(1024 * 4, np.uint64)
lrec = np.zeros(4, np.uint64)
eng.run_epochs_device([deps[i % 3] for i in range(6)], d)
assert lib.dv_debug_bucket_stamps(buf.ctypes.data, lrec.ctypes.data) == 0
eng.run_epochs_device([deps[i % 3] for i in range(epochs)], d)
torch.cuda.synchronize()
assert lib.dv_debug_bucket_stamps(buf.ctypes.data, lrec.ctypes.data) == 0
w = buf.reshape(1024, 4).astype(np.float64)
used = w[:, 0] > 0
w = w[used]
us = w[:, 1] / w[:, 0] * 0.01
keys = w[:, 2] / w[:, 0]
order = np.argsort(keys)
dec = [{"keys": float(keys[order[i]]), "us": float(us[order[i]])}
       for i in np.linspace(0, len(order) - 1, 12).astype(int)]
nl = max(1, int(lrec[0]))
out = {"epochs": epochs, "buckets": int(used.sum()), "launches": int(lrec[0]),
       "launch_slowest_bucket_us": float(lrec[1]) / nl * 0.01, "launch_slowest_bucket_keys": float(lrec[2]) / nl,
       "bucket_us_mean": float(us.mean()), "bucket_keys_mean": float(keys.mean()),
       "bucket_us_max_mean": float(us.max()), "keys_of_slowest_mean_bucket": float(keys[np.argmax(us)]),
       "us_vs_keys_fit": [float(v) for v in np.polyfit(keys, us, 1)], "by_size": dec}
print(json.dumps(out))
eng.close()
