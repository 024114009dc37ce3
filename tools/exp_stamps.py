"""k_round_async's per-iteration breakdown: config D on
one context with the DVCC_ASYNC_STAMPS measurement build
(tools/exp_variant.sh stamps dvcc_rounds.hip -DDVCC_ASYNC_STAMPS; run with
DVCC_LIB=exp_build/stamps/libdvcc.so).  Thread 0 of every workgroup stamps
each iteration with the 100-MHz wall clock: facts loaded, carry walk done,
decide/compact/publish done, back-off.  Prints one JSON line."""
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
lib.dv_debug_async_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
lib.dv_debug_async_launches.argtypes = [ctypes.c_void_p]
lrec = np.zeros(4, np.uint64)
buf = np.zeros(512 * 8, np.uint64)
eng.run_epochs_device([deps[i % 3] for i in range(6)], d)
assert lib.dv_debug_async_stamps(buf.ctypes.data, buf.size) == 0
assert lib.dv_debug_async_launches(lrec.ctypes.data) == 0
sts = eng.run_epochs_device([deps[i % 3] for i in range(epochs)], d)
torch.cuda.synchronize()
assert lib.dv_debug_async_stamps(buf.ctypes.data, buf.size) == 0
assert lib.dv_debug_async_launches(lrec.ctypes.data) == 0
w = buf.reshape(512, 8).astype(np.float64)
used = w[:, 0] > 0
w = w[used]
tick_us = 0.01
tot = w.sum(axis=0)
it = tot[1]
out = {"epochs": epochs, "workgroups": int(used.sum()), "launches_per_wg": float(w[:, 0].mean()),
       "iters_per_wg_launch": float(it / tot[0]),
       "iters_max_per_launch_mean": float((w[:, 1] / w[:, 0]).max()),
       "us_in_loop_per_wg_launch": float(tot[2] / tot[0] * tick_us),
       "per_iteration_us": {"facts": float(tot[3] / it * tick_us), "carry_walk": float(tot[4] / it * tick_us),
                            "work": float(tot[5] / it * tick_us), "backoff": float(tot[6] / it * tick_us)},
       "moved_frac": float(tot[7] / it),
       "per_launch": {"launches": int(lrec[0]),
                      "mean_of_wg_iterations": float(lrec[2]) / 1024.0 / max(1, int(lrec[0])),
                      "max_wg_iterations": float(lrec[1]) / max(1, int(lrec[0]))},
       "rounds_mean": float(np.mean([s.rounds for s in sts])),
       "async_live_per_epoch": float(np.mean([s.async_live for s in sts]))}
print(json.dumps(out))
eng.close()
