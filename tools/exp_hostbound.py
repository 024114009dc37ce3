"""Is the driver's short run host-bound?  Config D over four decision lanes:
ms per epoch of a W=5 / K=20 run (the driver's arguments) and of a K=100 run
after it, with `n_buf` distinct epoch buffers.  DVCC_HOST_PROF=1 prints the
host's queueing vs waiting per epoch to stderr; DVCC_GRAPH_AFTER /
DVCC_NO_GRAPHS steer the epoch graphs.  Prints one JSON line."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deneva-plus_amd"))
import dvcc  # noqa: E402

rows, n_txn = 16_777_216, 1_048_576
n_buf = int(sys.argv[1]) if len(sys.argv) > 1 else 5
n_lanes = int(sys.argv[2]) if len(sys.argv) > 2 else 4
gen = dvcc.YCSBQueryGenerator(rows, part_cnt=1, req_per_query=10, zipf_theta=0.9, txn_write_perc=1.0,
                              tup_write_perc=0.5, part_per_txn=1, strict_ppt=1, mpr=-1.0)
deps = [dvcc.DeviceEpoch(gen.gen(n_txn, dvcc.epoch_seed(0, e))) for e in range(n_buf)]
torch.cuda.set_stream(torch.cuda.Stream())
eng = dvcc.CCEngine("NO_WAIT", n_txn, n_txn * 10)
eng.set_stream(torch.cuda.current_stream().cuda_stream)
eng.load_ycsb_partition(rows)
lanes = [eng.open_lane() for _ in range(n_lanes - 1)]
d = torch.zeros(n_txn, dtype=torch.uint8, device="cuda")


def batch(first, k):
    return eng.run_epochs_lanes(lanes, [deps[(first + i) % n_buf] for i in range(k)], d)


out = {"n_buf": n_buf, "lanes": n_lanes}
batch(0, 5)
torch.cuda.synchronize()
for name, first, k in (("k20", 5, 20), ("k100", 25, 100), ("k20_after", 125, 20)):
    t0 = time.perf_counter()
    batch(first, k)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    out[name] = (t2 - t0) / k * 1e3
    out[name + "_call_ms"] = (t1 - t0) * 1e3
    out[name + "_sync_ms"] = (t2 - t1) * 1e3
    sys.stderr.flush()
# the wrapper's pieces around the C call (run_epochs_lanes inline)
import ctypes  # noqa: E402
from dvcc import _lib as L  # noqa: E402
from dvcc.engine import _after_torch_all  # noqa: E402
ctxs = [eng] + lanes
sel = [deps[i % n_buf] for i in range(20)]
torch.cuda.synchronize()
t0 = time.perf_counter()
_after_torch_all(ctxs)
t1 = time.perf_counter()
arr = (L.EpochDev * 20)(*[x.desc() for x in sel])
cps = (ctypes.c_void_p * 20)(*([int(d.data_ptr())] * 20))
sts = (L.Stats * 20)()
lp = (ctypes.c_void_p * len(ctxs))(*[e._ctx.value for e in ctxs])
t2 = time.perf_counter()
L.check(L.lib().dv_epoch_run_device_lanes(lp, len(ctxs), arr, 20, cps, sts), "lanes")
t3 = time.perf_counter()
torch.cuda.synchronize()
t4 = time.perf_counter()
out["split_ms"] = {"after_torch": (t1 - t0) * 1e3, "args": (t2 - t1) * 1e3, "call": (t3 - t2) * 1e3,
                   "sync": (t4 - t3) * 1e3}
print(json.dumps(out))
for ln in lanes:
    ln.close()
eng.close()
