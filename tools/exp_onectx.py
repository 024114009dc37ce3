"""One context, config D: ms per epoch of a pipelined batch (no profiling)
and, after it, every kernel's average launch time from its own dispatch
timestamps (DV_FLAG_KERNEL_PROFILE).  For A/B of experiment libraries
(DVCC_LIB=exp_build/<name>/libdvcc.so).  Prints one JSON line."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deneva-plus_amd"))
import dvcc  # noqa: E402

rows, n_txn = 16_777_216, 1_048_576
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
lanes_n = int(sys.argv[2]) if len(sys.argv) > 2 else 1
gen = dvcc.YCSBQueryGenerator(rows, part_cnt=1, req_per_query=10, zipf_theta=0.9, txn_write_perc=1.0,
                              tup_write_perc=0.5, part_per_txn=1, strict_ppt=1, mpr=-1.0)
deps = [dvcc.DeviceEpoch(gen.gen(n_txn, dvcc.epoch_seed(0, e))) for e in range(5)]
torch.cuda.set_stream(torch.cuda.Stream())
eng = dvcc.CCEngine("NO_WAIT", n_txn, n_txn * 10)
eng.set_stream(torch.cuda.current_stream().cuda_stream)
eng.load_ycsb_partition(rows)
lanes = [eng.open_lane() for _ in range(lanes_n - 1)]
d = torch.zeros(n_txn, dtype=torch.uint8, device="cuda")


def run(k):
    eps = [deps[i % 5] for i in range(k)]
    return eng.run_epochs_lanes(lanes, eps, d) if lanes else eng.run_epochs_device(eps, d)


run(10)
torch.cuda.synchronize()
t0 = time.perf_counter()
sts = run(steps)
torch.cuda.synchronize()
el = time.perf_counter() - t0
eng.set_timing(False, profile=True)
eng.kernel_times(reset=True)
eng.run_epochs_device([deps[i % 5] for i in range(10)], d)
kt = eng.kernel_times(reset=True)
eng.set_timing(False)
out = {"ms_per_epoch": el / steps * 1e3, "committed": int(sum(s.committed for s in sts)) // steps,
       "yields": int(sum(s.async_yields for s in sts)), "declined": int(sum(s.async_declined for s in sts)),
       "kernels_us": {k: round(ms / n * 1e3, 2) for k, (n, ms) in sorted(kt.items(), key=lambda kv: -kv[1][1])[:12]},
       "kernel_us_per_epoch": round(sum(ms for _, ms in kt.values()) / 10 * 1e3, 1)}
print(json.dumps(out))
for ln in lanes:
    ln.close()
eng.close()
