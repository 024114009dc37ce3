"""The closed loop at config D: ms per epoch of
dv_epoch_run_closed_loop (one context, 20 epochs) and of
dv_epoch_run_closed_loop_lanes (four lanes, 32 epochs), then the one-context
loop's per-kernel launch averages (DV_FLAG_KERNEL_PROFILE).  For A/B of
experiment libraries (DVCC_LIB=exp_build/<name>/libdvcc.so).  Prints one JSON
line."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deneva-plus_amd"))
import dvcc  # noqa: E402

rows, n_txn = 16_777_216, 1_048_576
gen = dvcc.YCSBQueryGenerator(rows, part_cnt=1, req_per_query=10, zipf_theta=0.9, txn_write_perc=1.0,
                              tup_write_perc=0.5, part_per_txn=1, strict_ppt=1, mpr=-1.0)
pool = gen.gen(2 * n_txn, dvcc.epoch_seed(0, 999))
dpool = dvcc.DeviceEpoch(pool)
pb = torch.from_numpy(pool.txn_begin.astype("int32")).cuda()
torch.cuda.set_stream(torch.cuda.Stream())
eng = dvcc.CCEngine("NO_WAIT", n_txn, n_txn * 10)
eng.set_stream(torch.cuda.current_stream().cuda_stream)
eng.load_ycsb_partition(rows)
out = {}
sts, bufs, cursor = eng.closed_loop(dpool, pb, n_txn, 2)
torch.cuda.synchronize()
t0 = time.perf_counter()
sts, bufs, cursor = eng.closed_loop(dpool, pb, n_txn, 20, cursor=cursor, bufs=bufs, resume=True)
torch.cuda.synchronize()
out["one_ctx_ms"] = (time.perf_counter() - t0) / 20 * 1e3
out["committed_one"] = sum(s.committed for s in sts)
eng.set_timing(False, profile=True)
eng.kernel_times(reset=True)
sts, bufs, cursor = eng.closed_loop(dpool, pb, n_txn, 10, cursor=cursor, bufs=bufs, resume=True)
kt = eng.kernel_times(reset=True)
eng.set_timing(False)
out["kernels_us"] = {k: round(ms / n * 1e3, 2) for k, (n, ms) in sorted(kt.items(), key=lambda kv: -kv[1][1])[:10]}
lanes = [eng.open_lane() for _ in range(3)]
sts, lb, cur = eng.closed_loop_lanes(lanes, dpool, pb, n_txn, 8)
torch.cuda.synchronize()
t0 = time.perf_counter()
sts, lb, cur = eng.closed_loop_lanes(lanes, dpool, pb, n_txn, 32, cursor=cur, bufs=lb, resume=True)
torch.cuda.synchronize()
out["lanes_ms"] = (time.perf_counter() - t0) / 32 * 1e3
out["committed_lanes"] = sum(s.committed for s in sts)
print(json.dumps(out))
for ln in lanes:
    ln.close()
eng.close()
