"""Where a decision lane's time goes at config D (four lanes, the headline's
entry point dv_epoch_run_device_lanes), from the DVCC_LANE_STAMPS
measurement build, its code kept out of the product's sources
(EXP_PATCH=tools/patches/lane_stamps.diff tools/exp_variant.sh lst
dvcc_kernels.hip,dvcc_runtime.hip -DDVCC_LANE_STAMPS [-DDVCC_DUMMY_LAUNCHES=20];
run with DVCC_LIB=exp_build/lst/libdvcc.so; argv: epochs, lanes).  Each
lane's epoch: clear -> turn wait begins (its decision done) -> wait ends (the
previous execution posted) -> post (its execution done) -> the lane's next
clear.  Prints one JSON line: per-phase means over the timed call's steady
epochs, and how many lanes were deciding at once."""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deneva-plus_amd"))
import dvcc  # noqa: E402
from dvcc import _lib as L  # noqa: E402

rows, n_txn = 16_777_216, 1_048_576
epochs = int(sys.argv[1]) if len(sys.argv) > 1 else 100
nl = int(sys.argv[2]) if len(sys.argv) > 2 else 4
gen = dvcc.YCSBQueryGenerator(rows, part_cnt=1, req_per_query=10, zipf_theta=0.9, txn_write_perc=1.0,
                              tup_write_perc=0.5, part_per_txn=1, strict_ppt=1, mpr=-1.0)
eps = [gen.gen(n_txn, dvcc.epoch_seed(0, e)) for e in range(5)]
deps = [dvcc.DeviceEpoch(e) for e in eps]
eng = dvcc.CCEngine("NO_WAIT", n_txn, max(e.n_acc for e in eps))
eng.set_stream(torch.cuda.current_stream().cuda_stream)
eng.load_ycsb_partition(rows)
lanes = [eng.open_lane() for _ in range(nl - 1)]
d = torch.zeros(n_txn, dtype=torch.uint8, device="cuda")
lib = L.lib()
lib.dv_debug_lane_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
buf = np.zeros(8192 * 2, np.uint64)
cnt = np.zeros(1, np.uint32)
run = (lambda r: eng.run_epochs_lanes(lanes, r, d)) if lanes else (lambda r: eng.run_epochs_device(r, d))
run([deps[i % 5] for i in range(10)])
assert lib.dv_debug_lane_stamps(buf.ctypes.data, buf.size, cnt.ctypes.data) == 0
torch.cuda.synchronize()
t0 = time.perf_counter()
run([deps[i % 5] for i in range(epochs)])
torch.cuda.synchronize()
el = time.perf_counter() - t0
assert lib.dv_debug_lane_stamps(buf.ctypes.data, buf.size, cnt.ctypes.data) == 0
n = int(cnt[0])
assert n <= 8192, n
ts = buf[0:2 * n:2].astype(np.int64)
tag = buf[1:2 * n:2]
ev = (tag & 3).astype(np.int64)
ctx = tag >> 2
us = 0.01
lane_ids = {c: i for i, c in enumerate(sorted(set(ctx.tolist())))}
phases = {"decide": [], "turn_wait": [], "exec": [], "idle": []}
starts, ends = [], []
per_lane = {}
for c, li in lane_ids.items():
    m = ctx == c
    order = np.argsort(ts[m], kind="stable")
    t_l, e_l = ts[m][order], ev[m][order]
    seq = list(zip(e_l.tolist(), t_l.tolist()))
    eps_l = []
    cur = {}
    for e, t in seq:
        if e == 0:
            if cur:
                eps_l.append(cur)
            cur = {0: t}
        else:
            cur[e] = t
    if cur:
        eps_l.append(cur)
    per_lane[li] = len(eps_l)
    for j, x in enumerate(eps_l):
        if not all(k in x for k in (0, 1, 2, 3)):
            continue
        phases["decide"].append((x[1] - x[0]) * us)
        phases["turn_wait"].append((x[2] - x[1]) * us)
        phases["exec"].append((x[3] - x[2]) * us)
        starts.append(x[0])
        ends.append(x[1])
        if j + 1 < len(eps_l) and 0 in eps_l[j + 1]:
            phases["idle"].append((eps_l[j + 1][0] - x[3]) * us)
span = (ts.max() - ts.min()) * us
# lanes deciding at once, time-weighted over the call
if not starts:  # (one context: no turn words, no phases)
    print(json.dumps({"epochs": epochs, "lanes": nl, "ms_per_epoch_host": el / epochs * 1e3}))
    sys.exit(0)
pts = sorted([(s, 1) for s in starts] + [(e, -1) for e in ends])
busy, lv, last, hist = 0.0, 0, pts[0][0], {}
for t, dlt in pts:
    hist[lv] = hist.get(lv, 0) + (t - last) * us
    lv += dlt
    last = t
# a short call (the driver's 20 epochs): every epoch's clear / decided /
# turn / posted, in us from the call's first stamp, lane by lane
timeline = None
if epochs <= 40:
    t_min = ts.min()
    timeline = {}
    for c, li in lane_ids.items():
        m = ctx == c
        order = np.argsort(ts[m], kind="stable")
        rows_l, cur = [], None
        for e, t in zip(ev[m][order].tolist(), ts[m][order].tolist()):
            if e == 0:
                if cur:
                    rows_l.append(cur)
                cur = [round((t - t_min) * us, 1), None, None, None]
            elif cur is not None:
                cur[e] = round((t - t_min) * us, 1)
        if cur:
            rows_l.append(cur)
        timeline[str(li)] = rows_l
out = {"epochs": epochs, "lanes": nl, "ms_per_epoch_host": el / epochs * 1e3, "stamp_span_us": span,
       "timeline": timeline,
       "us_per_epoch_device": span / epochs, "lane_epochs": per_lane,
       "mean_us": {k: float(np.mean(v)) for k, v in phases.items() if v},
       "p90_us": {k: float(np.percentile(v, 90)) for k, v in phases.items() if v},
       "deciding_at_once_us": {str(k): round(v, 1) for k, v in sorted(hist.items())}}
print(json.dumps(out))
for ln in lanes:
    ln.close()
eng.close()
