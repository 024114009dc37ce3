"""Measurement only: two independent engines (own tables, own streams) each
running config-D epochs through dv_epoch_run_device_batch from its own host
thread, against one engine alone -- how much decision work of two epochs
overlaps on one GPU (the async rounds are latency-bound).
    python tools/exp_two_lanes.py [epochs]"""
import os
import sys
import threading
import time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "deneva-plus_amd"))
import torch
import dvcc
from dvcc import CCEngine, DeviceEpoch, YCSBQueryGenerator

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
rows, n = 1 << 24, 1 << 20
g = YCSBQueryGenerator(rows, zipf_theta=0.9, txn_write_perc=1.0, tup_write_perc=0.5)
host = [g.gen(n, dvcc.epoch_seed(0, e)) for e in range(4)]


def make():
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        eng = CCEngine("NO_WAIT", n, n * 10)
        eng.set_stream(s.cuda_stream)
        eng.load_ycsb_partition(rows)
        deps = [DeviceEpoch(e) for e in host]
        d = torch.zeros(n, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    return eng, deps, d


lanes = [make(), make()]


def run(lane, k, out):
    eng, deps, d = lane
    sts = eng.run_epochs_device([deps[i % 4] for i in range(k)], d)
    out.append(sts)


for ln in lanes:  # warm-up
    run(ln, 3, [])
torch.cuda.synchronize()
t0 = time.perf_counter()
one = []
run(lanes[0], K, one)
torch.cuda.synchronize()
t1 = time.perf_counter() - t0
res = [[], []]
ths = [threading.Thread(target=run, args=(lanes[i], K, res[i])) for i in range(2)]
t0 = time.perf_counter()
for t in ths:
    t.start()
for t in ths:
    t.join()
torch.cuda.synchronize()
t2 = time.perf_counter() - t0
y = sum(st.async_yields for r in res for sts in r for st in sts)
print(f"one lane: {t1 / K * 1e3:.4f} ms/epoch; two lanes: {t2 / (2 * K) * 1e3:.4f} ms/epoch aggregate "
      f"({t1 / K / (t2 / (2 * K)):.2f}x), async yields {y}")
