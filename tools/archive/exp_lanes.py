"""Measurement only: config-D epochs through dv_epoch_run_device_lanes with
1..3 lanes, the owner on torch's stream (as bench.py) or on its own stream.
    python tools/exp_lanes.py [epochs] [own]"""
import os
import sys
import time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "deneva-plus_amd"))
import torch
import dvcc
from dvcc import CCEngine, DeviceEpoch, YCSBQueryGenerator

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
own = len(sys.argv) > 2 and sys.argv[2] == "own"
rows, n = 1 << 24, 1 << 20
g = YCSBQueryGenerator(rows, zipf_theta=0.9, txn_write_perc=1.0, tup_write_perc=0.5)
host = [g.gen(n, dvcc.epoch_seed(0, e)) for e in range(4)]
if not own:
    torch.cuda.set_stream(torch.cuda.Stream())
eng = CCEngine("NO_WAIT", n, n * 10)
if not own:
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
eng.load_ycsb_partition(rows)
deps = [DeviceEpoch(e) for e in host]
d = torch.zeros(n, dtype=torch.uint8, device="cuda")
lanes = [eng.open_lane() for _ in range(int(os.environ.get('EXP_NLANES', '2')) - 1)]
for L in (1, 2) if len(sys.argv) > 3 else tuple(int(x) for x in os.environ.get('EXP_LSEQ', '1,2,1,2,1,2').split(',')):
    run = lambda k: eng.run_epochs_lanes(lanes[:L - 1], [deps[i % 4] for i in range(k)], d)
    run(4)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sts = run(K)
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    print(f"lanes {L} ({'own' if own else 'torch'} stream): {t / K * 1e3:.4f} ms/epoch, "
          f"yields {sum(s.async_yields for s in sts)}, committed {sum(s.committed for s in sts)}", flush=True)
eng.close()
