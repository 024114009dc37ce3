"""Prefix size under four decision lanes (config D): ms per epoch of a
60-epoch pipelined call for each prefix size in argv (txns; 0 = the
automatic n/32), alternated twice.  Prints one JSON line."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deneva-plus_amd"))
import dvcc  # noqa: E402

rows, n_txn = 16_777_216, 1_048_576
sizes = [int(a) for a in sys.argv[1:]] or [0, 16384, 49152, 65536]
gen = dvcc.YCSBQueryGenerator(rows, part_cnt=1, req_per_query=10, zipf_theta=0.9, txn_write_perc=1.0,
                              tup_write_perc=0.5, part_per_txn=1, strict_ppt=1, mpr=-1.0)
deps = [dvcc.DeviceEpoch(gen.gen(n_txn, dvcc.epoch_seed(0, e))) for e in range(5)]
torch.cuda.set_stream(torch.cuda.Stream())
eng = dvcc.CCEngine("NO_WAIT", n_txn, n_txn * 10)
eng.set_stream(torch.cuda.current_stream().cuda_stream)
eng.load_ycsb_partition(rows)
lanes = [eng.open_lane() for _ in range(3)]
d = torch.zeros(n_txn, dtype=torch.uint8, device="cuda")
res = {str(k): [] for k in sizes}
commits = {}
for rep in range(2):
    for k in sizes:
        for e in [eng] + lanes:
            e.set_prefix(k)
        eng.run_epochs_lanes(lanes, [deps[i % 5] for i in range(10)], d)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sts = eng.run_epochs_lanes(lanes, [deps[i % 5] for i in range(60)], d)
        torch.cuda.synchronize()
        res[str(k)].append(round((time.perf_counter() - t0) / 60 * 1e3, 4))
        commits[str(k)] = sum(s.committed for s in sts[:5])
print(json.dumps({"ms_per_epoch": res, "committed_first5": commits}))
for ln in lanes:
    ln.close()
eng.close()
