"""Round-by-round live / undecided counts of config D's decision stages, with
the synchronous rounds only (no asynchronous launch, no tail kernel): the
prefix (its K txns run as an epoch of their own) and the survivors' stage
(dv_round_log of a prefix-kill epoch).  Measurement only.
    python tools/exp_rounds.py [rows] [n_txn]"""
import sys
import os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "deneva-plus_amd"))
import numpy as np
import dvcc
from dvcc import CCEngine, DeviceEpoch, YCSBQueryGenerator
import torch

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 24
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
g = YCSBQueryGenerator(rows, zipf_theta=0.9, txn_write_perc=1.0, tup_write_perc=0.5)
e = g.gen(n, dvcc.epoch_seed(0, 0))
K = n // 32
for cc in (dvcc.NO_WAIT, dvcc.OCC):
    eng = CCEngine(cc, n, e.n_acc, tail=False, asynchronous=False)
    eng.load_ycsb_partition(rows)
    eng.set_prefix(None)
    tb = e.txn_begin
    pre = dvcc.Epoch(e.keys[:tb[K]].copy(), e.types[:tb[K]].copy(), tb[:K + 1].copy())
    d = torch.zeros(n, dtype=torch.uint8, device="cuda")
    st = eng.run_epoch_device(DeviceEpoch(pre), d)
    live, und = eng.round_log()
    print(f"cc {cc} prefix K={K}: committed {st.committed} rounds {st.rounds}")
    print("  live", live)
    print("  und ", und)
    eng.close()
    eng = CCEngine(cc, n, e.n_acc, tail=False, asynchronous=False)
    eng.load_ycsb_partition(rows)
    eng.set_prefix(0)
    st = eng.run_epoch_device(DeviceEpoch(e), d)
    live, und = eng.round_log()
    print(f"cc {cc} epoch: committed {st.committed} prefix_acc {st.prefix_acc} surv_txn {st.surv_txn} "
          f"surv_acc {st.surv_acc} rounds {st.rounds}")
    print("  survivors live", live)
    print("  survivors und ", und)
    eng.close()
