"""Experiment: time the first decision-round passes of one config-D epoch
under variant builds (DVCC_LIB selects the library).  Uses the staged API
(begin / round_local / round_apply) for a fixed number of rounds, so variants
that break decisions still run a bounded amount of work.

    DVCC_LIB=... rocprofv3 --kernel-trace -- python tools/exp_pass.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deneva-plus_amd"))
import torch  # noqa: E402
import dvcc  # noqa: E402

rows, n_txn = 1 << 24, 1 << 20
g = dvcc.YCSBQueryGenerator(rows, zipf_theta=0.9)
e = g.gen(n_txn, 1)
eng = dvcc.CCEngine(dvcc.NO_WAIT, n_txn, e.n_acc)
eng.load_ycsb_partition(rows)
dep = dvcc.DeviceEpoch(e)
v = torch.zeros(n_txn, dtype=torch.uint8, device="cuda")
for it in range(4):
    eng.begin(dep)
    for r in range(3):
        eng.round_local(v)
        try:
            eng.round_apply(v)
        except Exception as ex:  # variants may trip the error checks
            print("round", r, ex)
            break
    try:
        eng.finish()
    except Exception as ex:
        print("finish", ex)
torch.cuda.synchronize()
print(os.environ.get("DVCC_LIB", "base"), "done")
