"""Regenerate the TPC-C golden epochs (tests/golden/tpcc/*.npz): small seeded
Payment + NewOrder epochs with the oracle's decisions, o_ids and the rows each
epoch changed (SURVEY.md 8(c) KAT 6 for config E).

Inputs come from the oracle's restatement of TPCCQueryGenerator
(tpcc_query.cpp:26-263, glibc rand pinned by tests/test_tpcc.py) and the
loader of tpcc_wl.cpp; decisions from the literal Row_lock / OptCC state
machines; execution from run_payment_1/3/5 and new_order_5/9.  Not reference
outputs (the reference cannot be built here).

    python tests/golden/make_golden_tpcc.py
"""
import os
import sys

import numpy as np

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tpcc")
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import _oracle as O  # noqa: E402

PARAMS = dict(num_wh=2, cust_per_dist=1000, max_items=2000)
LOAD_SEED = 7
# name: (cc, n_txn, epoch seed, perc_payment)
CASES = {
    "nowait": (O.NO_WAIT, 2000, 21, 0.5),
    "waitdie": (O.WAIT_DIE, 2000, 22, 0.5),
    "occ": (O.OCC, 2000, 23, 0.5),
    "calvin": (O.CALVIN, 2000, 24, 0.5),
    "calvin_payment": (O.CALVIN, 1500, 25, 1.0),
}


def make(name):
    cc, n_txn, seed, perc = CASES[name]
    p = O.tpcc_params(perc_payment=perc, **PARAMS)
    keys, types, tables, args, tb, tt, own = O.tpcc_gen(p, n_txn, seed)
    db = O.TpccDB(p, LOAD_SEED)
    before = [db.table(t) for t in range(5)]
    commit, oid, st = db.epoch(cc, keys, types, tables, args, tb)
    out = dict(cc=np.int32(cc), perc=np.float64(perc), keys=keys, types=types, tables=tables, args=args,
               txn_begin=tb, commit=commit, oid=oid,
               stats=np.array([st.committed, st.aborted, st.write_cnt], np.uint64))
    for t in range(5):
        after = db.table(t)
        cols_b = np.stack(before[t][1:], 1)
        cols_a = np.stack(after[1:], 1)
        rows = np.flatnonzero((cols_a != cols_b).any(1))
        out[f"rows_{t}"] = rows.astype(np.int64)
        out[f"vals_{t}"] = cols_a[rows]
    return out


if __name__ == "__main__":
    os.makedirs(HERE, exist_ok=True)
    for name in CASES:
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **make(name))
        print("wrote", name)
