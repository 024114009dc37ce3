"""Regenerate the golden epochs (SURVEY.md 8(c) KAT 6): small seeded YCSB
epochs with the oracle's E-schedule decisions and state digests.

The inputs come from the oracle restatement of gen_requests_zipf
(ycsb_query.cpp:303-376) and the decisions from its literal Row_lock / OptCC
state machines (row_lock.cpp:52-382, occ.cpp:116-327).  The reference binary
cannot be built here, so these fixtures pin the oracle
against regressions and the GPU engine against the oracle; they are not
reference outputs.

    python tests/golden/make_golden.py      # rewrites tests/golden/*.npz
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import _oracle as O  # noqa: E402

# name: (cc, rows, n_txn, zipf_theta, txn_write_perc, tup_write_perc, req, seed)
CASES = {
    "nowait_z09": (O.NO_WAIT, 4096, 4000, 0.9, 1.0, 0.5, 10, 11),
    "waitdie_z09": (O.WAIT_DIE, 4096, 4000, 0.9, 1.0, 0.5, 10, 12),
    "occ_z09": (O.OCC, 4096, 4000, 0.9, 1.0, 0.5, 10, 13),
    "calvin_z06": (O.CALVIN, 4096, 4000, 0.6, 1.0, 0.5, 10, 14),
    "nowait_mix_z06": (O.NO_WAIT, 1024, 2000, 0.6, 0.5, 0.5, 10, 15),
    "occ_hot_z099": (O.OCC, 512, 3000, 0.99, 1.0, 0.5, 4, 16),
}


def make(name):
    cc, rows, n_txn, theta, twp, tup, req, seed = CASES[name]
    p = O.ycsb_params(rows, 1, req, theta, twp, tup)
    keys, types, tb = O.ycsb_gen(p, seed, 0, n_txn)
    tab = O.YcsbTable(rows)
    f0 = tab.f0.copy()
    commit, grant, st = O.epoch_run(cc, tab.ix, f0, n_txn, tb, keys, types,
                                    want_grant=(cc == O.CALVIN))
    out = dict(cc=np.int32(cc), rows=np.int64(rows), keys=keys, types=types, txn_begin=tb,
               commit=commit, f0=f0,
               stats=np.array([st.committed, st.aborted, st.read_digest, st.write_cnt], np.uint64))
    if grant is not None:
        out["grant"] = grant
    return out


if __name__ == "__main__":
    for name in CASES:
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **make(name))
        print("wrote", name)
