"""Diagnose a partitioned TPC-C mismatch: run dv_tpcc_epoch_run_part over
`world` contexts and report, per table and partition, the rows whose state
differs from the one-partition oracle (key, engine columns, oracle columns).

    python tools/debug_tpcc_e.py <cc> <num_wh> <world> <n_txn> [cust_per_dist max_items]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "deneva-plus_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import _oracle as O  # noqa: E402
import dvcc  # noqa: E402
import test_tpcc_gpu as TG  # noqa: E402
from dvcc import tpcc as T  # noqa: E402


def main():
    cc = {"WAIT_DIE": dvcc.WAIT_DIE, "CALVIN": dvcc.CALVIN, "NO_WAIT": dvcc.NO_WAIT, "OCC": dvcc.OCC}[sys.argv[1]]
    num_wh, world, n_txn = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    cpd = int(sys.argv[5]) if len(sys.argv) > 5 else 3000
    items = int(sys.argv[6]) if len(sys.argv) > 6 else 100000
    kw = dict(num_wh=num_wh, cust_per_dist=cpd, max_items=items, part_per_txn=2, mpr=1.0)
    engines, pp, batches, out = TG._tpcc_group(cc, kw, world, n_txn, 5, 60)
    db = O.TpccDB(O.tpcc_params(**dict(kw, part_cnt=1)), 5)
    keys, types, tables, args, tb = TG._global(batches)
    c_ref, o_ref, st_ref = db.epoch(TG.ORACLE_CC[cc], keys, types, tables, args, tb)
    for r, x in enumerate(out):
        if isinstance(x, Exception):
            print("rank", r, "error", x)
            return
        c, o, st = x
        print("rank", r, "commit mismatches", int((c != c_ref).sum()), "oid mismatches", int((o != o_ref).sum()))
    n_bad = 0
    for tid in range(5):
        ref = db.table(tid)
        pos = {int(k): i for i, k in enumerate(ref[0])} if tid != T.L.T_STOCK else None
        for p, eng in enumerate(engines):
            pk = T.table(pp, 5, tid, p)[0]
            cols = [eng.read_col(tid, col) for col in range(3)]
            if pos is None:
                idx = np.searchsorted(ref[0], pk) if (np.diff(ref[0].astype(np.int64)) > 0).all() else None
                if idx is None:
                    order = np.argsort(ref[0])
                    idx = order[np.searchsorted(ref[0][order], pk)]
            else:
                idx = np.array([pos[int(k)] for k in pk])
            bad = np.zeros(len(pk), bool)
            for col in range(3):
                bad |= cols[col] != ref[1 + col][idx]
            nb = int(bad.sum())
            n_bad += nb
            if nb:
                print(f"table {tid} partition {p}: {nb} rows differ")
                for i in np.flatnonzero(bad)[:8]:
                    k = int(pk[i])
                    acc = np.flatnonzero((keys == k) & (tables == tid))
                    txns = np.searchsorted(tb, acc, side="right") - 1
                    print("  key", k, "engine", [int(cols[c][i]) for c in range(3)], "oracle",
                          [int(ref[1 + c][idx[i]]) for c in range(3)], "direct accesses by txns", txns.tolist()[:10])
    print("rows differing:", n_bad)
    for eng in engines:
        eng.close()


if __name__ == "__main__":
    main()
