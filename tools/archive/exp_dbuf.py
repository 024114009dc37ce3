"""Double-buffered host input on config D: per-epoch wall time and the
asynchronous-round outcome (yields / declines) with the next epoch's copy in
flight, against the serial path.

    python tools/exp_dbuf.py [epochs]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deneva-plus_amd"))

import torch  # noqa: E402

import dvcc  # noqa: E402


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    rows, n_txn = 16_777_216, 1_048_576
    gen = dvcc.YCSBQueryGenerator(rows, zipf_theta=0.9, txn_write_perc=1.0, tup_write_perc=0.5)
    epochs = [gen.gen(n_txn, dvcc.epoch_seed(0, e)) for e in range(2)]
    eng = dvcc.CCEngine(dvcc.NO_WAIT, n_txn, max(e.n_acc for e in epochs))
    eng.load_ycsb_partition(rows)
    bufs = [(torch.from_numpy(e.to_access_array().view(np.uint8)).pin_memory(),
             torch.from_numpy(np.ascontiguousarray(e.txn_begin, dtype=np.uint32)).pin_memory(), e.n_acc, e.n_txn)
            for e in epochs]
    commit = torch.zeros(n_txn, dtype=torch.uint8).pin_memory()
    eng.run_epoch_host(*bufs[0], commit)
    for i in range(k):
        t0 = time.perf_counter()
        st = eng.run_epoch_host(*bufs[i % 2], commit)
        print(f"serial {i}: {1e3 * (time.perf_counter() - t0):.3f} ms yields {st.async_yields} "
              f"declined {st.async_declined} rounds {st.rounds}", flush=True)
    eng.stage_host(0, *bufs[0])
    for i in range(k):
        t0 = time.perf_counter()
        if i + 1 < k:
            eng.stage_host((i + 1) % 2, *bufs[(i + 1) % 2])
        t1 = time.perf_counter()
        st = eng.run_staged(i % 2, commit)
        t2 = time.perf_counter()
        print(f"staged {i}: stage {1e3 * (t1 - t0):.3f} ms run {1e3 * (t2 - t1):.3f} ms yields {st.async_yields} "
              f"declined {st.async_declined} rounds {st.rounds}", flush=True)
    eng.close()


if __name__ == "__main__":
    main()
