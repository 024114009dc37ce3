"""What one decider of the N > 1 headline decides: an epoch of 1,048,576 txns
made of N origins' batches (1,048,576 / N each, MPR gate, 2 partitions per
multi-partition txn) in Calvin's origin-major order, over the global row space
(N x 16,777,216 rows), on one context -- its stage sizes and time per epoch
(the prefix is the first 1/32 of the sequence, i.e. origin 0's first txns).

    python tools/exp_multiorigin.py [N ...] [--mpr 0.1] [--steps 10]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deneva-plus_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import dvcc  # noqa: E402


def interleave(batches):
    """position-major order: txn j of origin 0, of origin 1, ..., then j + 1"""
    n = len(batches)
    m = batches[0].n_txn
    off = np.cumsum([0] + [int(b.n_acc) for b in batches[:-1]])
    starts = np.stack([b.txn_begin[:m].astype(np.int64) + off[q] for q, b in enumerate(batches)], axis=1).ravel()
    lens = np.stack([np.diff(b.txn_begin.astype(np.int64))[:m] for b in batches], axis=1).ravel()
    tb = np.zeros(n * m + 1, np.int64)
    tb[1:] = np.cumsum(lens)
    idx = np.repeat(starts - tb[:-1], lens) + np.arange(int(tb[-1]))
    allk = np.concatenate([b.keys for b in batches])
    allt = np.concatenate([b.types for b in batches])
    return dvcc.Epoch(allk[idx], allt[idx], tb.astype(np.uint32))


def main():
    args = sys.argv[1:]
    mpr = float(args[args.index("--mpr") + 1]) if "--mpr" in args else 0.1
    steps = int(args[args.index("--steps") + 1]) if "--steps" in args else 10
    ns = [int(x) for x in args if x.isdigit() and (args.index(x) == 0 or args[args.index(x) - 1] not in
                                                    ("--mpr", "--steps"))] or [1, 2, 8]
    rows_pp, total = 16_777_216, 1_048_576
    for n in ns:
        rows = rows_pp * n
        gen = dvcc.YCSBQueryGenerator(rows, part_cnt=n, req_per_query=10, zipf_theta=0.9, txn_write_perc=1.0,
                                      tup_write_perc=0.5, part_per_txn=min(2, n), strict_ppt=1,
                                      mpr=mpr if n > 1 else -1.0)
        eps = []
        for e in range(3):
            batches = [gen.gen(total // n, dvcc.epoch_seed(r, e), r) for r in range(n)]
            eps.append(interleave(batches) if "--interleave" in args else
                       (dvcc.sequence(batches) if n > 1 else batches[0]))
        eng = dvcc.CCEngine(dvcc.NO_WAIT, total, max(e.n_acc for e in eps))
        eng.load_ycsb_partition(rows)
        deps = [dvcc.DeviceEpoch(e) for e in eps]
        d = torch.zeros(total, dtype=torch.uint8, device="cuda")
        eng.run_epochs_device([deps[i % 3] for i in range(3)], d)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sts = eng.run_epochs_device([deps[i % 3] for i in range(steps)], d)
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / steps
        st = sts[-1]
        print(f"N={n} mpr={mpr}{' interleaved' if '--interleave' in args else ''}: {el * 1e3:.3f} ms per decided epoch, committed {st.committed}, prefix "
              f"{st.prefix_txn} txns / {st.prefix_acc} acc, survivors {st.surv_txn} txns / {st.surv_acc} acc, "
              f"rounds {st.rounds}, async {st.async_launches} ({st.async_declined} declined)", flush=True)
        eng.close()
        del deps, eps


if __name__ == "__main__":
    main()
