"""YCSB epoch builder (client query generation + sequencer ordering).

Mirrors YCSBQueryGenerator (benchmarks/ycsb_query.cpp:29-376) through the
host-side generator in libdvcc (dv_ycsb_gen) and Deneva's sequencing rules:
the global lock order of a Calvin epoch is (epoch, origin node, position in
that node's batch) (system/work_queue.cpp:105-151, sequencer.cpp:207-211).
"""
import ctypes

import numpy as np

from . import _lib as L
from .engine import Epoch

SEED = 1  # explicit seed replacing the clock seeds of hazard H2


def epoch_seed(partition, epoch, seed=SEED):
    """myrand seed of (partition, epoch): SEED + 97*partition + epoch."""
    return seed + 97 * partition + epoch


class YCSBQueryGenerator:
    """g_* knobs of the reference (system/global.cpp:65-195, parser.cpp:76-179)."""

    def __init__(self, synth_table_size, part_cnt=1, req_per_query=10, zipf_theta=0.6,
                 txn_write_perc=1.0, tup_write_perc=0.5, part_per_txn=None, strict_ppt=0,
                 mpr=-1.0):
        self.p = L.YcsbParams(synth_table_size, part_cnt, req_per_query, zipf_theta,
                              txn_write_perc, tup_write_perc,
                              part_cnt if part_per_txn is None else part_per_txn, strict_ppt, mpr)

    @property
    def rows_per_part(self):
        return self.p.synth_table_size // self.p.part_cnt

    def gen(self, n_txn, seed, home_part=0):
        R = self.p.req_per_query
        keys = np.zeros(n_txn * R, dtype=np.uint64)
        types = np.zeros(n_txn * R, dtype=np.uint8)
        tb = np.zeros(n_txn + 1, dtype=np.uint32)
        L.check(L.lib().dv_ycsb_gen(ctypes.byref(self.p), seed, home_part, n_txn,
                                    keys.ctypes.data_as(ctypes.c_void_p),
                                    types.ctypes.data_as(ctypes.c_void_p),
                                    tb.ctypes.data_as(ctypes.c_void_p)), "dv_ycsb_gen")
        return Epoch(keys, types, tb)


def sequence(batches):
    """Concatenates per-origin-node batches into one epoch in Calvin lock order:
    node 0's batch, then node 1's, ... (QWorkQueue::sched_dequeue)."""
    keys = np.concatenate([b.keys for b in batches])
    types = np.concatenate([b.types for b in batches])
    sizes = [b.txn_begin[1:] - b.txn_begin[:-1] for b in batches]
    tb = np.zeros(sum(len(s) for s in sizes) + 1, dtype=np.uint32)
    tb[1:] = np.cumsum(np.concatenate(sizes))
    return Epoch(keys, types, tb)


def sequence_position(batches, txns_per_rank=None):
    """The same batches merged txn by txn (DV_COMM_POSITION_ORDER): origin q's
    txn j is sequence number j * P + q, for j < txns_per_rank (default: the
    longest batch); a batch shorter than that leaves empty txns (no accesses,
    they commit) in its slots -- the epoch a position-major epoch group
    decides."""
    P = len(batches)
    tpr = txns_per_rank or max(b.n_txn for b in batches)
    lens = np.zeros((tpr, P), dtype=np.int64)
    starts = np.zeros((tpr, P), dtype=np.int64)
    off = 0
    for q, b in enumerate(batches):
        tb = b.txn_begin.astype(np.int64)
        assert b.n_txn <= tpr, "a batch longer than txns_per_rank"
        lens[:b.n_txn, q] = np.diff(tb)
        starts[:b.n_txn, q] = tb[:-1] + off
        off += int(tb[-1])
    lens, starts = lens.ravel(), starts.ravel()
    tb = np.zeros(tpr * P + 1, dtype=np.int64)
    tb[1:] = np.cumsum(lens)
    idx = np.repeat(starts - tb[:-1], lens) + np.arange(int(tb[-1]))
    keys = np.concatenate([b.keys for b in batches])
    types = np.concatenate([b.types for b in batches])
    return Epoch(keys[idx], types[idx], tb.astype(np.uint32))
