"""TPC-C on the engine (config E): loader, epoch builder and the per-epoch call.

Mirrors TPCCWorkload (benchmarks/tpcc_wl.cpp), TPCCQueryGenerator
(tpcc_query.cpp:26-263) and TPCCTxnManager's Payment / NewOrder
(tpcc_txn.cpp:117-244, 500-933) through libdvcc (dv_tpcc_*).  Decisions and
table state equal one worker thread running the epoch in sequence order
(SURVEY.md 8.0); inserted ORDER / NEW_ORDER / ORDER_LINE rows are determined by
the query, the commit byte and the o_id this path returns.
"""
import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib as L
from .engine import CCEngine, DeviceEpoch, Epoch, _ptr

TABLES = {"WAREHOUSE": L.T_WAREHOUSE, "DISTRICT": L.T_DISTRICT, "CUSTOMER": L.T_CUSTOMER,
          "ITEM": L.T_ITEM, "STOCK": L.T_STOCK, "CUST_LAST": L.T_CUST_LAST}


def tpcc_params(num_wh, dist_per_wh=10, cust_per_dist=3000, max_items=100000, max_items_per_txn=15,
                part_cnt=1, part_per_txn=2, wh_update=1, perc_payment=0.5, mpr=1.0):
    """g_* knobs (config.h:181-223; config E: PERC_PAYMENT 0.5, MPR 1.0)."""
    return L.TpccParams(num_wh, dist_per_wh, cust_per_dist, max_items, max_items_per_txn, part_cnt,
                        part_per_txn, wh_update, perc_payment, mpr)


@dataclass
class TpccEpoch(Epoch):
    args: np.ndarray = None      # uint64 [n_acc] op << 56 | operand
    txn_type: np.ndarray = None  # uint8 [n_txn] 1 Payment, 2 NewOrder
    owner: np.ndarray = None     # uint8 [n_acc] partition that runs the access


def table_rows(p, table, part_id=0):
    n = ctypes.c_uint64()
    L.check(L.lib().dv_tpcc_table_rows(ctypes.byref(p), part_id, table, ctypes.byref(n)), "dv_tpcc_table_rows")
    return n.value


def table(p, seed, table_id, part_id=0):
    """keys and the three state columns of one table as loaded (dv_tpcc_table)."""
    n = table_rows(p, table_id, part_id)
    out = [np.zeros(n, dtype=np.uint64) for _ in range(4)]
    L.check(L.lib().dv_tpcc_table(ctypes.byref(p), seed, part_id, table_id, *[_ptr(a) for a in out]),
            "dv_tpcc_table")
    return out


def gen(p, n_txn, seed, home_part=0):
    cap = n_txn * (3 + 2 * p.max_items_per_txn)
    keys = np.zeros(cap, dtype=np.uint64)
    types = np.zeros(cap, dtype=np.uint8)
    tables = np.zeros(cap, dtype=np.uint8)
    args = np.zeros(cap, dtype=np.uint64)
    tb = np.zeros(n_txn + 1, dtype=np.uint32)
    tt = np.zeros(n_txn, dtype=np.uint8)
    own = np.zeros(cap, dtype=np.uint8)
    L.check(L.lib().dv_tpcc_gen(ctypes.byref(p), seed, home_part, n_txn, _ptr(keys), _ptr(types),
                                _ptr(tables), _ptr(args), _ptr(tb), _ptr(tt), _ptr(own)), "dv_tpcc_gen")
    n = int(tb[-1])
    return TpccEpoch(keys[:n].copy(), types[:n].copy(), tb, tables[:n].copy(), args[:n].copy(), tt,
                     own[:n].copy())


class TpccEngine(CCEngine):
    """A DV_TPCC context: the six tables of one partition in HBM."""

    def __init__(self, cc_alg, params, max_txn, device=0, part_id=0, seed=1, **kw):
        max_acc = max_txn * (3 + 2 * params.max_items_per_txn)
        super().__init__(cc_alg, max_txn, max_acc, device=device, part_cnt=params.part_cnt,
                         part_id=part_id, workload=L.TPCC, **kw)
        self.params = params
        L.check(L.lib().dv_tpcc_load(self._ctx, ctypes.byref(params), seed), "dv_tpcc_load")

    def read_col(self, table_id, col, first=0, n=None):
        if n is None:
            n = table_rows(self.params, table_id, self.part_id) - first
        out = np.zeros(n, dtype=np.uint64)
        L.check(L.lib().dv_read_table_col(self._ctx, table_id, col, first, n, _ptr(out)), "dv_read_table_col")
        return out

    def begin_tpcc(self, dep, d_args, d_oid=None):
        """Staged form (partitioned epochs): rounds and finish as CCEngine's."""
        self._after_torch()
        self._desc = dep.desc()
        self._keep = (d_args, d_oid)  # alive until finish
        L.check(L.lib().dv_tpcc_epoch_begin(self._ctx, ctypes.byref(self._desc), _ptr(d_args), _ptr(d_oid)),
                "dv_tpcc_epoch_begin")

    def run_tpcc_epoch_device(self, dep, d_args, d_commit, d_oid=None):
        self._after_torch()
        st = L.Stats()
        L.check(L.lib().dv_tpcc_epoch_run_device(self._ctx, ctypes.byref(dep.desc()), _ptr(d_args),
                                                 _ptr(d_commit), _ptr(d_oid), ctypes.byref(st)),
                "dv_tpcc_epoch_run_device")
        return st


    def run_tpcc_epochs_device(self, deps, d_args, d_commits=None, d_oids=None, lanes=None):
        """Several TPC-C epochs back to back (dv_tpcc_epoch_run_device_batch):
        epoch k+1 is queued before epoch k is read back.  deps / d_args: one
        DeviceEpoch and operation-word tensor per epoch; d_commits / d_oids:
        one device tensor per epoch, one tensor for all, or None.  lanes:
        decision lanes (open_lane) -- dv_tpcc_epoch_run_device_lanes over
        [self] + lanes.  Returns the list of stats."""
        ctxs = [self] + list(lanes or [])
        for e in ctxs:
            e._after_torch()
        n = len(deps)

        def ptrs(x):
            if x is None:
                return None
            xs = x if isinstance(x, (list, tuple)) else [x] * n
            return (ctypes.c_void_p * n)(*[_ptr(t) for t in xs])
        descs = (L.EpochDev * n)(*[d.desc() for d in deps])
        args = ptrs(list(d_args))
        sts = (L.Stats * n)()
        self._keep = (deps, d_args, d_commits, d_oids)
        if len(ctxs) > 1:
            lp = (ctypes.c_void_p * len(ctxs))(*[e._ctx.value for e in ctxs])
            L.check(L.lib().dv_tpcc_epoch_run_device_lanes(lp, len(ctxs), descs, args, n, ptrs(d_commits),
                                                           ptrs(d_oids), sts), "dv_tpcc_epoch_run_device_lanes")
        else:
            L.check(L.lib().dv_tpcc_epoch_run_device_batch(self._ctx, descs, args, n, ptrs(d_commits),
                                                           ptrs(d_oids), sts), "dv_tpcc_epoch_run_device_batch")
        return list(sts)

    def run_tpcc_epoch_part(self, home, d_args, d_owner, txns_per_rank, d_commit, d_oid=None):
        """Config E from the engine (dv_tpcc_epoch_run_part): this rank's
        client batch `home` (DeviceEpoch), its operation words and owner
        bytes; d_commit / d_oid sized for the global epoch (ranks x
        txns_per_rank), d_oid equal on every rank afterwards."""
        self._after_torch()
        st = L.Stats()
        L.check(L.lib().dv_tpcc_epoch_run_part(self._ctx, ctypes.byref(home.desc()), _ptr(d_args), _ptr(d_owner),
                                               txns_per_rank, _ptr(d_commit), _ptr(d_oid), ctypes.byref(st)),
                "dv_tpcc_epoch_run_part")
        return st


def device_epoch(e, device="cuda"):
    """(DeviceEpoch, args tensor) of a TpccEpoch."""
    import torch
    dep = DeviceEpoch(e, device)
    return dep, torch.from_numpy(e.args.view(np.int64)).to(device)
