"""Host-side mirror of Deneva's CC plugin surface over the HIP engine.

`CCEngine` is what a workload driver calls once per epoch instead of calling
Row_lock::lock_get/lock_release, OptCC::validate/finish, Row_occ and
IndexHash::index_read once per access (concurrency_control/row_lock.cpp:52-373,
occ.cpp:42-294, row_occ.cpp:33-79, storage/index_hash.cpp:137-153).  Return
values keep the reference's meaning: commit byte 1 == RCOK/Commit, 0 == Abort.

Everything here is plumbing around libdvcc.so: no decision is computed in
Python, and nothing falls back to the CPU.
"""
import ctypes
import os
import sys
import time
from dataclasses import dataclass

import numpy as np

from . import _lib as L


def _ptr(a):
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data_as(ctypes.c_void_p)
    return ctypes.c_void_p(int(a.data_ptr()))  # torch tensor (device memory)


def comm_unique_id():
    """A fresh RCCL unique id (128 bytes) for dv_comm_init; make it on rank 0
    and hand it to the other ranks."""
    buf = ctypes.create_string_buffer(128)
    L.check(L.lib().dv_comm_unique_id(buf), "dv_comm_unique_id")
    return buf.raw


@dataclass
class Epoch:
    """One host-side epoch in sequence order."""
    keys: np.ndarray       # uint64 [n_acc]
    types: np.ndarray      # uint8  [n_acc] RD/WR/SCAN
    txn_begin: np.ndarray  # uint32 [n_txn+1]
    tables: np.ndarray = None  # uint8 [n_acc] or None (all table 0)

    @property
    def n_txn(self):
        return len(self.txn_begin) - 1

    @property
    def n_acc(self):
        return int(self.txn_begin[-1])

    def max_txn_acc(self):
        return int(np.diff(self.txn_begin.astype(np.int64)).max()) if self.n_txn else 0

    def acc_txn(self):
        counts = np.diff(self.txn_begin.astype(np.int64))
        return np.repeat(np.arange(self.n_txn, dtype=np.uint32), counts)

    def to_row_records(self):
        """4-byte records for dv_epoch_stage_host_rows: key | write << 31
        (table 0 reads / writes, keys below 2^31)"""
        if self.n_acc and (int(self.keys.max()) >> 31 or (self.types > 1).any()
                           or (self.tables is not None and self.tables.any())):
            raise ValueError("4-byte records hold table-0 reads / writes of keys below 2^31")
        return (self.keys.astype(np.uint32) | (self.types.astype(np.uint32) << 31)).astype(np.uint32)

    def to_access_array(self):
        a = np.zeros(self.n_acc, dtype=[("key", "<u8"), ("txn_seq", "<u4"), ("type", "u1"),
                                        ("table", "u1"), ("flags", "<u2")])
        a["key"] = self.keys
        a["txn_seq"] = self.acc_txn()
        a["type"] = self.types
        if self.tables is not None:
            a["table"] = self.tables
        return a


# DVCC_PY_PROF=1: the lanes wrapper's own time around the C call, to stderr
_PY_PROF = bool(os.environ.get("DVCC_PY_PROF"))


class DeviceEpoch:
    """An epoch resident in HBM (torch tensors used as device buffers)."""

    def __setattr__(self, name, value):
        # every public attribute set bumps the version the descriptor cache
        # (desc, desc_bytes) is keyed on
        object.__setattr__(self, name, value)
        if name[0] != "_":
            object.__setattr__(self, "_ver", self.__dict__.get("_ver", 0) + 1)

    def __init__(self, epoch, device="cuda", txn_begin=True, recs32=True):
        import torch
        self.n_txn = epoch.n_txn
        self.n_acc = epoch.n_acc
        self.max_txn_acc = epoch.max_txn_acc()
        self.keys = torch.from_numpy(epoch.keys.view(np.int64)).to(device)
        self.types = torch.from_numpy(epoch.types).to(device)
        self.acc_txn = torch.from_numpy(epoch.acc_txn().view(np.int32)).to(device)
        self.tables = (torch.from_numpy(epoch.tables).to(device)
                       if epoch.tables is not None else None)
        # the txns' boundaries too (dv_epoch_dev.txn_begin): a prefix-kill
        # epoch then reads ranges from them (acc_txn stays, other paths read it)
        self.txn_begin = torch.from_numpy(epoch.txn_begin.astype(np.int32)).to(device) if txn_begin else None
        # ... and its accesses as 4-byte records (key | write << 31) where they
        # fit one (dv_epoch_dev::recs32: table-0 reads / writes, keys < 2^31)
        self.recs32 = None
        if txn_begin and recs32:
            try:
                self.recs32 = torch.from_numpy(epoch.to_row_records().view(np.int32)).to(device)
            except ValueError:
                pass
        # every txn id below the last one used has an access (what the compact
        # epoch-group batches need, dv_epoch_group_run); None = unknown
        n = np.diff(epoch.txn_begin.astype(np.int64))
        used = np.flatnonzero(n)
        self.dense = bool(used.size == 0 or (n[:used[-1] + 1] > 0).all())

    @classmethod
    def from_tensors(cls, keys, types, acc_txn, n_txn, tables=None, max_txn_acc=0):
        """max_txn_acc: bound on one txn's accesses (0 = unknown, the engine
        then assumes the 128-access maximum)."""
        self = cls.__new__(cls)
        self.keys, self.types, self.acc_txn, self.tables = keys, types, acc_txn, tables
        self.txn_begin = self.recs32 = None
        self.n_acc = int(keys.numel())
        self.n_txn = int(n_txn)
        self.max_txn_acc = int(max_txn_acc)
        self.dense = None
        return self

    @classmethod
    def concat(cls, first, second):
        """`first`'s txns, then `second`'s (renumbered after them): the next
        epoch of the abort carry-over, carried txns ahead of the new ones."""
        import torch
        tabs = None
        if first.tables is not None or second.tables is not None:
            tabs = torch.cat([t.tables if t.tables is not None
                              else torch.zeros_like(t.types) for t in (first, second)])
        return cls.from_tensors(torch.cat([first.keys, second.keys]),
                                torch.cat([first.types, second.types]),
                                torch.cat([first.acc_txn, second.acc_txn + first.n_txn]),
                                first.n_txn + second.n_txn, tables=tabs,
                                max_txn_acc=max(first.max_txn_acc, second.max_txn_acc))

    def desc(self):
        """the dv_epoch_dev of these buffers (kept until an attribute is set
        again: the pipelined entry points take one per epoch, and data_ptr()
        is a few microseconds a call)"""
        memo = self.__dict__.get("_desc_memo")
        if memo is not None and memo[0] == self._ver:
            return memo[1]
        ts = getattr(self, "ts", None)
        tb = getattr(self, "txn_begin", None)
        r32 = getattr(self, "recs32", None)
        d = L.EpochDev(self.keys.data_ptr(), self.types.data_ptr(), self.acc_txn.data_ptr(),
                       self.tables.data_ptr() if self.tables is not None else None,
                       self.n_acc, self.n_txn, self.max_txn_acc, ts.data_ptr() if ts is not None else None,
                       None, tb.data_ptr() if tb is not None else None, r32.data_ptr() if r32 is not None else None)
        self._desc_memo = (self._ver, d, bytes(d))
        return d

    def desc_bytes(self):
        """desc() as bytes (cached the same way)"""
        memo = self.__dict__.get("_desc_memo")
        if memo is None or memo[0] != self._ver:
            self.desc()
            memo = self._desc_memo
        return memo[2]


class ClosedLoopBufs:
    """The closed loop's two epoch buffers (dv_epoch_run_closed_loop).  With
    n_txn (and no table bytes) they also hold the tb form -- 4-byte records and
    txn boundaries -- which the refill then writes instead of keys / types /
    txn ids when the pool has records too (the engine's tb-mode path)."""

    def __init__(self, cap, tables, device, n_txn=None):
        import torch
        self.cap = int(cap)
        n = max(1, self.cap)
        self.keys = [torch.empty(n, dtype=torch.int64, device=device) for _ in range(2)]
        self.types = [torch.empty(n, dtype=torch.uint8, device=device) for _ in range(2)]
        self.acc_txn = [torch.empty(n, dtype=torch.int32, device=device) for _ in range(2)]
        self.tables = [torch.empty(n, dtype=torch.uint8, device=device) for _ in range(2)] if tables else None
        self.n_acc = [torch.zeros(1, dtype=torch.int32, device=device) for _ in range(2)]
        tb = n_txn is not None and not tables
        self.recs32 = [torch.empty(n, dtype=torch.int32, device=device) for _ in range(2)] if tb else None
        self.txn_begin = ([torch.zeros(int(n_txn) + 1, dtype=torch.int32, device=device) for _ in range(2)]
                          if tb else None)
        self.tb = False  # (set by the engine: the last call wrote the tb form)

    def desc(self, b):
        return L.EpochDev(self.keys[b].data_ptr(), self.types[b].data_ptr(), self.acc_txn[b].data_ptr(),
                          self.tables[b].data_ptr() if self.tables is not None else None, 0, 0, 0, None,
                          self.n_acc[b].data_ptr(),
                          self.txn_begin[b].data_ptr() if self.txn_begin is not None else None,
                          self.recs32[b].data_ptr() if self.recs32 is not None else None)

    def swap(self):
        """after a call of n_epochs odd: the next epoch moves to buffer 0"""
        for a in (self.keys, self.types, self.acc_txn, self.tables, self.n_acc, self.recs32, self.txn_begin):
            if a is not None:
                a.reverse()

    def epoch(self, b, n_txn, max_txn_acc):
        """buffer b's epoch as a DeviceEpoch (reads its access count)"""
        import torch
        n = int(self.n_acc[b].item())
        if self.tb:  # (keys / types / txn ids from the tb form)
            r = self.recs32[b][:n].to(torch.int64) & 0xFFFFFFFF
            keys = r & 0x7FFFFFFF
            types = (r >> 31).to(torch.uint8)
            tb = self.txn_begin[b][:n_txn + 1].to(torch.int64)
            acc_txn = torch.repeat_interleave(torch.arange(n_txn, device=keys.device, dtype=torch.int32),
                                              tb[1:] - tb[:-1])
            return DeviceEpoch.from_tensors(keys, types, acc_txn, n_txn, max_txn_acc=max_txn_acc)
        return DeviceEpoch.from_tensors(self.keys[b][:n], self.types[b][:n], self.acc_txn[b][:n], n_txn,
                                        tables=self.tables[b][:n] if self.tables is not None else None,
                                        max_txn_acc=max_txn_acc)


def _loop_tb(pool, bufs):
    """dv_epoch_run_closed_loop writes the tb form (loop_tb, dvcc_runtime.hip)"""
    import os
    return (not os.environ.get("DVCC_LOOP_NO_TB") and getattr(pool, "recs32", None) is not None
            and pool.tables is None and all(b.recs32 is not None for b in bufs))


def _commit_ptrs(d_commits, n):
    """the n commit-byte pointers: one device tensor (or None) for every
    epoch, or a list of them"""
    if d_commits is None or not isinstance(d_commits, (list, tuple)):
        p = int(d_commits.data_ptr()) if d_commits is not None else None
        return (ctypes.c_void_p * n)(*([p] * n))
    return (ctypes.c_void_p * n)(*[(int(t.data_ptr()) if t is not None else None) for t in d_commits])


def _after_torch_all(engines):
    """CCEngine._after_torch for several contexts: one event recorded on
    torch's current stream, every other context's stream waits on it"""
    import sys
    torch = sys.modules.get("torch")
    if torch is None or not torch.cuda.is_initialized():
        return
    cur = torch.cuda.current_stream()
    if cur.query():  # (nothing queued on it is unfinished: its results are visible to any later launch)
        return
    ev = None
    for e in engines:
        sp = e.stream_ptr or 0
        if sp == cur.cuda_stream:
            continue
        if ev is None:
            ev = getattr(engines[0], "_ev_all", None)
            if ev is None:
                ev = engines[0]._ev_all = torch.cuda.Event()
            ev.record(cur)
        if getattr(e, "_ext", None) is None or e._ext.cuda_stream != sp:
            e._ext = torch.cuda.ExternalStream(sp)
        e._ext.wait_event(ev)


class CCEngine:
    """One context = one GPU (one process per GPU)."""

    def __init__(self, cc_alg, max_txn, max_acc, device=0, part_cnt=1, part_id=0, timing=False,
                 workload=L.YCSB, tail=True, el64=False, asynchronous=True, lsd_sort=False):
        """tail=False keeps every decision round in the multi-workgroup pass
        (no single-workgroup tail kernel); el64=True forces 64-bit round
        elements; asynchronous=False never finishes the rounds in the
        asynchronous kernel; lsd_sort=True sorts with the plain LSD passes
        (no bucket sort of small sorts).  Decisions are the same either way
        (testing knobs)."""
        if isinstance(cc_alg, str):
            cc_alg = L.CC_NAMES[cc_alg.upper()]
        self.cc_alg = cc_alg
        self.part_cnt, self.part_id = part_cnt, part_id
        self.max_txn, self.max_acc = max_txn, max_acc
        # timing: True = per-stage events, "kernel" = only the scatter / pass
        # launches' own dispatch timestamps (no marker packets between kernels)
        tflag = L.FLAG_KERNEL_TIMING if timing == "kernel" else (L.FLAG_TIMING if timing else 0)
        flags = (tflag | (0 if tail else L.FLAG_NO_TAIL)
                 | (L.FLAG_EL64 if el64 else 0) | (0 if asynchronous else L.FLAG_NO_ASYNC)
                 | (L.FLAG_LSD_SORT if lsd_sort else 0))
        cfg = L.Config(device, cc_alg, workload, part_cnt, part_id, max_txn, max_acc, flags, 0)
        self._ctx = ctypes.c_void_p()
        L.check(L.lib().dv_open(ctypes.byref(self._ctx), ctypes.byref(cfg)), "dv_open")

    def close(self):
        for lane in getattr(self, "_lanes", []):  # (a lane closes before its owner)
            lane.close()
        self._lanes = []
        if self._ctx:
            L.lib().dv_close(self._ctx)
            self._ctx = ctypes.c_void_p()
        self._owner = None

    def open_lane(self):
        """A decision lane (dv_open_lane): a second context of the same
        configuration over this engine's tables (loaded first; frozen while
        lanes are open).  Closed with, or before, this engine."""
        lane = type(self).__new__(type(self))
        lane.__dict__.update({k: v for k, v in self.__dict__.items() if k not in ("_ctx", "_lanes", "_ev", "_ext")})
        lane._ctx = ctypes.c_void_p()
        L.check(L.lib().dv_open_lane(self._ctx, ctypes.byref(lane._ctx)), "dv_open_lane")
        lane._owner, lane._lanes = self, []
        if not hasattr(self, "_lanes"):
            self._lanes = []
        self._lanes.append(lane)
        return lane

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream_ptr(self):
        return L.lib().dv_stream(self._ctx)

    def _after_torch(self):
        """Orders the engine's stream after the work torch has queued on its
        current stream: device epochs built by torch kernels (cat, slices,
        arithmetic) are inputs of the next launch, and the context's own
        stream is non-blocking, so without this wait it can read them early
        (no host synchronisation: an event record + stream wait)."""
        import sys
        torch = sys.modules.get("torch")
        if torch is None or not torch.cuda.is_initialized():
            return
        cur = torch.cuda.current_stream()
        sp = self.stream_ptr or 0
        if sp == cur.cuda_stream:
            return
        if getattr(self, "_ev", None) is None:
            self._ev = torch.cuda.Event()
            self._ext = torch.cuda.ExternalStream(sp)
        elif self._ext.cuda_stream != sp:
            self._ext = torch.cuda.ExternalStream(sp)
        self._ev.record(cur)
        self._ext.wait_event(self._ev)

    def set_stream(self, stream):
        """Run on the hipStream_t handle `stream` (an int such as
        torch.cuda.current_stream().cuda_stream; 0 is the default stream);
        None returns to the context's own stream."""
        if stream is None:
            stream = L.lib().dv_own_stream(self._ctx)
        L.check(L.lib().dv_set_stream(self._ctx, stream), "dv_set_stream")

    def set_async_limits(self, max_iters=0, idle_us=0):
        """Asynchronous rounds: a workgroup yields after max_iters iterations
        or idle_us without a decision (0 = defaults); testing knob."""
        L.check(L.lib().dv_set_async_limits(self._ctx, max_iters, idle_us), "dv_set_async_limits")

    def set_prefix(self, prefix_txns=0):
        """Prefix-kill decisions (dv_set_prefix): 0 automatic, None off, or
        the prefix size in txns."""
        v = 0xFFFFFFFF if prefix_txns is None else int(prefix_txns)
        L.check(L.lib().dv_set_prefix(self._ctx, v), "dv_set_prefix")

    def set_timing(self, timing, profile=False):
        """Between epochs: True = per-stage events, "kernel" = only the scatter
        and pass launches' dispatch timestamps, False = none; profile=True
        also times every launch on its own (kernel_times)."""
        flag = L.FLAG_KERNEL_TIMING if timing == "kernel" else (L.FLAG_TIMING if timing else 0)
        L.check(L.lib().dv_set_timing(self._ctx, flag | (L.FLAG_KERNEL_PROFILE if profile else 0)),
                "dv_set_timing")

    def kernel_times(self, reset=True):
        """{kernel name: (launches, total ms)} of the launches timed while
        set_timing(..., profile=True) was on (dv_kernel_times)."""
        cap = 128
        arr = (L.KernelTime * cap)()
        n = L.lib().dv_kernel_times(self._ctx, arr, cap, 1 if reset else 0)
        if n < 0:
            L.check(n, "dv_kernel_times")
        return {arr[i].name.decode(): (int(arr[i].launches), float(arr[i].ms_total)) for i in range(min(n, cap))}

    # ---- storage (Workload::init_schema / init_table; IndexHash::index_insert)
    def load_ycsb_partition(self, rows_per_part):
        L.check(L.lib().dv_load_ycsb_partition(self._ctx, rows_per_part), "dv_load_ycsb_partition")

    def create_table(self, table, capacity_rows, nbuckets, hash_kind=L.HASH_MOD):
        L.check(L.lib().dv_create_table(self._ctx, table, capacity_rows, nbuckets, hash_kind),
                "dv_create_table")

    def load_table(self, table, keys, f0=None):
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        f0 = None if f0 is None else np.ascontiguousarray(f0, dtype=np.uint64)
        L.check(L.lib().dv_load_table(self._ctx, table, _ptr(keys), _ptr(f0), len(keys)),
                "dv_load_table")

    def read_table(self, first_row, n, table=0):
        out = np.zeros(n, dtype=np.uint64)
        L.check(L.lib().dv_read_table(self._ctx, table, first_row, n, _ptr(out)), "dv_read_table")
        return out

    def read_rows(self, keys, table=0):
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        out = np.zeros(len(keys), dtype=np.uint64)
        L.check(L.lib().dv_read_rows(self._ctx, table, _ptr(keys), len(keys), _ptr(out)),
                "dv_read_rows")
        return out

    # ---- one epoch from host buffers
    def run_epoch(self, epoch, want_grant=False):
        acc = epoch.to_access_array()
        tb = np.ascontiguousarray(epoch.txn_begin, dtype=np.uint32)
        commit = np.zeros(max(1, epoch.n_txn), dtype=np.uint8)
        grant = np.zeros(max(1, epoch.n_acc), dtype=np.uint32) if want_grant else None
        st = L.Stats()
        L.check(L.lib().dv_epoch_run(self._ctx, _ptr(acc), epoch.n_acc, _ptr(tb), epoch.n_txn,
                                     None, _ptr(commit), _ptr(grant), ctypes.byref(st)),
                "dv_epoch_run")
        return commit[:epoch.n_txn], (grant[:epoch.n_acc] if want_grant else None), st

    def run_epoch_host(self, acc, tb, n_acc, n_txn, commit):
        """dv_epoch_run on prebuilt host buffers (any objects _ptr accepts:
        numpy arrays or pinned torch tensors): 16-B access records, txn_begin,
        and the commit-byte output.  Returns the stats."""
        st = L.Stats()
        L.check(L.lib().dv_epoch_run(self._ctx, _ptr(acc), n_acc, _ptr(tb), n_txn, None, _ptr(commit),
                                     None, ctypes.byref(st)), "dv_epoch_run")
        return st

    def stage_host(self, slot, acc, tb, n_acc, n_txn):
        """dv_epoch_stage_host: queue the H2D copy of host records (pinned
        for an asynchronous copy) into staging slot 0 / 1."""
        L.check(L.lib().dv_epoch_stage_host(self._ctx, slot, _ptr(acc), n_acc, _ptr(tb), n_txn),
                "dv_epoch_stage_host")

    def stage_host_rows(self, slot, row_wr, tb, n_acc, n_txn):
        """dv_epoch_stage_host_rows: the same from 4-byte records (key |
        write << 31, table 0, keys below 2^31) and txn_begin."""
        L.check(L.lib().dv_epoch_stage_host_rows(self._ctx, slot, _ptr(row_wr), n_acc, _ptr(tb), n_txn),
                "dv_epoch_stage_host_rows")

    def run_staged(self, slot, commit):
        """dv_epoch_run_staged: run the epoch in `slot`; commit bytes to host."""
        st = L.Stats()
        L.check(L.lib().dv_epoch_run_staged(self._ctx, slot, None, _ptr(commit), None, ctypes.byref(st)),
                "dv_epoch_run_staged")
        return st

    # ---- one epoch already resident in HBM
    def run_epoch_device(self, dep, d_commit=None, d_grant=None):
        st = L.Stats()
        self._after_torch()
        desc = dep.desc()
        L.check(L.lib().dv_epoch_run_device(self._ctx, ctypes.byref(desc), _ptr(d_commit),
                                            _ptr(d_grant), ctypes.byref(st)), "dv_epoch_run_device")
        return st

    def run_epochs_device(self, deps, d_commits=None):
        """Several epochs back to back (dv_epoch_run_device_batch): epoch
        k+1 is queued before epoch k's outcome is read.  d_commits: one device
        tensor (or None) per epoch, or one tensor for all.  Returns the list of
        stats."""
        self._after_torch()
        n = len(deps)
        arr = self._epoch_array(deps)
        cps = _commit_ptrs(d_commits, n)
        sts = (L.Stats * n)()
        L.check(L.lib().dv_epoch_run_device_batch(self._ctx, arr, n, cps, sts), "dv_epoch_run_device_batch")
        return list(sts)

    def lanes_order(self, lanes):
        """dv_lanes_order over [self] + lanes: each on its own CU-masked
        stream, and their epoch groups (run_epoch_group / run_epoch_groups,
        each lane from its own host thread, group g on lane g % len) executed
        in group order across them.  lanes=[]: this engine alone again."""
        ctxs = [self] + list(lanes)
        if len(ctxs) == 1 and getattr(self, "_order", None):
            # every lane of the previous order alone again too (its CU-masked
            # stream and the shared order released), so it can be ordered anew
            for e in self._order[1:]:
                one = (ctypes.c_void_p * 1)(e._ctx.value)
                L.check(L.lib().dv_lanes_order(one, 1), "dv_lanes_order")
        lp = (ctypes.c_void_p * len(ctxs))(*[e._ctx.value for e in ctxs])
        L.check(L.lib().dv_lanes_order(lp, len(ctxs)), "dv_lanes_order")
        self._order = ctxs if len(ctxs) > 1 else None
        self._order_next = 0  # the lane of the next group (tickets continue across calls)

    def run_ordered(self, n, call):
        """n epochs over the ordered lanes (lanes_order) for the per-epoch
        partitioned drivers: epoch i of the call on lane (epochs so far + i)
        % L, each lane from its own host thread running call(ctx, i) for its
        epochs in order (e.g. ctx.run_epoch_part / ctx.run_tpcc_epoch_part);
        executions in epoch order.  Returns the list of call results; raises
        the first lane's error."""
        import threading
        ctxs = self._order
        nl = len(ctxs)
        base = self._order_next
        out, errs = [None] * n, []

        def body(ln):
            try:
                for i in range(n):
                    if (base + i) % nl == ln:
                        out[i] = call(ctxs[ln], i)
            except Exception as ex:  # noqa: BLE001 -- re-raised below
                errs.append(ex)
        th = [threading.Thread(target=body, args=(ln,)) for ln in range(nl)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        self._order_next = (base + n) % nl
        if errs:
            errs.sort(key=lambda e: getattr(e, "code", 0) == L.DV_ERR_STATE)
            raise errs[0]
        return out

    def run_epoch_groups_ordered(self, groups, txns_per_rank, d_commits=None):
        """Epoch groups over the ordered lanes (lanes_order): group i of the
        call on lane (groups so far + i) % L, every lane from its own host
        thread (dv_epoch_group_run_batch over its groups), executions in
        group order.  d_commits: one device tensor (or None) per group.
        Returns the list of stats; raises the first lane's error."""
        import threading
        ctxs = self._order
        n, nl = len(groups), len(ctxs)
        if d_commits is None or not isinstance(d_commits, (list, tuple)):
            d_commits = [d_commits] * n
        base = self._order_next
        out, errs = [None] * n, []

        def body(ln):
            mine = [i for i in range(n) if (base + i) % nl == ln]
            if not mine:
                return
            try:
                sts = ctxs[ln].run_epoch_groups([groups[i] for i in mine], txns_per_rank,
                                                [d_commits[i] for i in mine])
                for i, st in zip(mine, sts):
                    out[i] = st
            except Exception as ex:  # noqa: BLE001 -- re-raised below
                errs.append(ex)
        th = [threading.Thread(target=body, args=(ln,)) for ln in range(nl)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        self._order_next = (base + n) % nl
        if errs:  # (the failing group's own error first; the others stopped behind it)
            errs.sort(key=lambda e: getattr(e, "code", 0) == L.DV_ERR_STATE)
            raise errs[0]
        return out

    @staticmethod
    def _epoch_array(deps):
        """the dv_epoch_dev array of `deps` (DeviceEpoch: one copy of the
        descriptors' cached bytes)"""
        n = len(deps)
        if all(isinstance(d, DeviceEpoch) for d in deps):
            return (L.EpochDev * n).from_buffer_copy(b"".join([d.desc_bytes() for d in deps]))
        return (L.EpochDev * n)(*[d.desc() for d in deps])

    def run_epochs_lanes(self, lanes, deps, d_commits=None):
        """dv_epoch_run_device_lanes over [self] + lanes (open_lane):
        epoch k decided on context k % len, executions in epoch order; same
        results as run_epochs_device.  Returns the list of stats."""
        prof = _PY_PROF and time.perf_counter()
        ctxs = [self] + list(lanes)
        _after_torch_all(ctxs)
        t_ev = _PY_PROF and time.perf_counter()
        n = len(deps)
        arr = self._epoch_array(deps)
        cps = _commit_ptrs(d_commits, n)
        sts = (L.Stats * n)()
        lp = (ctypes.c_void_p * len(ctxs))(*[e._ctx.value for e in ctxs])
        t1 = _PY_PROF and time.perf_counter()
        L.check(L.lib().dv_epoch_run_device_lanes(lp, len(ctxs), arr, n, cps, sts), "dv_epoch_run_device_lanes")
        t_ret = _PY_PROF and time.perf_counter()
        out = list(sts)
        if _PY_PROF:
            t2 = time.perf_counter()
            print(f"dvcc python: {n} epochs over {len(ctxs)} lanes, {(t1 - prof) * 1e6:.1f} us before the call "
                  f"({(t_ev - prof) * 1e6:.1f} ordering after torch), {(t_ret - t1) * 1e6:.1f} us in it, "
                  f"{(t2 - t_ret) * 1e6:.1f} after", file=sys.stderr)
        return out

    # ---- partitioned epochs over RCCL from the engine (dv_comm_init)
    def comm_init(self, unique_id, nranks, rank):
        """unique_id: the 128 bytes comm_unique_id() returned on rank 0."""
        buf = ctypes.create_string_buffer(bytes(unique_id), 128)
        L.check(L.lib().dv_comm_init(self._ctx, buf, nranks, rank), "dv_comm_init")

    @staticmethod
    def comm_init_local(engines):
        """Partitioned epochs among engines of this process (engine q owns
        partition q), e.g. several partitions on one GPU: drive each engine's
        run_epoch_part from its own thread."""
        arr = (ctypes.c_void_p * len(engines))(*[e._ctx.value for e in engines])
        L.check(L.lib().dv_comm_init_local(arr, len(engines)), "dv_comm_init_local")

    def comm_init_ipc(self, name, nranks, rank):
        """Partitioned epochs among PROCESSES of this node (dv_comm_init_ipc):
        every rank passes the same fresh shared-memory name ("/...")."""
        L.check(L.lib().dv_comm_init_ipc(self._ctx, name.encode(), nranks, rank), "dv_comm_init_ipc")

    def comm_set_mode(self, mode):
        """dv_comm_set_mode: 0 automatic, 1 list protocol, 2 replicated when
        possible; | DV_COMM_WIDE_BATCHES (8-byte group batches), |
        DV_COMM_POSITION_ORDER (epoch groups sequenced position-major,
        dvcc.sequence_position)."""
        L.check(L.lib().dv_comm_set_mode(self._ctx, mode), "dv_comm_set_mode")
        self._comm_mode = mode

    def _wide_for(self, batches):
        """Epoch groups move compact 4-byte batches only when every rank's txn
        ids are dense; a batch with an empty txn in the middle would fail the
        group (DV_ERR_ARG).  Such a batch switches this rank to the 8-byte
        form for the call -- the group's vote then takes it on every rank, so
        the results are the same -- and the previous mode is returned."""
        mode = getattr(self, "_comm_mode", 0)
        if mode & L.DV_COMM_WIDE_BATCHES or all(getattr(b, "dense", None) is not False for b in batches):
            return None
        L.check(L.lib().dv_comm_set_mode(self._ctx, mode | L.DV_COMM_WIDE_BATCHES), "dv_comm_set_mode")
        return mode

    def run_epoch_part(self, home, txns_per_rank, d_commit=None):
        """One partitioned epoch from this rank's client batch (DeviceEpoch,
        txn ids local); d_commit: nranks * txns_per_rank device bytes."""
        self._after_torch()
        st = L.Stats()
        L.check(L.lib().dv_epoch_run_part(self._ctx, ctypes.byref(home.desc()), txns_per_rank,
                                          _ptr(d_commit), ctypes.byref(st)), "dv_epoch_run_part")
        return st

    def run_epoch_group(self, homes, txns_per_rank, d_commit=None):
        """One epoch group (dv_epoch_group_run): homes[e] is this rank's
        client batch (DeviceEpoch) of epoch e of the group, one per rank;
        d_commit: nranks * txns_per_rank device bytes, this rank's txns'
        commit bytes of epoch e at e * txns_per_rank."""
        self._after_torch()
        st = L.Stats()
        arr = (L.EpochDev * len(homes))(*[h.desc() for h in homes])
        prev = self._wide_for(homes)
        try:
            L.check(L.lib().dv_epoch_group_run(self._ctx, arr, len(homes), txns_per_rank, _ptr(d_commit),
                                               ctypes.byref(st)), "dv_epoch_group_run")
        finally:
            if prev is not None:
                L.lib().dv_comm_set_mode(self._ctx, prev)
        return st

    def run_epoch_groups(self, groups, txns_per_rank, d_commits=None):
        """Several epoch groups back to back (dv_epoch_group_run_batch), as
        many run_epoch_group calls with one host wait between two groups.
        groups: a list of group batch lists (one DeviceEpoch per rank each);
        d_commits: one device tensor (or None) per group, or one for all.
        Returns the list of stats."""
        self._after_torch()
        n = len(groups)
        P = len(groups[0]) if n else 0
        if any(len(g) != P for g in groups):
            raise ValueError("every group holds one batch per rank")
        arr = self._epoch_array([h for g in groups for h in g])
        cps = _commit_ptrs(d_commits, n)
        sts = (L.Stats * n)()
        prev = self._wide_for([h for g in groups for h in g])
        try:
            L.check(L.lib().dv_epoch_group_run_batch(self._ctx, arr, n, P, txns_per_rank, cps, sts),
                    "dv_epoch_group_run_batch")
        finally:
            if prev is not None:
                L.lib().dv_comm_set_mode(self._ctx, prev)
        return list(sts)

    def closed_loop(self, pool, pool_begin, n_txn, n_epochs, cursor=None, bufs=None, d_commits=None,
                    resume=False):
        """The closed loop on the device (dv_epoch_run_closed_loop): n_epochs
        epochs of n_txn txns, each the previous one's aborted txns then fresh
        ones from `pool` (a DeviceEpoch with max_txn_acc > 0; pool_begin: its
        n_txn + 1 access offsets, int32 device tensor) from the device word
        `cursor` (int32 tensor, advanced).  bufs: ClosedLoopBufs (allocated when
        None); d_commits: a device tensor per epoch (or None).  Returns (stats
        list, bufs, cursor); the next epoch is in bufs.epoch(n_epochs & 1)."""
        import torch
        dev = pool.keys.device
        if cursor is None:
            cursor = torch.zeros(1, dtype=torch.int32, device=dev)
        if bufs is None:
            bufs = ClosedLoopBufs(n_txn * pool.max_txn_acc, pool.tables is not None, dev, n_txn=n_txn)
        bufs.tb = _loop_tb(pool, [bufs])
        arr = (L.EpochDev * 2)(*[bufs.desc(b) for b in range(2)])
        if d_commits is None or not isinstance(d_commits, (list, tuple)):
            d_commits = [d_commits] * n_epochs
        cps = (ctypes.c_void_p * max(1, n_epochs))(*[(int(t.data_ptr()) if t is not None else None)
                                                     for t in d_commits])
        sts = (L.Stats * max(1, n_epochs))()
        self._after_torch()
        L.check(L.lib().dv_epoch_run_closed_loop(self._ctx, ctypes.byref(pool.desc()), _ptr(pool_begin),
                                                 _ptr(cursor), n_txn, arr, bufs.cap, n_epochs, int(resume),
                                                 cps, sts), "dv_epoch_run_closed_loop")
        return list(sts)[:n_epochs], bufs, cursor

    def closed_loop_lanes(self, lanes, pool, pool_begin, n_txn, n_epochs, cursor=None, bufs=None,
                          d_commits=None, resume=False):
        """dv_epoch_run_closed_loop_lanes over [self] + lanes: epoch k on
        context k % L, each context's epochs a closed loop of their own
        (aborted txns retried L epochs later), the pool cursor shared.  bufs:
        one ClosedLoopBufs per context (allocated when None).  Returns (stats
        list, bufs, cursor); resume needs the previous call's n_epochs to be a
        multiple of 2 L."""
        import torch
        ctxs = [self] + list(lanes)
        nl = len(ctxs)
        dev = pool.keys.device
        if cursor is None:
            cursor = torch.zeros(1, dtype=torch.int32, device=dev)
        if bufs is None:
            bufs = [ClosedLoopBufs(n_txn * pool.max_txn_acc, pool.tables is not None, dev, n_txn=n_txn)
                    for _ in range(nl)]
        tb = _loop_tb(pool, bufs)
        for b in bufs:
            b.tb = tb
        arr = (L.EpochDev * (2 * nl))(*[b.desc(i) for b in bufs for i in range(2)])
        if d_commits is None or not isinstance(d_commits, (list, tuple)):
            d_commits = [d_commits] * n_epochs
        cps = (ctypes.c_void_p * max(1, n_epochs))(*[(int(t.data_ptr()) if t is not None else None)
                                                     for t in d_commits])
        sts = (L.Stats * max(1, n_epochs))()
        lp = (ctypes.c_void_p * nl)(*[e._ctx.value for e in ctxs])
        for e in ctxs:
            e._after_torch()
        L.check(L.lib().dv_epoch_run_closed_loop_lanes(lp, nl, ctypes.byref(pool.desc()), _ptr(pool_begin),
                                                       _ptr(cursor), n_txn, arr, bufs[0].cap, n_epochs,
                                                       int(resume), cps, sts), "dv_epoch_run_closed_loop_lanes")
        return list(sts)[:n_epochs], bufs, cursor

    def group_carry(self, homes, d_commit, txns_per_rank, max_txn=None):
        """Retries across epoch groups (dv_epoch_group_carry): for each of this
        rank's batches of the group just run (DeviceEpochs), a DeviceEpoch of
        its aborted txns (commit byte 0 in d_commit at e * txns_per_rank), in
        sequence order, at most max_txn each -- the head of the same epoch
        slot's batch in the next group."""
        import torch
        outs, keep = [], []
        for h in homes:
            dev = h.keys.device
            n = max(1, h.n_acc)
            t = (torch.empty(n, dtype=torch.int64, device=dev), torch.empty(n, dtype=torch.uint8, device=dev),
                 torch.empty(n, dtype=torch.int32, device=dev),
                 torch.empty(n, dtype=torch.uint8, device=dev) if h.tables is not None else None)
            keep.append(t)
            outs.append(L.EpochDev(t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(),
                                   t[3].data_ptr() if t[3] is not None else None, 0, 0, 0))
        arr = (L.EpochDev * len(homes))(*[h.desc() for h in homes])
        oarr = (L.EpochDev * len(homes))(*outs)
        cap = txns_per_rank if max_txn is None else max_txn
        self._after_torch()
        L.check(L.lib().dv_epoch_group_carry(self._ctx, arr, len(homes), txns_per_rank, _ptr(d_commit), cap, oarr),
                "dv_epoch_group_carry")
        res = []
        for o, t in zip(oarr, keep):
            n = int(o.n_acc)
            res.append(DeviceEpoch.from_tensors(t[0][:n], t[1][:n], t[2][:n], int(o.n_txn),
                                                tables=t[3][:n] if t[3] is not None else None,
                                                max_txn_acc=int(o.max_txn_acc)))
        return res

    def carry(self, dep, max_txn=None):
        """Abort carry-over: a DeviceEpoch of the last epoch's (`dep`'s)
        aborted txns, in sequence order, at most max_txn of them."""
        import torch
        dev = dep.keys.device
        keys = torch.empty(max(1, dep.n_acc), dtype=torch.int64, device=dev)
        types = torch.empty(max(1, dep.n_acc), dtype=torch.uint8, device=dev)
        txn = torch.empty(max(1, dep.n_acc), dtype=torch.int32, device=dev)
        tabs = torch.empty(max(1, dep.n_acc), dtype=torch.uint8, device=dev) if dep.tables is not None else None
        out = L.EpochDev(keys.data_ptr(), types.data_ptr(), txn.data_ptr(),
                         tabs.data_ptr() if tabs is not None else None, 0, 0, 0)
        cap = dep.n_txn if max_txn is None else max_txn
        self._after_torch()
        L.check(L.lib().dv_epoch_carry(self._ctx, ctypes.byref(dep.desc()), cap, ctypes.byref(out)),
                "dv_epoch_carry")
        n = int(out.n_acc)
        return DeviceEpoch.from_tensors(keys[:n], types[:n], txn[:n], int(out.n_txn),
                                        tables=tabs[:n] if tabs is not None else None,
                                        max_txn_acc=int(out.max_txn_acc))

    def round_log(self):
        """(live accesses entering, undecided txns before) per decision round
        of the last epoch."""
        live = (ctypes.c_uint32 * 64)()
        und = (ctypes.c_uint32 * 64)()
        n = L.lib().dv_round_log(self._ctx, live, und, 64)
        return list(live[:n]), list(und[:n])

    # ---- staged form (multi-partition epochs)
    def begin(self, dep, d_grant=None):
        self._after_torch()
        self._desc = dep.desc()
        L.check(L.lib().dv_epoch_begin(self._ctx, ctypes.byref(self._desc), _ptr(d_grant)),
                "dv_epoch_begin")

    def round_local(self, d_verdict):
        self._after_torch()  # (d_verdict may come from a torch kernel still queued)
        L.check(L.lib().dv_epoch_round_local(self._ctx, _ptr(d_verdict)), "dv_epoch_round_local")

    def round_apply(self, d_verdict, wait=True):
        """Applies the combined verdicts; wait=False only enqueues the apply
        (read its outcome with round_wait)."""
        self._after_torch()
        und = ctypes.c_uint32()
        L.check(L.lib().dv_epoch_round_apply(self._ctx, _ptr(d_verdict),
                                             ctypes.byref(und) if wait else None),
                "dv_epoch_round_apply")
        return und.value if wait else None

    def round_wait(self, r):
        """Undecided txns after round r (or after a later, already applied one)."""
        und = ctypes.c_uint32()
        L.check(L.lib().dv_epoch_round_wait(self._ctx, r, ctypes.byref(und)), "dv_epoch_round_wait")
        return und.value

    def errors_local(self, d_word):
        """Partitioned epochs: enqueue this partition's input-error bits into
        the device int32 tensor d_word (combine with MAX across ranks)."""
        self._after_torch()
        L.check(L.lib().dv_epoch_errors_local(self._ctx, _ptr(d_word)), "dv_epoch_errors_local")

    def errors_combined(self, d_word):
        """... and hand the combined word back: an error anywhere rejects the
        epoch on every partition, at the same round."""
        self._after_torch()
        L.check(L.lib().dv_epoch_errors_combined(self._ctx, _ptr(d_word)), "dv_epoch_errors_combined")

    def finish(self, d_commit=None):
        self._after_torch()  # (d_commit may be a torch.zeros still queued)
        st = L.Stats()
        L.check(L.lib().dv_epoch_finish(self._ctx, _ptr(d_commit), ctypes.byref(st)),
                "dv_epoch_finish")
        return st
