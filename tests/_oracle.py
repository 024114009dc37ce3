"""ctypes binding of the CPU oracle (oracle/liboracle.so) -- the CHECKER.

Test infrastructure only: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product package.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, "oracle", "build", "liboracle.so")

NO_WAIT, WAIT_DIE, OCC, CALVIN = 1, 2, 8, 10
RD, WR = 0, 1


class YcsbParams(ctypes.Structure):
    _fields_ = [
        ("synth_table_size", ctypes.c_uint64),
        ("part_cnt", ctypes.c_uint32),
        ("req_per_query", ctypes.c_uint32),
        ("zipf_theta", ctypes.c_double),
        ("txn_write_perc", ctypes.c_double),
        ("tup_write_perc", ctypes.c_double),
        ("part_per_txn", ctypes.c_uint32),
        ("strict_ppt", ctypes.c_uint32),
        ("mpr", ctypes.c_double),
    ]


class EpochStats(ctypes.Structure):
    _fields_ = [
        ("committed", ctypes.c_uint64),
        ("aborted", ctypes.c_uint64),
        ("read_digest", ctypes.c_uint64),
        ("write_cnt", ctypes.c_uint64),
    ]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.POINTER
        u8p, u32p, u64p = P(ctypes.c_uint8), P(ctypes.c_uint32), P(ctypes.c_uint64)
        L.or_myrand_next.argtypes = [u64p]
        L.or_myrand_next.restype = ctypes.c_uint64
        L.or_zeta.argtypes = [ctypes.c_uint64, ctypes.c_double]
        L.or_zeta.restype = ctypes.c_double
        L.or_ycsb_gen.argtypes = [P(YcsbParams), ctypes.c_uint64, ctypes.c_uint32,
                                  ctypes.c_uint32, u64p, u8p, u32p]
        L.or_ycsb_gen.restype = ctypes.c_int
        L.or_index_create.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_uint64]
        L.or_index_create.restype = ctypes.c_void_p
        L.or_index_free.argtypes = [ctypes.c_void_p]
        L.or_index_insert.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64]
        L.or_index_insert.restype = ctypes.c_int
        L.or_index_read.argtypes = [ctypes.c_void_p, ctypes.c_uint64, u64p]
        L.or_index_read.restype = ctypes.c_int
        L.or_ycsb_f0_init.argtypes = [ctypes.c_uint64]
        L.or_ycsb_f0_init.restype = ctypes.c_uint64
        L.or_ycsb_load.argtypes = [ctypes.c_void_p, u64p, ctypes.c_uint64, ctypes.c_uint32,
                                   ctypes.c_uint32]
        L.or_ycsb_load.restype = ctypes.c_int
        L.or_index_insert_many.argtypes = [ctypes.c_void_p, u64p, u64p, ctypes.c_uint64]
        L.or_index_insert_many.restype = ctypes.c_int
        L.or_conflict_lock.argtypes = [ctypes.c_int, ctypes.c_int]
        L.or_conflict_lock.restype = ctypes.c_int
        L.or_mix64.argtypes = [ctypes.c_uint64]
        L.or_mix64.restype = ctypes.c_uint64
        L.or_table_digest.argtypes = [u64p, ctypes.c_uint64]
        L.or_table_digest.restype = ctypes.c_uint64
        L.or_epoch_run.argtypes = [ctypes.c_int, ctypes.c_void_p, u64p, ctypes.c_uint64,
                                   ctypes.c_uint32, u32p, u64p, u8p, u8p, u32p, ctypes.c_int,
                                   P(EpochStats)]
        L.or_epoch_run.restype = ctypes.c_int
        L.or_mt_epoch_run.argtypes = [ctypes.c_void_p, u64p, u32p, ctypes.c_uint64, ctypes.c_uint32, u32p,
                                      u64p, u8p, ctypes.c_int, u64p, u64p]
        L.or_mt_epoch_run.restype = ctypes.c_int
        L.or_mt_lock_words.argtypes = [ctypes.c_uint64]
        L.or_mt_lock_words.restype = ctypes.c_uint64
        L.or_index_read_mid.argtypes = [ctypes.c_void_p, ctypes.c_uint64, u64p]
        L.or_index_read_mid.restype = ctypes.c_int
        L.or_grand_seed.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        L.or_grand_next.argtypes = [ctypes.c_void_p]
        L.or_grand_next.restype = ctypes.c_uint32
        L.or_tpcc_load.argtypes = [P(TpccParams), ctypes.c_uint64, ctypes.c_uint32]
        L.or_tpcc_load.restype = ctypes.c_void_p
        L.or_tpcc_free.argtypes = [ctypes.c_void_p]
        L.or_tpcc_rows.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        L.or_tpcc_rows.restype = ctypes.c_uint64
        L.or_tpcc_table.argtypes = [ctypes.c_void_p, ctypes.c_uint32, u64p, u64p, u64p, u64p]
        L.or_tpcc_table.restype = ctypes.c_int
        L.or_tpcc_gen.argtypes = [P(TpccParams), ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                  u64p, u8p, u8p, u64p, u32p, u8p, u8p]
        L.or_tpcc_gen.restype = ctypes.c_int
        L.or_tpcc_epoch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32, u32p, u64p, u8p, u8p,
                                    u64p, u8p, u64p, P(EpochStats)]
        L.or_tpcc_epoch.restype = ctypes.c_int
        L.or_tpcc_load_layout.argtypes = [P(TpccParams), ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32]
        L.or_tpcc_load_layout.restype = ctypes.c_void_p
        L.or_tpcc_epoch_owner.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32, u32p, u64p, u8p, u8p,
                                          u64p, u8p, u8p, u64p, P(EpochStats)]
        L.or_tpcc_epoch_owner.restype = ctypes.c_int
        _lib = L
    return _lib


class TpccParams(ctypes.Structure):
    _fields_ = [("num_wh", ctypes.c_uint32), ("dist_per_wh", ctypes.c_uint32),
                ("cust_per_dist", ctypes.c_uint32), ("max_items", ctypes.c_uint32),
                ("max_items_per_txn", ctypes.c_uint32), ("part_cnt", ctypes.c_uint32),
                ("part_per_txn", ctypes.c_uint32), ("wh_update", ctypes.c_uint32),
                ("perc_payment", ctypes.c_double), ("mpr", ctypes.c_double)]


def tpcc_params(num_wh, dist_per_wh=10, cust_per_dist=3000, max_items=100000, max_items_per_txn=15,
                part_cnt=1, part_per_txn=2, wh_update=1, perc_payment=0.5, mpr=1.0):
    return TpccParams(num_wh, dist_per_wh, cust_per_dist, max_items, max_items_per_txn, part_cnt,
                      part_per_txn, wh_update, perc_payment, mpr)


class GlibcRand:
    """oracle restatement of glibc srand()/rand() (random_r TYPE_3)."""

    def __init__(self, seed):
        self.buf = ctypes.create_string_buffer(31 * 4 + 8)
        lib().or_grand_seed(self.buf, seed)

    def next(self):
        return lib().or_grand_next(self.buf)


def tpcc_gen(p, n_txn, seed, home_part=0):
    cap = n_txn * (3 + 2 * p.max_items_per_txn)
    keys = np.zeros(cap, dtype=np.uint64)
    types = np.zeros(cap, dtype=np.uint8)
    tables = np.zeros(cap, dtype=np.uint8)
    args = np.zeros(cap, dtype=np.uint64)
    tb = np.zeros(n_txn + 1, dtype=np.uint32)
    tt = np.zeros(max(1, n_txn), dtype=np.uint8)
    own = np.zeros(cap, dtype=np.uint8)
    assert lib().or_tpcc_gen(ctypes.byref(p), seed, home_part, n_txn, _p(keys, ctypes.c_uint64),
                             _p(types, ctypes.c_uint8), _p(tables, ctypes.c_uint8),
                             _p(args, ctypes.c_uint64), _p(tb, ctypes.c_uint32), _p(tt, ctypes.c_uint8),
                             _p(own, ctypes.c_uint8)) == 0
    n = int(tb[-1])
    return keys[:n].copy(), types[:n].copy(), tables[:n].copy(), args[:n].copy(), tb, tt[:n_txn], own[:n].copy()


class TpccDB:
    """Oracle TPC-C partition (oracle/tpcc.c)."""

    def __init__(self, p, seed, part_id=0, index_parts=1):
        """index_parts > 1: last-name lists per partition of that layout
        (or_tpcc_load_layout), for epochs of a partitioned run."""
        self.p = p
        self.db = lib().or_tpcc_load_layout(ctypes.byref(p), seed, part_id, index_parts)
        assert self.db

    def table(self, t):
        n = lib().or_tpcc_rows(self.db, t)
        out = [np.zeros(n, dtype=np.uint64) for _ in range(4)]
        assert lib().or_tpcc_table(self.db, t, *[_p(a, ctypes.c_uint64) for a in out]) == 0
        return out

    def epoch(self, cc, keys, types, tables, args, tb, owner=None):
        n_txn = len(tb) - 1
        commit = np.zeros(max(1, n_txn), dtype=np.uint8)
        oid = np.zeros(max(1, n_txn), dtype=np.uint64)
        st = EpochStats()
        own = None if owner is None else np.ascontiguousarray(owner, dtype=np.uint8)
        rc = lib().or_tpcc_epoch_owner(self.db, cc, n_txn, _p(tb, ctypes.c_uint32), _p(keys, ctypes.c_uint64),
                                       _p(types, ctypes.c_uint8), _p(tables, ctypes.c_uint8),
                                       _p(args, ctypes.c_uint64), _p(own, ctypes.c_uint8) if own is not None
                                       else None, _p(commit, ctypes.c_uint8),
                                       _p(oid, ctypes.c_uint64), ctypes.byref(st))
        if rc != 0:
            raise RuntimeError(f"oracle tpcc epoch failed rc={rc}")
        return commit[:n_txn], oid[:n_txn], st

    def __del__(self):
        try:
            lib().or_tpcc_free(self.db)
        except Exception:
            pass


def _p(a, t):
    return a.ctypes.data_as(ctypes.POINTER(t))


def ycsb_params(synth_table_size, part_cnt=1, req_per_query=10, zipf_theta=0.9,
                txn_write_perc=1.0, tup_write_perc=0.5, part_per_txn=None, strict_ppt=0, mpr=-1.0):
    return YcsbParams(synth_table_size, part_cnt, req_per_query, zipf_theta, txn_write_perc,
                      tup_write_perc, part_cnt if part_per_txn is None else part_per_txn,
                      strict_ppt, mpr)


def ycsb_gen(params, seed, home_part, n_txn):
    R = params.req_per_query
    keys = np.zeros(n_txn * R, dtype=np.uint64)
    types = np.zeros(n_txn * R, dtype=np.uint8)
    tb = np.zeros(n_txn + 1, dtype=np.uint32)
    rc = lib().or_ycsb_gen(ctypes.byref(params), seed, home_part, n_txn, _p(keys, ctypes.c_uint64),
                           _p(types, ctypes.c_uint8), _p(tb, ctypes.c_uint32))
    assert rc == 0, rc
    return keys, types, tb


class YcsbTable:
    """Oracle YCSB partition: keys part, part+P, ... with rows in key order
    (ycsb_wl.cpp:144-203) and the YCSB index hash (index_hash.h:86-89)."""

    def __init__(self, rows_per_part, part_cnt=1, part_id=0):
        self.nrows = rows_per_part
        L = lib()
        self.ix = L.or_index_create(rows_per_part, part_cnt, 1, rows_per_part)
        self.f0 = np.zeros(rows_per_part, dtype=np.uint64)
        assert L.or_ycsb_load(self.ix, _p(self.f0, ctypes.c_uint64), rows_per_part, part_cnt,
                              part_id) == 0

    def __del__(self):
        try:
            lib().or_index_free(self.ix)
        except Exception:
            pass


class MultiIndex:
    """Oracle index over explicit (key,row) pairs (general chained hash)."""

    def __init__(self, nbuckets, part_cnt, ycsb_hash, pairs):
        keys = np.ascontiguousarray([k for k, _ in pairs], dtype=np.uint64)
        rows = np.ascontiguousarray([r for _, r in pairs], dtype=np.uint64)
        self.ix = lib().or_index_create(nbuckets, part_cnt, ycsb_hash, max(1, len(pairs)))
        assert lib().or_index_insert_many(self.ix, _p(keys, ctypes.c_uint64),
                                          _p(rows, ctypes.c_uint64), len(keys)) == 0

    def __del__(self):
        try:
            lib().or_index_free(self.ix)
        except Exception:
            pass


def mt_lock(rows):
    """The zeroed lock array mt_epoch_run takes for `rows` rows (the hot rows'
    words one per cache line, or_mt_lock_words)."""
    return np.zeros(lib().or_mt_lock_words(rows), np.uint32)


def mt_epoch_run(ix, f0, lock, n_txn, tb, keys, types, threads):
    """SURVEY.md 8(d)(ii) baseline: Deneva-style multi-threaded NO_WAIT
    (oracle/mt_engine.c).  lock: mt_lock(len(f0)).  Returns (committed, read
    digest); its aborts depend on the interleaving."""
    assert len(lock) >= lib().or_mt_lock_words(len(f0))
    c, d = ctypes.c_uint64(), ctypes.c_uint64()
    rc = lib().or_mt_epoch_run(ix, _p(f0, ctypes.c_uint64), _p(lock, ctypes.c_uint32), len(f0), n_txn,
                               _p(tb, ctypes.c_uint32), _p(keys, ctypes.c_uint64), _p(types, ctypes.c_uint8),
                               threads, ctypes.byref(c), ctypes.byref(d))
    assert rc == 0, rc
    return c.value, d.value


def epoch_run(cc, ix, f0, n_txn, tb, keys, types, want_grant=False, occ_literal=False):
    """Runs one E-schedule epoch; mutates f0 in place. Returns (commit, grant, stats)."""
    commit = np.zeros(max(1, n_txn), dtype=np.uint8)
    n_acc = int(tb[n_txn])
    grant = np.zeros(max(1, n_acc), dtype=np.uint32) if want_grant else None
    st = EpochStats()
    rc = lib().or_epoch_run(cc, ix, _p(f0, ctypes.c_uint64), len(f0), n_txn, _p(tb, ctypes.c_uint32),
                            _p(keys, ctypes.c_uint64), _p(types, ctypes.c_uint8),
                            _p(commit, ctypes.c_uint8),
                            _p(grant, ctypes.c_uint32) if grant is not None else None,
                            1 if occ_literal else 0, ctypes.byref(st))
    if rc != 0:
        raise RuntimeError(f"oracle epoch failed rc={rc}")
    return commit[:n_txn], (grant[:n_acc] if grant is not None else None), st


def table_digest(f0):
    return lib().or_table_digest(_p(f0, ctypes.c_uint64), len(f0))
