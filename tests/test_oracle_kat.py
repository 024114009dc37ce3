"""Pins the CPU oracle with known answers derived by hand from the reference
source text (SURVEY.md 8c "KATs the build must derive"): the reference has no
tests or fixtures of its own and cannot be built here, so these are the pins.

A tiny pure-Python restatement of myrand/zipf/gen_requests_zipf (small cases
only) gives an independent second derivation of the generator.
"""
import math

import numpy as np
import pytest

import _oracle as O


# ---------------------------------------------------------------- myrand
def py_myrand(seed, n):
    """system/helper.cpp:140-147 with Python big ints (wrap at 2^64 first)."""
    out = []
    for _ in range(n):
        seed = ((seed * 1103515247 + 12345) % (1 << 64)) % (1 << 63)
        out.append((seed // 65537) % 2147483647)
    return out, seed


def test_myrand_kat_seed0():
    # by hand: s1 = 12345 -> 12345 // 65537 = 0; s2 = 12345*1103515248 = 13622895736560
    # -> 13622895736560 // 65537 = 207865720
    seed = O.ctypes.c_uint64(0)
    got = [O.lib().or_myrand_next(O.ctypes.byref(seed)) for _ in range(5)]
    assert got[:2] == [0, 207865720]
    assert got == py_myrand(0, 5)[0]


@pytest.mark.parametrize("seed", [1, 98, 1234567, 2**62 + 5])
def test_myrand_matches_python(seed):
    s = O.ctypes.c_uint64(seed)
    got = [O.lib().or_myrand_next(O.ctypes.byref(s)) for _ in range(200)]
    assert got == py_myrand(seed, 200)[0]


# ------------------------------------------------------------------ zipf
def test_zeta_small():
    # zeta(n, theta) = sum_{i=1..n} pow(1.0/i, theta)  (ycsb_query.cpp:181-186)
    for n, th in [(1, 0.9), (2, 0.6), (10, 0.9), (1000, 0.3)]:
        ref = 0.0
        for i in range(1, n + 1):
            ref += math.pow(1.0 / i, th)
        assert O.lib().or_zeta(n, th) == ref


class PyYcsbGen:
    """Pure-Python restatement of gen_requests_zipf (ycsb_query.cpp:303-376)."""

    def __init__(self, table_size_total, part_cnt, R, theta, txn_wr, tup_wr, ppt, strict, mpr, seed):
        self.seed = seed
        self.n = table_size_total // part_cnt - 1
        self.theta = theta
        self.zetan = sum(math.pow(1.0 / i, theta) for i in range(1, self.n + 1))
        self.z2 = 1.0 + math.pow(1.0 / 2, theta)
        self.P, self.R, self.ppt, self.strict, self.mpr = part_cnt, R, ppt, strict, mpr
        self.txn_read = 1.0 - txn_wr
        self.tup_read = 1.0 - tup_wr

    def rnd(self):
        self.seed = ((self.seed * 1103515247 + 12345) % (1 << 64)) % (1 << 63)
        return (self.seed // 65537) % 2147483647

    def zipf(self):
        n, th = self.n, self.theta
        alpha = 1 / (1 - th)
        eta = (1 - math.pow(2.0 / n, 1 - th)) / (1 - self.z2 / self.zetan)
        u = float(self.rnd() % 10000000) / 10000000
        uz = u * self.zetan
        if uz < 1:
            return 1
        if uz < 1 + math.pow(0.5, th):
            return 2
        return 1 + int(n * math.pow(eta * u - eta + 1, alpha))

    def txn(self, home):
        gate = self.mpr >= 0
        limit = self.ppt
        if gate:
            r_mpt = float(self.rnd() % 10000) / 10000
            limit = self.ppt if r_mpt < self.mpr else 1
        r_twr = float(self.rnd() % 10000) / 10000
        keys, types, parts = [], [], []
        while len(keys) < self.R:
            r = float(self.rnd() % 10000) / 10000
            if not keys or (gate and limit == 1):
                pid = home
            else:
                pid = self.rnd() % self.P
                if self.strict and limit <= self.P:
                    while (len(parts) < limit and pid in parts) or (len(parts) == limit and pid not in parts):
                        pid = self.rnd() % self.P
                elif gate:
                    while len(parts) == limit and pid not in parts:
                        pid = self.rnd() % self.P
            t = 0 if (r_twr < self.txn_read or r < self.tup_read) else 1
            key = self.zipf() * self.P + pid
            self.rnd()  # value
            if key in keys:
                continue
            keys.append(key)
            types.append(t)
            if pid not in parts:
                parts.append(pid)
        return keys, types


@pytest.mark.parametrize("cfg", [
    dict(table=2000, P=1, R=10, theta=0.9, txn_wr=1.0, tup_wr=0.5, ppt=1, strict=0, mpr=-1.0),
    dict(table=5000, P=1, R=10, theta=0.6, txn_wr=0.5, tup_wr=0.5, ppt=1, strict=0, mpr=-1.0),
    dict(table=8000, P=4, R=10, theta=0.9, txn_wr=1.0, tup_wr=0.5, ppt=2, strict=1, mpr=-1.0),
    dict(table=8000, P=4, R=8, theta=0.9, txn_wr=1.0, tup_wr=0.5, ppt=2, strict=1, mpr=0.3),
    dict(table=9000, P=3, R=4, theta=0.3, txn_wr=0.0, tup_wr=0.0, ppt=3, strict=0, mpr=-1.0),
])
def test_generator_matches_python_restatement(cfg):
    n_txn, seed, home = 50, 4242, cfg["P"] - 1
    p = O.ycsb_params(cfg["table"], part_cnt=cfg["P"], req_per_query=cfg["R"], zipf_theta=cfg["theta"],
                      txn_write_perc=cfg["txn_wr"], tup_write_perc=cfg["tup_wr"],
                      part_per_txn=cfg["ppt"], strict_ppt=cfg["strict"], mpr=cfg["mpr"])
    keys, types, tb = O.ycsb_gen(p, seed, home, n_txn)
    g = PyYcsbGen(cfg["table"], cfg["P"], cfg["R"], cfg["theta"], cfg["txn_wr"], cfg["tup_wr"],
                  cfg["ppt"], cfg["strict"], cfg["mpr"], seed)
    for t in range(n_txn):
        k, ty = g.txn(home)
        assert list(keys[t * cfg["R"]:(t + 1) * cfg["R"]]) == k
        assert list(types[t * cfg["R"]:(t + 1) * cfg["R"]]) == ty
    assert list(tb) == [t * cfg["R"] for t in range(n_txn + 1)]
    # invariants: first request on the home partition, keys unique per txn, rows in [1, n]
    K = keys.reshape(n_txn, cfg["R"])
    assert (K[:, 0] % cfg["P"] == home).all()
    assert all(len(set(r)) == cfg["R"] for r in K.tolist())
    rows = K // cfg["P"]
    assert rows.min() >= 1 and rows.max() <= cfg["table"] // cfg["P"] - 1


def test_zipf_edge_rules():
    # uz < 1 -> row 1; uz < 1 + 0.5^theta -> row 2 (ycsb_query.cpp:199-200): for
    # theta = 0.9 over 1000 rows P(row 1) = 1/zeta ~ 0.13, P(row 2) ~ 0.07
    p = O.ycsb_params(1001, zipf_theta=0.9, req_per_query=1, txn_write_perc=0.0)
    keys, _, _ = O.ycsb_gen(p, 99, 0, 20000)
    z = O.lib().or_zeta(1000, 0.9)
    f1, f2 = (keys == 1).mean(), (keys == 2).mean()
    assert abs(f1 - 1.0 / z) < 0.01
    assert abs(f2 - math.pow(0.5, 0.9) / z) < 0.01
    assert 0 not in set(keys.tolist())


# ------------------------------------------------------------ lock table
def test_conflict_lock_truth_table():
    EX, SH, NONE = 0, 1, 2
    want = {(EX, EX): 1, (EX, SH): 1, (SH, EX): 1, (SH, SH): 0,
            (NONE, EX): 0, (NONE, SH): 0, (EX, NONE): 0, (SH, NONE): 0, (NONE, NONE): 0}
    for (a, b), v in want.items():
        assert O.lib().or_conflict_lock(a, b) == v


def test_f0_init_layout():
    # set_value(0,&key,8) then "hello\0" over bytes [0,6) (ycsb_wl.cpp:173-186)
    assert O.lib().or_ycsb_f0_init(0) == int.from_bytes(b"hello\x00\x00\x00", "little")
    k = 0x0123456789ABCDEF
    assert O.lib().or_ycsb_f0_init(k) == int.from_bytes(b"hello\x00" + k.to_bytes(8, "little")[6:], "little")


def _epoch(txns):
    keys, types, tb = [], [], [0]
    for acc in txns:
        for k, t in acc:
            keys.append(k)
            types.append(t)
        tb.append(len(keys))
    return (np.array(keys, dtype=np.uint64), np.array(types, dtype=np.uint8),
            np.array(tb, dtype=np.uint32))


R_, W_ = O.RD, O.WR
A, B, C = 1, 2, 3
HAND = [[(A, W_)], [(A, R_)], [(B, R_), (C, W_)], [(B, R_)], [(B, W_)], [(C, R_)]]


def _run(cc, txns, nrows=8, grant=False, literal=False):
    keys, types, tb = _epoch(txns)
    tab = O.YcsbTable(nrows)
    f0 = tab.f0.copy()
    c, g, st = O.epoch_run(cc, tab.ix, f0, len(txns), tb, keys, types, want_grant=grant,
                           occ_literal=literal)
    return c, g, st, f0


def test_hand_no_wait_and_wait_die():
    # T0 W(a) holds EX; T1 R(a) aborts; T2 R(b) W(c); T3 R(b) shares SH;
    # T4 W(b) conflicts with SH owners -> abort; T5 R(c) conflicts with T2's EX
    for cc in (O.NO_WAIT, O.WAIT_DIE):
        c, _, st, f0 = _run(cc, HAND)
        assert c.tolist() == [1, 0, 1, 1, 0, 0]
        assert st.committed == 3 and st.write_cnt == 2
        assert f0[A] == 0 and f0[C] == 0 and f0[B] != 0


def test_hand_occ():
    # backward validation: only earlier committed WRITE sets kill (occ.cpp:185-199);
    # T4 W(b) after readers of b commits
    for lit in (False, True):
        c, _, _, f0 = _run(O.OCC, HAND, literal=lit)
        assert c.tolist() == [1, 0, 1, 1, 1, 0]
        assert f0[B] == 0


def test_hand_calvin_grant_groups():
    c, g, st, _ = _run(O.CALVIN, HAND, grant=True)
    assert c.tolist() == [1] * 6
    assert g.tolist() == [0, 1, 0, 0, 0, 1, 1]


def test_calvin_runs_of_shared():
    X = 5
    seq = [R_, R_, W_, R_, R_, W_, W_, R_]
    c, g, _, _ = _run(O.CALVIN, [[(X, t)] for t in seq], grant=True)
    assert g.tolist() == [0, 0, 1, 2, 2, 3, 4, 5]


def test_calvin_reads_see_earlier_writes():
    # T0 R(x) sees the initial F0, T1 W(x), T2 R(x) sees 0 (serial order)
    X = 4
    keys, types, tb = _epoch([[(X, R_)], [(X, W_)], [(X, R_)]])
    tab = O.YcsbTable(8)
    f0 = tab.f0.copy()
    init = int(f0[X])
    _, _, st = O.epoch_run(O.CALVIN, tab.ix, f0, 3, tb, keys, types)
    mix = O.lib().or_mix64
    want = (mix(init ^ mix((0 << 32) ^ X)) + mix(0 ^ mix((2 << 32) ^ X))) % (1 << 64)
    assert st.read_digest == want


def test_occ_literal_equals_indexed():
    p = O.ycsb_params(1 << 12, zipf_theta=0.9)
    keys, types, tb = O.ycsb_gen(p, 77, 0, 1500)
    tab = O.YcsbTable(1 << 12)
    a = O.epoch_run(O.OCC, tab.ix, tab.f0.copy(), 1500, tb, keys, types, occ_literal=True)[0]
    b = O.epoch_run(O.OCC, tab.ix, tab.f0.copy(), 1500, tb, keys, types, occ_literal=False)[0]
    assert (a == b).all()


def test_no_wait_greedy_predicate():
    """i aborts <=> some earlier survivor shares a row with it and one of the two
    writes it -- checked by brute force on a contended epoch."""
    p = O.ycsb_params(1 << 10, zipf_theta=0.9, req_per_query=4)
    keys, types, tb = O.ycsb_gen(p, 5, 0, 400)
    tab = O.YcsbTable(1 << 10)
    c = O.epoch_run(O.NO_WAIT, tab.ix, tab.f0.copy(), 400, tb, keys, types)[0]
    K = keys.reshape(400, 4)
    T = types.reshape(400, 4)
    surv = []
    for i in range(400):
        acc = dict(zip(K[i].tolist(), T[i].tolist()))
        bad = False
        for j in surv:
            for k, t in zip(K[j].tolist(), T[j].tolist()):
                if k in acc and (t == 1 or acc[k] == 1):
                    bad = True
        assert c[i] == (0 if bad else 1)
        if not bad:
            surv.append(i)


# A txn touching one row twice.  Hand-derived from the text:
# 2PL re-locks through get_row (txn.cpp:790-803); conflict_lock(SH, SH) is
# free, anything with EX conflicts with the txn's own lock (row_lock.cpp:69):
# NO_WAIT aborts (86-90), WAIT_DIE dies (the reference asserts at 106).  OCC
# never validates a txn against itself (occ.cpp:185-199): the row is in its
# write set if any access writes it.
REP = [[(A, R_), (A, R_)],          # T0: shared twice -> commits
       [(B, R_), (B, W_)],          # T1: SH then EX on its own row
       [(C, W_), (C, R_)],          # T2: EX then SH
       [(B, R_)],                   # T3: reads b
       [(C, R_), (4, W_), (C, R_)]]  # T4: c twice (shared), writes d


def test_repeated_rows_2pl():
    for cc in (O.NO_WAIT, O.WAIT_DIE):
        c, _, st, f0 = _run(cc, REP)
        # T1 and T2 abort on themselves; T3 then finds b free; T4 too
        assert c.tolist() == [1, 0, 0, 1, 1], cc
        assert st.write_cnt == 1 and f0[4] == 0 and f0[B] != 0 and f0[C] != 0


def test_repeated_rows_occ():
    for lit in (False, True):
        c, _, st, f0 = _run(O.OCC, REP, literal=lit)
        # T1 and T2 commit (b, c in their write sets); T3 reads b -> aborts;
        # T4 reads c -> aborts
        assert c.tolist() == [1, 1, 1, 0, 0], lit
        assert st.write_cnt == 2 and f0[B] == 0 and f0[C] == 0


def test_repeated_rows_occ_reads_see_the_epoch_image():
    # OCC reads in the access phase (row_occ.cpp:38-46): T0's read of a after its
    # own write of a still sees the initial value
    keys, types, tb = _epoch([[(A, W_), (A, R_)]])
    tab = O.YcsbTable(8)
    f0 = tab.f0.copy()
    init = int(f0[A])
    _, _, st = O.epoch_run(O.OCC, tab.ix, f0, 1, tb, keys, types)
    mix = O.lib().or_mix64
    assert st.read_digest == mix(init ^ mix((0 << 32) ^ A)) and f0[A] == 0


def test_missing_key_is_an_error():
    keys, types, tb = _epoch([[(100, R_)]])
    tab = O.YcsbTable(8)
    with pytest.raises(RuntimeError):
        O.epoch_run(O.NO_WAIT, tab.ix, tab.f0.copy(), 1, tb, keys, types)


def test_empty_epoch():
    tab = O.YcsbTable(8)
    c, g, st = O.epoch_run(O.CALVIN, tab.ix, tab.f0.copy(), 0, np.zeros(1, np.uint32),
                           np.zeros(1, np.uint64), np.zeros(1, np.uint8), want_grant=True)
    assert st.committed == 0 and len(c) == 0


def test_mt_baseline_engine():
    """SURVEY.md 8(d)(ii) CPU baseline: one worker runs txns one at a time, so
    nothing conflicts and everything commits; several workers under zipf 0.9
    abort some txns, and every lock is free again at the end."""
    rows, n = 1 << 12, 4000
    p = O.ycsb_params(rows, zipf_theta=0.9, txn_write_perc=1.0, tup_write_perc=0.5)
    keys, types, tb = O.ycsb_gen(p, 11, 0, n)
    for threads in (1, 4):
        tab = O.YcsbTable(rows)
        f0 = tab.f0.copy()
        lock = O.mt_lock(rows)
        committed, _ = O.mt_epoch_run(tab.ix, f0, lock, n, tb, keys, types, threads)
        assert not lock.any()
        if threads == 1:
            assert committed == n
            assert (f0[keys[types == O.WR].astype(np.int64)] == 0).all()
        else:
            assert 0 < committed <= n
