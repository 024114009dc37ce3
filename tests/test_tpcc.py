"""TPC-C (config E) on the CPU: the oracle's generator pinned to glibc's own
rand(), hand-derived known answers from tpcc_helper.cpp / tpcc_txn.cpp, and
the product's host-side loader and epoch builder (libdvcc, no GPU needed)
against the oracle's restatement."""
import ctypes
import os

import numpy as np
import pytest

import _oracle as O

OR_WR, OR_RD = 1, 0


def test_glibc_rand_kat():
    """or_grand_* == glibc srand()/rand() (the reference's RAND, tpcc_helper.cpp:91-93)."""
    libc = ctypes.CDLL("libc.so.6")
    libc.rand.restype = ctypes.c_int
    for seed in (0, 1, 2, 97, 12345, 2**31 - 1, 4000000000):
        libc.srand(ctypes.c_uint(seed))
        g = O.GlibcRand(seed)
        assert [libc.rand() for _ in range(2000)] == [g.next() for _ in range(2000)], seed
    g = O.GlibcRand(1)
    assert [g.next() for _ in range(3)] == [1804289383, 846930886, 1681692777]


def _lastname(num):  # tpcc_helper.cpp:81-89
    n = ["BAR", "OUGHT", "ABLE", "PRI", "PRES", "ESE", "ANTI", "CALLY", "ATION", "EING"]
    return n[num // 100] + n[(num // 10) % 10] + n[num % 10]


def _custnp(last, d, w, dpw=10):  # tpcc_helper.cpp:35-43
    key = 0
    for ch in last:
        key = (key << 1) + (ord(ch) - ord("A"))
    return (key << 10) + w * dpw + d


def test_key_functions_kat():
    assert _lastname(0) == "BARBARBAR"
    assert _lastname(371) == "PRICALLYOUGHT"
    assert _lastname(999) == "EINGEINGEING"
    # "BARBARBAR": B=1 A=0 R=17 folded with key = 2*key + c
    k = 0
    for c in [1, 0, 17] * 3:
        k = 2 * k + c
    assert _custnp("BARBARBAR", 3, 2) == (k << 10) + 23
    # H8: w*10+d exceeds 10 bits past warehouse 102 and collides into the name bits
    assert _custnp("BARBARBAR", 4, 103) == (k << 10) + 1034


def test_mid_selection_kat():
    """run_payment_4: element floor(n/2) of the item list, newest insert first."""
    L = O.lib()
    for n in range(1, 9):
        ix = L.or_index_create(7, 1, 0, 16)
        for r in range(n):
            assert L.or_index_insert(ix, 42, 100 + r) == 0
        row = ctypes.c_uint64()
        assert L.or_index_read_mid(ix, 42, ctypes.byref(row)) == 0
        assert row.value == 100 + (n - 1 - n // 2), n
        L.or_index_free(ix)


def _small(nw=2, **kw):
    return O.tpcc_params(nw, cust_per_dist=1000, max_items=2000, **kw)


def _epoch(accs):
    """[(table, key, type, op, value), ...] per txn -> arrays"""
    keys, types, tables, args, tb = [], [], [], [], [0]
    for txn in accs:
        for t, k, ty, op, v in txn:
            keys.append(k); types.append(ty); tables.append(t); args.append(op << 56 | v)
        tb.append(len(keys))
    return (np.array(keys, np.uint64), np.array(types, np.uint8), np.array(tables, np.uint8),
            np.array(args, np.uint64), np.array(tb, np.uint32))


def _as_f(u):
    return np.asarray(u, np.uint64).view(np.float64)


def _payment(w, d, c, h, dpw=10, cpd=1000):
    return [(0, w, OR_WR, 1, h), (1, w * dpw + d, OR_WR, 2, h), (2, (w * dpw + d) * cpd + c, OR_WR, 3, h)]


def _new_order(w, d, c, items, dpw=10, cpd=1000, nitems=2000):
    a = [(0, w, OR_RD, 0, 0), (2, (w * dpw + d) * cpd + c, OR_RD, 0, 0), (1, w * dpw + d, OR_WR, 4, 0)]
    for i, sw, q in items:
        a += [(3, i, OR_RD, 0, 0), (4, sw * nitems + i, OR_WR, 5, q)]
    return a


def test_tpcc_scenarios_kat():
    """Hand-built epochs: Payment/NewOrder conflicts and their effects."""
    p = _small()
    e = _epoch([_payment(1, 1, 5, 100), _payment(1, 2, 6, 7), _new_order(2, 3, 9, [(10, 2, 4), (11, 2, 9)]),
                _new_order(2, 3, 10, [(10, 2, 3)]), _new_order(2, 4, 11, [(12, 2, 1)])])
    for cc in (O.NO_WAIT, O.WAIT_DIE, O.OCC):
        db = O.TpccDB(p, 3)
        wh0, dist0, cust0, _, st0 = db.table(0), db.table(1), db.table(2), None, db.table(4)
        commit, oid, st = db.epoch(cc, *e)
        # txn1 writes WH 1 after txn0 -> abort; txn3 shares district (2,3) with txn2 -> abort;
        # txn4 reads WH 2 like txn2 (RD-RD) and touches other rows -> commits
        assert commit.tolist() == [1, 0, 1, 0, 1], cc
        assert oid.tolist() == [0, 0, 3002, 0, 3002]
        wh, dist, cust, stock = db.table(0), db.table(1), db.table(2), db.table(4)
        assert _as_f(wh[1])[0] == 300100.0 and _as_f(wh[1])[1] == _as_f(wh0[1])[1]
        assert _as_f(dist[1])[0] == 30100.0 and dist[2][0] == 3001       # D_YTD / D_NEXT_O_ID of (1,1)
        assert dist[2][(2 - 1) * 10 + 2] == 3002                         # district (2,3)
        ci = 4  # customer (1,1,5) is row 4
        assert _as_f(cust[1])[ci] == -110.0 and _as_f(cust[2])[ci] == 110.0 and _as_f(cust[3])[ci] == 1.0
        srow = (2 - 1) * 2000 + 10 - 1 if p.num_wh == 2 else None
        s0 = int(st0[1][srow])
        exp = s0 - 4 if s0 > 14 else s0 - 4 + 91
        assert int(stock[1][srow]) == exp and int(stock[2][srow]) == 4 and int(stock[3][srow]) == 1
    db = O.TpccDB(p, 3)
    st0 = db.table(4)
    commit, oid, st = db.epoch(O.CALVIN, *e)
    assert commit.tolist() == [1] * 5 and oid.tolist() == [0, 0, 3002, 3003, 3002]
    wh, dist, stock = db.table(0), db.table(1), db.table(4)
    assert _as_f(wh[1])[0] == 300107.0
    assert dist[2][(2 - 1) * 10 + 2] == 3003
    srow = 2000 + 9
    s = int(st0[1][srow])
    for q in (4, 3):  # serial in sequence order
        s = s - q if s > q + 10 else s - q + 91
    assert int(stock[1][srow]) == s and int(stock[2][srow]) == 7 and int(stock[3][srow]) == 2


@pytest.fixture(scope="module")
def dv():
    from dvcc import tpcc
    return tpcc


@pytest.mark.parametrize("nw,parts,home", [(1, 1, 0), (2, 1, 0), (4, 2, 1), (200, 1, 0)])
def test_product_gen_matches_oracle(dv, nw, parts, home):
    for seed in (1, 98, 12345):
        po = _small(nw, part_cnt=parts)
        pp = dv.tpcc_params(nw, cust_per_dist=1000, max_items=2000, part_cnt=parts)
        a = O.tpcc_gen(po, 2000, seed, home)
        e = dv.gen(pp, 2000, seed, home)
        for x, y in zip(a[:5] + a[6:], [e.keys, e.types, e.tables, e.args, e.txn_begin, e.owner]):
            assert (x == y).all()
        assert (a[5] == e.txn_type).all()


def test_product_loader_matches_oracle(dv):
    po = _small(4, part_cnt=2)
    pp = dv.tpcc_params(4, cust_per_dist=1000, max_items=2000, part_cnt=2)
    for part in (0, 1):
        db = O.TpccDB(po, 5, part)
        for t in range(5):
            for x, y in zip(db.table(t), dv.table(pp, 5, t, part)):
                assert (x == y).all(), (part, t)
        # the secondary index: custNPKey of every customer, col 0 = its custKey
        ck, cl, _, _ = dv.table(pp, 5, 5, part)
        cust = dv.table(pp, 5, 2, part)[0]
        assert (cl == cust).all() and len(set(ck.tolist())) < len(ck)


def test_generator_mix(dv):
    """create_query / gen_payment / gen_new_order shape (tpcc_query.cpp)."""
    p = dv.tpcc_params(8, cust_per_dist=1000, max_items=2000, perc_payment=0.5)
    e = dv.gen(p, 20000, 3)
    n = np.diff(e.txn_begin.astype(np.int64))
    pay = e.txn_type == 1
    assert abs(pay.mean() - 0.5) < 0.02
    assert (n[pay] == 3).all()
    assert ((n[~pay] >= 3 + 10) & (n[~pay] <= 3 + 30) & ((n[~pay] - 3) % 2 == 0)).all()
    first = e.txn_begin[:-1][pay]
    by_name = (e.tables[first + 2] == 5).mean()
    assert abs(by_name - 0.6) < 0.03


GOLDEN_TPCC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "tpcc")


def _golden_names():
    return sorted(f[:-4] for f in os.listdir(GOLDEN_TPCC) if f.endswith(".npz"))


def test_tpcc_golden_set_complete():
    from golden.make_golden_tpcc import CASES
    assert sorted(CASES) == _golden_names()


@pytest.mark.parametrize("name", _golden_names())
def test_oracle_reproduces_tpcc_golden(name):
    from golden.make_golden_tpcc import make
    with np.load(os.path.join(GOLDEN_TPCC, name + ".npz")) as z:
        g = {k: z[k] for k in z.files}
    m = make(name)
    assert sorted(g) == sorted(m)
    for k in g:
        assert np.array_equal(g[k], m[k]), k


@pytest.mark.parametrize("name", _golden_names())
def test_product_generator_matches_tpcc_golden(dv, name):
    from golden.make_golden_tpcc import CASES, PARAMS
    cc, n_txn, seed, perc = CASES[name]
    e = dv.gen(dv.tpcc_params(perc_payment=perc, **PARAMS), n_txn, seed)
    with np.load(os.path.join(GOLDEN_TPCC, name + ".npz")) as z:
        for k, v in (("keys", e.keys), ("types", e.types), ("tables", e.tables), ("args", e.args),
                     ("txn_begin", e.txn_begin)):
            assert np.array_equal(z[k], v), k


def test_oracle_index_layout_matches_partition_loads():
    """or_tpcc_load_layout: the all-warehouse image with last-name lists per
    partition equals, partition by partition, the oracle loaded as that one
    partition (or_tpcc_load, PART_CNT 4) -- with 128 warehouses custNPKey's
    w * 10 + d overflows its 10 bits (tpcc_helper.cpp:35-43), so the lists
    really differ from the one-partition image's (checked too)."""
    P, nw = 4, 128
    kw = dict(cust_per_dist=1000, max_items=2000, perc_payment=1.0, mpr=0.0)
    p1 = O.tpcc_params(nw, part_cnt=1, **kw)
    pP = O.tpcc_params(nw, part_cnt=P, **kw)
    img = O.TpccDB(p1, 3, index_parts=P)
    flat = O.TpccDB(p1, 3)
    differs = False
    for q in range(P):
        keys, types, tables, args, tb, _, own = O.tpcc_gen(pP, 3000, 50 + q, home_part=q)
        # the txns that run on partition q only (no remote customer)
        local = [t for t in range(len(tb) - 1) if (own[tb[t]:tb[t + 1]] == q).all()]
        sel = np.concatenate([np.arange(tb[t], tb[t + 1]) for t in local])
        sizes = np.array([tb[t + 1] - tb[t] for t in local], np.int64)
        tbl = np.zeros(len(local) + 1, np.uint32)
        tbl[1:] = np.cumsum(sizes)
        e = (keys[sel], types[sel], tables[sel], args[sel], tbl)
        part = O.TpccDB(pP, 3, part_id=q)
        c_part, _, _ = part.epoch(O.CALVIN, *e)
        c_img, _, _ = img.epoch(O.CALVIN, *e, owner=own[sel])
        assert (c_part == c_img).all()
        ck, cref = part.table(2)[0], part.table(2)[1:]
        ik, icols = img.table(2)[0], img.table(2)[1:]
        idx = np.searchsorted(ik, ck)
        assert (ik[idx] == ck).all()
        for col in range(3):
            assert (icols[col][idx] == cref[col]).all(), (q, col)
        flat.epoch(O.CALVIN, *e)
    fk, fcols = flat.table(2)[0], flat.table(2)[1:]
    ik, icols = img.table(2)[0], img.table(2)[1:]
    assert (fk == ik).all()
    differs = any((fcols[c] != icols[c]).any() for c in range(3))
    assert differs, "expected the flat index to pick other customers at 128 warehouses"
