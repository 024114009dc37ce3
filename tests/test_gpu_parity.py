"""GPU parity: the HIP engine (through the C ABI) against the CPU oracle on the
same seeded epochs.  Integer work, so everything is bit-exact: per-txn commit
bytes, Calvin grant groups, the final F0 column of every row, the committed
read digest and the committed write count."""
import numpy as np
import pytest

import _oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import dvcc  # noqa: E402
from dvcc import CCEngine, DeviceEpoch, Epoch, YCSBQueryGenerator  # noqa: E402

CCS = [dvcc.NO_WAIT, dvcc.WAIT_DIE, dvcc.OCC, dvcc.CALVIN]
ORACLE_CC = {dvcc.NO_WAIT: O.NO_WAIT, dvcc.WAIT_DIE: O.WAIT_DIE, dvcc.OCC: O.OCC,
             dvcc.CALVIN: O.CALVIN}


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    yield


def _oracle_epoch(cc, tab, f0, e):
    return O.epoch_run(ORACLE_CC[cc], tab.ix, f0, e.n_txn, e.txn_begin, e.keys, e.types,
                       want_grant=(cc == dvcc.CALVIN))


def _gpu_epoch(eng, e, path):
    want_grant = eng.cc_alg == dvcc.CALVIN
    if path == "host":
        return eng.run_epoch(e, want_grant=want_grant)
    dep = DeviceEpoch(e)
    d_commit = torch.zeros(max(1, e.n_txn), dtype=torch.uint8, device="cuda")
    d_grant = (torch.zeros(max(1, e.n_acc), dtype=torch.int32, device="cuda")
               if want_grant else None)
    st = eng.run_epoch_device(dep, d_commit, d_grant)
    c = d_commit.cpu().numpy()[:e.n_txn]
    g = d_grant.cpu().numpy().view(np.uint32)[:e.n_acc] if want_grant else None
    return c, g, st


def _check(cc, rows, epochs, path="device", max_txn=None, max_acc=None, tail=True, el64=False,
           asynchronous=True, prefix=0, async_iters=0, lsd_sort=False):
    """prefix: dv_set_prefix (0 automatic -- epochs from 131,072 txns --, None
    off, else the prefix size for every longer epoch)."""
    tab = O.YcsbTable(rows)
    f0 = tab.f0.copy()
    eng = CCEngine(cc, max_txn or max(1, max(e.n_txn for e in epochs)),
                   max_acc or max(1, max(e.n_acc for e in epochs)), tail=tail, el64=el64,
                   asynchronous=asynchronous, lsd_sort=lsd_sort)
    eng.set_prefix(prefix)
    if async_iters:
        eng.set_async_limits(async_iters, 0)
    eng.load_ycsb_partition(rows)
    assert (eng.read_table(0, rows) == f0).all()
    for e in epochs:
        c_ref, g_ref, st_ref = _oracle_epoch(cc, tab, f0, e)
        c, g, st = _gpu_epoch(eng, e, path)
        assert (c == c_ref).all(), f"commit mismatch: {int((c != c_ref).sum())} txns"
        if cc == dvcc.CALVIN:
            assert (g == g_ref).all(), f"grant mismatch: {int((g != g_ref).sum())}"
        assert st.committed == st_ref.committed
        assert st.aborted == st_ref.aborted
        assert st.write_cnt == st_ref.write_cnt
        assert st.read_digest == st_ref.read_digest
        assert (eng.read_table(0, rows) == f0).all(), "table state mismatch"
    eng.close()
    return st


@pytest.mark.parametrize("cc", CCS)
def test_hand_scenario(cc):
    txns = [[(1, 1)], [(1, 0)], [(2, 0), (3, 1)], [(2, 0)], [(2, 1)], [(3, 0)]]
    keys = np.array([k for t in txns for k, _ in t], np.uint64)
    types = np.array([ty for t in txns for _, ty in t], np.uint8)
    tb = np.array([0] + list(np.cumsum([len(t) for t in txns])), np.uint32)
    _check(cc, 8, [Epoch(keys, types, tb)])


@pytest.mark.parametrize("path", ["device", "host"])
@pytest.mark.parametrize("cc", CCS)
def test_contended_epoch(cc, path):
    g = YCSBQueryGenerator(1 << 12, zipf_theta=0.9)
    _check(cc, 1 << 12, [g.gen(4096, 1234)], path=path)


@pytest.mark.parametrize("cc", CCS)
@pytest.mark.parametrize("n_txn,rows,theta", [(1, 1000, 0.9), (7, 1000, 0.6), (409, 999, 0.9),
                                              (5000, 77777, 0.3), (20000, 1 << 16, 0.99)])
def test_ragged_sizes(cc, n_txn, rows, theta):
    g = YCSBQueryGenerator(rows, zipf_theta=theta, txn_write_perc=0.5, tup_write_perc=0.5)
    _check(cc, rows, [g.gen(n_txn, 7 + n_txn)])


@pytest.mark.parametrize("cc", CCS)
def test_double_buffered_host_input(cc):
    """dv_epoch_stage_host / dv_epoch_run_staged: epoch k+1's records copied
    on the copy stream while epoch k runs, alternating slots -- the same
    decisions and table state as the oracle epoch after epoch; an empty slot
    is DV_ERR_STATE, a malformed txn_begin DV_ERR_ARG."""
    rows = 1 << 14
    g = YCSBQueryGenerator(rows, zipf_theta=0.9)
    epochs = [g.gen(3000, s) for s in (11, 12, 13, 14, 15)]
    tab = O.YcsbTable(rows)
    f0 = tab.f0.copy()
    eng = CCEngine(cc, 3000, max(e.n_acc for e in epochs))
    try:
        eng.load_ycsb_partition(rows)
        bufs = [(torch.from_numpy(e.to_access_array().view(np.uint8)).pin_memory(),
                 torch.from_numpy(np.ascontiguousarray(e.txn_begin, dtype=np.uint32)).pin_memory(),
                 e.n_acc, e.n_txn) for e in epochs]
        commit = torch.zeros(3000, dtype=torch.uint8).pin_memory()
        with pytest.raises(dvcc.DvccError) as ex:
            eng.run_staged(1, commit)
        assert ex.value.code == dvcc._lib.DV_ERR_STATE
        bad_tb = bufs[0][1].clone()
        bad_tb[5] = bad_tb[7]  # not monotone
        with pytest.raises(dvcc.DvccError) as ex:
            eng.stage_host(0, bufs[0][0], bad_tb, bufs[0][2], bufs[0][3])
        assert ex.value.code == dvcc._lib.DV_ERR_ARG
        eng.stage_host(0, *bufs[0])
        for i, e in enumerate(epochs):
            if i + 1 < len(epochs):
                eng.stage_host((i + 1) % 2, *bufs[i + 1])
            st = eng.run_staged(i % 2, commit)
            c_ref, _, st_ref = _oracle_epoch(cc, tab, f0, e)
            assert (commit.numpy()[:e.n_txn] == c_ref).all(), i
            assert st.committed == st_ref.committed and st.read_digest == st_ref.read_digest
        assert (eng.read_table(0, rows) == f0).all()
    finally:
        eng.close()


@pytest.mark.parametrize("cc", CCS)
def test_double_buffered_row_records(cc):
    """dv_epoch_stage_host_rows: 4-byte records (key | write << 31) with
    txn_begin, slots alternating with 16-byte records; epochs with empty txns
    (equal starts) and a txn count that is no multiple of a wave's 64"""
    rows = 1 << 14
    g = YCSBQueryGenerator(rows, zipf_theta=0.9)
    epochs = [g.gen(n, s) for n, s in ((3001, 21), (2999, 22), (3000, 23))]
    rng = np.random.default_rng(3)
    lens = rng.integers(0, 9, size=1777)  # empty txns among them
    lens[:3] = 0
    tb = np.zeros(len(lens) + 1, np.uint32)
    tb[1:] = np.cumsum(lens)
    epochs.append(Epoch(rng.integers(0, rows, size=int(tb[-1])).astype(np.uint64),
                        (rng.random(int(tb[-1])) < 0.4).astype(np.uint8), tb))
    tab = O.YcsbTable(rows)
    f0 = tab.f0.copy()
    eng = CCEngine(cc, 3001, max(e.n_acc for e in epochs))
    try:
        eng.load_ycsb_partition(rows)

        def stage(slot, e):
            tbp = torch.from_numpy(np.ascontiguousarray(e.txn_begin, dtype=np.uint32)).pin_memory()
            if slot == 0:
                eng.stage_host_rows(0, torch.from_numpy(e.to_row_records()).pin_memory(), tbp, e.n_acc, e.n_txn)
            else:
                eng.stage_host(1, torch.from_numpy(e.to_access_array().view(np.uint8)).pin_memory(), tbp,
                               e.n_acc, e.n_txn)
        commit = torch.zeros(3001, dtype=torch.uint8).pin_memory()
        stage(0, epochs[0])
        for i, e in enumerate(epochs):
            if i + 1 < len(epochs):
                stage((i + 1) % 2, epochs[i + 1])
            st = eng.run_staged(i % 2, commit)
            c_ref, _, st_ref = _oracle_epoch(cc, tab, f0, e)
            assert (commit.numpy()[:e.n_txn] == c_ref).all(), i
            assert st.committed == st_ref.committed and st.read_digest == st_ref.read_digest
        assert (eng.read_table(0, rows) == f0).all()
        with pytest.raises(ValueError):
            Epoch(np.array([1 << 31], np.uint64), np.zeros(1, np.uint8), np.array([0, 1], np.uint32)).to_row_records()
    finally:
        eng.close()


@pytest.mark.parametrize("cc", CCS)
def test_epochs_carry_table_state(cc):
    g = YCSBQueryGenerator(1 << 14, zipf_theta=0.8)
    _check(cc, 1 << 14, [g.gen(3000, s) for s in (1, 2, 3)])


@pytest.mark.parametrize("cc", CCS)
def test_medium_epoch(cc):
    g = YCSBQueryGenerator(1 << 20, zipf_theta=0.9)
    _check(cc, 1 << 20, [g.gen(1 << 16, 99)])


@pytest.mark.parametrize("cc", CCS)
def test_empty_epoch(cc):
    e = Epoch(np.zeros(0, np.uint64), np.zeros(0, np.uint8), np.zeros(1, np.uint32))
    _check(cc, 16, [e], max_txn=4, max_acc=16)


def test_missing_key_reports_error():
    eng = CCEngine(dvcc.NO_WAIT, 4, 16)
    eng.load_ycsb_partition(16)
    e = Epoch(np.array([3, 1000], np.uint64), np.array([0, 1], np.uint8), np.array([0, 2], np.uint32))
    with pytest.raises(dvcc.DvccError) as ex:
        eng.run_epoch(e)
    assert ex.value.code == dvcc._lib.DV_ERR_KEY_NOT_FOUND
    # the context stays usable
    e2 = Epoch(np.array([3], np.uint64), np.array([1], np.uint8), np.array([0, 1], np.uint32))
    c, _, st = eng.run_epoch(e2)
    assert c.tolist() == [1] and st.committed == 1


@pytest.mark.parametrize("hash_kind,part_cnt", [(dvcc._lib.HASH_MOD, 1), (dvcc._lib.HASH_YCSB, 1),
                                                (dvcc._lib.HASH_YCSB, 4)])
def test_direct_map_key_tags(hash_kind, part_cnt):
    """Implicit-row direct maps probe a one-byte key tag (key_tag,
    dvcc_internal.h) and the pkey word only behind the wide-tag sentinel:
    every loaded key is found, whether its tag is narrow, at the edge
    (codes 253-255) or wide; keys sharing a bucket with a loaded row but not
    loaded -- other quotient, other residue -- are DV_ERR_KEY_NOT_FOUND."""
    nb = 64
    P = part_cnt if hash_kind == dvcc._lib.HASH_YCSB else 1
    rng = np.random.default_rng(3)
    # key of bucket b: (q * nb + b) * P + lo, quotients from narrow to wide
    qs = rng.choice([0, 1, 2, 60, 63, 254 // max(P, 1), 255, 256, 10 ** 6, 2 ** 40], size=nb)
    lo = rng.integers(0, P, size=nb) if P > 1 else np.zeros(nb, np.int64)
    keys = ((qs.astype(np.uint64) * np.uint64(nb) + np.arange(nb, dtype=np.uint64)) * np.uint64(P)
            + lo.astype(np.uint64))
    eng = CCEngine(dvcc.NO_WAIT, 8, 64, part_cnt=part_cnt if hash_kind == dvcc._lib.HASH_YCSB else 1)
    try:
        eng.create_table(0, nb, nb, hash_kind)
        f0 = np.arange(nb, dtype=np.uint64) * np.uint64(7) + np.uint64(11)
        eng.load_table(0, keys, f0)
        assert (eng.read_rows(keys) == f0).all()
        for b in range(nb):
            others = [((int(qs[b]) + d) * nb + b) * P + int(lo[b]) for d in (1, -1) if int(qs[b]) + d >= 0]
            if P > 1:
                others.append((int(qs[b]) * nb + b) * P + (int(lo[b]) + 1) % P)
            for k in others:
                with pytest.raises(dvcc.DvccError) as ex:
                    eng.read_rows(np.array([k], np.uint64))
                assert ex.value.code == dvcc._lib.DV_ERR_KEY_NOT_FOUND, (b, k)
        # and through an epoch's probe
        e = _epoch_of([[(int(keys[3]), 1), (int(keys[9]), 0)], [(int(keys[3]) + nb * P, 1)]])
        with pytest.raises(dvcc.DvccError) as ex:
            eng.run_epoch(e)
        assert ex.value.code == dvcc._lib.DV_ERR_KEY_NOT_FOUND
        c, _, st = eng.run_epoch(_epoch_of([[(int(keys[3]), 1), (int(keys[9]), 0)], [(int(keys[60]), 1)]]))
        assert st.committed == 2
    finally:
        eng.close()


def _epoch_of(txns):
    keys = np.array([k for t in txns for k, _ in t], np.uint64)
    types = np.array([ty for t in txns for _, ty in t], np.uint8)
    tb = np.array([0] + list(np.cumsum([len(t) for t in txns])), np.uint32)
    return Epoch(keys, types, tb)


@pytest.mark.parametrize("cc", CCS)
def test_repeated_rows_hand(cc):
    """A txn touching one row several times: NO_WAIT /
    WAIT_DIE abort it unless every access to the row reads (its own lock
    conflicts, row_lock.cpp:69, 86-90); OCC puts the row in its write set if
    any access writes it; CALVIN locks it once (txn.cpp:778-788)."""
    txns = [[(1, 0), (1, 0)], [(2, 0), (2, 1)], [(3, 1), (3, 0)], [(2, 0)], [(3, 0), (4, 1), (3, 0)]]
    _check(cc, 8, [_epoch_of(txns)])


@pytest.mark.parametrize("cc", CCS)
@pytest.mark.parametrize("rows,R,theta", [(64, 6, 0.5), (1 << 12, 10, 0.9), (1 << 14, 16, 0.99)])
def test_repeated_rows_random(cc, rows, R, theta):
    """Keys drawn with replacement inside a txn (the YCSB generator never
    repeats one), over several epochs and all decision-path knobs."""
    rng = np.random.default_rng(rows + R)
    epochs = []
    for k in range(2):
        n_txn = 3000
        lens = rng.integers(1, R + 1, size=n_txn)
        tb = np.zeros(n_txn + 1, np.uint32)
        tb[1:] = np.cumsum(lens)
        n = int(tb[-1])
        hot = max(4, rows // 64)
        keys = np.where(rng.random(n) < theta, rng.integers(0, hot, size=n), rng.integers(0, rows, size=n))
        # force a repeat in about a third of the txns
        for t in range(0, n_txn, 3):
            a, b = int(tb[t]), int(tb[t + 1])
            if b - a >= 2:
                keys[b - 1] = keys[a]
        types = (rng.random(n) < 0.5).astype(np.uint8)
        epochs.append(Epoch(keys.astype(np.uint64), types, tb))
    for knobs in (dict(), dict(asynchronous=False), dict(tail=False, asynchronous=False), dict(el64=True)):
        _check(cc, rows, epochs, **knobs)


def test_txn_longer_than_declared_bound_is_rejected():
    """max_txn_acc under-declared (ERRB_BIG): the epoch fails with DV_ERR_ARG
    before anything executes, and the context stays usable."""
    rows = 64
    e = _epoch_of([[(k, 1) for k in range(20)], [(30, 1)]])
    for cc in (dvcc.NO_WAIT, dvcc.WAIT_DIE, dvcc.OCC):  # CALVIN: any length <= 128
        eng = CCEngine(cc, 4, 64)
        eng.load_ycsb_partition(rows)
        before = eng.read_table(0, rows)
        dep = DeviceEpoch(e)
        dep.max_txn_acc = 16  # the first txn has 20 accesses
        with pytest.raises(dvcc.DvccError) as ex:
            eng.run_epoch_device(dep, torch.zeros(4, dtype=torch.uint8, device="cuda"))
        assert ex.value.code == dvcc._lib.DV_ERR_ARG
        assert (eng.read_table(0, rows) == before).all(), "a rejected epoch changed the table"
        c, _, st = eng.run_epoch(e)
        assert st.committed == 2
        eng.close()


@pytest.mark.parametrize("cc", CCS)
def test_rejected_epoch_leaves_table_unchanged(cc):
    """A missing key (and, from host buffers, a record outside its txn's range)
    rejects the whole epoch before execution: no row changes, for every CC
    (CALVIN has no rounds in between, so the gate is on the execution)."""
    rows = 64
    eng = CCEngine(cc, 8, 64)
    eng.load_ycsb_partition(rows)
    before = eng.read_table(0, rows)
    bad = _epoch_of([[(1, 1), (2, 1)], [(3, 1), (1000, 1)], [(5, 1)]])
    with pytest.raises(dvcc.DvccError) as ex:
        eng.run_epoch(bad)
    assert ex.value.code == dvcc._lib.DV_ERR_KEY_NOT_FOUND
    assert (eng.read_table(0, rows) == before).all()
    good = _epoch_of([[(1, 1), (2, 1)], [(3, 1), (4, 1)], [(5, 1)]])
    acc = good.to_access_array()
    acc["txn_seq"][2] = 0  # the first access of txn 1 claims txn 0
    commit = np.zeros(3, np.uint8)
    with pytest.raises(dvcc.DvccError) as ex:
        eng.run_epoch_host(acc, np.ascontiguousarray(good.txn_begin), good.n_acc, good.n_txn, commit)
    assert ex.value.code == dvcc._lib.DV_ERR_TXN_RANGE
    assert (eng.read_table(0, rows) == before).all()
    c, _, st = eng.run_epoch(good)
    assert st.committed == 3 and st.write_cnt == 5
    eng.close()


def test_wait_die_timestamps_must_rise_in_sequence_order():
    """dv_epoch_run's ts: WAIT_DIE decisions equal sequence order only when ts
    rises with it (otherwise the reference waits, row_lock.cpp:119-147)."""
    import ctypes
    e = _epoch_of([[(1, 1)], [(1, 0)], [(2, 1)]])
    eng = CCEngine(dvcc.WAIT_DIE, 4, 16)
    eng.load_ycsb_partition(8)
    acc = e.to_access_array()
    tb = np.ascontiguousarray(e.txn_begin)
    commit = np.zeros(3, np.uint8)
    st = dvcc._lib.Stats()
    L = dvcc._lib.lib()
    for ts, ok in (([5, 9, 12], True), ([5, 5, 12], False), ([9, 5, 12], False)):
        t = np.array(ts, np.uint64)
        rc = L.dv_epoch_run(eng._ctx, acc.ctypes.data, e.n_acc, tb.ctypes.data, 3, t.ctypes.data,
                            commit.ctypes.data, None, ctypes.byref(st))
        assert (rc == 0) == ok, (ts, rc)
        if ok:
            assert commit.tolist() == [1, 0, 1]
    eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n_txn,prefix", [(3000, None), (40_000, 512)])
def test_wait_die_device_timestamps(n_txn, prefix):
    """dv_epoch_dev.ts on the device entry points (the plain path and a
    prefix-kill epoch): rising timestamps give the sequence-order decisions;
    a pair that does not rise is DV_ERR_ARG from the probe, and no row
    changes; NO_WAIT never reads them."""
    rows = 1 << 16
    g = YCSBQueryGenerator(rows, zipf_theta=0.9, txn_write_perc=1.0, tup_write_perc=0.5)
    e = g.gen(n_txn, 31)
    tab = O.YcsbTable(rows)
    f0 = tab.f0.copy()
    c_ref, _, st_ref = _oracle_epoch(dvcc.WAIT_DIE, tab, f0, e)
    eng = CCEngine(dvcc.WAIT_DIE, n_txn, e.n_acc)
    eng.load_ycsb_partition(rows)
    eng.set_prefix(prefix)
    before = eng.read_table(0, rows)
    dep = DeviceEpoch(e)
    ts = torch.arange(n_txn, dtype=torch.int64, device="cuda") * 3 + 7
    ts[n_txn // 2] = ts[n_txn // 2 - 1]  # not rising
    dep.ts = ts
    d = torch.zeros(n_txn, dtype=torch.uint8, device="cuda")
    with pytest.raises(dvcc.DvccError) as ei:
        eng.run_epoch_device(dep, d)
    assert ei.value.code == dvcc._lib.DV_ERR_ARG
    assert (eng.read_table(0, rows) == before).all()
    ts[n_txn // 2] += 1
    st = eng.run_epoch_device(dep, d)
    assert (d.cpu().numpy() == c_ref).all()
    assert (st.committed, st.read_digest) == (st_ref.committed, st_ref.read_digest)
    assert (eng.read_table(0, rows) == f0).all()
    eng.close()
    nw = CCEngine(dvcc.NO_WAIT, n_txn, e.n_acc)
    nw.load_ycsb_partition(rows)
    ts[3] = 0
    nw.run_epoch_device(dep, d)  # (ignored)
    nw.close()


@pytest.mark.parametrize("cc", [dvcc.NO_WAIT, dvcc.OCC])
@pytest.mark.parametrize("max_iters", [1, 3])
def test_async_rounds_yield_and_resume(cc, max_iters):
    """Forward progress of the asynchronous rounds: workgroups forced to yield
    after max_iters iterations; the host resumes the synchronous rounds from
    the launch's input state and decisions stay bit-exact."""
    rows = 1 << 20
    g = YCSBQueryGenerator(rows, zipf_theta=0.9)
    epochs = [g.gen(1 << 16, 95), g.gen(1 << 16, 94)]
    tab = O.YcsbTable(rows)
    f0 = tab.f0.copy()
    eng = CCEngine(cc, 1 << 16, max(e.n_acc for e in epochs))
    eng.load_ycsb_partition(rows)
    eng.set_async_limits(max_iters, 0)
    yields = 0
    for e in epochs:
        c_ref, _, st_ref = _oracle_epoch(cc, tab, f0, e)
        c, _, st = _gpu_epoch(eng, e, "device")
        assert (c == c_ref).all()
        assert st.read_digest == st_ref.read_digest and st.write_cnt == st_ref.write_cnt
        assert (eng.read_table(0, rows) == f0).all()
        yields += st.async_yields
    assert yields > 0, "no asynchronous launch yielded"
    eng.close()


def test_calvin_repeat_access_keeps_first_lock_type():
    # TxnManager::get_lock dedups on calvin_locked_rows (txn.cpp:778-788)
    txns = [[(5, 0), (5, 1)], [(5, 0)], [(6, 1), (5, 1)], [(5, 0), (6, 0), (5, 0)]]
    keys = np.array([k for t in txns for k, _ in t], np.uint64)
    types = np.array([ty for t in txns for _, ty in t], np.uint8)
    tb = np.array([0] + list(np.cumsum([len(t) for t in txns])), np.uint32)
    e = Epoch(keys, types, tb)
    tab = O.YcsbTable(8)
    c_ref, g_ref, _ = O.epoch_run(O.CALVIN, tab.ix, tab.f0.copy(), 4, tb, keys, types, want_grant=True)
    eng = CCEngine(dvcc.CALVIN, 4, 16)
    eng.load_ycsb_partition(8)
    c, g, _ = eng.run_epoch(e, want_grant=True)
    assert (c == c_ref).all() and (g == g_ref).all()


def test_chained_index_table():
    # dv_load_table with key % nbuckets chains (index_hash.cpp:69-83, 217-231)
    rows = 5000
    rng = np.random.default_rng(3)
    keys = rng.permutation(np.arange(rows, dtype=np.uint64) * 7 + 3)
    f0 = rng.integers(1, 2**63, size=rows, dtype=np.uint64)
    ix = O.MultiIndex(97, 1, 0, list(zip(keys.tolist(), range(rows))))
    n_txn, R = 2000, 6
    ak = keys[rng.integers(0, rows // 10, size=n_txn * R)]
    at = rng.integers(0, 2, size=n_txn * R).astype(np.uint8)
    # drop repeated keys inside a txn
    for t in range(n_txn):
        seen = set()
        for j in range(R):
            while int(ak[t * R + j]) in seen:
                ak[t * R + j] = keys[rng.integers(0, rows)]
            seen.add(int(ak[t * R + j]))
    tb = (np.arange(n_txn + 1) * R).astype(np.uint32)
    for cc in CCS:
        ref_f0 = f0.copy()
        c_ref, g_ref, st_ref = O.epoch_run(ORACLE_CC[cc], ix.ix, ref_f0, n_txn, tb, ak, at,
                                           want_grant=cc == dvcc.CALVIN)
        eng = CCEngine(cc, n_txn, n_txn * R)
        eng.create_table(0, rows, 97, dvcc.HASH_MOD)
        eng.load_table(0, keys, f0)
        c, g, st = eng.run_epoch(Epoch(ak, at, tb), want_grant=cc == dvcc.CALVIN)
        assert (c == c_ref).all()
        if cc == dvcc.CALVIN:
            assert (g == g_ref).all()
        assert st.read_digest == st_ref.read_digest
        assert (eng.read_table(0, rows) == ref_f0).all()
        assert (eng.read_rows(keys[:100]) == ref_f0[:100]).all()
        eng.close()


def test_host_records_must_match_txn_begin():
    """dv_epoch_run checks every record's txn_seq against the CSR txn_begin
    (on the device); a record placed in another txn's range is rejected."""
    g = YCSBQueryGenerator(1 << 12, zipf_theta=0.6)
    e = g.gen(500, 5)
    eng = CCEngine(dvcc.NO_WAIT, 500, 5000)
    eng.load_ycsb_partition(1 << 12)
    acc = e.to_access_array()
    tb = np.ascontiguousarray(e.txn_begin, dtype=np.uint32)
    commit = np.zeros(500, np.uint8)
    st = eng.run_epoch_host(acc, tb, e.n_acc, e.n_txn, commit)
    assert st.n_txn == 500
    acc["txn_seq"][int(tb[7])] = 8  # first access of txn 7 claims txn 8
    with pytest.raises(dvcc.DvccError):
        eng.run_epoch_host(acc, tb, e.n_acc, e.n_txn, commit)
    eng.close()


@pytest.mark.parametrize("order", ["bucket", "shuffled"])
def test_direct_index_table(order):
    """dv_load_table with one key per bucket: keys loaded in bucket order give
    an implicit-row map (probes read the primary-key column), shuffled keys a
    {key, row} entry per bucket.  Same decisions, table and digests either
    way, and a key that is not in the table is reported."""
    rows = 4096
    rng = np.random.default_rng(11)
    keys = np.arange(rows, dtype=np.uint64) + np.uint64(5 * rows)  # key % rows: distinct buckets
    if order == "shuffled":
        keys = rng.permutation(keys)
    f0 = rng.integers(1, 2**63, size=rows, dtype=np.uint64)
    ix = O.MultiIndex(rows, 1, 0, list(zip(keys.tolist(), range(rows))))
    n_txn, R = 1500, 8
    ak = np.empty(n_txn * R, np.uint64)
    for t in range(n_txn):
        ak[t * R:(t + 1) * R] = keys[rng.choice(rows // 4, size=R, replace=False)]
    at = rng.integers(0, 2, size=n_txn * R).astype(np.uint8)
    tb = (np.arange(n_txn + 1) * R).astype(np.uint32)
    for cc in CCS:
        ref_f0 = f0.copy()
        c_ref, g_ref, st_ref = O.epoch_run(ORACLE_CC[cc], ix.ix, ref_f0, n_txn, tb, ak, at,
                                           want_grant=cc == dvcc.CALVIN)
        eng = CCEngine(cc, n_txn, n_txn * R)
        eng.create_table(0, rows, rows, dvcc.HASH_MOD)
        eng.load_table(0, keys, f0)
        c, g, st = eng.run_epoch(Epoch(ak, at, tb), want_grant=cc == dvcc.CALVIN)
        assert (c == c_ref).all()
        if cc == dvcc.CALVIN:
            assert (g == g_ref).all()
        assert st.read_digest == st_ref.read_digest
        assert (eng.read_table(0, rows) == ref_f0).all()
        missing = ak.copy()
        missing[7] = np.uint64(3 * rows + 1)  # bucket 1 holds another key
        with pytest.raises(dvcc.DvccError):
            eng.run_epoch(Epoch(missing, at, tb))
        eng.close()


@pytest.mark.parametrize("cc", [dvcc.NO_WAIT, dvcc.WAIT_DIE, dvcc.OCC])
def test_dense_ycsb_table_beside_a_second_table(cc):
    """A dense YCSB partition (table 0) beside a chained table 1 in one
    context: the execution takes a table-0 read's primary key from its row
    (row - base, the dense map), but a table-1 row's from its pkey column --
    the committed-read digest and both tables equal the oracle's over the
    combined key space."""
    rows0, n1 = 1 << 14, 3000
    rng = np.random.default_rng(21)
    keys1 = (np.uint64(rows0 * 10) + rng.permutation(n1 * 4)[:n1].astype(np.uint64))
    f01 = rng.integers(1, 2**63, size=n1, dtype=np.uint64)
    base = O.YcsbTable(rows0)
    ix = O.MultiIndex(rows0 + n1, 1, 0, list(zip(range(rows0), range(rows0)))
                      + list(zip(keys1.tolist(), range(rows0, rows0 + n1))))
    n_txn, R = 2000, 8
    ak = np.empty(n_txn * R, np.uint64)
    tabs = np.zeros(n_txn * R, np.uint8)
    at = rng.integers(0, 2, size=n_txn * R).astype(np.uint8)
    for t in range(n_txn):
        half = R // 2
        ak[t * R:t * R + half] = rng.choice(rows0 // 4, size=half, replace=False).astype(np.uint64)
        ak[t * R + half:(t + 1) * R] = keys1[rng.choice(n1, size=R - half, replace=False)]
        tabs[t * R + half:(t + 1) * R] = 1
    tb = (np.arange(n_txn + 1) * R).astype(np.uint32)
    ref_f0 = np.concatenate([base.f0, f01])
    c_ref, _, st_ref = O.epoch_run(ORACLE_CC[cc], ix.ix, ref_f0, n_txn, tb, ak, at)
    eng = CCEngine(cc, n_txn, n_txn * R)
    try:
        eng.load_ycsb_partition(rows0)
        eng.create_table(1, n1, 2 * n1, dvcc.HASH_MOD)
        eng.load_table(1, keys1, f01)
        c, _, st = eng.run_epoch(Epoch(ak, at, tb, tables=tabs))
        assert (c == c_ref).all()
        assert (st.committed, st.read_digest, st.write_cnt) == (st_ref.committed, st_ref.read_digest,
                                                               st_ref.write_cnt)
        assert (eng.read_table(0, rows0) == ref_f0[:rows0]).all()
        assert (eng.read_rows(keys1, table=1) == ref_f0[rows0:]).all()
    finally:
        eng.close()


# ---- BASELINE.json sizes (configs B, C, D at N=1), bit-exact against the oracle
@pytest.mark.slow
def test_config_b_calvin_full():
    g = YCSBQueryGenerator(16_777_216, zipf_theta=0.6, txn_write_perc=1.0, tup_write_perc=0.5)
    _check(dvcc.CALVIN, 16_777_216, [g.gen(65_536, dvcc.epoch_seed(0, 0))])


@pytest.mark.slow
def test_config_c_occ_full():
    g = YCSBQueryGenerator(100_000_000, zipf_theta=0.9, txn_write_perc=1.0, tup_write_perc=0.5)
    st = _check(dvcc.OCC, 100_000_000, [g.gen(1_048_576, dvcc.epoch_seed(0, 0))])
    assert st.rounds > 1


@pytest.mark.slow
@pytest.mark.parametrize("cc", [dvcc.NO_WAIT, dvcc.OCC])
def test_config_d_single_partition_full(cc):
    g = YCSBQueryGenerator(16_777_216, zipf_theta=0.9, txn_write_perc=1.0, tup_write_perc=0.5)
    _check(cc, 16_777_216, [g.gen(1_048_576, dvcc.epoch_seed(0, 1))])


@pytest.mark.parametrize("tail,el64,asyn", [(True, False, True), (True, False, False),
                                            (False, False, False), (True, True, True),
                                            (False, True, True)])
@pytest.mark.parametrize("rows,req,theta", [(64, 4, 0.5), (1 << 14, 8, 0.95), (1 << 12, 16, 0.99)])
@pytest.mark.parametrize("cc", [dvcc.NO_WAIT, dvcc.OCC])
def test_many_rounds(cc, rows, req, theta, tail, el64, asyn):
    """Long decision chains: the pipelined round loop (rounds queued ahead of
    the host, no-op rounds past the fixpoint) over many rounds, with and
    without the single-workgroup tail kernel."""
    gen = YCSBQueryGenerator(rows, zipf_theta=theta, req_per_query=req)
    epochs = [gen.gen(20_000, 300 + k) for k in range(2)]
    st = _check(cc, rows, epochs, tail=tail, el64=el64, asynchronous=asyn)
    assert st.rounds >= 2


# ---- prefix-kill epochs (dvcc_prefix.hip): the prefix decided alone, later
# txns conflicting with its commits killed, the survivors decided as a
# renumbered sub-epoch -- bit-exact against the oracle however the epoch is cut
@pytest.mark.parametrize("cc", [dvcc.NO_WAIT, dvcc.WAIT_DIE, dvcc.OCC])
@pytest.mark.parametrize("prefix", [1, 17, 500, 4096])
def test_prefix_kill_sizes(cc, prefix):
    """each stage: round 0, then one asynchronous launch whose statuses stay
    in the fact words for the stage's consumer (no finalize)"""
    g = YCSBQueryGenerator(1 << 16, zipf_theta=0.9)
    _check(cc, 1 << 16, [g.gen(20_000, 61), g.gen(20_000, 62)], prefix=prefix)


@pytest.mark.parametrize("knobs", [dict(asynchronous=False), dict(tail=False, asynchronous=False),
                                   dict(el64=True), dict(async_iters=1), dict(async_iters=2),
                                   dict(async_iters=3)])
@pytest.mark.parametrize("cc", [dvcc.NO_WAIT, dvcc.OCC])
def test_prefix_kill_knobs(cc, knobs):
    """the stages' rounds on every decision path: pipelined passes, no tail,
    64-bit elements, asynchronous launches forced to yield (both stages then
    resume synchronously)"""
    g = YCSBQueryGenerator(1 << 18, zipf_theta=0.95, req_per_query=12)
    _check(cc, 1 << 18, [g.gen(30_000, 71)], prefix=2000, **knobs)


@pytest.mark.parametrize("theta", [0.0, 0.5, 0.99])
@pytest.mark.parametrize("cc", [dvcc.NO_WAIT, dvcc.OCC])
def test_prefix_kill_automatic(cc, theta):
    """the default cut of a 131,072-txn epoch, uniform to very skewed keys
    (uniform: the kill removes little, the survivors' sub-epoch is most of
    the epoch)"""
    g = YCSBQueryGenerator(1 << 20, zipf_theta=theta)
    _check(cc, 1 << 20, [g.gen(131_072, 81)])


def test_prefix_kill_repeated_rows():
    rng = np.random.default_rng(5)
    n_txn = 6000
    lens = rng.integers(1, 11, size=n_txn)
    tb = np.zeros(n_txn + 1, np.uint32)
    tb[1:] = np.cumsum(lens)
    n = int(tb[-1])
    keys = np.where(rng.random(n) < 0.8, rng.integers(0, 64, size=n), rng.integers(0, 4096, size=n))
    for t in range(0, n_txn, 2):
        a, b = int(tb[t]), int(tb[t + 1])
        if b - a >= 2:
            keys[b - 1] = keys[a]
    e = Epoch(keys.astype(np.uint64), (rng.random(n) < 0.5).astype(np.uint8), tb)
    for cc in (dvcc.NO_WAIT, dvcc.WAIT_DIE, dvcc.OCC):
        _check(cc, 4096, [e], prefix=300)


@pytest.mark.parametrize("cc", CCS)
def test_sorts_past_2_20_rows(cc):
    """rows past 2^20 (24-bit sort keys, 3 passes of 8 bits): whole epochs,
    and prefix and survivors stages (their count only on the device)"""
    rows = 1 << 22
    g = YCSBQueryGenerator(rows, zipf_theta=0.9)
    eps = [g.gen(30_000, 131), g.gen(7_000, 132), g.gen(1, 133)]
    _check(cc, rows, eps, prefix=None)
    if cc != dvcc.CALVIN:
        _check(cc, rows, eps[:2], prefix=3000)


def _hot_read_epoch(rows, n_txn, seed, hot=0, R=4):
    """every txn reads row `hot` first, then R - 1 random rows (half written):
    one sort bucket holds every txn's hot access -- more than a workgroup's
    LDS takes (k_bucket_sort's global-memory passes)"""
    rng = np.random.default_rng(seed)
    keys = rng.integers(0, rows, size=(n_txn, R)).astype(np.uint64)
    keys[:, 0] = hot
    types = (rng.random((n_txn, R)) < 0.5).astype(np.uint8)
    types[:, 0] = 0
    tb = (np.arange(n_txn + 1) * R).astype(np.uint32)
    return Epoch(keys.reshape(-1), types.reshape(-1), tb)


@pytest.mark.parametrize("cc", CCS)
@pytest.mark.parametrize("rows", [1 << 16, 1 << 20, 1 << 24])
def test_bucket_sort_oversized_bucket(cc, rows):
    """row bits above the bucket digit: 8 (one pass), 12 and 16 (two passes,
    the result copied out of the scratch region); a 40,000-key bucket and the
    rest in LDS; whole epochs and, for the 2PL / OCC algorithms, prefix and
    survivors stages (counts on the device)"""
    e = _hot_read_epoch(rows, 40_000, 7)
    _check(cc, rows, [e], prefix=None)
    if cc != dvcc.CALVIN:
        _check(cc, rows, [e], prefix=5000)


@pytest.mark.parametrize("cc", CCS)
def test_lsd_sort_knob(cc):
    """DV_FLAG_LSD_SORT: the plain LSD passes on the sizes that take the
    bucket sort by default, same decisions"""
    rows = 1 << 22
    g = YCSBQueryGenerator(rows, zipf_theta=0.9)
    eps = [g.gen(30_000, 141), _hot_read_epoch(rows, 20_000, 8)]
    _check(cc, rows, eps, prefix=None, lsd_sort=True)
    if cc != dvcc.CALVIN:
        _check(cc, rows, eps, prefix=3000, lsd_sort=True)


def _repeat_epoch(rows, n_txn, seed, R=6):
    """txns that touch some row two or three times (mixed types): round 0's
    repeats -- transparent, the group's first access carrying the OR of the
    types"""
    rng = np.random.default_rng(seed)
    keys = rng.integers(0, rows, size=(n_txn, R)).astype(np.uint64)
    keys[:, 3] = keys[:, 1]
    keys[::3, 5] = keys[::3, 1]
    types = (rng.random((n_txn, R)) < 0.3).astype(np.uint8)
    tb = (np.arange(n_txn + 1) * R).astype(np.uint32)
    return Epoch(keys.reshape(-1), types.reshape(-1), tb)


@pytest.mark.parametrize("cc", [dvcc.NO_WAIT, dvcc.WAIT_DIE, dvcc.OCC])
@pytest.mark.parametrize("lsd", [False, True])
def test_small_sorts_round0(cc, lsd):
    """round 0 behind the small sorts (bucket sort, or DV_FLAG_LSD_SORT's
    passes): zipf, repeat-access and one-hot-row epochs, two txns; whole
    epochs and prefix-kill stages, asynchronous rounds and synchronous"""
    rows = 1 << 20
    g = YCSBQueryGenerator(rows, zipf_theta=0.9)
    eps = [g.gen(30_000, 151), _repeat_epoch(1 << 12, 9_000, 152), _hot_read_epoch(rows, 20_000, 9),
           g.gen(2, 153)]
    _check(cc, rows, eps, prefix=None, lsd_sort=lsd)
    _check(cc, rows, eps, prefix=3000, lsd_sort=lsd)
    _check(cc, rows, eps[:2], prefix=None, lsd_sort=lsd, asynchronous=False, tail=False)


@pytest.mark.parametrize("cc", [dvcc.NO_WAIT, dvcc.WAIT_DIE, dvcc.OCC])
def test_medium_epoch_without_tail(cc):
    g = YCSBQueryGenerator(1 << 20, zipf_theta=0.9)
    _check(cc, 1 << 20, [g.gen(1 << 16, 98)], tail=False, asynchronous=False)


@pytest.mark.parametrize("cc", [dvcc.NO_WAIT, dvcc.WAIT_DIE, dvcc.OCC])
def test_medium_epoch_tail_only(cc):
    g = YCSBQueryGenerator(1 << 20, zipf_theta=0.9)
    _check(cc, 1 << 20, [g.gen(1 << 16, 96)], asynchronous=False)


@pytest.mark.parametrize("cc", [dvcc.NO_WAIT, dvcc.OCC])
def test_medium_epoch_el64(cc):
    g = YCSBQueryGenerator(1 << 20, zipf_theta=0.9)
    _check(cc, 1 << 20, [g.gen(1 << 16, 97)], el64=True)


@pytest.mark.parametrize("case", range(24))
def test_randomized_sweep(case):
    """Seeded random configurations across sizes, request counts, skew, write
    mixes, CC algorithms and the decision-path knobs (tail kernel, 64-bit
    elements, asynchronous rounds), each bit-exact against the oracle over two
    consecutive epochs (table state carried)."""
    rng = np.random.default_rng(1000 + case)
    R = int(rng.integers(1, 17))
    rows = int(rng.integers(max(R, 16), 1 << 16))
    n_txn = int(rng.integers(1, 8000))
    theta = float(rng.choice([0.0, 0.3, 0.6, 0.9, 0.99]))
    cc = CCS[case % len(CCS)]
    g = YCSBQueryGenerator(rows, req_per_query=R, zipf_theta=theta,
                           txn_write_perc=float(rng.choice([0.0, 0.5, 1.0])),
                           tup_write_perc=float(rng.choice([0.1, 0.5, 0.9])))
    knobs = dict(tail=bool(rng.integers(0, 2)), el64=bool(rng.integers(0, 2)),
                 asynchronous=bool(rng.integers(0, 2)))
    _check(cc, rows, [g.gen(n_txn, 77 + case), g.gen(n_txn, 78 + case)], **knobs)


def _check_batch(cc, rows, epochs, prefix=None, max_iters=None, lanes=1, stream=None, reuse=False):
    """dv_epoch_run_device_batch (lanes > 1: dv_epoch_run_device_lanes over
    the engine and lanes - 1 decision lanes) against the oracle run over the
    same epochs one after the other: every epoch's commit bytes, digest and
    write count, and the table after the batch.  reuse: an epoch listed again
    runs from the same device buffers (so its decision is captured into an
    epoch graph the second time and replayed after)."""
    tab = O.YcsbTable(rows)
    f0 = tab.f0.copy()
    refs = [_oracle_epoch(cc, tab, f0, e) for e in epochs]
    eng = CCEngine(cc, max(e.n_txn for e in epochs), max(e.n_acc for e in epochs))
    if stream is not None:
        eng.set_stream(stream.cuda_stream)
    eng.load_ycsb_partition(rows)
    eng.set_prefix(prefix)
    extra = [eng.open_lane() for _ in range(lanes - 1)]
    for e in [eng] + extra:
        if max_iters:
            e.set_async_limits(max_iters, 0)
    if reuse:
        made = {}
        deps = [made.setdefault(id(e), DeviceEpoch(e)) for e in epochs]
    else:
        deps = [DeviceEpoch(e) for e in epochs]
    commits = [torch.zeros(max(1, e.n_txn), dtype=torch.uint8, device="cuda") for e in epochs]
    if lanes > 1:
        sts = eng.run_epochs_lanes(extra, deps, commits)
    else:
        sts = eng.run_epochs_device(deps, commits)
    for k, (e, (c_ref, _, st_ref), st) in enumerate(zip(epochs, refs, sts)):
        c = commits[k].cpu().numpy()[:e.n_txn]
        assert (c == c_ref).all(), f"epoch {k}: {(c != c_ref).sum()} mismatches"
        assert (st.committed, st.read_digest, st.write_cnt) == (st_ref.committed, st_ref.read_digest,
                                                               st_ref.write_cnt), f"epoch {k}"
    assert (eng.read_table(0, rows) == f0).all()
    eng.close()
    return sts


@pytest.mark.gpu
@pytest.mark.parametrize("cc", [dvcc.NO_WAIT, dvcc.WAIT_DIE, dvcc.OCC])
def test_batch_pipelined_prefix_epochs(cc):
    """Pipelined epochs (each queued before the previous one is read back)
    give the results of running them one at a time."""
    rows = 1 << 18
    g = YCSBQueryGenerator(rows, zipf_theta=0.9, txn_write_perc=1.0, tup_write_perc=0.5)
    _check_batch(cc, rows, [g.gen(20_000, 300 + k) for k in range(5)], prefix=512)


@pytest.mark.gpu
def test_batch_mixed_and_halted_epochs():
    """A batch mixing prefix-kill epochs with small ones (run one at a time),
    and asynchronous rounds forced to yield: a halted epoch and the one queued
    behind it run again synchronously, results unchanged."""
    rows = 1 << 18
    g = YCSBQueryGenerator(rows, zipf_theta=0.9, txn_write_perc=1.0, tup_write_perc=0.5)
    sizes = [20_000, 20_000, 1, 20_000, 20_000, 20_000]
    epochs = [g.gen(n, 400 + k) for k, n in enumerate(sizes)]
    _check_batch(dvcc.NO_WAIT, rows, epochs, prefix=512)
    sts = _check_batch(dvcc.NO_WAIT, rows, epochs, prefix=512, max_iters=1)
    assert sum(st.async_yields for st in sts) > 0, "no asynchronous launch yielded"


@pytest.mark.gpu
def test_batch_error_stops_before_execution():
    """A missing key in the third epoch: the batch returns the error, the first
    two epochs are applied, nothing of the third or later ones is."""
    rows = 1 << 16
    g = YCSBQueryGenerator(rows, zipf_theta=0.9, txn_write_perc=1.0, tup_write_perc=0.5)
    epochs = [g.gen(8_000, 500 + k) for k in range(5)]
    epochs[2].keys[17] = np.uint64(rows + 3)
    tab = O.YcsbTable(rows)
    f0 = tab.f0.copy()
    for e in epochs[:2]:
        _oracle_epoch(dvcc.NO_WAIT, tab, f0, e)
    eng = CCEngine(dvcc.NO_WAIT, 8_000, max(e.n_acc for e in epochs))
    eng.load_ycsb_partition(rows)
    eng.set_prefix(256)
    with pytest.raises(dvcc.DvccError) as ei:
        eng.run_epochs_device([DeviceEpoch(e) for e in epochs])
    assert ei.value.code == dvcc._lib.DV_ERR_KEY_NOT_FOUND
    assert (eng.read_table(0, rows) == f0).all()
    eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("what", ["n_txn", "n_acc"])
def test_batch_setup_error_after_pipelined_epochs(what):
    """Pipelined epochs followed by one the context cannot hold (n_txn past
    max_txn / n_acc past max_acc): the epoch fails in its setup, before any
    epoch clear would write the previous epoch's deferred counter read-back.
    The call returns DV_ERR_ARG at once (the read-back is flushed, no 120-s
    wait), the earlier epochs are applied and their stats filled, and the
    context runs epochs again."""
    import ctypes
    import time
    from dvcc import _lib as L
    rows = 1 << 16
    g = YCSBQueryGenerator(rows, zipf_theta=0.9, txn_write_perc=1.0, tup_write_perc=0.5)
    epochs = [g.gen(8_000, 600 + k) for k in range(3)]
    big = g.gen(8_001 if what == "n_txn" else 8_000, 700)
    tab = O.YcsbTable(rows)
    f0 = tab.f0.copy()
    refs = [_oracle_epoch(dvcc.NO_WAIT, tab, f0, e) for e in epochs]
    cap_acc = max(e.n_acc for e in epochs)
    if what == "n_acc":
        big = dvcc.Epoch(np.concatenate([big.keys, big.keys[:64]]), np.concatenate([big.types, big.types[:64]]),
                         np.concatenate([big.txn_begin[:-1], [big.txn_begin[-1] + 64]]).astype(np.uint32))
        assert big.n_acc > cap_acc
    eng = CCEngine(dvcc.NO_WAIT, 8_000, cap_acc)
    eng.load_ycsb_partition(rows)
    eng.set_prefix(256)
    deps = [DeviceEpoch(e) for e in epochs + [big]]
    arr = (L.EpochDev * 4)(*[d.desc() for d in deps])
    sts = (L.Stats * 4)()
    t0 = time.perf_counter()
    rc = L.lib().dv_epoch_run_device_batch(eng._ctx, arr, 4, None, sts)
    assert rc == L.DV_ERR_ARG and time.perf_counter() - t0 < 30
    for k, (_, _, st_ref) in enumerate(refs):
        assert (sts[k].committed, sts[k].read_digest) == (st_ref.committed, st_ref.read_digest), k
    assert (eng.read_table(0, rows) == f0).all()
    e2 = g.gen(8_000, 800)
    _, _, st_ref = _oracle_epoch(dvcc.NO_WAIT, tab, f0, e2)
    st = eng.run_epoch_device(DeviceEpoch(e2))
    assert (st.committed, st.read_digest) == (st_ref.committed, st_ref.read_digest)
    assert (eng.read_table(0, rows) == f0).all()
    eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("cc,lanes", [(dvcc.NO_WAIT, 2), (dvcc.WAIT_DIE, 2), (dvcc.OCC, 2), (dvcc.NO_WAIT, 4),
                                      (dvcc.OCC, 3), (dvcc.WAIT_DIE, 8)])
def test_lanes_pipelined_prefix_epochs(cc, lanes):
    """Decision lanes: epochs decided on alternating contexts, executed in
    epoch order -- commit bytes, read digests (reads see every earlier
    epoch's writes) and the final table equal the sequential oracle's."""
    rows = 1 << 18
    g = YCSBQueryGenerator(rows, zipf_theta=0.9, txn_write_perc=1.0, tup_write_perc=0.5)
    _check_batch(cc, rows, [g.gen(20_000, 900 + k) for k in range(7)], prefix=512, lanes=lanes)


@pytest.mark.gpu
def test_lanes_mixed_and_halted_epochs():
    """Lanes with a small epoch (run synchronously) in the middle and
    asynchronous rounds forced to yield: a halted epoch and every epoch queued
    behind it (on any lane) run again in order, results unchanged."""
    rows = 1 << 18
    g = YCSBQueryGenerator(rows, zipf_theta=0.9, txn_write_perc=1.0, tup_write_perc=0.5)
    sizes = [20_000, 20_000, 20_000, 1, 20_000, 20_000, 20_000, 20_000, 20_000, 20_000]
    epochs = [g.gen(n, 1000 + k) for k, n in enumerate(sizes)]
    _check_batch(dvcc.NO_WAIT, rows, epochs, prefix=512, lanes=4)
    sts = _check_batch(dvcc.NO_WAIT, rows, epochs, prefix=512, max_iters=1, lanes=4)
    assert sum(st.async_yields for st in sts) > 0, "no asynchronous launch yielded"


@pytest.mark.gpu
@pytest.mark.parametrize("cc,lanes", [(dvcc.CALVIN, 1), (dvcc.CALVIN, 4), (dvcc.NO_WAIT, 1), (dvcc.NO_WAIT, 4),
                                      (dvcc.WAIT_DIE, 3), (dvcc.OCC, 1), (dvcc.OCC, 4)])
def test_small_epochs_pipelined(cc, lanes):
    """Epochs below the prefix-kill size queue without a host wait too (CALVIN,
    and round 0 + one asynchronous launch for the others): through the batch
    and the decision lanes, ragged sizes and a one-txn epoch included, every
    epoch equals the sequential oracle's."""
    rows = 1 << 16
    g = YCSBQueryGenerator(rows, zipf_theta=0.8, txn_write_perc=1.0, tup_write_perc=0.5)
    sizes = [5000, 5000, 1, 3000, 5000, 5000, 4000, 5000, 5000]
    _check_batch(cc, rows, [g.gen(n, 1200 + k) for k, n in enumerate(sizes)], lanes=lanes)


@pytest.mark.gpu
@pytest.mark.parametrize("lanes", [1, 4])
def test_small_epochs_pipelined_halted(lanes):
    """... with the asynchronous rounds forced to yield: a halted small epoch
    and every epoch queued behind it run again in order, results unchanged."""
    rows = 1 << 16
    g = YCSBQueryGenerator(rows, zipf_theta=0.9, txn_write_perc=1.0, tup_write_perc=0.5)
    epochs = [g.gen(5000, 1300 + k) for k in range(8)]
    sts = _check_batch(dvcc.NO_WAIT, rows, epochs, max_iters=1, lanes=lanes)
    assert sum(st.async_yields for st in sts) > 0, "no asynchronous launch yielded"


@pytest.mark.gpu
@pytest.mark.parametrize("cc,lanes,prefix", [(dvcc.CALVIN, 1, None), (dvcc.CALVIN, 4, None), (dvcc.NO_WAIT, 1, None),
                                             (dvcc.OCC, 4, None), (dvcc.WAIT_DIE, 3, None), (dvcc.NO_WAIT, 1, 512),
                                             (dvcc.OCC, 4, 512)])
def test_epoch_graphs_replayed(cc, lanes, prefix):
    """Epochs from the same device buffers, again and again (as the bench
    cycles them): the third time a (lane, buffers) pair comes, its decision
    is captured into a graph, from the fourth on it is replayed -- every
    epoch's results equal the sequential oracle's, small epochs (prefix-kill
    ones run as they are), batch and lanes."""
    import math
    rows = 1 << 18
    g = YCSBQueryGenerator(rows, zipf_theta=0.9, txn_write_perc=1.0, tup_write_perc=0.5)
    n = 20_000 if prefix else 5000
    base = [g.gen(n, 1400 + k) for k in range(3)]
    period = lanes * 3 // math.gcd(lanes, 3)  # (every lane meets every buffer once per period)
    _check_batch(cc, rows, [base[k % 3] for k in range(5 * period)], prefix=prefix, lanes=lanes, reuse=True)


@pytest.mark.gpu
@pytest.mark.parametrize("lanes", [1, 4])
def test_epoch_graphs_new_content_and_halts(lanes):
    """The same device buffers refilled with new epochs of the same sizes
    between calls (a graph replays whatever the buffers hold), and forced
    yields: every epoch equals the oracle's, halted ones run again."""
    rows = 1 << 16
    g = YCSBQueryGenerator(rows, zipf_theta=0.9, txn_write_perc=1.0, tup_write_perc=0.5)
    tab = O.YcsbTable(rows)
    f0 = tab.f0.copy()
    eng = CCEngine(dvcc.NO_WAIT, 5000, 50_000)
    eng.load_ycsb_partition(rows)
    eng.set_prefix(None)
    extra = [eng.open_lane() for _ in range(lanes - 1)]
    bufs = [DeviceEpoch(g.gen(5000, 1500 + k)) for k in range(lanes)]
    commits = [torch.zeros(5000, dtype=torch.uint8, device="cuda") for _ in range(lanes)]
    yields = 0
    for call in range(9):  # (a key's graph: captured at its 3rd call, replayed from its 4th)
        if call == 4:
            for e in [eng] + extra:
                e.set_async_limits(1, 0)  # (forced yields from here on)
        epochs = [g.gen(5000, 1600 + lanes * call + k) for k in range(lanes)]
        for b, e in zip(bufs, epochs):
            b.keys.copy_(torch.from_numpy(e.keys.view(np.int64)))
            b.types.copy_(torch.from_numpy(e.types))
            b.acc_txn.copy_(torch.from_numpy(e.acc_txn().view(np.int32)))
            b.txn_begin.copy_(torch.from_numpy(e.txn_begin.astype(np.int32)))
            if b.recs32 is not None:
                b.recs32.copy_(torch.from_numpy(e.to_row_records().view(np.int32)))
        torch.cuda.synchronize()
        sts = eng.run_epochs_lanes(extra, bufs, commits) if extra else eng.run_epochs_device(bufs, commits)
        for k, (e, st) in enumerate(zip(epochs, sts)):
            c_ref, _, st_ref = _oracle_epoch(dvcc.NO_WAIT, tab, f0, e)
            assert (commits[k].cpu().numpy() == c_ref).all(), (call, k)
            assert (st.committed, st.read_digest, st.write_cnt) == (st_ref.committed, st_ref.read_digest,
                                                                   st_ref.write_cnt), (call, k)
            yields += st.async_yields
    assert (eng.read_table(0, rows) == f0).all()
    assert yields > 0, "no asynchronous launch yielded"
    for ln in extra:
        ln.close()
    eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("cc,lanes", [(dvcc.NO_WAIT, 1), (dvcc.NO_WAIT, 4), (dvcc.CALVIN, 1), (dvcc.OCC, 3)])
def test_epoch_graphs_after_table_changes(cc, lanes):
    """Graphs captured, then the tables change under them: a
    second table created (the state columns f0 / pkey / ktag reallocated and
    copied, the dense primary-key shortcut off), then table 0 reloaded (its
    bucket bitmap reallocated, every row back to its initial F0).  The same
    epoch buffers run again -- no graph captured before the change may replay
    against the freed storage: every epoch equals the oracle's."""
    rows = 1 << 16
    n = 5000
    g = YCSBQueryGenerator(rows, zipf_theta=0.9, txn_write_perc=1.0, tup_write_perc=0.5)
    tab = O.YcsbTable(rows)
    f0 = tab.f0.copy()
    eng = CCEngine(cc, n, 60_000)
    eng.load_ycsb_partition(rows)
    eng.set_prefix(None)
    bufs_src = [g.gen(n, 1700 + k) for k in range(lanes)]
    bufs = [DeviceEpoch(e) for e in bufs_src]
    commits = [torch.zeros(n, dtype=torch.uint8, device="cuda") for _ in range(lanes)]

    def run(calls):
        extra = [eng.open_lane() for _ in range(lanes - 1)]
        for _ in range(calls):
            sts = eng.run_epochs_lanes(extra, bufs, commits) if extra else eng.run_epochs_device(bufs, commits)
            for k, (e, st) in enumerate(zip(bufs_src, sts)):
                c_ref, _, st_ref = _oracle_epoch(cc, tab, f0, e)
                assert (commits[k].cpu().numpy() == c_ref).all(), k
                assert (st.committed, st.read_digest, st.write_cnt) == (st_ref.committed, st_ref.read_digest,
                                                                       st_ref.write_cnt), k
        for ln in extra:
            ln.close()
        assert (eng.read_table(0, rows) == f0).all()

    run(6)  # (captured at a key's 3rd call, replayed from its 4th)
    eng.create_table(1, 4096, 4096)
    eng.load_table(1, np.arange(4096, dtype=np.uint64) * 7 + 3)
    run(6)
    eng.load_ycsb_partition(rows)
    f0[:] = tab.f0
    run(6)
    eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("cc", CCS)
@pytest.mark.parametrize("offset", [1, 5])
def test_unaligned_commit_buffer(cc, offset):
    """Commit bytes into a caller's buffer at an odd offset:
    every commit byte and count equals the oracle's, guard bytes on both
    sides of the slice untouched."""
    rows, n = 1 << 16, 5000
    g = YCSBQueryGenerator(rows, zipf_theta=0.9, txn_write_perc=1.0, tup_write_perc=0.5)
    tab = O.YcsbTable(rows)
    f0 = tab.f0.copy()
    eng = CCEngine(cc, n, 60_000)
    eng.load_ycsb_partition(rows)
    for k in range(3):
        e = g.gen(n - k, 1900 + k)
        c_ref, _, st_ref = _oracle_epoch(cc, tab, f0, e)
        big = torch.full((e.n_txn + offset + 32,), 0xAB, dtype=torch.uint8, device="cuda")
        d_commit = big[offset:offset + e.n_txn]
        d_grant = torch.zeros(e.n_acc, dtype=torch.int32, device="cuda") if cc == dvcc.CALVIN else None
        st = eng.run_epoch_device(DeviceEpoch(e), d_commit, d_grant)
        hb = big.cpu().numpy()
        assert (hb[:offset] == 0xAB).all() and (hb[offset + e.n_txn:] == 0xAB).all()
        assert (hb[offset:offset + e.n_txn] == c_ref).all(), k
        assert (st.committed, st.read_digest, st.write_cnt) == (st_ref.committed, st_ref.read_digest,
                                                               st_ref.write_cnt), k
    assert (eng.read_table(0, rows) == f0).all()
    eng.close()


@pytest.mark.gpu
def test_epoch_graphs_default_capture_mode():
    """The epoch graphs with HIP's default graph capture (the package no
    longer sets DEBUG_CLR_GRAPH_PACKET_CAPTURE; the suite's
    conftest does, as the bench): tests/graph_mode_check.py replays epoch
    graphs through the batch and four lanes in a fresh process with the
    variable unset and checks every epoch against the oracle."""
    import os
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "DVCC_PACKET_CAPTURE")}
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, os.path.join(here, "graph_mode_check.py")], env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "graph mode ok" in r.stdout, r.stdout[-2000:]


@pytest.mark.gpu
def test_lanes_rotated_orders_and_ragged_calls():
    """Decision lanes handed over in different orders from call to call (the
    shared order word is lanes[0]'s, each context's turn its own) and calls of
    1 to 5 epochs, from the same device buffers refilled with new epochs (so
    the graphs, keyed by the lanes' order, replay): every epoch equals the
    sequential oracle's and the table ends as the oracle's."""
    rows = 1 << 16
    g = YCSBQueryGenerator(rows, zipf_theta=0.9, txn_write_perc=1.0, tup_write_perc=0.5)
    tab = O.YcsbTable(rows)
    f0 = tab.f0.copy()
    eng = CCEngine(dvcc.NO_WAIT, 5000, 50_000)
    eng.load_ycsb_partition(rows)
    eng.set_prefix(None)
    l1, l2 = eng.open_lane(), eng.open_lane()
    orders = [(eng, [l1, l2]), (l1, [l2, eng]), (l2, [eng, l1])]
    bufs = [DeviceEpoch(g.gen(5000, 1700 + k)) for k in range(5)]
    commits = [torch.zeros(5000, dtype=torch.uint8, device="cuda") for _ in range(5)]
    seed = 1800
    for call in range(12):
        first, rest = orders[call % 3]
        n = (1, 3, 5, 2)[call % 4]
        epochs = [g.gen(5000, seed + k) for k in range(n)]
        seed += n
        for b, e in zip(bufs, epochs):
            b.keys.copy_(torch.from_numpy(e.keys.view(np.int64)))
            b.types.copy_(torch.from_numpy(e.types))
            b.acc_txn.copy_(torch.from_numpy(e.acc_txn().view(np.int32)))
            b.txn_begin.copy_(torch.from_numpy(e.txn_begin.astype(np.int32)))
            if b.recs32 is not None:
                b.recs32.copy_(torch.from_numpy(e.to_row_records().view(np.int32)))
        torch.cuda.synchronize()
        sts = first.run_epochs_lanes(rest, bufs[:n], commits[:n])
        for k, (e, st) in enumerate(zip(epochs, sts)):
            c_ref, _, st_ref = _oracle_epoch(dvcc.NO_WAIT, tab, f0, e)
            assert (commits[k].cpu().numpy() == c_ref).all(), (call, k)
            assert (st.committed, st.read_digest, st.write_cnt) == (st_ref.committed, st_ref.read_digest,
                                                                   st_ref.write_cnt), (call, k)
    assert (eng.read_table(0, rows) == f0).all()
    for ln in (l1, l2):
        ln.close()
    eng.close()


@pytest.mark.gpu
@pytest.mark.slow
def test_config_b_lanes_timed_path():
    """The bench's config-B leg as timed: 65,536-txn CALVIN epochs (zipf 0.6,
    16,777,216 rows), three distinct epochs cycled over four decision lanes."""
    rows = 16_777_216
    g = YCSBQueryGenerator(rows, zipf_theta=0.6, txn_write_perc=1.0, tup_write_perc=0.5)
    base = [g.gen(65_536, dvcc.epoch_seed(0, e)) for e in range(3)]
    _check_batch(dvcc.CALVIN, rows, [base[k % 3] for k in range(12)], lanes=4, reuse=True)


@pytest.mark.gpu
@pytest.mark.parametrize("bad", [1, 2, 3])
def test_lanes_error_stops_before_execution(bad):
    """A missing key in epoch `bad` (either lane): the call returns the error,
    the epochs before it are applied, nothing of it or the epochs queued
    behind it on the other lane is."""
    rows = 1 << 16
    g = YCSBQueryGenerator(rows, zipf_theta=0.9, txn_write_perc=1.0, tup_write_perc=0.5)
    epochs = [g.gen(8_000, 1100 + k) for k in range(5)]
    epochs[bad].keys[17] = np.uint64(rows + 3)
    tab = O.YcsbTable(rows)
    f0 = tab.f0.copy()
    for e in epochs[:bad]:
        _oracle_epoch(dvcc.NO_WAIT, tab, f0, e)
    eng = CCEngine(dvcc.NO_WAIT, 8_000, max(e.n_acc for e in epochs))
    eng.load_ycsb_partition(rows)
    eng.set_prefix(256)
    lane = eng.open_lane()
    more = [eng.open_lane() for _ in range(2)]
    with pytest.raises(dvcc.DvccError) as ei:
        eng.run_epochs_lanes([lane] + more, [DeviceEpoch(e) for e in epochs])
    assert ei.value.code == dvcc._lib.DV_ERR_KEY_NOT_FOUND
    assert (eng.read_table(0, rows) == f0).all()
    # both contexts run epochs again afterwards
    e2 = g.gen(8_000, 1200)
    _, _, st_ref = _oracle_epoch(dvcc.NO_WAIT, tab, f0, e2)
    st = lane.run_epoch_device(DeviceEpoch(e2))
    assert (st.committed, st.read_digest) == (st_ref.committed, st_ref.read_digest)
    assert (eng.read_table(0, rows) == f0).all()
    eng.close()


@pytest.mark.gpu
def test_lane_tables_frozen_and_shared():
    """A lane sees the owner's tables (no copy) and the owner's tables cannot
    be reloaded while it is open; lanes of a different owner are refused."""
    from dvcc import _lib as L
    rows = 1 << 12
    eng = CCEngine(dvcc.NO_WAIT, 1024, 16_384)
    with pytest.raises(dvcc.DvccError):
        eng.open_lane()  # (no tables yet)
    eng.load_ycsb_partition(rows)
    lane = eng.open_lane()
    assert (lane.read_table(0, rows) == eng.read_table(0, rows)).all()
    with pytest.raises(dvcc.DvccError) as ei:
        eng.load_ycsb_partition(rows)
    assert ei.value.code == L.DV_ERR_STATE
    other = CCEngine(dvcc.NO_WAIT, 1024, 16_384)
    other.load_ycsb_partition(rows)
    g = YCSBQueryGenerator(rows, zipf_theta=0.9, txn_write_perc=1.0, tup_write_perc=0.5)
    with pytest.raises(dvcc.DvccError) as ei:
        eng.run_epochs_lanes([other], [DeviceEpoch(g.gen(100, 1))])
    assert ei.value.code == L.DV_ERR_ARG
    more = [eng.open_lane() for _ in range(8)]
    with pytest.raises(dvcc.DvccError) as ei:  # (eight lanes at most)
        eng.run_epochs_lanes([lane] + more, [DeviceEpoch(g.gen(100, 1))])
    assert ei.value.code == L.DV_ERR_ARG
    with pytest.raises(dvcc.DvccError) as ei:  # (each context once)
        eng.run_epochs_lanes([lane, lane], [DeviceEpoch(g.gen(100, 1))])
    assert ei.value.code == L.DV_ERR_ARG
    for m in more:
        m.close()
    other.close()
    lane.close()
    eng.load_ycsb_partition(rows)  # (unfrozen once its lanes are closed)
    eng.close()


@pytest.mark.gpu
def test_lanes_setup_error_and_short_batches():
    """Four lanes: a batch shorter than the lanes (0, 1 and 3 epochs), and an
    epoch the contexts cannot hold (n_txn past max_txn) at position 3 -- the
    call returns DV_ERR_ARG at once, the earlier epochs are applied and their
    stats filled, and the lanes run epochs again."""
    import ctypes
    import time
    from dvcc import _lib as L
    rows = 1 << 16
    g = YCSBQueryGenerator(rows, zipf_theta=0.9, txn_write_perc=1.0, tup_write_perc=0.5)
    tab = O.YcsbTable(rows)
    f0 = tab.f0.copy()
    eng = CCEngine(dvcc.NO_WAIT, 8_000, 8_000 * 10)
    eng.load_ycsb_partition(rows)
    eng.set_prefix(256)
    lanes = [eng.open_lane() for _ in range(3)]
    try:
        assert eng.run_epochs_lanes(lanes, []) == []
        seed = 1300
        for count in (1, 3):
            es = [g.gen(8_000, seed + k) for k in range(count)]
            seed += count
            refs = [_oracle_epoch(dvcc.NO_WAIT, tab, f0, e) for e in es]
            sts = eng.run_epochs_lanes(lanes, [DeviceEpoch(e) for e in es])
            for st, (_, _, st_ref) in zip(sts, refs):
                assert (st.committed, st.read_digest) == (st_ref.committed, st_ref.read_digest)
            assert (eng.read_table(0, rows) == f0).all()
        es = [g.gen(8_000, seed + k) for k in range(3)] + [g.gen(8_001, seed + 3), g.gen(8_000, seed + 4)]
        refs = [_oracle_epoch(dvcc.NO_WAIT, tab, f0, e) for e in es[:3]]
        deps = [DeviceEpoch(e) for e in es]
        arr = (L.EpochDev * 5)(*[d.desc() for d in deps])
        sts = (L.Stats * 5)()
        lp = (ctypes.c_void_p * 4)(*[e._ctx.value for e in [eng] + lanes])
        t0 = time.perf_counter()
        rc = L.lib().dv_epoch_run_device_lanes(lp, 4, arr, 5, None, sts)
        assert rc == L.DV_ERR_ARG and time.perf_counter() - t0 < 30
        for k, (_, _, st_ref) in enumerate(refs):
            assert (sts[k].committed, sts[k].read_digest) == (st_ref.committed, st_ref.read_digest), k
        assert (eng.read_table(0, rows) == f0).all()
        e2 = [g.gen(8_000, seed + 10 + k) for k in range(5)]
        refs = [_oracle_epoch(dvcc.NO_WAIT, tab, f0, e) for e in e2]
        sts = eng.run_epochs_lanes(lanes, [DeviceEpoch(e) for e in e2])
        for st, (_, _, st_ref) in zip(sts, refs):
            assert (st.committed, st.read_digest) == (st_ref.committed, st_ref.read_digest)
        assert (eng.read_table(0, rows) == f0).all()
    finally:
        eng.close()


@pytest.mark.gpu
@pytest.mark.slow
def test_bench_timed_path_config_d_lanes():
    """bench.py's timed region at its own size: dv_epoch_run_device_lanes over
    the engine and three decision lanes, config D (16,777,216 rows,
    1,048,576-txn epochs, zipf 0.9, NO_WAIT, automatic n/32 prefix), the
    bench's 5 distinct epochs (seeds epoch_seed(0, e)) cycled twice, so every
    epoch is decided on two different lanes, on a torch stream as in the
    bench -- commit bytes, read digest, write count of every epoch and the
    final F0 column against the oracle running the 10 epochs in order."""
    rows, n_txn = 16_777_216, 1_048_576
    g = YCSBQueryGenerator(rows, part_cnt=1, req_per_query=10, zipf_theta=0.9, txn_write_perc=1.0,
                           tup_write_perc=0.5, part_per_txn=1, strict_ppt=1, mpr=-1.0)
    es = [g.gen(n_txn, dvcc.epoch_seed(0, e), 0) for e in range(5)]
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        sts = _check_batch(dvcc.NO_WAIT, rows, es + es, prefix=0, lanes=4, stream=s)
    assert all(st.prefix_txn == n_txn // 32 for st in sts), [st.prefix_txn for st in sts]
    assert sum(st.async_yields for st in sts) == 0


@pytest.mark.gpu
def test_lanes_order_release_and_reorder():
    """lanes_order([]) releases the whole order (every lane back on its own
    stream), so the same lanes can be ordered again; the owner then still
    decides epochs bit-exact."""
    rows = 1 << 14
    g = YCSBQueryGenerator(rows, zipf_theta=0.9, txn_write_perc=1.0, tup_write_perc=0.5)
    e = g.gen(3000, 1234)
    eng = CCEngine(dvcc.NO_WAIT, 3000, e.n_acc)
    eng.load_ycsb_partition(rows)
    lanes = [eng.open_lane() for _ in range(2)]
    for _ in range(2):
        eng.lanes_order(lanes)
        eng.lanes_order([])
    tab = O.YcsbTable(rows)
    f0 = tab.f0.copy()
    c_ref, _, st_ref = _oracle_epoch(dvcc.NO_WAIT, tab, f0, e)
    c, _, st = _gpu_epoch(eng, e, "device")
    assert (c == c_ref).all() and st.read_digest == st_ref.read_digest
    for ln in lanes:
        ln.close()
    eng.close()


# ---- prefix-kill epochs with their txn boundaries (dv_epoch_dev::txn_begin:
#      k_probe_tb probes the prefix, k_kill / k_kill_emit the later accesses)
def _prefix_engine(cc, rows, n_txn, n_acc, prefix):
    eng = CCEngine(cc, n_txn, n_acc)
    eng.load_ycsb_partition(rows)
    eng.set_prefix(prefix)
    return eng


@pytest.mark.parametrize("cc", [dvcc.NO_WAIT, dvcc.WAIT_DIE, dvcc.OCC])
@pytest.mark.parametrize("rows,R,theta", [(1 << 18, 10, 0.9), (1 << 12, 16, 0.99), (1 << 16, 4, 0.5),
                                          (1 << 20, 48, 0.5), (1 << 22, 64, 0.3)])
def test_prefix_epochs_with_and_without_txn_begin(cc, rows, R, theta):
    """The same prefix-kill epochs through both range sources -- the epoch's
    own boundaries (with its accesses as 4-byte records or as keys and types)
    and acc_txn -- give the oracle's commit bytes, digests, write counts and
    table, epoch after epoch (repeated rows included).  R = 48 / 64: survivors
    longer than one 32-bit skip word, several hundred of them with skipped
    reads (k_kill_emit takes their kept accesses from k_kill's skip bits)."""
    g = YCSBQueryGenerator(rows, zipf_theta=theta, req_per_query=R, txn_write_perc=1.0, tup_write_perc=0.5)
    es = [g.gen(9_000, 1300 + k) for k in range(3)]
    for with_tb, recs in ((True, True), (True, False), (False, False)):  # (+ 4-byte records, dv_epoch_dev::recs32)
        tab = O.YcsbTable(rows)
        f0 = tab.f0.copy()
        eng = _prefix_engine(cc, rows, 9_000, max(e.n_acc for e in es), 700)
        for e in es:
            c_ref, _, st_ref = _oracle_epoch(cc, tab, f0, e)
            d = torch.zeros(e.n_txn, dtype=torch.uint8, device="cuda")
            dep = DeviceEpoch(e, txn_begin=with_tb, recs32=recs)
            assert (dep.recs32 is not None) == recs
            st = eng.run_epoch_device(dep, d)
            assert st.prefix_txn == 700, st.prefix_txn
            assert (d.cpu().numpy() == c_ref).all(), with_tb
            assert (st.committed, st.read_digest, st.write_cnt) == (st_ref.committed, st_ref.read_digest,
                                                                   st_ref.write_cnt), with_tb
            assert (eng.read_table(0, rows) == f0).all(), with_tb
        eng.close()


@pytest.mark.parametrize("where", ["prefix", "later", "survivor"])
def test_txn_begin_prefix_epoch_missing_key(where):
    """A key no row holds -- in the prefix (k_probe_tb), in a later txn the
    prefix kills or in one that survives (k_kill probes both) -- rejects the
    whole epoch with DV_ERR_KEY_NOT_FOUND and no row changed; the context
    then decides the next epoch bit-exact."""
    rows = 1 << 16
    g = YCSBQueryGenerator(rows, zipf_theta=0.9, txn_write_perc=1.0, tup_write_perc=0.5)
    e = g.gen(6_000, 1400)
    i = {"prefix": 3, "later": int(e.txn_begin[3000]) + 1, "survivor": int(e.txn_begin[-2])}[where]
    e.keys[i] = np.uint64(rows + 17)
    eng = _prefix_engine(dvcc.NO_WAIT, rows, 6_000, e.n_acc, 500)
    before = eng.read_table(0, rows)
    with pytest.raises(dvcc.DvccError) as ex:
        eng.run_epoch_device(DeviceEpoch(e), torch.zeros(6_000, dtype=torch.uint8, device="cuda"))
    assert ex.value.code == dvcc._lib.DV_ERR_KEY_NOT_FOUND
    assert (eng.read_table(0, rows) == before).all()
    e2 = g.gen(6_000, 1401)
    tab = O.YcsbTable(rows)
    f0 = tab.f0.copy()
    c_ref, _, st_ref = _oracle_epoch(dvcc.NO_WAIT, tab, f0, e2)
    d = torch.zeros(6_000, dtype=torch.uint8, device="cuda")
    st = eng.run_epoch_device(DeviceEpoch(e2), d)
    assert (d.cpu().numpy() == c_ref).all() and st.read_digest == st_ref.read_digest
    eng.close()


@pytest.mark.parametrize("bad", ["descending", "past_end", "short_end", "nonzero_start", "too_long"])
def test_txn_begin_bad_boundaries(bad):
    """Boundaries that do not describe an epoch (descending, past n_acc, not
    ending at n_acc, not starting at 0) are DV_ERR_TXN_RANGE; a txn longer than
    the declared bound DV_ERR_ARG -- before anything executes."""
    rows = 1 << 14
    g = YCSBQueryGenerator(rows, zipf_theta=0.9, req_per_query=20 if bad == "too_long" else 10)
    e = g.gen(3_000, 1500)
    eng = _prefix_engine(dvcc.NO_WAIT, rows, 3_000, e.n_acc, 256)
    before = eng.read_table(0, rows)
    dep = DeviceEpoch(e)
    tb = dep.txn_begin
    if bad == "descending":
        tb[1000] = tb[1001] + 1
    elif bad == "past_end":
        tb[2000] = e.n_acc + 5
    elif bad == "short_end":
        tb[-1] = e.n_acc - 1
    elif bad == "nonzero_start":
        tb[0] = 1
    else:
        dep.max_txn_acc = 16  # 20 accesses per txn
    with pytest.raises(dvcc.DvccError) as ex:
        eng.run_epoch_device(dep, torch.zeros(3_000, dtype=torch.uint8, device="cuda"))
    assert ex.value.code == (dvcc._lib.DV_ERR_ARG if bad == "too_long" else dvcc._lib.DV_ERR_TXN_RANGE), ex.value.code
    assert (eng.read_table(0, rows) == before).all()
    eng.close()


def _max_len_epoch(rows, n_txn, seed, longest=128):
    """Ragged txns of 0..longest accesses (one in ten exactly `longest`, the
    first one too; a few empty), half the keys from a hot set, every fifth
    txn ending on its own first row again."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(1, longest + 1, size=n_txn)
    lens[rng.random(n_txn) < 0.1] = longest
    lens[rng.random(n_txn) < 0.02] = 0
    lens[0] = longest
    tb = np.zeros(n_txn + 1, np.uint32)
    tb[1:] = np.cumsum(lens)
    n = int(tb[-1])
    hot = max(8, rows // 256)
    keys = np.where(rng.random(n) < 0.5, rng.integers(0, hot, size=n), rng.integers(0, rows, size=n))
    for t in range(0, n_txn, 5):
        a, b = int(tb[t]), int(tb[t + 1])
        if b - a >= 2:
            keys[b - 1] = keys[a]
    types = (rng.random(n) < 0.5).astype(np.uint8)
    return Epoch(keys.astype(np.uint64), types, tb)


@pytest.mark.parametrize("cc", CCS)
def test_longest_txns(cc):
    """Txns of up to 128 accesses -- the engine's bound (kMaxPos, a txn's
    positions in 7 bits of a sort key) -- mixed with short and empty ones:
    every decision path (one context without and with the prefix kill, which
    takes the epoch's own boundaries; the synchronous rounds alone; 64-bit
    round elements) gives the oracle's commit bytes, digest, write count and
    table, epoch after epoch."""
    rows = 1 << 16
    epochs = [_max_len_epoch(rows, 3000, 1600 + k) for k in range(2)]
    assert max(int(np.diff(e.txn_begin).max()) for e in epochs) == 128
    _check(cc, rows, epochs, prefix=None)
    _check(cc, rows, epochs, prefix=None, asynchronous=False, tail=False)
    _check(cc, rows, epochs, prefix=None, el64=True)
    if cc != dvcc.CALVIN:  # (CALVIN takes no prefix)
        st = _check(cc, rows, epochs, prefix=300)
        assert st.prefix_txn == 300, st.prefix_txn


@pytest.mark.parametrize("cc", [dvcc.NO_WAIT, dvcc.OCC, dvcc.CALVIN])
def test_longest_txns_lanes(cc):
    """The same 128-access txns through the pipelined batch and four decision
    lanes (prefix-kill epochs with 4-byte records for NO_WAIT / OCC, small
    pipelined epochs for CALVIN)."""
    rows = 1 << 16
    epochs = [_max_len_epoch(rows, 2500, 1700 + k) for k in range(6)]
    prefix = None if cc == dvcc.CALVIN else 256
    _check_batch(cc, rows, epochs, prefix=prefix)
    _check_batch(cc, rows, epochs, prefix=prefix, lanes=4)


@pytest.mark.parametrize("declared", [True, False])
@pytest.mark.parametrize("cc", CCS)
def test_txn_past_the_longest_is_rejected(cc, declared):
    """A txn of 129 accesses, one past the bound: declared (max_txn_acc 129)
    the epoch is refused before any launch, undeclared (0) the probe finds
    it (ERRB_BIG) -- DV_ERR_ARG either way, no row changed, and the context
    decides the next epoch bit-exact."""
    rows = 1 << 12
    bad = _max_len_epoch(rows, 400, 1800, longest=129)
    assert int(np.diff(bad.txn_begin).max()) == 129
    tab = O.YcsbTable(rows)
    f0 = tab.f0.copy()
    eng = CCEngine(cc, 400, bad.n_acc)
    try:
        eng.load_ycsb_partition(rows)
        before = eng.read_table(0, rows)
        dep = DeviceEpoch(bad)
        assert dep.max_txn_acc == 129
        if not declared:
            dep.max_txn_acc = 0
        with pytest.raises(dvcc.DvccError) as ex:
            eng.run_epoch_device(dep, torch.zeros(400, dtype=torch.uint8, device="cuda"))
        assert ex.value.code == dvcc._lib.DV_ERR_ARG, ex.value.code
        assert (eng.read_table(0, rows) == before).all(), "a rejected epoch changed the table"
        good = _max_len_epoch(rows, 400, 1801)
        c_ref, _, st_ref = _oracle_epoch(cc, tab, f0, good)
        c, _, st = _gpu_epoch(eng, good, "device")
        assert (c == c_ref).all() and st.read_digest == st_ref.read_digest
        assert (eng.read_table(0, rows) == f0).all()
    finally:
        eng.close()
