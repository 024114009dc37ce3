"""TPC-C GPU parity (config E): dv_tpcc_epoch_run_device through the C ABI
against the oracle on the same seeded epochs.  Integer work (the double
columns hold integer values), so bit-exact: commit bytes, o_id of every
committed NewOrder, and every state column of every table."""
import numpy as np
import pytest

import _oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import dvcc  # noqa: E402
from dvcc import tpcc as T  # noqa: E402

ORACLE_CC = {dvcc.NO_WAIT: O.NO_WAIT, dvcc.WAIT_DIE: O.WAIT_DIE, dvcc.OCC: O.OCC, dvcc.CALVIN: O.CALVIN}
CCS = [dvcc.NO_WAIT, dvcc.WAIT_DIE, dvcc.OCC, dvcc.CALVIN]


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    yield


def _params(kind, **kw):
    if kind == "small":
        d = dict(num_wh=4, cust_per_dist=1000, max_items=2000)
    else:  # config E, one GPU's share: 32 warehouses, full item / customer counts
        d = dict(num_wh=32, cust_per_dist=3000, max_items=100000)
    d.update(kw)
    return O.tpcc_params(**d), T.tpcc_params(**d)


def _check_tables(eng, db, p):
    for t in range(5):
        ref = db.table(t)
        for col in range(3):
            got = eng.read_col(t, col)
            assert (got == ref[1 + col]).all(), f"table {t} col {col}: {np.flatnonzero(got != ref[1 + col])[:5]}"


def _run(eng, e, offset=0):
    """offset: the commit bytes land `offset` bytes into a larger buffer
    (an unaligned slice), whose guard bytes on either side must survive."""
    dep, d_args = T.device_epoch(e)
    n = max(1, e.n_txn)
    big = torch.full((n + offset + 32,), 0xAB, dtype=torch.uint8, device="cuda")
    d_commit = big[offset:offset + n]
    d_oid = torch.zeros(n, dtype=torch.int64, device="cuda")
    st = eng.run_tpcc_epoch_device(dep, d_args, d_commit, d_oid)
    hb = big.cpu().numpy()
    assert (hb[:offset] == 0xAB).all() and (hb[offset + n:] == 0xAB).all(), "commit bytes outside the slice"
    return d_commit.cpu().numpy()[:e.n_txn], d_oid.cpu().numpy().view(np.uint64)[:e.n_txn], st


@pytest.mark.parametrize("cc", CCS)
@pytest.mark.parametrize("kind,n_txn,perc", [("small", 4096, 0.5), ("small", 3000, 0.0), ("small", 3000, 1.0),
                                             ("small", 1, 0.5), ("e", 65536, 0.5)])
def test_tpcc_epoch_parity(cc, kind, n_txn, perc):
    po, pp = _params(kind, perc_payment=perc)
    db = O.TpccDB(po, 5)
    eng = T.TpccEngine(cc, pp, n_txn, seed=5)
    try:
        e = T.gen(pp, n_txn, 11)
        c_ref, o_ref, st_ref = db.epoch(ORACLE_CC[cc], e.keys, e.types, e.tables, e.args, e.txn_begin)
        c, o, st = _run(eng, e)
        assert (c == c_ref).all(), f"commit mismatch at {np.flatnonzero(c != c_ref)[:5]}"
        assert (o == o_ref).all(), f"o_id mismatch at {np.flatnonzero(o != o_ref)[:5]}"
        assert st.committed == st_ref.committed and st.write_cnt == st_ref.write_cnt
        _check_tables(eng, db, pp)
    finally:
        eng.close()


@pytest.mark.parametrize("cc", CCS)
@pytest.mark.parametrize("offset", [1, 3, 8])
def test_tpcc_unaligned_commit_buffer(cc, offset):
    """The caller's commit-byte buffer at an odd offset (the
    commit-byte pass's scalar path ran past its own 16 txns when `out` was not
    16-byte aligned): commit bytes, counts and tables still equal the oracle's,
    and nothing outside the slice is written."""
    po, pp = _params("small")
    db = O.TpccDB(po, 5)
    eng = T.TpccEngine(cc, pp, 4096, seed=5)
    try:
        e = T.gen(pp, 4000, 13)
        c_ref, o_ref, st_ref = db.epoch(ORACLE_CC[cc], e.keys, e.types, e.tables, e.args, e.txn_begin)
        c, o, st = _run(eng, e, offset=offset)
        assert (c == c_ref).all(), f"commit mismatch at {np.flatnonzero(c != c_ref)[:5]}"
        assert (o == o_ref).all()
        assert st.committed == st_ref.committed and st.write_cnt == st_ref.write_cnt
        _check_tables(eng, db, pp)
    finally:
        eng.close()


@pytest.mark.parametrize("cc", [dvcc.WAIT_DIE, dvcc.CALVIN])
def test_tpcc_epochs_accumulate(cc):
    """State carries across epochs (D_NEXT_O_ID, YTD sums, stock levels)."""
    po, pp = _params("small", num_wh=2)
    db = O.TpccDB(po, 9)
    eng = T.TpccEngine(cc, pp, 2048, seed=9)
    try:
        for ep in range(4):
            e = T.gen(pp, 2048, 100 + ep)
            c_ref, o_ref, _ = db.epoch(ORACLE_CC[cc], e.keys, e.types, e.tables, e.args, e.txn_begin)
            c, o, _ = _run(eng, e)
            assert (c == c_ref).all() and (o == o_ref).all(), ep
        _check_tables(eng, db, pp)
    finally:
        eng.close()


@pytest.mark.parametrize("cc", CCS)
@pytest.mark.parametrize("kind,n_txn,epochs,lanes", [("small", 2048, 5, 1), ("e", 10_000, 3, 1),
                                                     ("small", 2048, 7, 2), ("e", 10_000, 9, 4)])
def test_tpcc_batch_pipelined(cc, kind, n_txn, epochs, lanes):
    """dv_tpcc_epoch_run_device_batch (epoch k+1 queued before k is read
    back; lanes 2: dv_tpcc_epoch_run_device_lanes, epochs decided alternately
    on two contexts) against the oracle running the epochs one after the
    other: commit bytes, o_id, stats of every epoch and every table after."""
    po, pp = _params(kind, num_wh=2) if kind == "small" else _params(kind)
    db = O.TpccDB(po, 9)
    eng = T.TpccEngine(cc, pp, n_txn, seed=9)
    extra = [eng.open_lane() for _ in range(lanes - 1)]
    try:
        es = [T.gen(pp, n_txn, 300 + k) for k in range(epochs)]
        refs = [db.epoch(ORACLE_CC[cc], e.keys, e.types, e.tables, e.args, e.txn_begin) for e in es]
        devs = [T.device_epoch(e) for e in es]
        commits = [torch.zeros(n_txn, dtype=torch.uint8, device="cuda") for _ in es]
        oids = [torch.zeros(n_txn, dtype=torch.int64, device="cuda") for _ in es]
        sts = eng.run_tpcc_epochs_device([d for d, _ in devs], [a for _, a in devs], commits, oids, lanes=extra)
        for k, (e, (c_ref, o_ref, st_ref), st) in enumerate(zip(es, refs, sts)):
            c = commits[k].cpu().numpy()
            o = oids[k].cpu().numpy().view(np.uint64)
            assert (c == c_ref).all(), f"epoch {k}: commit mismatch at {np.flatnonzero(c != c_ref)[:5]}"
            assert (o == o_ref).all(), f"epoch {k}: o_id mismatch at {np.flatnonzero(o != o_ref)[:5]}"
            assert st.committed == st_ref.committed and st.write_cnt == st_ref.write_cnt, k
        _check_tables(eng, db, pp)
    finally:
        eng.close()


@pytest.mark.parametrize("lanes", [1, 2, 4])
def test_tpcc_batch_halted_epochs_rerun(lanes):
    """Asynchronous rounds forced to yield in a pipelined TPC-C batch (or over
    two decision lanes): the halted epoch and the ones queued behind it run
    again synchronously, results unchanged."""
    po, pp = _params("small", num_wh=2)
    db = O.TpccDB(po, 9)
    eng = T.TpccEngine(dvcc.WAIT_DIE, pp, 2048, seed=9)
    extra = [eng.open_lane() for _ in range(lanes - 1)]
    for e in [eng] + extra:
        e.set_async_limits(1, 0)
    try:
        es = [T.gen(pp, 2048, 400 + k) for k in range(4)]
        refs = [db.epoch(O.WAIT_DIE, e.keys, e.types, e.tables, e.args, e.txn_begin) for e in es]
        devs = [T.device_epoch(e) for e in es]
        commits = [torch.zeros(2048, dtype=torch.uint8, device="cuda") for _ in es]
        oids = [torch.zeros(2048, dtype=torch.int64, device="cuda") for _ in es]
        sts = eng.run_tpcc_epochs_device([d for d, _ in devs], [a for _, a in devs], commits, oids, lanes=extra)
        assert sum(st.async_yields for st in sts) > 0, "no asynchronous launch yielded"
        for k, (c_ref, o_ref, _) in enumerate(refs):
            assert (commits[k].cpu().numpy() == c_ref).all(), k
            assert (oids[k].cpu().numpy().view(np.uint64) == o_ref).all(), k
        _check_tables(eng, db, pp)
    finally:
        eng.close()


def test_tpcc_missing_last_name():
    """A last-name key with no customer is fatal in the reference
    (M_ASSERT_V, index_hash.cpp:225): DV_ERR_KEY_NOT_FOUND."""
    po, pp = _params("small", perc_payment=1.0)
    eng = T.TpccEngine(dvcc.NO_WAIT, pp, 16, seed=5)
    try:
        e = T.gen(pp, 16, 3)
        name = np.flatnonzero(e.tables == T.L.T_CUST_LAST)
        assert len(name)
        e.keys[name[0]] = 12345  # no custNPKey has this value
        with pytest.raises(dvcc.DvccError) as ei:
            _run(eng, e)
        assert ei.value.code == -4
    finally:
        eng.close()


def _global_position(batches):
    """Origin batches -> one epoch in position-major order
    (DV_COMM_POSITION_ORDER: origin q's txn j is sequence number j * P + q);
    also the index of every access in the origin-major concatenation"""
    P = len(batches)
    tpr = batches[0].n_txn
    assert all(b.n_txn == tpr for b in batches)
    offs = np.cumsum([0] + [len(b.keys) for b in batches])
    idx = []
    for j in range(tpr):
        for q, b in enumerate(batches):
            lo, hi = int(b.txn_begin[j]), int(b.txn_begin[j + 1])
            idx.append(np.arange(offs[q] + lo, offs[q] + hi))
    idx = np.concatenate(idx).astype(np.int64)
    keys, types, tables, args, _ = _global(batches)
    sizes = np.array([int(b.txn_begin[j + 1] - b.txn_begin[j]) for j in range(tpr) for b in batches], np.int64)
    tb = np.zeros(len(sizes) + 1, np.uint32)
    tb[1:] = np.cumsum(sizes)
    return (keys[idx], types[idx], tables[idx], args[idx], tb), idx


def _origin_order(v, world, n_txn):
    """per-txn values of a position-major sequence in origin order (q * n_txn + j)"""
    return np.asarray(v).reshape(n_txn, world).T.reshape(-1)


def _global(batches):
    """Origin batches -> one epoch in Calvin's global order (rank-major)."""
    keys = np.concatenate([b.keys for b in batches])
    types = np.concatenate([b.types for b in batches])
    tables = np.concatenate([b.tables for b in batches])
    args = np.concatenate([b.args for b in batches])
    sizes = np.concatenate([np.diff(b.txn_begin.astype(np.int64)) for b in batches])
    tb = np.zeros(len(sizes) + 1, np.uint32)
    tb[1:] = np.cumsum(sizes)
    return keys, types, tables, args, tb


@pytest.mark.parametrize("cc", CCS)
@pytest.mark.parametrize("world", [2, 4, 8])
def test_tpcc_partitioned_engines(cc, world):
    """config E's layout on one GPU: `world` contexts, each the partition of
    its warehouses ((w-1) % PART_CNT, ITEM replicated); fragments routed by
    owner in origin order, verdicts combined by MAX (the all-reduce) -- equal
    to the single-thread E-schedule over the whole epoch."""
    from dvcc.partitioned import split_by_owner, owner_order
    n_txn = 1500
    kw = dict(num_wh=2 * world, cust_per_dist=1000, max_items=2000, part_cnt=world, part_per_txn=2, mpr=1.0)
    pp = T.tpcc_params(**kw)
    batches = [T.gen(pp, n_txn, 40 + r, home_part=r) for r in range(world)]
    kw1 = dict(kw, part_cnt=1)
    db = O.TpccDB(O.tpcc_params(**kw1), 5)
    c_ref, o_ref, st_ref = db.epoch(ORACLE_CC[cc], *_global(batches))
    N = n_txn * world
    engines, parts = [], []
    for p in range(world):
        ks, ts, xs, tbs, ags = [], [], [], [], []
        for r, b in enumerate(batches):
            k, t, x, counts = split_by_owner(b, r * n_txn, world)
            _, order = owner_order(b, world)
            lo = int(counts[:p].sum()); hi = lo + int(counts[p])
            ks.append(k[lo:hi]); ts.append(t[lo:hi]); xs.append(x[lo:hi])
            tbs.append(b.tables[order][lo:hi]); ags.append(b.args[order][lo:hi])
        k = np.concatenate(ks); t = np.concatenate(ts); x = np.concatenate(xs)
        eng = T.TpccEngine(cc, pp, N, part_id=p, seed=5)
        dep = dvcc.DeviceEpoch.from_tensors(torch.from_numpy(k.view(np.int64)).cuda(), torch.from_numpy(t).cuda(),
                                            torch.from_numpy(x).cuda(), N,
                                            tables=torch.from_numpy(np.concatenate(tbs)).cuda(), max_txn_acc=33)
        args = torch.from_numpy(np.concatenate(ags).view(np.int64)).cuda()
        oid = torch.zeros(N, dtype=torch.int64, device="cuda")
        eng.begin_tpcc(dep, args, oid)
        engines.append(eng)
        parts.append((dep, args, oid))
    if cc != dvcc.CALVIN:
        for _ in range(N + 1):
            vs = []
            for eng in engines:
                v = torch.zeros((N + 3) // 4 * 4, dtype=torch.uint8, device="cuda")
                eng.round_local(v)
                vs.append(v)
            torch.cuda.synchronize()
            comb = torch.stack(vs).max(dim=0).values.contiguous()
            copies = [comb.clone() for _ in engines]
            torch.cuda.synchronize()
            und = [eng.round_apply(cp) for eng, cp in zip(engines, copies)]
            assert len(set(und)) == 1
            if und[0] == 0:
                break
    oid_sum = np.zeros(N, np.uint64)
    committed = 0
    for p, eng in enumerate(engines):
        commit = torch.zeros(N, dtype=torch.uint8, device="cuda")
        st = eng.finish(commit)
        committed += st.committed
        assert (commit.cpu().numpy() == c_ref).all(), p
        oid_sum += parts[p][2].cpu().numpy().view(np.uint64)
        for tid in range(5):
            ref = db.table(tid)
            mine = np.isin(ref[0], T.table(pp, 5, tid, p)[0])
            for col in range(3):
                assert (eng.read_col(tid, col) == ref[1 + col][mine]).all(), (p, tid, col)
        eng.close()
    assert (oid_sum == o_ref).all()


def _tpcc_group(cc, kw, world, n_txn, seed, gen_seed, position=False):
    """`world` TPC-C contexts on this GPU joined by the in-process transport
    (dv_comm_init_local), one epoch through dv_tpcc_epoch_run_part on one
    host thread each; returns (engines, params, batches, per-rank results).
    position: DV_COMM_POSITION_ORDER (the list protocol sequences the
    origins' batches txn by txn)."""
    import threading
    pp = T.tpcc_params(part_cnt=world, **kw)
    batches = [T.gen(pp, n_txn, gen_seed + r, home_part=r) for r in range(world)]
    engines = [T.TpccEngine(cc, pp, n_txn * world, part_id=p, seed=seed) for p in range(world)]
    dvcc.CCEngine.comm_init_local(engines)
    if position:
        for eng in engines:
            eng.comm_set_mode(dvcc._lib.DV_COMM_POSITION_ORDER)
    out = [None] * world

    def body(r):
        try:
            b = batches[r]
            dep, d_args = T.device_epoch(b)
            own = torch.from_numpy(b.owner).cuda()
            d_commit = torch.zeros(n_txn * world, dtype=torch.uint8, device="cuda")
            d_oid = torch.zeros(n_txn * world, dtype=torch.int64, device="cuda")
            st = engines[r].run_tpcc_epoch_part(dep, d_args, own, n_txn, d_commit, d_oid)
            out[r] = (d_commit.cpu().numpy(), d_oid.cpu().numpy().view(np.uint64), st)
        except Exception as ex:  # noqa: BLE001 -- reported per rank
            out[r] = ex
    th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
        assert not t.is_alive(), "a rank hung in the partitioned TPC-C epoch"
    return engines, pp, batches, out


def _check_tpcc_group(cc, kw, world, n_txn, full_tables, position=False):
    engines, pp, batches, out = _tpcc_group(cc, kw, world, n_txn, 5, 60, position=position)
    try:
        # the oracle's all-warehouse image with last-name lists per partition
        # of this layout (custNPKey collides across warehouses from 103 on)
        db = O.TpccDB(O.tpcc_params(**dict(kw, part_cnt=1)), 5, index_parts=world)
        owner = np.concatenate([b.owner for b in batches])
        if position and cc != dvcc.CALVIN:  # (CALVIN keeps the sequencer's origin order)
            ep, idx = _global_position(batches)
            c_ref, o_ref, st_ref = db.epoch(ORACLE_CC[cc], *ep, owner=owner[idx])
            c_ref, o_ref = _origin_order(c_ref, world, n_txn), _origin_order(o_ref, world, n_txn)
        else:
            c_ref, o_ref, st_ref = db.epoch(ORACLE_CC[cc], *_global(batches), owner=owner)
        committed = 0
        for r, x in enumerate(out):
            assert not isinstance(x, Exception), f"rank {r}: {x}"
            c, o, st = x
            assert (c == c_ref).all(), f"rank {r}: {(c != c_ref).sum()} commit mismatches"
            assert (o == o_ref).all(), f"rank {r}: o_id (RFWD all-reduce) differs"
            committed = st.committed
        assert committed == st_ref.committed
        for tid in range(5):
            ref = db.table(tid)
            if full_tables or tid == T.L.T_ITEM:  # (ITEM: replicated on every partition)
                for p, eng in enumerate(engines):
                    mine = np.isin(ref[0], T.table(pp, 5, tid, p)[0])
                    for col in range(3):
                        assert (eng.read_col(tid, col) == ref[1 + col][mine]).all(), (p, tid, col)
            else:  # order-free digest of every (key, column) pair over all partitions
                def dig(keys, cols):
                    h = keys * np.uint64(0x9E3779B97F4A7C15)
                    for j, c in enumerate(cols):
                        h ^= (c + np.uint64(j + 1)) * np.uint64(0xC2B2AE3D27D4EB4F)
                    return int(h.sum(dtype=np.uint64))
                want = dig(ref[0], ref[1:])
                got = sum(dig(T.table(pp, 5, tid, p)[0], [eng.read_col(tid, col) for col in range(3)])
                          for p, eng in enumerate(engines)) % (1 << 64)
                assert got == want, f"table {tid}"
    finally:
        for eng in engines:
            eng.close()


@pytest.mark.parametrize("cc", CCS)
@pytest.mark.parametrize("world", [2, 8])
def test_tpcc_engine_driver(cc, world):
    """dv_tpcc_epoch_run_part: owner split by the per-access owner byte,
    records with table and operation word, per-partition last-name lookup,
    decisions and execution, o_id all-reduced to every rank -- equal to the
    single-thread E-schedule over the sequenced global epoch."""
    kw = dict(num_wh=2 * world, cust_per_dist=1000, max_items=2000, part_per_txn=2, mpr=1.0)
    _check_tpcc_group(cc, kw, world, 1500, full_tables=True)


@pytest.mark.parametrize("cc", CCS)
@pytest.mark.parametrize("world", [2, 4])
def test_tpcc_engine_driver_position_order(cc, world):
    """dv_tpcc_epoch_run_part under DV_COMM_POSITION_ORDER: each owner
    interleaves the records it receives txn by txn (origin q's txn j at
    j * P + q; CALVIN keeps the origin order) -- commit bytes and o_id, in
    origin order, equal the oracle over the position-major sequence, and so
    do the rows."""
    kw = dict(num_wh=2 * world, cust_per_dist=1000, max_items=2000, part_per_txn=2, mpr=1.0)
    _check_tpcc_group(cc, kw, world, 1500, full_tables=True, position=True)


@pytest.mark.slow
@pytest.mark.parametrize("cc", [dvcc.WAIT_DIE, dvcc.CALVIN])
def test_tpcc_config_e_full_layout(cc):
    """Config E's full layout: 256 warehouses over 8 partitions (32 each),
    full item / customer counts, MPR 1.0, PERC_PAYMENT 0.5 -- 8 contexts on
    this GPU driven by the engine's partitioned protocol."""
    kw = dict(num_wh=256, cust_per_dist=3000, max_items=100000, part_per_txn=2, mpr=1.0)
    _check_tpcc_group(cc, kw, 8, 1250, full_tables=False)


def test_tpcc_engine_driver_bad_owner():
    """An owner byte >= the partition count: DV_ERR_ARG on every rank, no
    rank hangs, no table changes."""
    world = 2
    kw = dict(num_wh=4, cust_per_dist=1000, max_items=2000, part_per_txn=2, mpr=1.0)
    pp = T.tpcc_params(part_cnt=world, **kw)
    batches = [T.gen(pp, 500, 70 + r, home_part=r) for r in range(world)]
    batches[1].owner[3] = 7
    engines = [T.TpccEngine(dvcc.WAIT_DIE, pp, 500 * world, part_id=p, seed=5) for p in range(world)]
    dvcc.CCEngine.comm_init_local(engines)
    import threading
    before = [[eng.read_col(t, 0) for t in range(5)] for eng in engines]
    out = [None] * world

    def body(r):
        try:
            dep, d_args = T.device_epoch(batches[r])
            own = torch.from_numpy(batches[r].owner).cuda()
            d_commit = torch.zeros(500 * world, dtype=torch.uint8, device="cuda")
            out[r] = engines[r].run_tpcc_epoch_part(dep, d_args, own, 500, d_commit)
        except Exception as ex:  # noqa: BLE001
            out[r] = ex
    th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
        assert not t.is_alive()
    try:
        for r, x in enumerate(out):
            assert isinstance(x, dvcc.DvccError) and x.code == dvcc._lib.DV_ERR_ARG, (r, x)
        for eng, b in zip(engines, before):
            assert all((eng.read_col(t, 0) == b[t]).all() for t in range(5))
    finally:
        for eng in engines:
            eng.close()


@pytest.mark.parametrize("cc", [dvcc.WAIT_DIE, dvcc.CALVIN])
def test_tpcc_runner_single_rank_rccl(cc):
    """The torch.distributed driver (RCCL) over a TPC-C engine, one rank."""
    import torch.distributed as dist
    from dvcc.partitioned import EnginePartition, PartitionedEpoch, PartitionedRunner
    if dist.is_initialized():
        dist.destroy_process_group()
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1)
    try:
        po, pp = _params("small")
        db = O.TpccDB(po, 5)
        eng = T.TpccEngine(cc, pp, 3000, seed=5)
        e = T.gen(pp, 3000, 21)
        c_ref, o_ref, _ = db.epoch(ORACLE_CC[cc], e.keys, e.types, e.tables, e.args, e.txn_begin)
        part = EnginePartition(eng)
        runner = PartitionedRunner(part, 1, 0)
        commit = torch.zeros(3000, dtype=torch.uint8, device="cuda")
        runner.run(PartitionedEpoch(e, 0, 1, 3000, "cuda"), commit=commit)
        assert (commit.cpu().numpy() == c_ref).all()
        assert (part.oid.cpu().numpy().view(np.uint64)[:3000] == o_ref).all()
        _check_tables(eng, db, pp)
        eng.set_stream(None)
        eng.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name", sorted(f[:-4] for f in __import__("os").listdir(
    __import__("os").path.join(__import__("os").path.dirname(__file__), "golden", "tpcc")) if f.endswith(".npz")))
def test_engine_matches_tpcc_golden(name):
    import os
    from golden.make_golden_tpcc import CASES, LOAD_SEED, PARAMS
    with np.load(os.path.join(os.path.dirname(__file__), "golden", "tpcc", name + ".npz")) as z:
        g = {k: z[k] for k in z.files}
    cc = {O.NO_WAIT: dvcc.NO_WAIT, O.WAIT_DIE: dvcc.WAIT_DIE, O.OCC: dvcc.OCC, O.CALVIN: dvcc.CALVIN}[int(g["cc"])]
    pp = T.tpcc_params(perc_payment=float(g["perc"]), **PARAMS)
    e = T.TpccEpoch(g["keys"], g["types"], g["txn_begin"], g["tables"], g["args"])
    eng = T.TpccEngine(cc, pp, e.n_txn, seed=LOAD_SEED)
    try:
        before = [[eng.read_col(t, c) for c in range(3)] for t in range(5)]
        c, o, st = _run(eng, e)
        assert np.array_equal(c, g["commit"]) and np.array_equal(o, g["oid"])
        assert (st.committed, st.aborted, st.write_cnt) == tuple(int(x) for x in g["stats"])
        for t in range(5):
            after = np.stack([eng.read_col(t, col) for col in range(3)], 1)
            rows = np.flatnonzero((after != np.stack(before[t], 1)).any(1))
            assert np.array_equal(rows, g[f"rows_{t}"]) and np.array_equal(after[rows], g[f"vals_{t}"]), t
    finally:
        eng.close()


@pytest.mark.slow
@pytest.mark.parametrize("cc", [dvcc.WAIT_DIE, dvcc.CALVIN])
@pytest.mark.parametrize("n_txn", [65_536, 10_000])
def test_tpcc_bench_timed_path_lanes(cc, n_txn):
    """bench.py's TPC-C leg at its own size: config E's share of one GPU (32
    warehouses, full counts, engine seed 1), the leg's 3 distinct epochs
    (seeds epoch_seed(0, e)) cycled twice over four decision lanes
    (dv_tpcc_epoch_run_device_lanes) -- commit bytes, o_id and stats of every
    epoch and every table after, against the oracle running them in order."""
    po, pp = _params("e")
    db = O.TpccDB(po, 1)
    eng = T.TpccEngine(cc, pp, n_txn, seed=1)
    extra = [eng.open_lane() for _ in range(3)]
    try:
        es = [T.gen(pp, n_txn, dvcc.epoch_seed(0, e)) for e in range(3)] * 2
        refs = [db.epoch(ORACLE_CC[cc], e.keys, e.types, e.tables, e.args, e.txn_begin) for e in es]
        devs = [T.device_epoch(e) for e in es]
        commits = [torch.zeros(n_txn, dtype=torch.uint8, device="cuda") for _ in es]
        oids = [torch.zeros(n_txn, dtype=torch.int64, device="cuda") for _ in es]
        sts = eng.run_tpcc_epochs_device([d for d, _ in devs], [a for _, a in devs], commits, oids, lanes=extra)
        for k, ((c_ref, o_ref, st_ref), st) in enumerate(zip(refs, sts)):
            assert (commits[k].cpu().numpy() == c_ref).all(), k
            assert (oids[k].cpu().numpy().view(np.uint64) == o_ref).all(), k
            assert st.committed == st_ref.committed and st.write_cnt == st_ref.write_cnt, k
        _check_tables(eng, db, pp)
    finally:
        eng.close()


def test_tpcc_part_txn_id_past_txns_per_rank_is_rejected():
    """dv_tpcc_epoch_run_part with a batch whose txn ids reach txns_per_rank:
    the owner split sends them as an invalid id, and every rank returns
    DV_ERR_TXN_RANGE with no row changed (the id would otherwise alias the next
    origin's txn 0 and merge two txns)."""
    import threading
    world, n_txn = 2, 300
    pp = T.tpcc_params(part_cnt=world, num_wh=4, cust_per_dist=1000, max_items=2000)
    batches = [T.gen(pp, n_txn, 70 + r, home_part=r) for r in range(world)]
    engines = [T.TpccEngine(dvcc.WAIT_DIE, pp, n_txn * world, part_id=p, seed=5) for p in range(world)]
    dvcc.CCEngine.comm_init_local(engines)
    before = [[eng.read_col(t, 0).copy() for t in range(5)] for eng in engines]
    out = [None] * world

    def body(r):
        try:
            dep, d_args = T.device_epoch(batches[r])
            if r == 1:
                t = dep.acc_txn.clone()
                t[-2:] = n_txn  # the last txn's accesses name txn n_txn
                dep = dvcc.DeviceEpoch.from_tensors(dep.keys, dep.types, t, n_txn, max_txn_acc=dep.max_txn_acc,
                                                    tables=dep.tables)
            own = torch.from_numpy(batches[r].owner).cuda()
            d_commit = torch.zeros(n_txn * world, dtype=torch.uint8, device="cuda")
            d_oid = torch.zeros(n_txn * world, dtype=torch.int64, device="cuda")
            out[r] = engines[r].run_tpcc_epoch_part(dep, d_args, own, n_txn, d_commit, d_oid)
        except Exception as ex:  # noqa: BLE001 -- reported per rank
            out[r] = ex
    th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
        assert not t.is_alive(), "a rank hung"
    try:
        for r, x in enumerate(out):
            assert isinstance(x, dvcc.DvccError) and x.code == dvcc._lib.DV_ERR_TXN_RANGE, (r, x)
        for eng, b in zip(engines, before):
            for t in range(5):
                assert (eng.read_col(t, 0) == b[t]).all()
    finally:
        for eng in engines:
            eng.close()
