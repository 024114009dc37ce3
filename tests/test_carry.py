"""Abort carry-over into the next epoch.

The reference retries an aborted txn with its query unchanged after a
penalty (WorkerThread::abort, worker_thread.cpp:160-172; AbortQueue::enqueue /
process, abort_queue.cpp:26-82).  The engine's rule: the penalty is one epoch;
the aborted txns of epoch k, in sequence order, open epoch k+1 ahead of its
new txns.  `host_carry` below restates that rule on the host (checker side);
every epoch of the closed loop is decided by the oracle's E-schedule and the
engine must match it bit for bit: decisions, digests, carried epochs and the
final table.
"""
import numpy as np
import pytest

import _oracle as O
import dvcc
from dvcc import CCEngine, DeviceEpoch, Epoch, YCSBQueryGenerator

ORACLE_CC = {dvcc.NO_WAIT: O.NO_WAIT, dvcc.WAIT_DIE: O.WAIT_DIE, dvcc.OCC: O.OCC}


def host_carry(ep, commit, max_txn):
    """The aborted txns of `ep` (commit byte 0), in order, at most max_txn."""
    tb = ep.txn_begin.astype(np.int64)
    ab = np.flatnonzero(commit[:ep.n_txn] == 0)[:max_txn]
    idx, ntb = _gather_txns(tb, ab)
    return Epoch(ep.keys[idx].copy(), ep.types[idx].copy(), ntb)


def _gather_txns(tb, ids):
    """access indices of txns `ids` (in that order) of an epoch with
    txn_begin `tb`, and the new txn_begin"""
    lens = tb[ids + 1] - tb[ids]
    ntb = np.zeros(len(ids) + 1, np.int64)
    ntb[1:] = np.cumsum(lens)
    idx = np.repeat(tb[ids] - ntb[:-1], lens) + np.arange(int(ntb[-1]), dtype=np.int64)
    return idx, ntb.astype(np.uint32)


def host_concat(a, b):
    tb = np.concatenate([a.txn_begin, b.txn_begin[1:] + a.txn_begin[-1]]).astype(np.uint32)
    return Epoch(np.concatenate([a.keys, b.keys]), np.concatenate([a.types, b.types]), tb)


def test_host_carry_rule():
    ep = Epoch(np.arange(7, dtype=np.uint64), np.array([0, 1, 1, 0, 1, 0, 1], np.uint8),
               np.array([0, 2, 3, 5, 7], np.uint32))
    c = host_carry(ep, np.array([1, 0, 0, 1], np.uint8), 8)
    assert c.n_txn == 2 and list(c.keys) == [2, 3, 4] and list(c.txn_begin) == [0, 1, 3]
    assert host_carry(ep, np.array([1, 0, 0, 1], np.uint8), 1).n_txn == 1
    nxt = host_concat(c, ep)
    assert nxt.n_txn == 6 and list(nxt.txn_begin) == [0, 1, 3, 5, 6, 8, 10]


def test_device_epoch_concat_cpu_tensors():
    torch = pytest.importorskip("torch")
    a = DeviceEpoch.from_tensors(torch.tensor([5, 6], dtype=torch.int64), torch.tensor([1, 0], dtype=torch.uint8),
                                 torch.tensor([0, 1], dtype=torch.int32), 2, max_txn_acc=1)
    b = DeviceEpoch.from_tensors(torch.tensor([7, 8, 9], dtype=torch.int64),
                                 torch.tensor([0, 0, 1], dtype=torch.uint8),
                                 torch.tensor([0, 0, 1], dtype=torch.int32), 2, max_txn_acc=2)
    c = DeviceEpoch.concat(a, b)
    assert c.n_txn == 4 and c.n_acc == 5 and c.max_txn_acc == 2
    assert c.acc_txn.tolist() == [0, 1, 2, 2, 3] and c.keys.tolist() == [5, 6, 7, 8, 9]


@pytest.mark.gpu
@pytest.mark.parametrize("cc", [dvcc.NO_WAIT, dvcc.WAIT_DIE, dvcc.OCC])
def test_closed_loop_carry(cc):
    """Fixed-size epochs: the carried txns first, new txns fill the rest."""
    import torch
    rows, N, R = 1 << 14, 3000, 10
    gen = YCSBQueryGenerator(rows, zipf_theta=0.9, txn_write_perc=1.0, tup_write_perc=0.5)
    eng = CCEngine(cc, N, N * R)
    eng.load_ycsb_partition(rows)
    tab = O.YcsbTable(rows)
    f0 = tab.f0.copy()
    host = gen.gen(N, dvcc.epoch_seed(0, 0))
    dev = DeviceEpoch(host)
    d_commit = torch.zeros(N, dtype=torch.uint8, device="cuda")
    carried_total = 0
    for k in range(5):
        c_ref, _, st_ref = O.epoch_run(ORACLE_CC[cc], tab.ix, f0, host.n_txn, host.txn_begin,
                                       host.keys, host.types)
        st = eng.run_epoch_device(dev, d_commit)
        assert np.array_equal(d_commit.cpu().numpy()[:host.n_txn], c_ref[:host.n_txn]), k
        assert (st.committed, st.read_digest, st.write_cnt) == (st_ref.committed, st_ref.read_digest,
                                                               st_ref.write_cnt)
        cap = N if k % 2 == 0 else N // 3  # also a cap below the aborted count
        hc = host_carry(host, c_ref, cap)
        dc = eng.carry(dev, cap)
        assert (dc.n_txn, dc.n_acc) == (hc.n_txn, hc.n_acc)
        assert np.array_equal(dc.keys.cpu().numpy().view(np.uint64), hc.keys)
        assert np.array_equal(dc.types.cpu().numpy(), hc.types)
        assert np.array_equal(dc.acc_txn.cpu().numpy().view(np.uint32), hc.acc_txn())
        carried_total += hc.n_txn
        new = gen.gen(N - hc.n_txn, dvcc.epoch_seed(0, k + 1))
        host = host_concat(hc, new)
        dev = DeviceEpoch.concat(dc, DeviceEpoch(new))
    assert carried_total > 0
    assert np.array_equal(eng.read_table(0, rows), f0)
    eng.close()


@pytest.mark.gpu
def test_carry_rejects_calvin_and_stale_epochs():
    import torch
    gen = YCSBQueryGenerator(1 << 10, zipf_theta=0.9)
    e = gen.gen(200, 1)
    eng = CCEngine(dvcc.CALVIN, 200, 2000)
    eng.load_ycsb_partition(1 << 10)
    dev = DeviceEpoch(e)
    eng.run_epoch_device(dev, torch.zeros(200, dtype=torch.uint8, device="cuda"))
    with pytest.raises(dvcc.DvccError):
        eng.carry(dev)
    eng.close()
    eng = CCEngine(dvcc.NO_WAIT, 400, 4000)
    eng.load_ycsb_partition(1 << 10)
    eng.run_epoch_device(dev, torch.zeros(200, dtype=torch.uint8, device="cuda"))
    with pytest.raises(dvcc.DvccError):  # not the epoch the context decided last
        eng.carry(DeviceEpoch(gen.gen(100, 2)))
    eng.close()


def host_take(pool, cur, n):
    """txns [cur, cur + n) of the pool, wrapping around it (the fresh txns of
    the device closed loop)"""
    ids = (cur + np.arange(n)) % pool.n_txn
    idx, ntb = _gather_txns(pool.txn_begin.astype(np.int64), ids)
    return Epoch(pool.keys[idx].copy(), pool.types[idx].copy(), ntb)


def host_closed_loop(cc, tab, f0, pool, cur, n_txn, n_epochs, first=None):
    """the oracle's closed loop: each epoch decided by the E-schedule, its
    aborts carried ahead of fresh pool txns.  Returns the per-epoch commit
    bytes and stats, the next epoch and the cursor."""
    host = first if first is not None else host_take(pool, cur, n_txn)
    if first is None:
        cur = (cur + n_txn) % pool.n_txn
    out = []
    for _ in range(n_epochs):
        c_ref, _, st_ref = O.epoch_run(ORACLE_CC[cc], tab.ix, f0, host.n_txn, host.txn_begin, host.keys,
                                       host.types)
        out.append((c_ref[:host.n_txn].copy(), st_ref, host))
        hc = host_carry(host, c_ref, n_txn)
        fresh = n_txn - hc.n_txn
        host = host_concat(hc, host_take(pool, cur, fresh))
        cur = (cur + fresh) % pool.n_txn
    return out, host, cur


def _pool(rows, n, seed, R=10):
    gen = YCSBQueryGenerator(rows, zipf_theta=0.9, txn_write_perc=1.0, tup_write_perc=0.5, req_per_query=R)
    return gen.gen(n, seed)


def _check_loop(eng, cc, rows, pool, n_txn, n_epochs, calls=1, cur0=0):
    import torch
    tab = O.YcsbTable(rows)
    f0 = tab.f0.copy()
    ref, nxt, cur_ref = host_closed_loop(cc, tab, f0, pool, cur0, n_txn, n_epochs * calls)
    dpool = DeviceEpoch(pool)
    pb = torch.from_numpy(pool.txn_begin.astype(np.int32)).cuda()
    cursor = torch.full((1,), cur0, dtype=torch.int32, device="cuda")
    commits = [torch.zeros(n_txn, dtype=torch.uint8, device="cuda") for _ in range(n_epochs)]
    bufs = None
    got = []
    for call in range(calls):
        sts, bufs, cursor = eng.closed_loop(dpool, pb, n_txn, n_epochs, cursor=cursor, bufs=bufs,
                                            d_commits=commits, resume=call > 0)
        got += [(c.cpu().numpy().copy(), s) for c, s in zip(commits, sts)]
        if n_epochs & 1:
            bufs.swap()
    for k, ((c, st), (c_ref, st_ref, host)) in enumerate(zip(got, ref)):
        assert np.array_equal(c, c_ref), k
        assert (st.n_txn, st.n_acc, st.committed) == (host.n_txn, host.n_acc, st_ref.committed), k
        assert (st.read_digest, st.write_cnt) == (st_ref.read_digest, st_ref.write_cnt), k
    # the next epoch the loop left, and the cursor
    assert int(cursor.item()) == cur_ref
    e = bufs.epoch(0, n_txn, pool.max_txn_acc())
    assert e.n_acc == nxt.n_acc
    assert np.array_equal(e.keys.cpu().numpy().view(np.uint64), nxt.keys)
    assert np.array_equal(e.types.cpu().numpy(), nxt.types)
    assert np.array_equal(e.acc_txn.cpu().numpy().view(np.uint32), nxt.acc_txn())
    assert np.array_equal(eng.read_table(0, rows), f0)


@pytest.mark.gpu
@pytest.mark.parametrize("cc", [dvcc.NO_WAIT, dvcc.WAIT_DIE, dvcc.OCC])
@pytest.mark.parametrize("prefix", [None, 400])
def test_device_closed_loop(cc, prefix):
    """dv_epoch_run_closed_loop against the oracle's host loop: epochs one at
    a time (prefix off) and pipelined prefix-kill epochs, the pool wrapping"""
    rows, N = 1 << 13, 2000
    pool = _pool(rows, 5000, 11)
    eng = CCEngine(cc, N, N * 10)
    eng.set_prefix(prefix)
    eng.load_ycsb_partition(rows)
    _check_loop(eng, cc, rows, pool, N, 6, cur0=1234)
    eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("cc", [dvcc.NO_WAIT, dvcc.OCC])
def test_device_closed_loop_halts_and_resume(cc):
    """asynchronous launches forced to yield (every epoch halts and is decided
    again before its successor is rebuilt), and a loop continued over three
    calls (resume) -- the same epochs as one host loop"""
    rows, N = 1 << 13, 3000
    pool = _pool(rows, 4000, 12, R=12)
    eng = CCEngine(cc, N, N * 12)
    eng.set_prefix(500)
    eng.set_async_limits(1, 0)
    eng.load_ycsb_partition(rows)
    _check_loop(eng, cc, rows, pool, N, 3, calls=3)
    eng.close()


@pytest.mark.gpu
def test_device_closed_loop_args():
    import torch
    rows = 1 << 10
    pool = _pool(rows, 300, 13)
    dpool = DeviceEpoch(pool)
    pb = torch.from_numpy(pool.txn_begin.astype(np.int32)).cuda()
    eng = CCEngine(dvcc.CALVIN, 300, 3000)
    eng.load_ycsb_partition(rows)
    with pytest.raises(dvcc.DvccError):  # no aborts to carry
        eng.closed_loop(dpool, pb, 100, 2)
    eng.close()
    eng = CCEngine(dvcc.NO_WAIT, 300, 3000)
    eng.load_ycsb_partition(rows)
    with pytest.raises(dvcc.DvccError):  # more txns per epoch than the pool holds
        eng.closed_loop(dpool, pb, 301, 2)
    with pytest.raises(dvcc.DvccError):  # an epoch's bound past the context's max_acc
        eng.closed_loop(DeviceEpoch(_pool(rows, 400, 14, R=16)), pb, 300, 1)
    eng.closed_loop(dpool, pb, 250, 2)
    eng.close()


def host_closed_loop_lanes(cc, tab, f0, pool, cur, n_txn, n_epochs, lanes):
    """the oracle of dv_epoch_run_closed_loop_lanes: each lane's first epoch
    fresh (lane 0 first), then epoch k + L = epoch k's aborts + fresh pool
    txns drawn in epoch order.  Returns the per-epoch results, the epochs left
    for k = n_epochs .. n_epochs + L - 1, and the cursor."""
    inputs = {}
    for ln in range(lanes):
        inputs[ln] = host_take(pool, cur, n_txn)
        cur = (cur + n_txn) % pool.n_txn
    out = []
    for k in range(n_epochs):
        host = inputs.pop(k)
        c_ref, _, st_ref = O.epoch_run(ORACLE_CC[cc], tab.ix, f0, host.n_txn, host.txn_begin, host.keys,
                                       host.types)
        out.append((c_ref[:host.n_txn].copy(), st_ref, host))
        hc = host_carry(host, c_ref, n_txn)
        fresh = n_txn - hc.n_txn
        inputs[k + lanes] = host_concat(hc, host_take(pool, cur, fresh))
        cur = (cur + fresh) % pool.n_txn
    return out, inputs, cur


def _check_loop_lanes(cc, rows, pool, n_txn, n_epochs, lanes, prefix, calls=1, async_iters=None):
    import torch
    eng = CCEngine(cc, n_txn, n_txn * pool.max_txn_acc())
    eng.set_prefix(prefix)
    eng.load_ycsb_partition(rows)
    extra = [eng.open_lane() for _ in range(lanes - 1)]
    if async_iters:
        for e in [eng] + extra:
            e.set_async_limits(async_iters, 0)
    try:
        tab = O.YcsbTable(rows)
        f0 = tab.f0.copy()
        ref, nxt, cur_ref = host_closed_loop_lanes(cc, tab, f0, pool, 0, n_txn, n_epochs * calls, lanes)
        dpool = DeviceEpoch(pool)
        pb = torch.from_numpy(pool.txn_begin.astype(np.int32)).cuda()
        commits = [torch.zeros(n_txn, dtype=torch.uint8, device="cuda") for _ in range(n_epochs)]
        cursor, bufs, got = None, None, []
        for call in range(calls):
            sts, bufs, cursor = eng.closed_loop_lanes(extra, dpool, pb, n_txn, n_epochs, cursor=cursor, bufs=bufs,
                                                      d_commits=commits, resume=call > 0)
            got += [(c.cpu().numpy().copy(), s) for c, s in zip(commits, sts)]
        for k, ((c, st), (c_ref, st_ref, host)) in enumerate(zip(got, ref)):
            assert np.array_equal(c, c_ref), k
            assert (st.n_txn, st.n_acc, st.committed) == (host.n_txn, host.n_acc, st_ref.committed), k
            assert (st.read_digest, st.write_cnt) == (st_ref.read_digest, st_ref.write_cnt), k
        assert int(cursor.item()) == cur_ref
        total = n_epochs * calls
        for ln in range(lanes):  # each lane's next epoch, in its first buffer
            k = total + ((ln - total) % lanes)
            e = bufs[ln].epoch((total // lanes) & 1 if total % lanes == 0 else 0, n_txn, pool.max_txn_acc())
            assert e.n_acc == nxt[k].n_acc, ln
            assert np.array_equal(e.keys.cpu().numpy().view(np.uint64), nxt[k].keys), ln
        assert np.array_equal(eng.read_table(0, rows), f0)
    finally:
        eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("cc,lanes,prefix", [(dvcc.NO_WAIT, 2, 400), (dvcc.WAIT_DIE, 4, 400), (dvcc.OCC, 2, 400),
                                             (dvcc.NO_WAIT, 3, None)])
def test_device_closed_loop_lanes(cc, lanes, prefix):
    """dv_epoch_run_closed_loop_lanes against the oracle's interleaved loops:
    every epoch's commit bytes and stats, the shared cursor, each lane's next
    epoch and the table"""
    rows, N = 1 << 13, 2000
    pool = _pool(rows, 5000, 21)
    _check_loop_lanes(cc, rows, pool, N, 4 * lanes, lanes, prefix)


@pytest.mark.gpu
def test_device_closed_loop_lanes_halts_and_resume():
    """forced yields (halted epochs and every epoch queued behind them run
    again in order) and a loop continued over two calls"""
    rows, N = 1 << 13, 3000
    pool = _pool(rows, 4000, 22, R=12)
    _check_loop_lanes(dvcc.NO_WAIT, rows, pool, N, 4, 2, 500, calls=2, async_iters=1)


@pytest.mark.gpu
@pytest.mark.slow
def test_device_closed_loop_lanes_config_d_full():
    """The bench's closed_loop_retry.lanes leg at its own size: config D
    (16,777,216 rows, 1,048,576-txn epochs, zipf 0.9, automatic prefix), four
    lanes, 8 epochs of the interleaved loops over a 2M-txn pool (the bench's
    pool seed) -- every epoch, the cursor, each lane's next epoch and the
    table against the oracle's loops"""
    rows, N = 16_777_216, 1_048_576
    gen = YCSBQueryGenerator(rows, zipf_theta=0.9, txn_write_perc=1.0, tup_write_perc=0.5)
    pool = gen.gen(2 * N, dvcc.epoch_seed(0, 999))
    _check_loop_lanes(dvcc.NO_WAIT, rows, pool, N, 8, 4, 0)
