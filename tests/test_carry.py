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
    lens = tb[ab + 1] - tb[ab]
    idx = np.concatenate([np.arange(tb[t], tb[t + 1]) for t in ab]) if len(ab) else np.zeros(0, np.int64)
    ntb = np.zeros(len(ab) + 1, np.uint32)
    ntb[1:] = np.cumsum(lens)
    return Epoch(ep.keys[idx].copy(), ep.types[idx].copy(), ntb)


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
