"""Deneva wire-format ingress and replies (dv_wire_*, SURVEY.md 8(f) transport
row) on the CPU: batches built byte by byte from copy_to_buf's field order
(transport/message.cpp) -- one spelled out in hex below, the rest by
tests/wire_fmt.py -- decode into the same epochs as the engine's own
generators (dv_ycsb_gen, dv_tpcc_gen); malformed batches are refused; the
replies parse back.  Parity unpinned: the reference's transport cannot run
here, so the layout is pinned by the source text alone."""
import struct

import numpy as np
import pytest

import wire_fmt as W

dvcc = pytest.importorskip("dvcc")
from dvcc import _lib as L  # noqa: E402
from dvcc import tpcc as T  # noqa: E402
from dvcc.wire import WireIngress, tpcc_gen_queries  # noqa: E402

U64 = (1 << 64) - 1


def _hex(s):
    return bytes.fromhex("".join(s.split()))


# One YCSB batch from client node 3 to server node 0, two CL_QRY messages,
# written out field by field (x86-64 little endian):
HAND_BATCH = _hex("""
00000000 03000000 02000000
03000000 ffffffffffffffff 0000000000000000
0000000000000000 0000000000000000 0000000000000000 0000000000000000
0000000000000000 0000000000000000 0000000000000000
0700000000000000 0100000000000000 0000000000000000
0200000000000000
01000000 abababab 2a00000000000000 11 cdcdcdcdcdcdcd
00000000 abababab 0500000000000000 22 cdcdcdcdcdcdcd
03000000 ffffffffffffffff 0000000000000000
0000000000000000 0000000000000000 0000000000000000 0000000000000000
0000000000000000 0000000000000000 0000000000000000
0900000000000000 0100000000000000 0000000000000000
0100000000000000
00000000 abababab 6300000000000000 33 cdcdcdcdcdcdcd
""")
# batch header: dest 0, src 3, count 2
# message 1: rtype CL_QRY (3), txn_id UINT64_MAX, mq_time 0, 7 latency doubles 0,
#   client_startts 7, 1 partition: 0, 2 requests: (WR, key 42, value 0x11), (RD, key 5)
#   (the 4 bytes after acctype and the 7 after value are the struct's padding:
#   COPY_BUF copies them as they lie in memory, so anything may be there)
# message 2: client_startts 9, 1 partition: 0, 1 request: (RD, key 99)


def _ycsb_ingress(max_txn=1024, max_acc=1 << 14, **kw):
    kw.setdefault("synth_table_size", 1 << 20)
    return WireIngress(L.YCSB, max_txn, max_acc, **kw)


def test_hand_built_batch():
    assert len(HAND_BATCH) == 12 + 2 * (76 + 24) + 2 * 8 + 3 * 24
    w = _ycsb_ingress(node_id=0, node_cnt=2)
    assert w.feed(HAND_BATCH) == []
    ep = w.take()
    assert ep.keys.tolist() == [42, 5, 99]
    assert ep.types.tolist() == [1, 0, 0]
    assert ep.txn_begin.tolist() == [0, 2, 3]
    assert ep.client_startts.tolist() == [7, 9]
    assert ep.return_node.tolist() == [3, 3]
    assert ep.txn_id.tolist() == [0, 2]  # node 0 + 2 nodes * k (get_next_txn_id, one worker)
    assert w.feed(HAND_BATCH) == [] and w.take().txn_id.tolist() == [4, 6]  # (the counter goes on)


def test_wire_fmt_reproduces_hand_batch():
    """The test encoder writes the same bytes (padding aside)."""
    msgs = [W.ycsb_query([(1, 42), (0, 5)], [0], 7), W.ycsb_query([(0, 99)], [0], 9)]
    b = W.batches(0, 3, msgs)
    assert len(b) == 1 and len(b[0]) == len(HAND_BATCH)
    pad = np.zeros(len(HAND_BATCH), bool)  # (the padding bytes differ)
    for off in (12 + 100 + 8, 12 + 100 + 8 + 24, 12 + 2 * 100 + 48 + 16):
        pad[off + 4:off + 8] = True
        pad[off + 16:off + 24] = True
    got, want = np.frombuffer(b[0], np.uint8), np.frombuffer(HAND_BATCH, np.uint8)
    assert (got[~pad] == want[~pad]).all()


@pytest.mark.parametrize("P,theta", [(1, 0.9), (4, 0.6)])
def test_ycsb_batches_decode_to_the_generators_epoch(P, theta):
    g = dvcc.YCSBQueryGenerator(P * (1 << 16), part_cnt=P, zipf_theta=theta)
    e = g.gen(3000, 77)
    batches = W.batches(1, 5, W.ycsb_epoch_messages(e, part_cnt=P))
    assert all(len(b) <= W.MSG_MAX for b in batches) and len(batches) > 100
    w = _ycsb_ingress(4096, 40_000, node_id=1, node_cnt=3, part_cnt=P, synth_table_size=P * (1 << 16))
    for b in batches:
        assert w.feed(b) == []
    d = w.take()
    assert (d.keys == e.keys).all() and (d.types == e.types).all() and (d.txn_begin == e.txn_begin).all()
    assert (d.owner == (e.keys % P)).all()
    assert (d.client_startts == np.arange(3000)).all()
    assert (d.txn_id == 1 + 3 * np.arange(3000, dtype=np.uint64)).all()


def test_decode_batches_in_one_call():
    """dv_wire_decode_batches over a receive queue equals batch-by-batch
    decoding, the epoch splits included; a refused batch stops it there."""
    g = dvcc.YCSBQueryGenerator(1 << 16, zipf_theta=0.9)
    e = g.gen(2000, 8)
    bs = W.batches(0, 1, W.ycsb_epoch_messages(e))
    w1, w2 = _ycsb_ingress(max_txn=300), _ycsb_ingress(max_txn=300)
    a = [x for b in bs for x in w1.feed(b)] + [w1.take()]
    c = w2.feed_many(bs) + [w2.take()]
    assert [x.n_txn for x in a] == [x.n_txn for x in c]
    assert all((x.keys == y.keys).all() and (x.txn_id == y.txn_id).all() for x, y in zip(a, c))
    assert (np.concatenate([x.keys for x in c]) == e.keys).all()
    w3 = _ycsb_ingress()
    _expect_refused(w3, bs[0][:4] + struct.pack("<I", 0) + bs[0][8:])  # (from itself)
    with pytest.raises(L.DvccError):
        w3.feed_many(bs[:3] + [bs[3][:-1]] + bs[4:])
    assert w3.take().n_txn == sum(struct.unpack_from("<I", b, 8)[0] for b in bs[:3])


def test_numpy_batches_equal_the_message_path():
    g = dvcc.YCSBQueryGenerator(1 << 16, zipf_theta=0.9)
    e = g.gen(500, 3)
    a = W.batches(0, 2, W.ycsb_epoch_messages(e))
    b = W.ycsb_epoch_batches_np(e, 0, 2)
    assert len(a) == len(b)
    for x, y in zip(a, b):  # (equal up to the padding and value bytes)
        w = _ycsb_ingress(node_id=0)
        w.feed(x)
        dx = w.take()
        w.feed(y)
        dy = w.take()
        assert (dx.keys == dy.keys).all() and (dx.types == dy.types).all() and (dx.txn_begin == dy.txn_begin).all()
        assert len(x) == len(y)


def test_capacity_splits_epochs():
    """An epoch that cannot take the next message is closed (DV_WIRE_MORE)
    and decoding goes on into the next: the concatenation is the stream."""
    g = dvcc.YCSBQueryGenerator(1 << 16, zipf_theta=0.9)
    e = g.gen(1000, 5)
    w = _ycsb_ingress(max_txn=97, max_acc=10_000)
    closed = []
    for b in W.batches(0, 1, W.ycsb_epoch_messages(e)):
        closed += w.feed(b)
    closed.append(w.take())
    assert [c.n_txn for c in closed[:-1]] == [97] * (1000 // 97)
    assert sum(c.n_txn for c in closed) == 1000
    assert (np.concatenate([c.keys for c in closed]) == e.keys).all()
    w2 = _ycsb_ingress(max_txn=1000, max_acc=95)  # the access bound closes them too
    cl = []
    for b in W.batches(0, 1, W.ycsb_epoch_messages(e)):
        cl += w2.feed(b)
    cl.append(w2.take())
    assert all(c.n_acc <= 95 for c in cl) and sum(c.n_txn for c in cl) == 1000


def _expect_refused(w, batch):
    with pytest.raises(L.DvccError) as ex:
        w.feed(batch)
    assert ex.value.code == L.DV_ERR_ARG


def test_malformed_batches_are_refused():
    ok = W.ycsb_query([(1, 4), (0, 8)], [0], 1)
    w = _ycsb_ingress(node_id=0, synth_table_size=1000, max_req=16)
    bad = {
        "wrong dest": struct.pack("<III", 1, 2, 1) + ok,
        "from itself": struct.pack("<III", 0, 0, 1) + ok,
        "empty": struct.pack("<III", 0, 2, 0),
        "truncated": struct.pack("<III", 0, 2, 1) + ok[:-5],
        "trailing bytes": struct.pack("<III", 0, 2, 1) + ok + b"\0",
        "count past the bytes": struct.pack("<III", 0, 2, 2) + ok,
        "unknown rtype": struct.pack("<III", 0, 2, 1) + struct.pack("<I", 7) + ok[4:],
        "RDONE without CALVIN": struct.pack("<III", 0, 2, 1) + W.rdone(0)[:76],
        "key past synth_table_size": W.batches(0, 2, [W.ycsb_query([(0, 1000)], [0])])[0],
        "SCAN access": W.batches(0, 2, [W.ycsb_query([(3, 5)], [0])])[0],
        "partition past part_cnt": W.batches(0, 2, [W.ycsb_query([(0, 5)], [1])])[0],
        "longer than max_req": W.batches(0, 2, [W.ycsb_query([(0, k) for k in range(17)], [0])])[0],
        "too long for one mbuf": struct.pack("<III", 0, 2, 1) + ok + b"\0" * 4096,
    }
    for name, b in bad.items():
        _expect_refused(w, b)
        assert w.take().n_txn == 0, name
    # a batch is checked whole before any of it is decoded
    _expect_refused(w, W.batches(0, 2, [ok, ok, W.ycsb_query([(0, 5000)], [0])])[0])
    assert w.take().n_txn == 0
    w.feed(W.batches(0, 2, [ok, ok])[0])
    ep = w.take()
    assert ep.n_txn == 2 and ep.keys.tolist() == [4, 8, 4, 8]


def _tpcc_wire_queries(q):
    out = []
    for x in q:
        d = dict(txn_type=x.txn_type, w_id=x.w_id, d_id=x.d_id, c_id=x.c_id, d_w_id=x.d_w_id, c_w_id=x.c_w_id,
                 c_d_id=x.c_d_id, c_last=bytes(x.c_last), h_amount=x.h_amount, by_last_name=x.by_last_name,
                 rbk=x.rbk, remote=x.remote, ol_cnt=x.ol_cnt, o_entry_d=x.o_entry_d,
                 parts=[x.parts[i] for i in range(x.n_parts)],
                 items=[(x.items[i].ol_i_id, x.items[i].ol_supply_w_id, x.items[i].ol_quantity)
                        for i in range(x.ol_cnt)])
        out.append(d)
    return out


@pytest.mark.parametrize("P,perc", [(1, 0.5), (4, 0.5), (2, 0.0), (2, 1.0)])
def test_tpcc_batches_decode_to_the_generators_epoch(P, perc):
    p = T.tpcc_params(num_wh=8, cust_per_dist=1000, max_items=2000, part_cnt=P, perc_payment=perc, mpr=0.5)
    n = 2000
    e = T.gen(p, n, 41, home_part=P - 1)
    qs = _tpcc_wire_queries(tpcc_gen_queries(p, n, 41, home_part=P - 1))
    assert [q["txn_type"] for q in qs] == e.txn_type.tolist()
    if 0 < perc < 1:
        assert any(q["by_last_name"] for q in qs) and any(len(q["parts"]) > 1 for q in qs) == (P > 1)
    msgs = [W.tpcc_query(q, client_startts=1000 + i) for i, q in enumerate(qs)]
    w = WireIngress(L.TPCC, n, n * 33, node_id=0, node_cnt=P, part_cnt=P, tpcc=p)
    for b in W.batches(0, P + 2, msgs):
        assert w.feed(b) == []
    d = w.take()
    for f in ("keys", "types", "tables", "args", "txn_begin", "txn_type", "owner"):
        assert (getattr(d, f) == getattr(e, f)).all(), f
    assert (d.client_startts == 1000 + np.arange(n)).all()


def test_tpcc_bad_fields_are_refused():
    p = T.tpcc_params(num_wh=4, cust_per_dist=1000, max_items=2000)
    q = _tpcc_wire_queries(tpcc_gen_queries(p, 50, 3))
    no = next(x for x in q if x["txn_type"] == 2)
    pay = next(x for x in q if x["txn_type"] == 1)
    w = WireIngress(L.TPCC, 64, 64 * 33, tpcc=p)
    bad = [dict(no, ol_cnt=no["ol_cnt"] + 1), dict(no, w_id=5), dict(no, items=[(2001, 1, 1)] * no["ol_cnt"]),
           dict(pay, c_w_id=0), dict(pay, d_id=11), dict(pay, by_last_name=False, c_id=1001),
           dict(pay, by_last_name=True, c_last=b"X" * 16), dict(no, txn_type=3)]
    for b in bad:
        _expect_refused(w, W.batches(0, 1, [W.tpcc_query(b)])[0])
        assert w.take().n_txn == 0, b
    w.feed(W.batches(0, 1, [W.tpcc_query(no), W.tpcc_query(pay)])[0])
    assert w.take().n_txn == 2


def test_calvin_sequencer_batches():
    """CALVIN: the sequencer forwards CL_QRY with its txn ids and batch id and
    ends each batch with RDONE (sequencer.cpp:207-326); a message of a later
    batch closes the epoch, an earlier one is refused."""
    g = dvcc.YCSBQueryGenerator(1 << 16, zipf_theta=0.6)
    e0, e1 = g.gen(40, 1), g.gen(30, 2)
    m0 = W.ycsb_epoch_messages(e0, batch_id=5, txn_ids=2 + 4 * np.arange(40))
    m1 = W.ycsb_epoch_messages(e1, batch_id=6, txn_ids=2 + 4 * np.arange(30))
    stream = m0 + [W.rdone(5)] + m1 + [W.rdone(6)]
    w = _ycsb_ingress(node_id=1, node_cnt=4, calvin=True)
    closed = []
    for b in W.batches(1, 2, stream):
        closed += w.feed(b)
    closed.append(w.take())
    assert len(closed) == 2
    a, b = closed
    assert (a.batch_id, a.rdone, a.n_txn) == (5, 1, 40) and (b.batch_id, b.rdone, b.n_txn) == (6, 1, 30)
    assert (a.keys == e0.keys).all() and (b.keys == e1.keys).all()
    assert (a.txn_id == 2 + 4 * np.arange(40)).all() and (a.return_node == 2).all()
    # an empty batch's RDONE alone still names it
    w.feed(W.batches(1, 2, [W.rdone(7)])[0])
    c = w.take()
    assert (c.batch_id, c.rdone, c.n_txn) == (7, 1, 0)
    # stale batch id
    w.feed(W.batches(1, 2, [W.rdone(9)])[0])
    _expect_refused(w, W.batches(1, 2, W.ycsb_epoch_messages(e1, batch_id=8))[0])
    # no batch id at all (UINT64_MAX)
    w.take()
    _expect_refused(w, W.batches(1, 2, [W.ycsb_query([(0, 1)], [0], batch_id=U64)])[0])


def test_client_responses():
    g = dvcc.YCSBQueryGenerator(1 << 16, zipf_theta=0.9)
    e = g.gen(2000, 9)
    msgs = W.ycsb_epoch_messages(e, client_startts=10_000 + np.arange(2000))
    w = _ycsb_ingress(4096, 40_000, node_id=2, node_cnt=3)
    for i, b in enumerate(W.batches(2, 0, msgs[:700]) + W.batches(2, 4, msgs[700:1500]) + W.batches(2, 3, msgs[1500:])):
        w.feed(b)
    ep = w.take()
    commit = (np.random.default_rng(1).random(2000) < 0.3).astype(np.uint8)
    out = w.respond(ep, commit)
    got = {}
    for b in out:
        assert len(b) <= W.MSG_MAX
        dest, src, ms = W.parse_batch(b)
        assert src == 2
        for m in ms:
            assert m["rtype"] == W.CL_RSP and m["mq_time"] == 0 and m["lat"] == (0.0,) * 7
            got[m["txn_id"]] = (dest, m["client_startts"])
    want = {int(ep.txn_id[t]): (int(ep.return_node[t]), 10_000 + t) for t in range(2000) if commit[t]}
    assert got == want
    dests = [W.parse_batch(b)[0] for b in out]
    assert dests == sorted(dests)  # destinations ascending, each destination's replies in txn order


def test_calvin_acks():
    g = dvcc.YCSBQueryGenerator(1 << 16, zipf_theta=0.6)
    e = g.gen(300, 1)
    w = _ycsb_ingress(node_id=1, node_cnt=4, calvin=True)
    for b in W.batches(1, 0, W.ycsb_epoch_messages(e, batch_id=3, txn_ids=4 * np.arange(300)) + [W.rdone(3)]):
        w.feed(b)
    ep = w.take()
    out = w.respond(ep)
    ms = [m for b in out for m in W.parse_batch(b, calvin=True)[2]]
    assert [m["txn_id"] for m in ms] == (4 * np.arange(300)).tolist()
    assert all(m["rtype"] == W.CALVIN_ACK and m["batch_id"] == 3 and m["rc"] == 0 for m in ms)
    assert all(W.parse_batch(b, calvin=True)[0] == 0 for b in out)
