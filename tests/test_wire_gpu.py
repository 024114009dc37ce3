"""The wire ingress on the GPU: client batches (tests/wire_fmt.py, from
copy_to_buf's field order) decoded by dv_wire_decode into host epochs, run
through the engine's C ABI and checked against the oracle on the same epochs
-- commit bytes, read digests, table state -- and the replies (CL_RSP /
CALVIN_ACK) name exactly the committed txns.  Parity unpinned for the byte
layout; the decisions are the oracle's."""
import numpy as np
import pytest

import _oracle as O
import wire_fmt as W

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import dvcc  # noqa: E402
from dvcc import _lib as L  # noqa: E402
from dvcc import tpcc as T  # noqa: E402
from dvcc.wire import WireIngress, tpcc_gen_queries  # noqa: E402

ORACLE_CC = {dvcc.NO_WAIT: O.NO_WAIT, dvcc.WAIT_DIE: O.WAIT_DIE, dvcc.OCC: O.OCC, dvcc.CALVIN: O.CALVIN}


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a visible MI355X")
    yield


@pytest.mark.parametrize("cc", [dvcc.NO_WAIT, dvcc.WAIT_DIE, dvcc.OCC])
def test_ycsb_client_batches_through_the_engine(cc):
    rows = 1 << 16
    g = dvcc.YCSBQueryGenerator(rows, zipf_theta=0.9)
    tab = O.YcsbTable(rows)
    f0 = tab.f0.copy()
    eng = dvcc.CCEngine(cc, 4000, 40_000)
    eng.load_ycsb_partition(rows)
    w = WireIngress(L.YCSB, 4000, 40_000, node_id=0, node_cnt=1, synth_table_size=rows)
    # three clients' streams, their batches interleaved as they arrive
    epochs = [g.gen(1500, 50 + c) for c in range(3)]
    streams = [W.batches(0, 1 + c, W.ycsb_epoch_messages(e, client_startts=100_000 * c + np.arange(1500)))
               for c, e in enumerate(epochs)]
    closed = []
    for i in range(max(len(s) for s in streams)):
        for s in streams:
            if i < len(s):
                closed += w.feed(s[i])
    closed.append(w.take())
    assert sum(ep.n_txn for ep in closed) == 4500 and len(closed) == 2
    for ep in closed:
        c_ref, _, st_ref = O.epoch_run(ORACLE_CC[cc], tab.ix, f0, ep.n_txn, ep.txn_begin, ep.keys, ep.types)
        d_commit = torch.zeros(ep.n_txn, dtype=torch.uint8, device="cuda")
        st = eng.run_epoch_device(dvcc.DeviceEpoch(ep), d_commit)
        c = d_commit.cpu().numpy()
        assert (c == c_ref).all()
        assert (st.committed, st.read_digest, st.write_cnt) == (st_ref.committed, st_ref.read_digest, st_ref.write_cnt)
        replies = [m for b in w.respond(ep, c) for m in W.parse_batch(b)[2]]
        assert sorted(m["txn_id"] for m in replies) == sorted(int(x) for x in ep.txn_id[c == 1])
    assert (eng.read_table(0, rows) == f0).all()
    eng.close()


def test_calvin_sequencer_streams_through_the_engine():
    """Two sequencers' batches for one Calvin epoch, each decoded into its own
    epoch and concatenated origin-major (dvcc.sequence): grant groups and
    table equal the oracle's; every txn acknowledged to its sequencer."""
    rows = 1 << 16
    g = dvcc.YCSBQueryGenerator(rows, zipf_theta=0.6, txn_write_perc=1.0, tup_write_perc=0.5)
    tab = O.YcsbTable(rows)
    f0 = tab.f0.copy()
    parts = []
    for node in range(2):
        e = g.gen(2000, 70 + node)
        ids = node + 2 * np.arange(2000)
        w = WireIngress(L.YCSB, 2000, 20_000, node_id=0, node_cnt=2, synth_table_size=rows, calvin=True)
        for b in W.batches(0, 10 + node, W.ycsb_epoch_messages(e, batch_id=4, txn_ids=ids) + [W.rdone(4)]):
            assert w.feed(b) == []
        d = w.take()
        assert d.rdone == 1 and d.batch_id == 4 and (d.keys == e.keys).all()
        acks = [m for b in w.respond(d) for m in W.parse_batch(b, calvin=True)[2]]
        assert [m["txn_id"] for m in acks] == ids.tolist()
        parts.append(d)
    ep = dvcc.sequence(parts)
    c_ref, g_ref, st_ref = O.epoch_run(O.CALVIN, tab.ix, f0, ep.n_txn, ep.txn_begin, ep.keys, ep.types,
                                       want_grant=True)
    eng = dvcc.CCEngine(dvcc.CALVIN, ep.n_txn, ep.n_acc)
    eng.load_ycsb_partition(rows)
    d_commit = torch.zeros(ep.n_txn, dtype=torch.uint8, device="cuda")
    d_grant = torch.zeros(ep.n_acc, dtype=torch.int32, device="cuda")
    st = eng.run_epoch_device(dvcc.DeviceEpoch(ep), d_commit, d_grant)
    assert (d_commit.cpu().numpy() == c_ref).all()
    assert (d_grant.cpu().numpy().view(np.uint32) == g_ref).all()
    assert st.read_digest == st_ref.read_digest
    assert (eng.read_table(0, rows) == f0).all()
    eng.close()


@pytest.mark.parametrize("cc", [dvcc.WAIT_DIE, dvcc.CALVIN])
def test_tpcc_client_batches_through_the_engine(cc):
    po = O.tpcc_params(num_wh=4, cust_per_dist=1000, max_items=2000)
    pp = T.tpcc_params(num_wh=4, cust_per_dist=1000, max_items=2000)
    db = O.TpccDB(po, 5)
    eng = T.TpccEngine(cc, pp, 3000, seed=5)
    try:
        qs = tpcc_gen_queries(pp, 3000, 17)
        msgs = []
        for i, x in enumerate(qs):
            msgs.append(W.tpcc_query(dict(
                txn_type=x.txn_type, w_id=x.w_id, d_id=x.d_id, c_id=x.c_id, d_w_id=x.d_w_id, c_w_id=x.c_w_id,
                c_d_id=x.c_d_id, c_last=bytes(x.c_last), h_amount=x.h_amount, by_last_name=x.by_last_name,
                ol_cnt=x.ol_cnt, o_entry_d=x.o_entry_d, parts=[x.parts[k] for k in range(x.n_parts)],
                items=[(x.items[k].ol_i_id, x.items[k].ol_supply_w_id, x.items[k].ol_quantity)
                       for k in range(x.ol_cnt)]), client_startts=i))
        w = WireIngress(L.TPCC, 3000, 3000 * 33, tpcc=pp)
        for b in W.batches(0, 1, msgs):
            w.feed(b)
        e = w.take()
        ref = T.gen(pp, 3000, 17)
        assert (e.keys == ref.keys).all() and (e.args == ref.args).all()
        c_ref, o_ref, st_ref = db.epoch(ORACLE_CC[cc], e.keys, e.types, e.tables, e.args, e.txn_begin)
        dep, d_args = T.device_epoch(e)
        d_commit = torch.zeros(3000, dtype=torch.uint8, device="cuda")
        d_oid = torch.zeros(3000, dtype=torch.int64, device="cuda")
        st = eng.run_tpcc_epoch_device(dep, d_args, d_commit, d_oid)
        c = d_commit.cpu().numpy()
        assert (c == c_ref).all()
        assert (d_oid.cpu().numpy().view(np.uint64) == o_ref).all()
        assert st.committed == st_ref.committed
        replies = [m for b in w.respond(e, c) for m in W.parse_batch(b)[2]]
        assert sorted(m["client_startts"] for m in replies) == np.flatnonzero(c).tolist()
    finally:
        eng.close()
