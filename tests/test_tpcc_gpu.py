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


def _run(eng, e):
    dep, d_args = T.device_epoch(e)
    d_commit = torch.zeros(max(1, e.n_txn), dtype=torch.uint8, device="cuda")
    d_oid = torch.zeros(max(1, e.n_txn), dtype=torch.int64, device="cuda")
    st = eng.run_tpcc_epoch_device(dep, d_args, d_commit, d_oid)
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
