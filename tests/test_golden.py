"""Golden epochs (tests/golden/*.npz, made by tests/golden/make_golden.py).

CPU: the oracle and the product generator reproduce the committed fixtures.
GPU: the HIP engine reproduces the fixture decisions and state bit-exactly.
"""
import os

import numpy as np
import pytest

import _oracle as O
import dvcc

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NAMES = sorted(f[:-4] for f in os.listdir(GOLDEN) if f.endswith(".npz"))
TO_DV = {O.NO_WAIT: dvcc.NO_WAIT, O.WAIT_DIE: dvcc.WAIT_DIE, O.OCC: dvcc.OCC, O.CALVIN: dvcc.CALVIN}


def _load(name):
    with np.load(os.path.join(GOLDEN, name + ".npz")) as z:
        return {k: z[k] for k in z.files}


def test_fixture_set_complete():
    from golden.make_golden import CASES
    assert sorted(CASES) == NAMES


@pytest.mark.parametrize("name", NAMES)
def test_oracle_reproduces_golden(name):
    from golden.make_golden import make
    g, m = _load(name), make(name)
    assert sorted(g) == sorted(m)
    for k in g:
        assert np.array_equal(g[k], m[k]), k


@pytest.mark.parametrize("name", NAMES)
def test_product_generator_matches_golden_inputs(name):
    from golden.make_golden import CASES
    cc, rows, n_txn, theta, twp, tup, req, seed = CASES[name]
    gen = dvcc.YCSBQueryGenerator(rows, zipf_theta=theta, req_per_query=req, txn_write_perc=twp,
                                  tup_write_perc=tup)
    e = gen.gen(n_txn, seed)
    g = _load(name)
    assert np.array_equal(e.keys, g["keys"])
    assert np.array_equal(e.types, g["types"])
    assert np.array_equal(e.txn_begin, g["txn_begin"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_engine_matches_golden(name):
    g = _load(name)
    cc = TO_DV[int(g["cc"])]
    rows = int(g["rows"])
    e = dvcc.Epoch(g["keys"], g["types"], g["txn_begin"])
    eng = dvcc.CCEngine(cc, e.n_txn, e.n_acc)
    try:
        eng.load_ycsb_partition(rows)
        commit, grant, st = eng.run_epoch(e, want_grant=(cc == dvcc.CALVIN))
        assert np.array_equal(commit, g["commit"])
        if cc == dvcc.CALVIN:
            assert np.array_equal(grant, g["grant"])
        committed, aborted, digest, wcnt = (int(x) for x in g["stats"])
        assert (st.committed, st.aborted, st.read_digest, st.write_cnt) == (committed, aborted,
                                                                               digest, wcnt)
        assert np.array_equal(eng.read_table(0, rows), g["f0"])
    finally:
        eng.close()
