"""The engine's own partitioned protocols (dvcc_comm.hip) across real
process boundaries: world-size-2 groups of PROCESSES sharing the one GPU,
joined by dv_comm_init_ipc (device IPC handles + a shared-memory barrier;
RCCL refuses two ranks per GPU).  Every rank process runs the C++ drivers
exactly as bench.py's ranks do over RCCL -- epoch groups (compact and wide
batches, batched groups), dv_epoch_run_part's list and replicated protocols,
TPC-C's dv_tpcc_epoch_run_part -- and the parent checks every rank's commit
bytes, digests and rows against the oracle running the sequenced epochs
(txn.cpp:544-554 vote combine, transport.cpp:224-304 fragments)."""
import multiprocessing as mp
import os
import uuid

import numpy as np
import pytest

import _oracle as O
import dvcc

pytestmark = pytest.mark.gpu

ORACLE_CC = {dvcc.NO_WAIT: O.NO_WAIT, dvcc.WAIT_DIE: O.WAIT_DIE, dvcc.OCC: O.OCC, dvcc.CALVIN: O.CALVIN}
WORLD = 2


def _ycsb_gen(world, rows_pp, mpr):
    return dvcc.YCSBQueryGenerator(rows_pp * world, part_cnt=world, zipf_theta=0.9, txn_write_perc=1.0,
                                   tup_write_perc=0.5, part_per_txn=2, strict_ppt=1, mpr=mpr)


def _group_batches(sc, world, rank):
    """[group][epoch] batches of `rank` (seeded SEED + 97 * rank + epoch)."""
    gen = _ycsb_gen(world, sc["rows_pp"], sc["mpr"])
    out = []
    for g in range(sc["groups"]):
        grp = []
        for e in range(world):
            b = gen.gen(sc["n_txn"], dvcc.epoch_seed(rank, sc["seed"] + g * world + e), rank)
            if sc.get("bad_key") == (rank, g, e):
                b.keys[5] = np.uint64(sc["rows_pp"] * world + 7)
            grp.append(b)
        out.append(grp)
    return out


def _part_batches(sc, world, rank):
    gen = _ycsb_gen(world, sc["rows_pp"], sc["mpr"])
    return [gen.gen(sc["n_txn"], dvcc.epoch_seed(rank, sc["seed"] + k), rank) for k in range(sc["epochs"])]


def _run_scenario(sc, world, rank, name):
    import torch
    from dvcc import tpcc as T
    kind = sc["kind"]
    if kind == "tpcc":
        kw = sc["kw"]
        pp = T.tpcc_params(part_cnt=world, **kw)
        b = T.gen(pp, sc["n_txn"], sc["seed"] + rank, home_part=rank)
        eng = T.TpccEngine(sc["cc"], pp, sc["n_txn"] * world, part_id=rank, seed=5, asynchronous=False)
        try:
            eng.comm_init_ipc(name, world, rank)
            dep, d_args = T.device_epoch(b)
            own = torch.from_numpy(b.owner).cuda()
            d_commit = torch.zeros(sc["n_txn"] * world, dtype=torch.uint8, device="cuda")
            d_oid = torch.zeros(sc["n_txn"] * world, dtype=torch.int64, device="cuda")
            st = eng.run_tpcc_epoch_part(dep, d_args, own, sc["n_txn"], d_commit, d_oid)
            cols = {t: [eng.read_col(t, c) for c in range(3)] for t in range(5)}
            return {"commit": d_commit.cpu().numpy(), "oid": d_oid.cpu().numpy().view(np.uint64),
                    "committed": st.committed, "cols": cols}
        finally:
            eng.close()
    rows_pp, n_txn, cc = sc["rows_pp"], sc["n_txn"], sc["cc"]
    mode = sc.get("mode", 2)
    cap = n_txn * world * 10 + 4096 if mode == 2 else max(64, int(n_txn * world * 10 * 1.2 / world) + 4096)
    eng = dvcc.CCEngine(cc, n_txn * world, cap, part_cnt=world, part_id=rank, asynchronous=sc.get("asyn", False))
    try:
        eng.load_ycsb_partition(rows_pp)
        # ordered lanes (bench.py --group-lanes): the lanes opened over this
        # partition's tables before any communicator, one communicator each
        lanes = [eng.open_lane() for _ in range(sc.get("lanes", 1) - 1)]
        for ln, ctx in enumerate([eng] + lanes):
            ctx.comm_init_ipc(name if ln == 0 else f"{name}_l{ln}", world, rank)
            ctx.comm_set_mode(mode | (dvcc._lib.DV_COMM_WIDE_BATCHES if sc.get("wide") else 0) |
                              (dvcc._lib.DV_COMM_POSITION_ORDER if sc.get("position") else 0))
        if lanes:
            eng.lanes_order(lanes)
        out = {}
        try:
            if kind == "group" and lanes:
                groups = [[dvcc.DeviceEpoch(b) for b in grp] for grp in _group_batches(sc, world, rank)]
                ds = [torch.zeros(n_txn * world, dtype=torch.uint8, device="cuda") for _ in groups]
                half = len(groups) // 2  # (two calls: the order continues across them)
                sts = eng.run_epoch_groups_ordered(groups[:half], n_txn, ds[:half])
                sts += eng.run_epoch_groups_ordered(groups[half:], n_txn, ds[half:])
                torch.cuda.synchronize()
                out["commit"] = [d.cpu().numpy() for d in ds]
                out["stats"] = [(s.committed, s.read_digest, s.write_cnt) for s in sts]
            elif kind == "group":
                groups = [[dvcc.DeviceEpoch(b) for b in grp] for grp in _group_batches(sc, world, rank)]
                ds = [torch.zeros(n_txn * world, dtype=torch.uint8, device="cuda") for _ in groups]
                sts = eng.run_epoch_groups(groups, n_txn, ds)
                out["commit"] = [d.cpu().numpy() for d in ds]
                out["stats"] = [(s.committed, s.read_digest, s.write_cnt) for s in sts]
            else:  # "part": one epoch per call
                out["commit"], out["stats"] = [], []
                for b in _part_batches(sc, world, rank):
                    d = torch.zeros(n_txn * world, dtype=torch.uint8, device="cuda")
                    st = eng.run_epoch_part(dvcc.DeviceEpoch(b), n_txn, d)
                    out["commit"].append(d.cpu().numpy())
                    out["stats"].append((st.committed, st.read_digest, st.write_cnt))
        except dvcc.DvccError as ex:
            out["error"] = ex.code
        out["table"] = eng.read_table(0, rows_pp)
        return out
    finally:
        eng.close()


def _worker(rank, world, names, scenarios, q):
    try:
        import torch
        torch.cuda.set_device(0)
        res = [_run_scenario(sc, world, rank, nm) for sc, nm in zip(scenarios, names)]
        q.put((rank, res))
    except BaseException as ex:  # noqa: BLE001 -- reported to the parent
        q.put((rank, repr(ex)))


def _run_ranks(scenarios, world=WORLD):
    """Every scenario on `world` rank processes (spawned: each opens its own
    HIP context on GPU 0); per rank the list of scenario results."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    tag = uuid.uuid4().hex[:12]
    names = [f"/dvcc_t{os.getpid()}_{tag}_{i}" for i in range(len(scenarios))]
    env_keep = os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY")
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"  # (dmabuf IPC: the only mode this host driver supports)
    try:
        procs = [ctx.Process(target=_worker, args=(r, world, names, scenarios, q)) for r in range(world)]
        for p in procs:
            p.start()
        got = dict(q.get(timeout=600) for _ in range(world))
        for p in procs:
            p.join(timeout=120)
    finally:
        if env_keep is None:
            os.environ.pop("HSA_ENABLE_IPC_MODE_LEGACY", None)
        else:
            os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = env_keep
    for r in range(world):
        assert not isinstance(got[r], str), f"rank {r}: {got[r]}"
    return [got[r] for r in range(world)]


def _position(sc):
    return sc.get("position", False) and sc["cc"] != dvcc.CALVIN


def _mine(c, sc, r, world):
    """Rank r's txns' commit bytes in a sequenced epoch's bytes."""
    n = sc["n_txn"]
    return c.reshape(n, world)[:, r] if _position(sc) else c[r * n:(r + 1) * n]


def _oracle_groups(sc, world):
    """Commit bytes and stats of every epoch of every group, the oracle running
    the sequenced epochs one after the other (origin-major, or position-major
    with sc["position"]: DV_COMM_POSITION_ORDER), and the final rows."""
    tab = O.YcsbTable(sc["rows_pp"] * world)
    f0 = tab.f0.copy()
    per_rank = [_group_batches(sc, world, r) for r in range(world)]
    refs = []
    for g in range(sc["groups"]):
        grp = []
        for e in range(world):
            b = [per_rank[r][g][e] for r in range(world)]
            q = dvcc.sequence_position(b) if _position(sc) else dvcc.sequence(b)
            c, _, st = O.epoch_run(ORACLE_CC[sc["cc"]], tab.ix, f0, q.n_txn, q.txn_begin, q.keys, q.types)
            grp.append((c, st))
        refs.append(grp)
    return refs, f0


GROUP_CASES = [dict(cc=dvcc.NO_WAIT, wide=False), dict(cc=dvcc.NO_WAIT, wide=True),
               dict(cc=dvcc.OCC, wide=False), dict(cc=dvcc.CALVIN, wide=False),
               dict(cc=dvcc.NO_WAIT, wide=False, position=True), dict(cc=dvcc.OCC, wide=True, position=True)]


def test_ipc_epoch_groups_two_processes():
    """Epoch groups (dv_epoch_group_run_batch, two groups of two epochs) over
    two processes: compact and wide batches, NO_WAIT / OCC / CALVIN, origin-
    and position-major sequences."""
    base = dict(kind="group", rows_pp=1 << 13, n_txn=1500, mpr=0.3, groups=2, seed=40)
    scs = [dict(base, **c) for c in GROUP_CASES]
    res = _run_ranks(scs)
    for i, sc in enumerate(scs):
        refs, f0 = _oracle_groups(sc, WORLD)
        n = sc["n_txn"]
        for g in range(sc["groups"]):
            committed = sum(st.committed for _, st in refs[g])
            digest = writes = 0
            for r in range(WORLD):
                out = res[r][i]
                assert "error" not in out, (sc, r, out.get("error"))
                for e in range(WORLD):
                    assert (out["commit"][g][e * n:(e + 1) * n] == _mine(refs[g][e][0], sc, r, WORLD)).all(), \
                        (sc, g, e, r)
                c, d, w = out["stats"][g]
                assert c == committed, (sc, g, r)
                digest = (digest + d) % (1 << 64)
                writes += w
            assert digest == sum(st.read_digest for _, st in refs[g]) % (1 << 64), (sc, g)
            assert writes == sum(st.write_cnt for _, st in refs[g]), (sc, g)
        for r in range(WORLD):
            assert (res[r][i]["table"] == f0[r::WORLD]).all(), (sc, r)


def test_ipc_epoch_groups_ordered_lanes_two_processes():
    """bench.py's N > 1 headline path (--group-lanes): each rank process opens
    three decision lanes over its partition, one communicator per lane,
    dv_lanes_order; 7 groups of two epochs over two calls, group g decided on
    lane g % 4 of both ranks, executions in group order -- every epoch's
    commit bytes, the digests and the rows against the oracle running the
    sequenced epochs in order.  Asynchronous rounds on (the bench's), NO_WAIT
    position-major (the bench's default order) and OCC origin-major."""
    base = dict(kind="group", rows_pp=1 << 13, n_txn=1500, mpr=0.3, groups=7, seed=140, lanes=4, asyn=True)
    scs = [dict(base, cc=dvcc.NO_WAIT, position=True), dict(base, cc=dvcc.OCC, wide=True)]
    res = _run_ranks(scs)
    for i, sc in enumerate(scs):
        refs, f0 = _oracle_groups(sc, WORLD)
        n = sc["n_txn"]
        for g in range(sc["groups"]):
            committed = sum(st.committed for _, st in refs[g])
            for r in range(WORLD):
                out = res[r][i]
                assert "error" not in out, (sc, r, out.get("error"))
                for e in range(WORLD):
                    assert (out["commit"][g][e * n:(e + 1) * n] == _mine(refs[g][e][0], sc, r, WORLD)).all(), \
                        (sc, g, e, r)
                assert out["stats"][g][0] == committed, (sc, g, r)
        for r in range(WORLD):
            assert (res[r][i]["table"] == f0[r::WORLD]).all(), (sc, r)


@pytest.mark.parametrize("cc", [dvcc.NO_WAIT, dvcc.CALVIN])
def test_ipc_part_protocols_two_processes(cc):
    """dv_epoch_run_part over two processes: the list protocol (owner split,
    all-to-allv of records, per-round verdict all-reduce) and the replicated
    one (all-gathered epoch), each in origin and in position order
    (DV_COMM_POSITION_ORDER: the origins' batches merged txn by txn; CALVIN
    keeps its origin order), two epochs each, and a missing key on one rank
    failing a group on both ranks with no row changed."""
    base = dict(kind="part", rows_pp=1 << 13, n_txn=2000, mpr=0.3, epochs=2, seed=20, cc=cc)
    bad = dict(kind="group", rows_pp=1 << 12, n_txn=800, mpr=0.3, groups=1, seed=60, cc=cc, bad_key=(1, 0, 1))
    scs = [dict(base, mode=1), dict(base, mode=2), dict(base, mode=2, position=True),
           dict(base, mode=1, position=True), bad]
    res = _run_ranks(scs)
    for i, sc in enumerate(scs[:4]):
        tab = O.YcsbTable(sc["rows_pp"] * WORLD)
        f0 = tab.f0.copy()
        per_rank = [_part_batches(sc, WORLD, r) for r in range(WORLD)]
        for k in range(sc["epochs"]):
            bk = [per_rank[r][k] for r in range(WORLD)]
            q = dvcc.sequence_position(bk, sc["n_txn"]) if _position(sc) else dvcc.sequence(bk)
            c_ref, _, st_ref = O.epoch_run(ORACLE_CC[cc], tab.ix, f0, q.n_txn, q.txn_begin, q.keys, q.types)
            if _position(sc):  # (the engine returns them in origin order)
                c_ref = c_ref.reshape(sc["n_txn"], WORLD).T.reshape(-1)
            digest = 0
            for r in range(WORLD):
                out = res[r][i]
                assert "error" not in out, (sc, r, out.get("error"))
                assert (out["commit"][k] == c_ref).all(), (sc, k, r)
                assert out["stats"][k][0] == st_ref.committed
                digest = (digest + out["stats"][k][1]) % (1 << 64)
            assert digest == st_ref.read_digest, (sc, k)
        for r in range(WORLD):
            assert (res[r][i]["table"] == f0[r::WORLD]).all(), (sc, r)
    fresh = O.YcsbTable(bad["rows_pp"] * WORLD).f0
    for r in range(WORLD):
        assert res[r][4].get("error") == dvcc._lib.DV_ERR_KEY_NOT_FOUND, (r, res[r][4].get("error"))
        assert (res[r][4]["table"] == fresh[r::WORLD]).all()


@pytest.mark.parametrize("cc", [dvcc.WAIT_DIE, dvcc.CALVIN])
def test_ipc_tpcc_two_processes(cc):
    """dv_tpcc_epoch_run_part over two processes (config E's protocol: records
    routed by the warehouse's partition with table and operation word,
    per-partition last-name lookup, o_id all-reduced to every rank)."""
    from dvcc import tpcc as T
    kw = dict(num_wh=4, cust_per_dist=1000, max_items=2000, part_per_txn=2, mpr=1.0)
    sc = dict(kind="tpcc", cc=cc, kw=kw, n_txn=1200, seed=60)
    res = _run_ranks([sc])
    pp = T.tpcc_params(part_cnt=WORLD, **kw)
    batches = [T.gen(pp, sc["n_txn"], sc["seed"] + r, home_part=r) for r in range(WORLD)]
    db = O.TpccDB(O.tpcc_params(**dict(kw, part_cnt=1)), 5, index_parts=WORLD)
    keys = np.concatenate([b.keys for b in batches])
    types = np.concatenate([b.types for b in batches])
    tables = np.concatenate([b.tables for b in batches])
    args = np.concatenate([b.args for b in batches])
    sizes = np.concatenate([np.diff(b.txn_begin.astype(np.int64)) for b in batches])
    tb = np.zeros(len(sizes) + 1, np.uint32)
    tb[1:] = np.cumsum(sizes)
    c_ref, o_ref, st_ref = db.epoch(ORACLE_CC[cc], keys, types, tables, args, tb,
                                    owner=np.concatenate([b.owner for b in batches]))
    for r in range(WORLD):
        out = res[r][0]
        assert (out["commit"] == c_ref).all(), r
        assert (out["oid"] == o_ref).all(), r
        assert out["committed"] == st_ref.committed
        for tid in range(5):
            ref = db.table(tid)
            mine = np.isin(ref[0], T.table(pp, 5, tid, r)[0])
            for col in range(3):
                assert (out["cols"][tid][col] == ref[1 + col][mine]).all(), (r, tid, col)
