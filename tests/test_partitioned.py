"""Partitioned (multi-GPU) epochs.

CPU: the PartitionedRunner protocol (owner split, all-to-all of fragments in
origin order, per-round verdict all-reduce MAX, termination) over gloo with
world_size 2, driving a numpy restatement of one partition's decision round
(test double); decisions must equal the single-node oracle E-schedule over the
sequenced global epoch.

GPU: two engine contexts on one device, each owning one partition, combined by
an element-wise MAX of their verdict tensors -- the same combine RCCL performs
across GPUs -- against the oracle; and the runner itself over a 1-rank
process group.
"""
import os
import socket
import types

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import _oracle as O
import dvcc
from dvcc.partitioned import PartitionedEpoch, PartitionedRunner, split_by_owner

ORACLE_CC = {dvcc.NO_WAIT: O.NO_WAIT, dvcc.WAIT_DIE: O.WAIT_DIE, dvcc.OCC: O.OCC}


class NumpyPartition:
    """Test double: one partition's decision round in numpy (checker side)."""

    needs_votes = True

    def __init__(self, cc, nkeys=None):
        self.nowait = cc != dvcc.OCC
        self.nkeys = nkeys  # keys >= nkeys are missing from the index

    def begin_partition(self, keys, types_, txn, n_txn, max_txn_acc=0):
        k = keys.numpy().view(np.uint64)
        self.err = int(self.nkeys is not None and bool((k >= self.nkeys).any()))  # ERRB_KEY
        self.peer = 0
        order = np.argsort(k, kind="stable")
        self.k, self.w, self.t = k[order], types_.numpy()[order] == 1, txn.numpy()[order].astype(np.int64)
        head = np.ones(len(self.k), bool)
        head[1:] = self.k[1:] != self.k[:-1]
        self.seg = np.cumsum(head) - 1
        self.n_txn = n_txn
        self.status = np.zeros(n_txn, np.int8)
        self.ulist = np.arange(n_txn)  # undecided txns, ascending
        self.log = []                  # undecided count after each applied round

    def _first(self, mask):
        n = len(self.k)
        fp = np.full(self.seg[-1] + 1 if n else 1, n, np.int64)
        np.minimum.at(fp, self.seg[mask], np.arange(n)[mask])
        return fp[self.seg] < np.arange(n)

    def round_local(self, verdict):
        v = np.zeros(verdict.numel(), np.uint8)
        if len(self.k):
            s = self.status[self.t]
            c, u, w = s == 1, s == 0, self.w
            cw, uw = self._first(c & w), self._first(u & w)
            if self.nowait:
                ca, ua = self._first(c), self._first(u)
                ab, wt = np.where(w, ca, cw), np.where(w, ua, uw)
            else:
                ab, wt = cw, uw
            mine = u
            np.maximum.at(v, self.t[mine & wt & ~ab], 1)
            np.maximum.at(v, self.t[mine & ab], 2)
        # list order: entry i is txn ulist[i]; bytes past the list are junk
        out = np.full(verdict.numel(), 0xEE, np.uint8)
        out[:len(self.ulist)] = v[self.ulist]
        verdict.copy_(torch.from_numpy(out))

    def errors_local(self, word):
        word.fill_(self.err)

    def errors_combined(self, word):
        self.peer = int(word.item())

    def round_apply(self, verdict, wait=True):
        v = verdict.numpy()[:len(self.ulist)]
        lst = self.ulist
        self.status[lst[(v & 2) != 0]] = 2
        self.status[lst[v == 0]] = 1
        self.ulist = lst[self.status[lst] == 0]
        self.log.append(len(self.ulist))
        return self.log[-1] if wait else None

    def round_wait(self, r):
        if self.err | self.peer:  # the engine reports the rejected epoch at the first round it reads
            raise dvcc.DvccError(dvcc._lib.DV_ERR_KEY_NOT_FOUND, "dv_epoch_round_wait")
        return self.log[r]

    def finish(self, commit=None):
        if commit is not None:
            commit[:self.n_txn] = torch.from_numpy((self.status == 1).astype(np.uint8))
        return types.SimpleNamespace(committed=int((self.status == 1).sum()), n_txn=self.n_txn)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _global_setup(world, n_txn, rows_pp, mpr, seed0=3):
    gen = dvcc.YCSBQueryGenerator(rows_pp * world, part_cnt=world, zipf_theta=0.9,
                                  part_per_txn=2, strict_ppt=1, mpr=mpr)
    batches = [gen.gen(n_txn, dvcc.epoch_seed(r, seed0), r) for r in range(world)]
    return gen, batches


def _oracle_global(cc, batches, world, rows_pp):
    e = dvcc.sequence(batches)
    n = rows_pp * world
    tab = O.YcsbTable(n)  # part_cnt 1 view: row == key
    f0 = tab.f0.copy()
    c, _, st = O.epoch_run(ORACLE_CC[cc], tab.ix, f0, e.n_txn, e.txn_begin, e.keys, e.types)
    return c, st, f0


def _gloo_worker(rank, world, port, cc, n_txn, rows_pp, mpr, q, position=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _, batches = _global_setup(world, n_txn, rows_pp, mpr)
        pe = PartitionedEpoch(batches[rank], rank, world, n_txn, "cpu", position=position)
        runner = PartitionedRunner(NumpyPartition(cc), world, rank, device="cpu")
        commit = torch.zeros(n_txn * world, dtype=torch.uint8)
        st, rounds = runner.run(pe, commit=commit)
        q.put((rank, commit.numpy().tobytes(), rounds))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("cc,mpr", [(dvcc.NO_WAIT, 0.3), (dvcc.OCC, 0.5), (dvcc.WAIT_DIE, 0.0),
                                    (dvcc.NO_WAIT, 1.0)])
def test_runner_protocol_gloo_world2(cc, mpr):
    world, n_txn, rows_pp = 2, 600, 1 << 10
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_worker, args=(r, world, port, cc, n_txn, rows_pp, mpr, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    _, batches = _global_setup(world, n_txn, rows_pp, mpr)
    c_ref, _, _ = _oracle_global(cc, batches, world, rows_pp)
    for rank, buf, rounds in res:
        got = np.frombuffer(buf, np.uint8)
        assert (got == c_ref).all(), f"rank {rank}: {(got != c_ref).sum()} mismatches"
        assert rounds >= 1


@pytest.mark.parametrize("cc,mpr", [(dvcc.NO_WAIT, 0.3), (dvcc.OCC, 0.5), (dvcc.WAIT_DIE, 0.1)])
def test_runner_protocol_gloo_world2_position_order(cc, mpr):
    """The torch.distributed list protocol with the origins' batches
    sequenced txn by txn (PartitionedEpoch(position=True): origin q's txn j
    is sequence number j * P + q, each owner merging its fragments by id):
    commit bytes, back in origin order, equal the oracle over
    dvcc.sequence_position of the same batches."""
    world, n_txn, rows_pp = 2, 600, 1 << 10
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_worker, args=(r, world, port, cc, n_txn, rows_pp, mpr, q, True))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    _, batches = _global_setup(world, n_txn, rows_pp, mpr)
    e = dvcc.sequence_position(batches, n_txn)
    tab = O.YcsbTable(rows_pp * world)
    c_pos, _, _ = O.epoch_run(ORACLE_CC[cc], tab.ix, tab.f0.copy(), e.n_txn, e.txn_begin, e.keys, e.types)
    c_ref = _origin_order(c_pos, world, n_txn)
    c_org, _, _ = _oracle_global(cc, batches, world, rows_pp)
    assert (c_ref != c_org).any(), "the two orders decide alike here: the test would not tell them apart"
    for rank, buf, rounds in res:
        got = np.frombuffer(buf, np.uint8)
        assert (got == c_ref).all(), f"rank {rank}: {(got != c_ref).sum()} mismatches"


def test_split_by_owner_orders_fragments():
    e = dvcc.Epoch(np.array([5, 2, 7, 4, 9, 6], np.uint64), np.array([0, 1, 0, 1, 1, 0], np.uint8),
                   np.array([0, 3, 6], np.uint32))
    k, t, x, counts = split_by_owner(e, 100, 2)
    assert counts.tolist() == [3, 3]
    assert k.tolist() == [2, 4, 6, 5, 7, 9]     # owner 0 first, request order kept
    assert x.tolist() == [100, 101, 101, 100, 100, 101]


def test_sequence_is_origin_major():
    _, batches = _global_setup(3, 50, 256, 0.5)
    e = dvcc.sequence(batches)
    assert e.n_txn == 150
    assert (e.keys[:500] == batches[0].keys).all() and (e.keys[500:1000] == batches[1].keys).all()


def test_sequence_position_interleaves_txns():
    """dvcc.sequence_position (DV_COMM_POSITION_ORDER's sequence): origin q's
    txn j is txn j * P + q, a shorter batch leaves empty txns in its slots."""
    _, batches = _global_setup(3, 50, 256, 0.5)
    short = dvcc.Epoch(batches[1].keys[:int(batches[1].txn_begin[20])], batches[1].types[:int(batches[1].txn_begin[20])],
                       batches[1].txn_begin[:21].copy())
    bs = [batches[0], short, batches[2]]
    e = dvcc.sequence_position(bs, 60)
    assert e.n_txn == 180 and e.n_acc == sum(b.n_acc for b in bs)
    for t in range(e.n_txn):
        j, q = divmod(t, 3)
        a, b = int(e.txn_begin[t]), int(e.txn_begin[t + 1])
        if j < bs[q].n_txn:
            s0, s1 = int(bs[q].txn_begin[j]), int(bs[q].txn_begin[j + 1])
            assert (e.keys[a:b] == bs[q].keys[s0:s1]).all() and (e.types[a:b] == bs[q].types[s0:s1]).all()
        else:
            assert a == b


# ------------------------------------------------------------------- GPU
def _gpu_two_partitions(cc, n_txn, rows_pp, mpr, world=2):
    _, batches = _global_setup(world, n_txn, rows_pp, mpr, seed0=9)
    c_ref, st_ref, f0_ref = _oracle_global(cc, batches, world, rows_pp)
    # owner fragments, then each owner's input in origin order (the all-to-all)
    frags = [split_by_owner(b, r * n_txn, world) for r, b in enumerate(batches)]
    engines, deps = [], []
    N = n_txn * world
    for p in range(world):
        ks, ts, xs = [], [], []
        for k, t, x, counts in frags:
            lo = int(counts[:p].sum())
            hi = lo + int(counts[p])
            ks.append(k[lo:hi]); ts.append(t[lo:hi]); xs.append(x[lo:hi])
        k = np.concatenate(ks); t = np.concatenate(ts); x = np.concatenate(xs)
        eng = dvcc.CCEngine(cc, N, max(16, len(k)), part_cnt=world, part_id=p)
        eng.load_ycsb_partition(rows_pp)
        dep = dvcc.DeviceEpoch.from_tensors(torch.from_numpy(k.view(np.int64)).cuda(),
                                            torch.from_numpy(t).cuda(),
                                            torch.from_numpy(x).cuda(), N)
        eng.begin(dep)
        engines.append(eng)
        deps.append(dep)
    rounds = 0
    while True:
        vs = []
        for eng in engines:
            v = torch.zeros((N + 3) // 4 * 4, dtype=torch.uint8, device="cuda")
            eng.round_local(v)
            vs.append(v)
        torch.cuda.synchronize()
        comb = torch.stack(vs).max(dim=0).values.contiguous()
        copies = [comb.clone() for _ in engines]
        torch.cuda.synchronize()  # engines run on their own streams
        und = [eng.round_apply(cp) for eng, cp in zip(engines, copies)]
        rounds += 1
        assert len(set(und)) == 1
        if und[0] == 0:
            break
        assert rounds < N
    digest = 0
    for p, eng in enumerate(engines):
        commit = torch.zeros(N, dtype=torch.uint8, device="cuda")
        st = eng.finish(commit)
        assert (commit.cpu().numpy() == c_ref).all()
        digest = (digest + st.read_digest) % (1 << 64)
        # partition p holds keys p, p+world, ...: oracle rows with the same keys
        assert (eng.read_table(0, rows_pp) == f0_ref[p::world]).all()
        eng.close()
    assert digest == st_ref.read_digest


@pytest.mark.gpu
@pytest.mark.parametrize("cc", [dvcc.NO_WAIT, dvcc.OCC, dvcc.WAIT_DIE])
@pytest.mark.parametrize("mpr", [0.0, 0.2, 1.0])
def test_gpu_two_partition_engines(cc, mpr):
    _gpu_two_partitions(cc, 3000, 1 << 12, mpr)


@pytest.mark.gpu
def test_gpu_four_partition_engines_large():
    _gpu_two_partitions(dvcc.NO_WAIT, 50_000, 1 << 18, 0.3, world=4)


@pytest.mark.gpu
def test_gpu_runner_single_rank_process_group():
    from dvcc.partitioned import EnginePartition
    if dist.is_initialized():
        dist.destroy_process_group()
    store = dist.HashStore()
    dist.init_process_group("nccl", store=store, rank=0, world_size=1)
    try:
        n_txn, rows = 20_000, 1 << 16
        gen = dvcc.YCSBQueryGenerator(rows, zipf_theta=0.9)
        e = gen.gen(n_txn, 5)
        tab = O.YcsbTable(rows)
        f0 = tab.f0.copy()
        c_ref, _, st_ref = O.epoch_run(O.NO_WAIT, tab.ix, f0, n_txn, e.txn_begin, e.keys, e.types)
        eng = dvcc.CCEngine(dvcc.NO_WAIT, n_txn, e.n_acc)
        eng.load_ycsb_partition(rows)
        runner = PartitionedRunner(EnginePartition(eng), 1, 0)
        commit = torch.zeros(n_txn, dtype=torch.uint8, device="cuda")
        st, rounds = runner.run(PartitionedEpoch(e, 0, 1, n_txn, "cuda"), commit=commit)
        assert (commit.cpu().numpy() == c_ref).all()
        assert st.read_digest == st_ref.read_digest
        assert (eng.read_table(0, rows) == f0).all()
        eng.set_stream(None)
        eng.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("cc", [dvcc.NO_WAIT, dvcc.OCC, dvcc.CALVIN])
def test_rccl_engine_driver_single_rank(cc, mode):
    """dv_comm_init + dv_epoch_run_part (RCCL called from the engine) on a
    one-rank communicator: mode 1, the owner split, all-to-all, list
    all-reduces and lagged rounds; mode 0, which picks the replicated epoch
    whenever it fits (one rank too), the all-gathers -- run for real and must
    decide exactly as the single-GPU path and the oracle.  (More ranks need
    more GPUs: the Python driver's protocol, which this mirrors, is covered
    with gloo above.)"""
    import torch
    rows, n_txn = 1 << 14, 6000
    gen = dvcc.YCSBQueryGenerator(rows, zipf_theta=0.9, txn_write_perc=1.0, tup_write_perc=0.5)
    e = gen.gen(n_txn, dvcc.epoch_seed(0, 3))
    ref = dvcc.CCEngine(cc, n_txn, e.n_acc)
    ref.load_ycsb_partition(rows)
    c_ref = torch.zeros(n_txn, dtype=torch.uint8, device="cuda")
    st_ref = ref.run_epoch_device(dvcc.DeviceEpoch(e), c_ref)
    eng = dvcc.CCEngine(cc, n_txn, e.n_acc, part_cnt=1, part_id=0)
    eng.load_ycsb_partition(rows)
    eng.comm_init(dvcc.comm_unique_id(), 1, 0)
    eng.comm_set_mode(mode)
    c = torch.zeros(n_txn, dtype=torch.uint8, device="cuda")
    for _ in range(2):  # the communicator and buffers are reused across epochs
        eng.load_ycsb_partition(rows)
        st = eng.run_epoch_part(dvcc.DeviceEpoch(e), n_txn, c)
        assert torch.equal(c, c_ref)
        assert (st.committed, st.read_digest, st.write_cnt) == (st_ref.committed, st_ref.read_digest,
                                                               st_ref.write_cnt)
    eng.close()
    ref.close()


def _gloo_error_worker(rank, world, port, cc, n_txn, rows_pp, bad_rank, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _, batches = _global_setup(world, n_txn, rows_pp, 0.5)
        b = batches[rank]
        if rank == bad_rank:  # a key no partition holds (IndexHash::index_read miss)
            b.keys = b.keys.copy()
            b.keys[7] = np.uint64(rows_pp * world * 4 + 1)
        pe = PartitionedEpoch(b, rank, world, n_txn, "cpu")
        runner = PartitionedRunner(NumpyPartition(cc, nkeys=rows_pp * world), world, rank, device="cpu")
        try:
            runner.run(pe, commit=torch.zeros(n_txn * world, dtype=torch.uint8))
            q.put((rank, "ok"))
        except dvcc.DvccError as ex:
            q.put((rank, ex.code))
        # the group still works: every rank left the round loop together
        t = torch.ones(1)
        dist.all_reduce(t)
        q.put((rank, int(t.item())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("cc,bad_rank", [(dvcc.NO_WAIT, 1), (dvcc.OCC, 0)])
def test_runner_error_is_collective_gloo_world2(cc, bad_rank):
    """A missing key on one rank: every rank raises the same error from the
    same round, and the process group is still in step afterwards (no rank
    left behind in a collective)."""
    world, n_txn, rows_pp = 2, 300, 1 << 10
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_error_worker, args=(r, world, port, cc, n_txn, rows_pp, bad_rank, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(2 * world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    codes = sorted(v for _, v in res)
    assert codes == sorted([dvcc._lib.DV_ERR_KEY_NOT_FOUND] * world + [world] * world), res


# ---- the engine's own partitioned driver (dv_epoch_run_part) with P ranks in
# one process: P contexts on one GPU, one host thread each, the in-process
# transport in place of RCCL (dv_comm_init_local) -- the same C++ protocol
# the bench runs over RCCL with one process per GPU.
def _run_group(engines, homes, n_txn):
    """run_epoch_part on every engine concurrently; (commit bytes, stats) or
    the exception, per rank."""
    import threading
    world = len(engines)
    out = [None] * world

    def body(r):
        try:
            d = torch.zeros(n_txn * world, dtype=torch.uint8, device="cuda")
            st = engines[r].run_epoch_part(homes[r], n_txn, d)
            out[r] = (d.cpu().numpy(), st)
        except Exception as ex:  # noqa: BLE001 -- reported per rank
            out[r] = ex
    th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
        assert not t.is_alive(), "a rank hung in the partitioned epoch"
    return out


def _engine_group(cc, world, rows_pp, n_txn, R=10, mode=1, async_iters=None):
    """mode: dv_comm_set_mode -- 1 the list protocol (capacity for this
    rank's share), 2 replicated (capacity for the whole epoch); + 8
    (DV_COMM_POSITION_ORDER) position-major replicated epochs.  async_iters:
    asynchronous rounds on every context, yielding after that many iterations
    (dv_set_async_limits; replicated contexts otherwise run without them)."""
    engines = []
    for p in range(world):
        rep = (mode & 3) == 2
        cap = n_txn * world * R + 4096 if rep else max(64, int(n_txn * world * R * 1.2 / world) + 4096)
        eng = dvcc.CCEngine(cc, n_txn * world, cap, part_cnt=world, part_id=p,
                            asynchronous=not rep or async_iters is not None)
        if async_iters is not None:
            eng.set_async_limits(async_iters, 0)
        eng.load_ycsb_partition(rows_pp)
        engines.append(eng)
    dvcc.CCEngine.comm_init_local(engines)
    for eng in engines:
        eng.comm_set_mode(mode)
    return engines


def _origin_order(c_pos, world, n_txn):
    """commit bytes of a position-major sequence (origin q's txn j at j * P +
    q) in origin order (q * n_txn + j), as the engine returns them"""
    return np.asarray(c_pos).reshape(n_txn, world).T.reshape(-1)


def _check_group(cc, world, rows_pp, n_txn, mpr, epochs=2, theta=0.9, mode=1, position=False):
    gen = dvcc.YCSBQueryGenerator(rows_pp * world, part_cnt=world, zipf_theta=theta, txn_write_perc=1.0,
                                  tup_write_perc=0.5, part_per_txn=2, strict_ppt=1, mpr=mpr)
    engines = _engine_group(cc, world, rows_pp, n_txn,
                            mode=mode | (dvcc._lib.DV_COMM_POSITION_ORDER if position else 0))
    tab = O.YcsbTable(rows_pp * world)  # one-partition view: row == key
    f0 = tab.f0.copy()
    pos = position and cc != dvcc.CALVIN  # (CALVIN keeps the sequencer's origin order)
    for k in range(epochs):
        batches = [gen.gen(n_txn, dvcc.epoch_seed(r, 20 + k), r) for r in range(world)]
        e = dvcc.sequence_position(batches, n_txn) if pos else dvcc.sequence(batches)
        c_ref, _, st_ref = O.epoch_run(ORACLE_CC.get(cc, O.CALVIN), tab.ix, f0, e.n_txn, e.txn_begin, e.keys,
                                       e.types)
        if pos:
            c_ref = _origin_order(c_ref, world, n_txn)
        res = _run_group(engines, [dvcc.DeviceEpoch(b) for b in batches], n_txn)
        digest = writes = 0
        for r, x in enumerate(res):
            assert not isinstance(x, Exception), f"rank {r}: {x}"
            c, st = x
            assert (c == c_ref).all(), f"rank {r}: {(c != c_ref).sum()} mismatches"
            assert st.committed == st_ref.committed
            digest = (digest + st.read_digest) % (1 << 64)
            writes += st.write_cnt
        assert digest == st_ref.read_digest and writes == st_ref.write_cnt
        for p, eng in enumerate(engines):
            assert (eng.read_table(0, rows_pp) == f0[p::world]).all(), f"partition {p} table"
    for eng in engines:
        eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("cc", [dvcc.NO_WAIT, dvcc.WAIT_DIE, dvcc.OCC, dvcc.CALVIN])
@pytest.mark.parametrize("mpr", [0.1, 0.5])
def test_engine_driver_8_partitions(cc, mpr):
    """SURVEY config D's protocol at 8 partitions: owner split, all-to-all of
    the records, list-ordered verdict MAX per round, execution per partition
    -- decisions, digests and every partition's rows equal the one-partition
    oracle E-schedule over the sequenced global epoch."""
    _check_group(cc, 8, 1 << 14, 4000, mpr)


@pytest.mark.gpu
@pytest.mark.parametrize("cc", [dvcc.NO_WAIT, dvcc.WAIT_DIE, dvcc.OCC, dvcc.CALVIN])
@pytest.mark.parametrize("world,mpr", [(2, 0.3), (8, 0.1), (8, 0.5)])
def test_engine_driver_replicated(cc, world, mpr):
    """The replicated protocol (dv_comm_set_mode 2): the epoch's accesses
    all-gathered, every rank decides the whole epoch with the single-GPU path
    and executes its own rows -- the same decisions, digests and rows as the
    oracle (and so as the list protocol).  (The contexts share one GPU, so
    their asynchronous rounds are off here.)"""
    _check_group(cc, world, 1 << 14, 4000, mpr, mode=2)


@pytest.mark.gpu
@pytest.mark.parametrize("cc", [dvcc.NO_WAIT, dvcc.WAIT_DIE, dvcc.OCC, dvcc.CALVIN])
@pytest.mark.parametrize("world,mpr,mode", [(2, 0.3, 2), (4, 0.1, 2), (8, 0.5, 2), (3, 0.3, 1), (8, 0.1, 0),
                                            (2, 0.3, 1), (8, 0.5, 1)])
def test_engine_driver_position_order(cc, world, mpr, mode):
    """DV_COMM_POSITION_ORDER for the per-epoch driver: a replicated epoch
    (mode 2, or mode 0 choosing it) merges the origins' batches txn by txn --
    origin q's txn j at j * P + q -- against the oracle over
    dvcc.sequence_position, commit bytes back in origin order; the list
    protocol (mode 1, or mode 0 choosing it) interleaves each owner's records
    the same way; CALVIN keeps the origin order under the flag."""
    _check_group(cc, world, 1 << 14, 3000, mpr, mode=mode, position=True)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [2, 1])
def test_engine_driver_position_order_malformed_batch(mode):
    """A position-major epoch (replicated, mode 2, or the list protocol, mode
    1) whose batch on one rank has txn ids that do not rise: the interleave
    refuses to move it (the list protocol: on the owners that receive the
    records, its refusal combined with the epoch's input errors) and every
    rank returns DV_ERR_TXN_RANGE before anything executes; the next epoch
    runs."""
    world, rows_pp, n_txn = 2, 1 << 12, 800
    gen = dvcc.YCSBQueryGenerator(rows_pp * world, part_cnt=world, zipf_theta=0.9, part_per_txn=2,
                                  strict_ppt=1, mpr=0.3)
    engines = _engine_group(dvcc.NO_WAIT, world, rows_pp, n_txn, mode=mode | dvcc._lib.DV_COMM_POSITION_ORDER)
    before = [eng.read_table(0, rows_pp) for eng in engines]
    batches = [gen.gen(n_txn, dvcc.epoch_seed(r, 70), r) for r in range(world)]
    homes = [dvcc.DeviceEpoch(b) for b in batches]
    t = homes[1].acc_txn.clone()
    a, b = int(batches[1].txn_begin[5]), int(batches[1].txn_begin[6])
    t[a:b] = 9  # (txn 5's accesses claim txn 9: the ids no longer rise)
    homes[1] = dvcc.DeviceEpoch.from_tensors(homes[1].keys, homes[1].types, t, n_txn, max_txn_acc=10)
    res = _run_group(engines, homes, n_txn)
    for r, x in enumerate(res):
        assert isinstance(x, dvcc.DvccError) and x.code == dvcc._lib.DV_ERR_TXN_RANGE, (r, x)
    for eng, b0 in zip(engines, before):
        assert (eng.read_table(0, rows_pp) == b0).all()
    batches = [gen.gen(n_txn, dvcc.epoch_seed(r, 71), r) for r in range(world)]
    e = dvcc.sequence_position(batches, n_txn)
    tab = O.YcsbTable(rows_pp * world)
    f0 = tab.f0.copy()
    c_ref, _, st_ref = O.epoch_run(O.NO_WAIT, tab.ix, f0, e.n_txn, e.txn_begin, e.keys, e.types)
    res = _run_group(engines, [dvcc.DeviceEpoch(b) for b in batches], n_txn)
    for r, x in enumerate(res):
        assert not isinstance(x, Exception), (r, x)
        assert (x[0] == _origin_order(c_ref, world, n_txn)).all(), r
    for eng in engines:
        eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [1, 2, 10])
def test_engine_driver_unequal_batches(mode):
    """Ranks with fewer txns than txns_per_rank (the rest of their sequence
    slots are empty txns): unequal parts through the list protocol and the
    replicated one (padded all-gather, then packed)."""
    world, rows_pp, tpr = 3, 1 << 13, 1000
    gen = dvcc.YCSBQueryGenerator(rows_pp * world, part_cnt=world, zipf_theta=0.9, txn_write_perc=1.0,
                                  tup_write_perc=0.5, part_per_txn=2, strict_ppt=1, mpr=0.3)
    batches = [gen.gen(n, dvcc.epoch_seed(r, 9), r) for r, n in enumerate((1000, 700, 851))]
    padded = []
    for b in batches:  # the oracle's epoch: each batch's unused slots as empty txns
        tb = np.concatenate([b.txn_begin, np.full(tpr - b.n_txn, b.txn_begin[-1], np.uint32)])
        padded.append(dvcc.Epoch(b.keys, b.types, tb))
    pos = mode & dvcc._lib.DV_COMM_POSITION_ORDER  # (mode 10: position-major replicated epochs)
    e = dvcc.sequence_position(padded, tpr) if pos else dvcc.sequence(padded)
    tab = O.YcsbTable(rows_pp * world)
    f0 = tab.f0.copy()
    c_ref, _, st_ref = O.epoch_run(O.NO_WAIT, tab.ix, f0, e.n_txn, e.txn_begin, e.keys, e.types)
    if pos:
        c_ref = _origin_order(c_ref, world, tpr)
    engines = _engine_group(dvcc.NO_WAIT, world, rows_pp, tpr, mode=mode)
    res = _run_group(engines, [dvcc.DeviceEpoch(b) for b in batches], tpr)
    digest = 0
    for r, x in enumerate(res):
        assert not isinstance(x, Exception), f"rank {r}: {x}"
        c, st = x
        assert (c == c_ref).all(), f"rank {r}: {(c != c_ref).sum()} mismatches"
        digest = (digest + st.read_digest) % (1 << 64)
    assert digest == st_ref.read_digest
    for p, eng in enumerate(engines):
        assert (eng.read_table(0, rows_pp) == f0[p::world]).all()
        eng.close()


@pytest.mark.gpu
@pytest.mark.slow
def test_engine_driver_replicated_prefix_kill():
    """Config-D-shaped epoch large enough for the prefix-kill path inside the
    replicated protocol: 4 partitions x 40,000 txns (160,000 in total), in
    origin and in position order."""
    _check_group(dvcc.NO_WAIT, 4, 1 << 18, 40_000, 0.1, epochs=1, mode=2)
    _check_group(dvcc.NO_WAIT, 4, 1 << 18, 40_000, 0.1, epochs=1, mode=2, position=True)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3, 4])
def test_engine_driver_other_widths(world):
    _check_group(dvcc.NO_WAIT, world, 1 << 13, 3000, 0.3, theta=0.99)


@pytest.mark.gpu
@pytest.mark.slow
@pytest.mark.parametrize("cc,mpr", [(dvcc.NO_WAIT, 0.1), (dvcc.OCC, 0.5)])
def test_config_d_8_partitions_full(cc, mpr):
    """Config D as written: 16,777,216 rows per partition, a 1,048,576-txn
    epoch in total (131,072 per rank), zipf 0.9, 8 partitions."""
    _check_group(cc, 8, 16_777_216, 131_072, mpr, epochs=1)


@pytest.mark.gpu
@pytest.mark.parametrize("cc,mode", [(dvcc.NO_WAIT, 1), (dvcc.CALVIN, 1), (dvcc.NO_WAIT, 2), (dvcc.CALVIN, 2)])
def test_engine_driver_error_is_collective(cc, mode):
    """A missing key on one rank: every rank returns DV_ERR_KEY_NOT_FOUND
    (none hangs in a collective), no table changes, and the group runs the
    next epoch normally -- list and replicated protocols."""
    world, rows_pp, n_txn = 4, 1 << 12, 1000
    gen = dvcc.YCSBQueryGenerator(rows_pp * world, part_cnt=world, zipf_theta=0.9, part_per_txn=2,
                                  strict_ppt=1, mpr=0.3)
    engines = _engine_group(cc, world, rows_pp, n_txn, mode=mode)
    before = [eng.read_table(0, rows_pp) for eng in engines]
    batches = [gen.gen(n_txn, dvcc.epoch_seed(r, 5), r) for r in range(world)]
    bad = [dvcc.Epoch(b.keys.copy(), b.types, b.txn_begin) for b in batches]
    bad[2].keys[11] = np.uint64(rows_pp * world * 3 + 2)
    res = _run_group(engines, [dvcc.DeviceEpoch(b) for b in bad], n_txn)
    for r, x in enumerate(res):
        assert isinstance(x, dvcc.DvccError) and x.code == dvcc._lib.DV_ERR_KEY_NOT_FOUND, (r, x)
    for eng, b in zip(engines, before):
        assert (eng.read_table(0, rows_pp) == b).all()
    res = _run_group(engines, [dvcc.DeviceEpoch(b) for b in batches], n_txn)
    assert all(not isinstance(x, Exception) for x in res), res
    for eng in engines:
        eng.close()


# ---- epoch groups (dv_epoch_group_run): P epochs per group, epoch e decided
# by rank e, committed accesses routed to their owners, executed in epoch
# order on every partition
def _run_group_epochs(engines, homes, n_txn):
    """run_epoch_group on every engine concurrently (homes[r] = rank r's
    batches of the group's epochs); (commit bytes, stats) or the exception."""
    import threading
    world = len(engines)
    out = [None] * world

    def body(r):
        try:
            d = torch.zeros(n_txn * world, dtype=torch.uint8, device="cuda")
            st = engines[r].run_epoch_group(homes[r], n_txn, d)
            out[r] = (d.cpu().numpy(), st)
        except Exception as ex:  # noqa: BLE001 -- reported per rank
            out[r] = ex
    th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
        assert not t.is_alive(), "a rank hung in the epoch group"
    return out


def _run_group_batches(engines, homes, n_txn, groups):
    """run_epoch_groups (one dv_epoch_group_run_batch call of `groups`
    groups) on every engine concurrently; homes[r][g] = rank r's batches of
    group g.  Per rank: ([commit bytes per group], [stats per group]) or the
    exception."""
    import threading
    world = len(engines)
    out = [None] * world

    def body(r):
        try:
            ds = [torch.zeros(n_txn * world, dtype=torch.uint8, device="cuda") for _ in range(groups)]
            sts = engines[r].run_epoch_groups(homes[r], n_txn, ds)
            out[r] = ([d.cpu().numpy() for d in ds], sts)
        except Exception as ex:  # noqa: BLE001 -- reported per rank
            out[r] = ex
    th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
        assert not t.is_alive(), "a rank hung in the epoch groups"
    return out


def _group_sequence(batches, n_txn, cc, position):
    """The epoch a group decides from these batches: origin-major (Calvin's
    order; batches padded with empty txns to n_txn each) or, position-major
    (DV_COMM_POSITION_ORDER, not CALVIN), txn by txn."""
    if position and cc != dvcc.CALVIN:
        return dvcc.sequence_position(batches, n_txn)
    padded = []
    for b in batches:
        tb = np.concatenate([b.txn_begin, np.full(n_txn - b.n_txn, b.txn_begin[-1], np.uint32)])
        padded.append(dvcc.Epoch(b.keys, b.types, tb))
    return dvcc.sequence(padded)


def _group_mine(c_ref, r, n_txn, world, cc, position):
    """Rank r's txns' commit bytes in a sequenced group epoch's bytes."""
    if position and cc != dvcc.CALVIN:
        return c_ref.reshape(n_txn, world)[:, r]
    return c_ref[r * n_txn:(r + 1) * n_txn]


def _check_epoch_groups(cc, world, rows_pp, n_txn, mpr, groups=2, theta=0.9, sizes=None, batch=False,
                        wide=False, position=False, prefix=0, async_iters=None):
    """Every epoch of every group against the one-partition oracle run over
    the sequenced epochs one after the other: commit bytes (each rank holds its
    own txns' bytes of every epoch), committed count, digest and writes summed
    over the partitions, and every partition's rows after each group.
    sizes: per-rank batch sizes (unequal batches; the rest of a rank's
    sequence slots are empty txns).  batch: all groups in one
    dv_epoch_group_run_batch call (rows checked after the last group).
    wide: 8-byte batches (DV_COMM_WIDE_BATCHES) instead of the compact ones.
    position: the origins' batches sequenced txn by txn (DV_COMM_POSITION_ORDER;
    CALVIN keeps origin order).  prefix: dv_set_prefix on every decider (a
    prefix-kill epoch at any size: the groups' boundaries path, tbx).
    async_iters: the deciders' asynchronous rounds on, yielding after that
    many iterations (_engine_group)."""
    gen = dvcc.YCSBQueryGenerator(rows_pp * world, part_cnt=world, zipf_theta=theta, txn_write_perc=1.0,
                                  tup_write_perc=0.5, part_per_txn=2, strict_ppt=1, mpr=mpr)
    engines = _engine_group(cc, world, rows_pp, n_txn, mode=2, async_iters=async_iters)
    if prefix:
        for eng in engines:
            eng.set_prefix(prefix)
    if wide or position:
        for eng in engines:
            eng.comm_set_mode(2 | (dvcc._lib.DV_COMM_WIDE_BATCHES if wide else 0) |
                              (dvcc._lib.DV_COMM_POSITION_ORDER if position else 0))
    tab = O.YcsbTable(rows_pp * world)
    f0 = tab.f0.copy()
    sizes = sizes or [n_txn] * world
    if batch:
        all_homes = [[] for _ in range(world)]  # [rank][group][epoch]
        all_refs = []
        for g in range(groups):
            homes = [[None] * world for _ in range(world)]
            refs = []
            for e in range(world):
                batches = [gen.gen(sizes[r], dvcc.epoch_seed(r, 40 + g * world + e), r) for r in range(world)]
                q = _group_sequence(batches, n_txn, cc, position)
                c_ref, _, st_ref = O.epoch_run(ORACLE_CC.get(cc, O.CALVIN), tab.ix, f0, q.n_txn, q.txn_begin,
                                               q.keys, q.types)
                refs.append((c_ref, st_ref))
                for r in range(world):
                    homes[r][e] = dvcc.DeviceEpoch(batches[r])
            for r in range(world):
                all_homes[r].append(homes[r])
            all_refs.append(refs)
        res = _run_group_batches(engines, all_homes, n_txn, groups)
        for r, x in enumerate(res):
            assert not isinstance(x, Exception), f"rank {r}: {x}"
        for g, refs in enumerate(all_refs):
            committed = sum(st.committed for _, st in refs)
            digest = writes = 0
            for r, (cs, sts) in enumerate(res):
                for e in range(world):
                    assert (cs[g][e * n_txn:(e + 1) * n_txn] ==
                            _group_mine(refs[e][0], r, n_txn, world, cc, position)).all(), f"group {g} epoch {e} rank {r}"
                assert sts[g].committed == committed and sts[g].n_txn == n_txn * world * world
                digest = (digest + sts[g].read_digest) % (1 << 64)
                writes += sts[g].write_cnt
            assert digest == sum(st.read_digest for _, st in refs) % (1 << 64), f"group {g} digest"
            assert writes == sum(st.write_cnt for _, st in refs), f"group {g} writes"
        for p, eng in enumerate(engines):
            assert (eng.read_table(0, rows_pp) == f0[p::world]).all(), f"partition {p} table"
        for eng in engines:
            eng.close()
        return
    for g in range(groups):
        homes = [[None] * world for _ in range(world)]  # [rank][epoch]
        refs = []
        for e in range(world):
            batches = [gen.gen(sizes[r], dvcc.epoch_seed(r, 40 + g * world + e), r) for r in range(world)]
            q = _group_sequence(batches, n_txn, cc, position)
            c_ref, _, st_ref = O.epoch_run(ORACLE_CC.get(cc, O.CALVIN), tab.ix, f0, q.n_txn, q.txn_begin, q.keys,
                                           q.types)
            refs.append((c_ref, st_ref))
            for r in range(world):
                homes[r][e] = dvcc.DeviceEpoch(batches[r])
        res = _run_group_epochs(engines, homes, n_txn)
        committed = sum(st.committed for _, st in refs)
        digest = writes = 0
        if async_iters == 1:  # (forced yields: some decider halted and finished after the vote)
            assert any(not isinstance(x, Exception) and x[1].async_yields for x in res), f"group {g}: no yield"
        for r, x in enumerate(res):
            assert not isinstance(x, Exception), f"rank {r}: {x}"
            c, st = x
            for e in range(world):
                mine = _group_mine(refs[e][0], r, n_txn, world, cc, position)
                assert (c[e * n_txn:(e + 1) * n_txn] == mine).all(), f"group {g} epoch {e} rank {r}"
            assert st.committed == committed and st.n_txn == n_txn * world * world
            digest = (digest + st.read_digest) % (1 << 64)
            writes += st.write_cnt
        assert digest == sum(st.read_digest for _, st in refs) % (1 << 64)
        assert writes == sum(st.write_cnt for _, st in refs)
        for p, eng in enumerate(engines):
            assert (eng.read_table(0, rows_pp) == f0[p::world]).all(), f"group {g} partition {p} table"
    for eng in engines:
        eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("cc", [dvcc.NO_WAIT, dvcc.WAIT_DIE, dvcc.OCC, dvcc.CALVIN])
@pytest.mark.parametrize("world,mpr", [(2, 0.3), (8, 0.1), (8, 0.5)])
def test_epoch_groups(cc, world, mpr):
    """Epoch-parallel scheduling: P epochs per group decided side by side (one
    per rank) and executed in epoch order on every partition -- the same
    commit bytes, digests and rows as the oracle running the epochs in
    sequence.  (The contexts share one GPU: asynchronous rounds off.)"""
    _check_epoch_groups(cc, world, 1 << 14, 3000, mpr)


@pytest.mark.gpu
@pytest.mark.parametrize("cc", [dvcc.NO_WAIT, dvcc.WAIT_DIE, dvcc.OCC, dvcc.CALVIN])
@pytest.mark.parametrize("world,mpr", [(2, 0.0), (2, 0.3), (8, 0.1)])
def test_epoch_groups_position_order(cc, world, mpr):
    """DV_COMM_POSITION_ORDER: the decider interleaves the origins' batches
    txn by txn (origin q's txn j at j * P + q) -- against the oracle over
    dvcc.sequence_position of the same batches, commit bytes back in origin
    order; CALVIN keeps its origin order under the flag."""
    _check_epoch_groups(cc, world, 1 << 14, 3000, mpr, position=True)


@pytest.mark.gpu
@pytest.mark.parametrize("cc,wide,batch,sizes", [
    (dvcc.NO_WAIT, True, False, None), (dvcc.OCC, True, False, None), (dvcc.WAIT_DIE, False, True, None),
    (dvcc.NO_WAIT, False, False, [1000, 640, 913]), (dvcc.OCC, True, False, [700, 1000, 1])])
def test_epoch_groups_position_order_forms(cc, wide, batch, sizes):
    """Position-major groups over the 8-byte batches (the senders' ids, bounds
    found by search), three groups in one batched call, and unequal batches
    (empty slots in the interleaved sequence)."""
    world = 3 if sizes else 4
    _check_epoch_groups(cc, world, 1 << 13, 1000, 0.3, groups=3 if batch else 2, batch=batch, wide=wide,
                        sizes=sizes, position=True)


@pytest.mark.gpu
@pytest.mark.slow
def test_epoch_groups_position_order_prefix_kill():
    """Position-major groups with epochs large enough for the decider's
    prefix-kill path (4 x 40,000 txns, MPR 0 and 0.1)."""
    _check_epoch_groups(dvcc.NO_WAIT, 4, 1 << 18, 40_000, 0.0, groups=1, position=True)
    _check_epoch_groups(dvcc.NO_WAIT, 4, 1 << 18, 40_000, 0.1, groups=1, position=True)


@pytest.mark.gpu
@pytest.mark.parametrize("cc", [dvcc.NO_WAIT, dvcc.WAIT_DIE, dvcc.OCC])
@pytest.mark.parametrize("world,position", [(2, False), (2, True), (4, True)])
def test_epoch_groups_with_boundaries(cc, world, position):
    """Prefix-kill deciders (a forced prefix of 400 txns) over batches that
    carry their txn_begin: the boundaries travel beside rows without start
    bits (the vote's tbx), the decider renumbers nothing -- origin-major as
    landed, position-major through the tile move -- against the oracle; and
    unequal batches (padded boundaries)."""
    _check_epoch_groups(cc, world, 1 << 13, 2000, 0.3, position=position, prefix=400)
    _check_epoch_groups(cc, 3, 1 << 13, 1000, 0.3, sizes=[1000, 640, 1], position=position, prefix=300)


@pytest.mark.gpu
@pytest.mark.parametrize("cc", [dvcc.NO_WAIT, dvcc.WAIT_DIE, dvcc.OCC])
@pytest.mark.parametrize("async_iters,prefix,batch", [(1, 0, False), (1, 400, False), (1, 400, True),
                                                      (1 << 18, 400, False)])
def test_epoch_groups_asynchronous_deciders(cc, async_iters, prefix, batch):
    """Deciders with asynchronous rounds, as the bench runs them: a decided
    group's counters reach the host with the outcome vote (no read of their
    own).  Forced yields (one iteration) halt every decision: the vote carries
    the halted decider, which finishes its rounds (and, prefix-kill, its
    prefix) and routes again, and every rank votes again -- against the
    oracle; then the same without forced yields."""
    _check_epoch_groups(cc, 2, 1 << 13, 2000, 0.3, position=True, prefix=prefix, async_iters=async_iters,
                        groups=3 if batch else 2, batch=batch)


@pytest.mark.gpu
def test_epoch_groups_bad_boundaries_fail_collectively():
    """A batch whose txn_begin falls inside (handed over as a DeviceEpoch with
    a tampered boundary): its sender's check fails the group with DV_ERR_ARG
    on every rank, no row changes, and the next group runs normally."""
    world, rows_pp, n_txn = 2, 1 << 12, 1500
    gen = dvcc.YCSBQueryGenerator(rows_pp * world, part_cnt=world, zipf_theta=0.9, part_per_txn=2,
                                  strict_ppt=1, mpr=0.3)
    engines = _engine_group(dvcc.NO_WAIT, world, rows_pp, n_txn, mode=2)
    for eng in engines:
        eng.set_prefix(300)
        eng.comm_set_mode(2 | dvcc._lib.DV_COMM_POSITION_ORDER)
    before = [eng.read_table(0, rows_pp) for eng in engines]
    homes = [[dvcc.DeviceEpoch(gen.gen(n_txn, dvcc.epoch_seed(r, 120 + e), r)) for e in range(world)]
             for r in range(world)]
    bad = dvcc.DeviceEpoch(gen.gen(n_txn, dvcc.epoch_seed(1, 130), 1))
    bad.txn_begin[9] = bad.txn_begin[11] + 1  # (not rising)
    bad_homes = [list(h) for h in homes]
    bad_homes[1][0] = bad
    res = _run_group_epochs(engines, bad_homes, n_txn)
    for r, x in enumerate(res):
        assert isinstance(x, dvcc.DvccError) and x.code == dvcc._lib.DV_ERR_ARG, (r, x)
    for eng, b0 in zip(engines, before):
        assert (eng.read_table(0, rows_pp) == b0).all()
    res = _run_group_epochs(engines, homes, n_txn)
    assert all(not isinstance(x, Exception) for x in res), res
    for eng in engines:
        eng.close()


@pytest.mark.gpu
def test_epoch_groups_position_order_malformed_wide_batch():
    """A raw wide batch whose txn ids do not rise (handed over as tensors):
    the position-major move refuses it -- DV_ERR_ARG on every rank, no row
    changes -- and the group then runs normally."""
    world, rows_pp, n_txn = 2, 1 << 12, 600
    gen = dvcc.YCSBQueryGenerator(rows_pp * world, part_cnt=world, zipf_theta=0.9, part_per_txn=2,
                                  strict_ppt=1, mpr=0.3)
    engines = _engine_group(dvcc.NO_WAIT, world, rows_pp, n_txn, mode=2)
    for eng in engines:
        eng.comm_set_mode(2 | dvcc._lib.DV_COMM_WIDE_BATCHES | dvcc._lib.DV_COMM_POSITION_ORDER)
    before = [eng.read_table(0, rows_pp) for eng in engines]
    homes = [[dvcc.DeviceEpoch(gen.gen(n_txn, dvcc.epoch_seed(r, 90 + e), r)) for e in range(world)]
             for r in range(world)]
    h = homes[1][0]
    txn = h.acc_txn.clone()
    a, b = int(txn.numel()) // 2, int(txn.numel()) // 2 + 40
    txn[a:b] = txn[a:b].flip(0)  # ids falling inside the batch
    bad = [list(x) for x in homes]
    bad[1][0] = dvcc.DeviceEpoch.from_tensors(h.keys, h.types, txn, h.n_txn, max_txn_acc=h.max_txn_acc)
    res = _run_group_epochs(engines, bad, n_txn)
    for r, x in enumerate(res):
        assert isinstance(x, dvcc.DvccError) and x.code == dvcc._lib.DV_ERR_ARG, (r, x)
    for eng, b0 in zip(engines, before):
        assert (eng.read_table(0, rows_pp) == b0).all()
    res = _run_group_epochs(engines, homes, n_txn)
    assert all(not isinstance(x, Exception) for x in res), res
    for eng in engines:
        eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("cc", [dvcc.NO_WAIT, dvcc.WAIT_DIE, dvcc.OCC, dvcc.CALVIN])
def test_epoch_groups_wide_batches(cc):
    """The 8-byte batch form (row id, txn id per access), which groups whose
    global row space reaches 2^30 take: the same results."""
    _check_epoch_groups(cc, 4, 1 << 13, 2000, 0.3, wide=True)


@pytest.mark.gpu
@pytest.mark.parametrize("cc,world", [(dvcc.NO_WAIT, 4), (dvcc.OCC, 2), (dvcc.CALVIN, 8)])
def test_epoch_group_batch(cc, world):
    """dv_epoch_group_run_batch: three groups in one call (each group's
    digest read with the next group's vote) equal the oracle's epochs in
    sequence, group by group."""
    _check_epoch_groups(cc, world, 1 << 13, 2000, 0.3, groups=3, batch=True)


@pytest.mark.gpu
def test_epoch_groups_unequal_batches():
    _check_epoch_groups(dvcc.NO_WAIT, 3, 1 << 13, 1000, 0.3, sizes=[1000, 640, 913])


@pytest.mark.gpu
@pytest.mark.slow
def test_epoch_groups_prefix_kill():
    """Epochs large enough for the prefix-kill path in the decider: 4
    partitions x 40,000 txns per batch (160,000-txn epochs)."""
    _check_epoch_groups(dvcc.NO_WAIT, 4, 1 << 18, 40_000, 0.1, groups=1)


@pytest.mark.gpu
@pytest.mark.slow
@pytest.mark.parametrize("position", [False, True])
def test_epoch_groups_config_d_size(position):
    """The N>1 headline's exact shape: config D at 8 partitions -- 16,777,216
    rows per partition, 131,072 txns per batch (1,048,576-txn epochs), zipf
    0.9, MPR 0.1 -- one group of 8 epochs, NO_WAIT: every epoch's commit
    bytes, the digests and every partition's rows against the oracle running
    the 8 sequenced epochs one after the other; origin-major and, as the
    bench runs it, position-major."""
    _check_epoch_groups(dvcc.NO_WAIT, 8, 16_777_216, 131_072, 0.1, groups=1, position=position)


@pytest.mark.gpu
def test_epoch_group_batch_stops_at_failing_group():
    """dv_epoch_group_run_batch with a bad key in its second group: every
    rank returns DV_ERR_KEY_NOT_FOUND, the first group's rows stay applied,
    the rest of the batch never runs, and the engines run groups again."""
    world, rows_pp, n_txn = 2, 1 << 12, 800
    gen = dvcc.YCSBQueryGenerator(rows_pp * world, part_cnt=world, zipf_theta=0.9, part_per_txn=2,
                                  strict_ppt=1, mpr=0.3)
    ref = _engine_group(dvcc.NO_WAIT, world, rows_pp, n_txn, mode=2)
    engines = _engine_group(dvcc.NO_WAIT, world, rows_pp, n_txn, mode=2)
    groups = [[[dvcc.DeviceEpoch(gen.gen(n_txn, dvcc.epoch_seed(r, 80 + g * world + e), r)) for e in range(world)]
               for g in range(3)] for r in range(world)]  # [rank][group][epoch]
    bad = gen.gen(n_txn, dvcc.epoch_seed(0, 99), 0)
    bad.keys[3] = np.uint64(rows_pp * world + 1)
    bad_groups = [[list(g) for g in gr] for gr in groups]
    bad_groups[0][1][1] = dvcc.DeviceEpoch(bad)
    res = _run_group_batches(engines, bad_groups, n_txn, 3)
    for r, x in enumerate(res):
        assert isinstance(x, dvcc.DvccError) and x.code == dvcc._lib.DV_ERR_KEY_NOT_FOUND, (r, x)
    res = _run_group_epochs(ref, [groups[r][0] for r in range(world)], n_txn)  # the first group alone
    assert all(not isinstance(x, Exception) for x in res), res
    for eng, e_ref in zip(engines, ref):
        assert (eng.read_table(0, rows_pp) == e_ref.read_table(0, rows_pp)).all()
    res = _run_group_batches(engines, [groups[r][1:] for r in range(world)], n_txn, 2)
    ref_res = _run_group_batches(ref, [groups[r][1:] for r in range(world)], n_txn, 2)
    for x, y in zip(res, ref_res):
        assert not isinstance(x, Exception) and not isinstance(y, Exception), (x, y)
        for g in range(2):
            assert (x[0][g] == y[0][g]).all()
            assert (x[1][g].committed, x[1][g].read_digest) == (y[1][g].committed, y[1][g].read_digest)
    for eng, e_ref in zip(engines, ref):
        assert (eng.read_table(0, rows_pp) == e_ref.read_table(0, rows_pp)).all()
    for eng in engines + ref:
        eng.close()


@pytest.mark.gpu
def test_epoch_groups_errors_are_collective():
    """A key out of range in one batch of one epoch fails the group on every
    rank with DV_ERR_KEY_NOT_FOUND and changes no row; a rank whose table is
    not a dense YCSB map makes every rank return DV_ERR_ARG; the group then
    runs normally."""
    world, rows_pp, n_txn = 4, 1 << 12, 1000
    gen = dvcc.YCSBQueryGenerator(rows_pp * world, part_cnt=world, zipf_theta=0.9, part_per_txn=2,
                                  strict_ppt=1, mpr=0.3)
    engines = _engine_group(dvcc.NO_WAIT, world, rows_pp, n_txn, mode=2)
    before = [eng.read_table(0, rows_pp) for eng in engines]
    homes = [[dvcc.DeviceEpoch(gen.gen(n_txn, dvcc.epoch_seed(r, 60 + e), r)) for e in range(world)]
             for r in range(world)]
    bad = gen.gen(n_txn, dvcc.epoch_seed(1, 62), 1)
    bad.keys[7] = np.uint64(rows_pp * world + 5)
    bad_homes = [list(h) for h in homes]
    bad_homes[1][2] = dvcc.DeviceEpoch(bad)
    res = _run_group_epochs(engines, bad_homes, n_txn)
    for r, x in enumerate(res):
        assert isinstance(x, dvcc.DvccError) and x.code == dvcc._lib.DV_ERR_KEY_NOT_FOUND, (r, x)
    for eng, b in zip(engines, before):
        assert (eng.read_table(0, rows_pp) == b).all()
    res = _run_group_epochs(engines, homes, n_txn)
    assert all(not isinstance(x, Exception) for x in res), res
    # an empty txn inside a batch (txn ids not dense) handed over as raw
    # device arrays (density unknown to the wrapper): the compact batch format
    # cannot number it, so the group fails with DV_ERR_ARG everywhere
    after = [eng.read_table(0, rows_pp) for eng in engines]
    gap = gen.gen(n_txn, dvcc.epoch_seed(2, 63), 2)
    tb = gap.txn_begin.copy()
    tb[5] = tb[4]
    gd = dvcc.DeviceEpoch(dvcc.Epoch(gap.keys, gap.types, tb))
    gap_homes = [list(h) for h in homes]
    gap_homes[2][0] = dvcc.DeviceEpoch.from_tensors(gd.keys, gd.types, gd.acc_txn, gd.n_txn,
                                                    max_txn_acc=gd.max_txn_acc)
    res = _run_group_epochs(engines, gap_homes, n_txn)
    for r, x in enumerate(res):
        assert isinstance(x, dvcc.DvccError) and x.code == dvcc._lib.DV_ERR_ARG, (r, x)
    for eng, b in zip(engines, after):
        assert (eng.read_table(0, rows_pp) == b).all()
    res = _run_group_epochs(engines, homes, n_txn)
    assert all(not isinstance(x, Exception) for x in res), res
    # partition 3 reloaded through dv_load_table (keys in bucket order, so an
    # implicit-row map, but not known dense): the group is refused everywhere
    keys = np.arange(rows_pp, dtype=np.uint64) * world + 3
    engines[3].load_table(0, keys, engines[3].read_table(0, rows_pp))
    res = _run_group_epochs(engines, homes, n_txn)
    for r, x in enumerate(res):
        assert isinstance(x, dvcc.DvccError) and x.code == dvcc._lib.DV_ERR_ARG, (r, x)
    for eng in engines:
        eng.close()


@pytest.mark.gpu
def test_epoch_groups_nondense_batch_goes_wide():
    """A host-built batch with an empty txn in the middle: the wrapper moves
    that rank to the 8-byte batch form for the call, the group's vote takes
    it on every rank, and the results equal the oracle over the sequenced
    epochs (the empty txn commits with no accesses, as on one GPU)."""
    world, rows_pp, n_txn = 2, 1 << 12, 700
    gen = dvcc.YCSBQueryGenerator(rows_pp * world, part_cnt=world, zipf_theta=0.9, part_per_txn=2,
                                  strict_ppt=1, mpr=0.3)
    engines = _engine_group(dvcc.NO_WAIT, world, rows_pp, n_txn, mode=2)
    tab = O.YcsbTable(rows_pp * world)
    f0 = tab.f0.copy()
    homes = [[None] * world for _ in range(world)]
    refs = []
    for e in range(world):
        batches = [gen.gen(n_txn, dvcc.epoch_seed(r, 70 + e), r) for r in range(world)]
        if e == 1:  # rank 0's batch of epoch 1: txn 9 loses its accesses
            b = batches[0]
            tb = b.txn_begin.astype(np.int64)
            keep = np.ones(b.n_acc, bool)
            keep[tb[9]:tb[10]] = False
            nt = np.diff(tb)
            nt[9] = 0
            batches[0] = dvcc.Epoch(b.keys[keep], b.types[keep],
                                    np.concatenate([[0], np.cumsum(nt)]).astype(np.uint32))
        q = dvcc.sequence(batches)
        c_ref, _, st_ref = O.epoch_run(O.NO_WAIT, tab.ix, f0, q.n_txn, q.txn_begin, q.keys, q.types)
        refs.append((c_ref, st_ref))
        for r in range(world):
            homes[r][e] = dvcc.DeviceEpoch(batches[r])
    assert homes[0][1].dense is False and homes[1][1].dense
    res = _run_group_epochs(engines, homes, n_txn)
    for r, x in enumerate(res):
        assert not isinstance(x, Exception), f"rank {r}: {x}"
        c, _ = x
        for e in range(world):
            assert (c[e * n_txn:(e + 1) * n_txn] == refs[e][0][r * n_txn:(r + 1) * n_txn]).all(), (r, e)
    for p, eng in enumerate(engines):
        assert (eng.read_table(0, rows_pp) == f0[p::world]).all()
        eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["group_wide", "replicated", "list"])
def test_txn_id_past_txns_per_rank_is_rejected(kind):
    """A batch whose device txn ids reach txns_per_rank (its n_txn within the
    bound): the id would alias the next origin's txn 0 in the global order, so
    the pack (the owner split, for the list protocol) sends it as an invalid
    id and every rank returns DV_ERR_TXN_RANGE with no row changed (the 8-byte
    epoch-group batches, the replicated and the list protocol; the compact
    batches reject it as non-dense)."""
    world, rows_pp, n_txn = 2, 1 << 12, 500
    gen = dvcc.YCSBQueryGenerator(rows_pp * world, part_cnt=world, zipf_theta=0.9, part_per_txn=2,
                                  strict_ppt=1, mpr=0.3)
    engines = _engine_group(dvcc.NO_WAIT, world, rows_pp, n_txn, mode=1 if kind == "list" else 2)
    if kind == "group_wide":
        for eng in engines:
            eng.comm_set_mode(2 | dvcc._lib.DV_COMM_WIDE_BATCHES)
    before = [eng.read_table(0, rows_pp) for eng in engines]
    batches = [[dvcc.DeviceEpoch(gen.gen(n_txn, dvcc.epoch_seed(r, 90 + e), r)) for e in range(world)]
               for r in range(world)]
    d = batches[0][0]
    t = d.acc_txn.clone()
    t[-3:] = n_txn  # the last txn's accesses name txn n_txn
    batches[0][0] = dvcc.DeviceEpoch.from_tensors(d.keys, d.types, t, n_txn, max_txn_acc=d.max_txn_acc)
    if kind == "group_wide":
        res = _run_group_epochs(engines, batches, n_txn)
    else:
        res = _run_group(engines, [batches[r][0] for r in range(world)], n_txn)
    for r, x in enumerate(res):
        assert isinstance(x, dvcc.DvccError) and x.code == dvcc._lib.DV_ERR_TXN_RANGE, (r, x)
    for eng, b in zip(engines, before):
        assert (eng.read_table(0, rows_pp) == b).all()
        eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("cc", [dvcc.NO_WAIT, dvcc.OCC, dvcc.CALVIN])
def test_rccl_epoch_group_single_rank(cc):
    """dv_epoch_group_run over RCCL on a one-rank communicator: the batch
    all-to-allv, route all-to-allv and commit-byte return run for real and
    must equal the single-GPU path."""
    rows, n_txn = 1 << 14, 6000
    gen = dvcc.YCSBQueryGenerator(rows, zipf_theta=0.9, txn_write_perc=1.0, tup_write_perc=0.5)
    e = gen.gen(n_txn, dvcc.epoch_seed(0, 3))
    ref = dvcc.CCEngine(cc, n_txn, e.n_acc)
    ref.load_ycsb_partition(rows)
    c_ref = torch.zeros(n_txn, dtype=torch.uint8, device="cuda")
    eng = dvcc.CCEngine(cc, n_txn, e.n_acc, part_cnt=1, part_id=0)
    eng.load_ycsb_partition(rows)
    eng.comm_init(dvcc.comm_unique_id(), 1, 0)
    c = torch.zeros(n_txn, dtype=torch.uint8, device="cuda")
    for _ in range(2):  # epochs in sequence: the second sees the first's writes
        st_ref = ref.run_epoch_device(dvcc.DeviceEpoch(e), c_ref)
        st = eng.run_epoch_group([dvcc.DeviceEpoch(e)], n_txn, c)
        assert torch.equal(c, c_ref)
        assert (st.committed, st.read_digest, st.write_cnt) == (st_ref.committed, st_ref.read_digest,
                                                               st_ref.write_cnt)
        assert (eng.read_table(0, rows) == ref.read_table(0, rows)).all()
    # three groups in one batch call
    cs = [torch.zeros(n_txn, dtype=torch.uint8, device="cuda") for _ in range(3)]
    sts = eng.run_epoch_groups([[dvcc.DeviceEpoch(e)]] * 3, n_txn, cs)
    for c, st in zip(cs, sts):
        st_ref = ref.run_epoch_device(dvcc.DeviceEpoch(e), c_ref)
        assert torch.equal(c, c_ref)
        assert (st.committed, st.read_digest, st.write_cnt) == (st_ref.committed, st_ref.read_digest,
                                                               st_ref.write_cnt)
    assert (eng.read_table(0, rows) == ref.read_table(0, rows)).all()
    eng.close()
    ref.close()


class NumpyTpccPartition(NumpyPartition):
    """Test double for TPC-C fragments: the last-name lookup (mid of the
    newest-first list, tpcc_txn.cpp:600-626) on the host, then rows keyed by
    (table, key); checks each access arrived with its own table and operation."""

    def __init__(self, cc, pp, seed, expect):
        super().__init__(cc)
        from dvcc import tpcc as T
        k, cust, _, _ = T.table(pp, seed, T.L.T_CUST_LAST, 0)
        lists = {}
        for a, c in zip(k.tolist(), cust.tolist()):
            lists.setdefault(a, []).insert(0, c)  # insert_item prepends
        self.mid = {a: v[len(v) // 2] for a, v in lists.items()}
        self.expect = expect

    def begin_partition(self, keys, types_, txn, n_txn, max_txn_acc=0, tables=None, args=None):
        k = keys.numpy().view(np.uint64).copy()
        tb = tables.numpy().copy()
        for i in np.flatnonzero(tb == 5):
            k[i] = self.mid[int(k[i])]
            tb[i] = 2
        trip = set(zip(txn.numpy().tolist(), keys.numpy().view(np.uint64).tolist(), tables.numpy().tolist(),
                       args.numpy().view(np.uint64).tolist()))
        assert trip <= self.expect
        rows = torch.from_numpy((k * np.uint64(8) + tb.astype(np.uint64)).view(np.int64))
        super().begin_partition(rows, types_, txn, n_txn, max_txn_acc)


def _tpcc_setup(world, n_txn):
    from dvcc import tpcc as T
    kw = dict(num_wh=2 * world, cust_per_dist=1000, max_items=2000, part_cnt=world)
    pp = T.tpcc_params(**kw)
    batches = [T.gen(pp, n_txn, 60 + r, home_part=r) for r in range(world)]
    return kw, pp, batches


def _tpcc_gloo_worker(rank, world, port, cc, n_txn, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        kw, pp, batches = _tpcc_setup(world, n_txn)
        expect = set()
        for r, b in enumerate(batches):
            expect |= set(zip((b.acc_txn().astype(np.int64) + r * n_txn).tolist(), b.keys.tolist(),
                              b.tables.tolist(), b.args.tolist()))
        pe = PartitionedEpoch(batches[rank], rank, world, n_txn, "cpu")
        runner = PartitionedRunner(NumpyTpccPartition(cc, dvcc.tpcc.tpcc_params(**dict(kw, part_cnt=1)), 5, expect),
                                   world, rank, device="cpu")
        commit = torch.zeros(n_txn * world, dtype=torch.uint8)
        runner.run(pe, commit=commit)
        q.put((rank, commit.numpy().tobytes()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("cc", [dvcc.NO_WAIT, dvcc.OCC])
def test_tpcc_runner_protocol_gloo_world2(cc):
    """TPC-C fragments (with tables and operation words) through the runner
    over gloo, world 2: decisions equal the global oracle E-schedule."""
    import dvcc.tpcc  # noqa: F401
    world, n_txn = 2, 400
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tpcc_gloo_worker, args=(r, world, port, cc, n_txn, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    kw, pp, batches = _tpcc_setup(world, n_txn)
    db = O.TpccDB(O.tpcc_params(**dict(kw, part_cnt=1)), 5)
    keys = np.concatenate([b.keys for b in batches])
    sizes = np.concatenate([np.diff(b.txn_begin.astype(np.int64)) for b in batches])
    tb = np.zeros(len(sizes) + 1, np.uint32)
    tb[1:] = np.cumsum(sizes)
    c_ref, _, _ = db.epoch(ORACLE_CC[cc], keys, np.concatenate([b.types for b in batches]),
                           np.concatenate([b.tables for b in batches]), np.concatenate([b.args for b in batches]), tb)
    assert 0 < c_ref.sum() < len(c_ref)
    for rank, buf in res:
        assert (np.frombuffer(buf, np.uint8) == c_ref).all(), rank


def _host_carry(ep, commit, max_txn):
    """The aborted txns of batch `ep` (commit byte 0), in order, at most
    max_txn (tests/test_carry.py's rule, restated for batches)."""
    tb = ep.txn_begin.astype(np.int64)
    ab = np.flatnonzero(commit[:ep.n_txn] == 0)[:max_txn]
    idx = np.concatenate([np.arange(tb[t], tb[t + 1]) for t in ab]) if len(ab) else np.zeros(0, np.int64)
    ntb = np.zeros(len(ab) + 1, np.uint32)
    ntb[1:] = np.cumsum(tb[ab + 1] - tb[ab])
    return dvcc.Epoch(ep.keys[idx].copy(), ep.types[idx].copy(), ntb)


def _host_concat(a, b):
    tb = np.concatenate([a.txn_begin, b.txn_begin[1:] + a.txn_begin[-1]]).astype(np.uint32)
    return dvcc.Epoch(np.concatenate([a.keys, b.keys]), np.concatenate([a.types, b.types]), tb)


@pytest.mark.gpu
@pytest.mark.parametrize("cc,world", [(dvcc.NO_WAIT, 2), (dvcc.WAIT_DIE, 2), (dvcc.OCC, 3)])
def test_epoch_group_retries(cc, world):
    """dv_epoch_group_carry: closed-loop epoch groups -- rank r's txns aborted
    in epoch e of group g open its batch of epoch e of group g + 1, in order,
    ahead of new txns (a penalty of one group), built on the device from the
    group's commit bytes.  Every epoch of three groups equals the oracle over
    the same sequenced epochs, and the carried batches equal the host rule."""
    rows_pp, n_txn = 1 << 13, 1500
    gen = dvcc.YCSBQueryGenerator(rows_pp * world, part_cnt=world, zipf_theta=0.9, txn_write_perc=1.0,
                                  tup_write_perc=0.5, part_per_txn=2, strict_ppt=1, mpr=0.3)
    engines = _engine_group(cc, world, rows_pp, n_txn, mode=2)
    tab = O.YcsbTable(rows_pp * world)
    f0 = tab.f0.copy()
    # group 0: all new txns
    host = [[gen.gen(n_txn, dvcc.epoch_seed(r, 70 + e), r) for e in range(world)] for r in range(world)]
    dev = [[dvcc.DeviceEpoch(b) for b in host[r]] for r in range(world)]
    carried_total = 0
    for g in range(3):
        refs = []
        for e in range(world):
            q = dvcc.sequence([host[r][e] for r in range(world)])
            c_ref, _, st_ref = O.epoch_run(ORACLE_CC.get(cc, O.CALVIN), tab.ix, f0, q.n_txn, q.txn_begin, q.keys,
                                           q.types)
            refs.append((c_ref, st_ref))
        res = _run_group_epochs(engines, dev, n_txn)
        for r, x in enumerate(res):
            assert not isinstance(x, Exception), f"group {g} rank {r}: {x}"
            c, st = x
            for e in range(world):
                assert (c[e * n_txn:e * n_txn + host[r][e].n_txn] ==
                        refs[e][0][r * n_txn:r * n_txn + host[r][e].n_txn]).all(), f"group {g} epoch {e} rank {r}"
            assert st.committed == sum(s.committed for _, s in refs)
        for p, eng in enumerate(engines):
            assert (eng.read_table(0, rows_pp) == f0[p::world]).all(), f"group {g} partition {p} table"
        # the next group's batches: this group's aborts first, then new txns
        nhost, ndev = [], []
        for r in range(world):
            d_commit = torch.from_numpy(res[r][0]).cuda()
            carried = engines[r].group_carry(dev[r], d_commit, n_txn)
            hb, db = [], []
            for e in range(world):
                hc = _host_carry(host[r][e], res[r][0][e * n_txn:(e + 1) * n_txn], n_txn)
                dc = carried[e]
                assert (dc.n_txn, dc.n_acc) == (hc.n_txn, hc.n_acc), f"group {g} rank {r} epoch {e}"
                assert np.array_equal(dc.keys.cpu().numpy().view(np.uint64), hc.keys)
                assert np.array_equal(dc.types.cpu().numpy(), hc.types)
                assert np.array_equal(dc.acc_txn.cpu().numpy().view(np.uint32), hc.acc_txn())
                carried_total += hc.n_txn
                new = gen.gen(n_txn - hc.n_txn, dvcc.epoch_seed(r, 80 + g * world + e), r)
                hb.append(_host_concat(hc, new))
                db.append(dvcc.DeviceEpoch.concat(dc, dvcc.DeviceEpoch(new)) if hc.n_txn else dvcc.DeviceEpoch(new))
            nhost.append(hb)
            ndev.append(db)
        host, dev = nhost, ndev
    assert carried_total > 0
    for eng in engines:
        eng.close()


# ---- epoch groups over ordered lanes (dv_lanes_order): each rank runs L
# contexts over its partition's tables, each with its own communicator and
# host thread; group g is decided on lane g % L and the groups execute in
# group order on every partition
def _check_epoch_groups_lanes(cc, world, rows_pp, n_txn, mpr, groups, lanes, theta=0.9, bad_group=None):
    import threading
    R = 10
    gen = dvcc.YCSBQueryGenerator(rows_pp * world, part_cnt=world, zipf_theta=theta, txn_write_perc=1.0,
                                  tup_write_perc=0.5, part_per_txn=2, strict_ppt=1, mpr=mpr)
    owners = []
    for p in range(world):
        eng = dvcc.CCEngine(cc, n_txn * world, n_txn * world * R + 4096, part_cnt=world, part_id=p,
                            asynchronous=False)
        eng.load_ycsb_partition(rows_pp)
        owners.append(eng)
    ctxs = [[o] + [o.open_lane() for _ in range(lanes - 1)] for o in owners]  # [rank][lane]
    for ln in range(lanes):
        dvcc.CCEngine.comm_init_local([ctxs[r][ln] for r in range(world)])
        for r in range(world):
            ctxs[r][ln].comm_set_mode(2)
    for r in range(world):
        ctxs[r][0].lanes_order(ctxs[r][1:])
    tab = O.YcsbTable(rows_pp * world)
    f0 = tab.f0.copy()
    homes = [[] for _ in range(world)]  # [rank][group][epoch]
    refs = []                           # [group][epoch] (commit bytes, stats)
    for g in range(groups):
        hg = [[None] * world for _ in range(world)]
        rg = []
        for e in range(world):
            batches = [gen.gen(n_txn, dvcc.epoch_seed(r, 60 + g * world + e), r) for r in range(world)]
            if bad_group == g and e == 1:
                batches[0].keys[5] = np.uint64(rows_pp * world + 7)
            q = dvcc.sequence(batches)
            if bad_group is None or g < bad_group:
                c_ref, _, st_ref = O.epoch_run(ORACLE_CC.get(cc, O.CALVIN), tab.ix, f0, q.n_txn, q.txn_begin,
                                               q.keys, q.types)
                rg.append((c_ref, st_ref))
            for r in range(world):
                hg[r][e] = dvcc.DeviceEpoch(batches[r])
        for r in range(world):
            homes[r].append(hg[r])
        refs.append(rg)
    out = {}

    def body(r, ln):
        mine = list(range(ln, groups, lanes))
        try:
            ds = [torch.zeros(n_txn * world, dtype=torch.uint8, device="cuda") for _ in mine]
            sts = ctxs[r][ln].run_epoch_groups([homes[r][g] for g in mine], n_txn, ds)
            torch.cuda.synchronize()
            for g, d, st in zip(mine, ds, sts):
                out[(r, g)] = (d.cpu().numpy(), st)
        except Exception as ex:  # noqa: BLE001 -- reported per rank and lane
            out[(r, "err", ln)] = ex
    th = [threading.Thread(target=body, args=(r, ln)) for r in range(world) for ln in range(lanes)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
        assert not t.is_alive(), "a lane hung in the ordered epoch groups"
    try:
        if bad_group is not None:
            errs = [v for k, v in out.items() if len(k) == 3]
            assert errs and all(isinstance(x, dvcc.DvccError) for x in errs), out
            # groups before the failing one are applied on every partition, nothing after them
            for p, eng in enumerate(owners):
                assert (eng.read_table(0, rows_pp) == f0[p::world]).all(), f"partition {p} table"
            # the order has ended: a later call on any lane returns DV_ERR_STATE
            # and changes no row (the failed ticket itself never executes)
            again = {}

            def body2(r, ln):
                try:
                    d = torch.zeros(n_txn * world, dtype=torch.uint8, device="cuda")
                    again[(r, ln)] = ctxs[r][ln].run_epoch_groups([homes[r][0]], n_txn, [d])
                except Exception as ex:  # noqa: BLE001 -- reported per rank and lane
                    again[(r, ln)] = ex
            th = [threading.Thread(target=body2, args=(r, ln)) for r in range(world) for ln in range(lanes)]
            for t in th:
                t.start()
            for t in th:
                t.join(timeout=300)
                assert not t.is_alive(), "a lane hung after the order ended"
            for k, x in again.items():
                assert isinstance(x, dvcc.DvccError) and x.code == dvcc._lib.DV_ERR_STATE, (k, x)
            for p, eng in enumerate(owners):
                assert (eng.read_table(0, rows_pp) == f0[p::world]).all(), f"partition {p} table after"
            return
        assert not [k for k in out if len(k) == 3], {k: v for k, v in out.items() if len(k) == 3}
        for g in range(groups):
            committed = sum(st.committed for _, st in refs[g])
            digest = writes = 0
            for r in range(world):
                cs, st = out[(r, g)]
                for e in range(world):
                    assert (cs[e * n_txn:(e + 1) * n_txn] == refs[g][e][0][r * n_txn:(r + 1) * n_txn]).all(), \
                        f"group {g} epoch {e} rank {r}"
                assert st.committed == committed
                digest = (digest + st.read_digest) % (1 << 64)
                writes += st.write_cnt
            assert digest == sum(st.read_digest for _, st in refs[g]) % (1 << 64), f"group {g} digest"
            assert writes == sum(st.write_cnt for _, st in refs[g]), f"group {g} writes"
        for p, eng in enumerate(owners):
            assert (eng.read_table(0, rows_pp) == f0[p::world]).all(), f"partition {p} table"
    finally:
        for o in owners:
            o.close()


@pytest.mark.gpu
@pytest.mark.parametrize("cc,world,lanes", [(dvcc.NO_WAIT, 2, 2), (dvcc.WAIT_DIE, 2, 4), (dvcc.OCC, 4, 2),
                                            (dvcc.CALVIN, 2, 2)])
def test_epoch_groups_ordered_lanes(cc, world, lanes):
    """Epoch groups over ordered lanes: groups decided concurrently on L
    contexts per rank (each with its own communicator and host thread),
    executed in group order on every partition -- every group's commit
    bytes, digests and writes, and every partition's rows, equal the oracle
    running all the epochs in sequence."""
    _check_epoch_groups_lanes(cc, world, 1 << 13, 2000, 0.3, groups=2 * lanes + 1, lanes=lanes)


@pytest.mark.gpu
def test_epoch_groups_ordered_lanes_failure():
    """A bad key in group 2 of 6 over two ordered lanes: that lane returns
    DV_ERR_KEY_NOT_FOUND on every rank, the other lane stops at its next
    turn (DV_ERR_STATE) instead of waiting for ever, and only groups 0 and 1
    reach the rows; calling the lanes again afterwards returns DV_ERR_STATE
    and changes nothing."""
    _check_epoch_groups_lanes(dvcc.NO_WAIT, 2, 1 << 13, 2000, 0.3, groups=6, lanes=2, bad_group=2)


# ---- the per-epoch partitioned driver (dv_epoch_run_part) over ordered lanes
@pytest.mark.gpu
@pytest.mark.parametrize("cc,mode,lanes", [(dvcc.NO_WAIT, 1, 2), (dvcc.WAIT_DIE, 2, 2), (dvcc.OCC, 1, 3),
                                           (dvcc.CALVIN, 1, 2)])
def test_part_epochs_ordered_lanes(cc, mode, lanes):
    """dv_epoch_run_part over ordered lanes (list protocol, mode 1, or
    replicated, mode 2): epoch k on lane k % L of every rank, each lane with
    its own communicator and host thread, executions in epoch order -- every
    epoch's commit bytes and the partitions' rows equal the oracle running
    the sequenced epochs one after the other."""
    import threading
    world, rows_pp, n_txn, R, epochs = 2, 1 << 13, 1500, 10, 2 * lanes + 1
    gen = dvcc.YCSBQueryGenerator(rows_pp * world, part_cnt=world, zipf_theta=0.9, txn_write_perc=1.0,
                                  tup_write_perc=0.5, part_per_txn=2, strict_ppt=1, mpr=0.3)
    owners = []
    for p in range(world):
        cap = n_txn * world * R + 4096
        eng = dvcc.CCEngine(cc, n_txn * world, cap, part_cnt=world, part_id=p, asynchronous=False)
        eng.load_ycsb_partition(rows_pp)
        owners.append(eng)
    ctxs = [[o] + [o.open_lane() for _ in range(lanes - 1)] for o in owners]
    for ln in range(lanes):
        dvcc.CCEngine.comm_init_local([ctxs[r][ln] for r in range(world)])
        for r in range(world):
            ctxs[r][ln].comm_set_mode(mode)
    for r in range(world):
        ctxs[r][0].lanes_order(ctxs[r][1:])
    tab = O.YcsbTable(rows_pp * world)
    f0 = tab.f0.copy()
    batches, refs = [], []
    for k in range(epochs):
        b = [gen.gen(n_txn, dvcc.epoch_seed(r, 80 + k), r) for r in range(world)]
        q = dvcc.sequence(b)
        c_ref, _, st_ref = O.epoch_run(ORACLE_CC.get(cc, O.CALVIN), tab.ix, f0, q.n_txn, q.txn_begin, q.keys,
                                       q.types)
        batches.append([dvcc.DeviceEpoch(x) for x in b])
        refs.append((c_ref, st_ref))
    res = [None] * world

    def rank_body(r):
        try:
            ds = [torch.zeros(n_txn * world, dtype=torch.uint8, device="cuda") for _ in range(epochs)]
            sts = owners[r].run_ordered(epochs, lambda ctx, i: ctx.run_epoch_part(batches[i][r], n_txn, ds[i]))
            torch.cuda.synchronize()
            res[r] = ([d.cpu().numpy() for d in ds], sts)
        except Exception as ex:  # noqa: BLE001 -- reported per rank
            res[r] = ex
    th = [threading.Thread(target=rank_body, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
        assert not t.is_alive(), "a rank hung in the ordered partitioned epochs"
    try:
        for r, x in enumerate(res):
            assert not isinstance(x, Exception), f"rank {r}: {x}"
        for k, (c_ref, st_ref) in enumerate(refs):
            digest = writes = 0
            for r in range(world):
                cs, sts = res[r]
                assert (cs[k] == c_ref).all(), f"epoch {k} rank {r}"
                assert sts[k].committed == st_ref.committed, f"epoch {k} rank {r}"
                digest = (digest + sts[k].read_digest) % (1 << 64)
                writes += sts[k].write_cnt
            assert digest == st_ref.read_digest and writes == st_ref.write_cnt, f"epoch {k}"
        for p, eng in enumerate(owners):
            assert (eng.read_table(0, rows_pp) == f0[p::world]).all(), f"partition {p} table"
    finally:
        for o in owners:
            o.close()
