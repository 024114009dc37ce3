"""Partitioned epochs across the GPUs of one node.

One process per GPU; rank r owns partition r (PART_CNT == world size,
GET_NODE_ID(part) == part, system/global.h:294).  Per epoch:

1. every rank holds the accesses of its own client batch (its "home" txns),
   grouped by owner rank = key % PART_CNT (YCSBWorkload::key_to_part,
   benchmarks/ycsb_wl.cpp:69-74) -- the host does this split;
2. one all-to-all moves each fragment to its owner -- it replaces RQRY
   messages through msg_queue/nanomsg (ycsb_txn.cpp:160-175,
   system/msg_queue.cpp, transport/transport.cpp:224-304);
3. received fragments are concatenated in origin order, which *is* Calvin's
   global lock order (epoch, origin node, position) (work_queue.cpp:105-151),
   so the owner sorts them stably by row;
4. NO_WAIT / WAIT_DIE / OCC: decision rounds; after each local round the
   verdict bytes of the still-undecided txns are combined with an
   all-reduce(MAX), which is the vote combine of TxnManager::received_response
   (system/txn.cpp:544-554) applied to every open txn of the epoch at once;
   CALVIN needs no votes.  Every rank holds the same statuses, hence the same
   ascending list of undecided txns: the bytes travel in list order, so the
   all-reduce shrinks with the list.  The host runs LAG rounds ahead of the
   outcomes it reads (rounds past the fixpoint are no-ops), sizing each
   all-reduce by the list length of LAG - 1 rounds earlier -- the same number
   on every rank;
5. every rank executes the committed accesses on its own rows.

Errors are collective: after the probe, one all-reduce(MAX) of every
partition's input-error bits (missing key, bad txn order, ...) makes every
rank treat the epoch as rejected, so all of them raise at the same round --
none is left waiting in a collective the others never reach.  The round loop's
other exits (stalled rounds) depend only on the combined verdicts, which are
identical on every rank.

Decisions are identical to the single-thread E-schedule over the whole
epoch, whatever the number of GPUs.

The collectives go through torch.distributed: backend "nccl" is RCCL over
xGMI on the GPU box; "gloo" runs the same protocol on CPU tensors in tests.
"""
import numpy as np
import torch
import torch.distributed as dist

from .engine import Epoch


def owner_order(epoch, world):
    """Owner rank of every access and the stable order grouping them by owner.
    YCSB: key % PART_CNT (ycsb_wl.cpp:69-74); TPC-C epochs carry the owner
    (wh_to_part of the access's warehouse, tpcc_helper.cpp:161-164)."""
    own = getattr(epoch, "owner", None)
    if own is not None:
        owner = own.astype(np.int64)
    else:
        owner = (epoch.keys % np.uint64(world)).astype(np.int64)
    return owner, np.argsort(owner, kind="stable")


def split_by_owner(epoch, txn_base, world, txn_stride=1):
    """Host-side split of one origin batch into per-owner fragments.

    Returns (keys, types, txn, counts): arrays ordered by owner rank and, inside
    an owner, by (txn, request position); txn is the global sequence number
    local txn index * txn_stride + txn_base (origin-major: stride 1, base
    rank * txns_per_rank; position-major: stride world, base rank)."""
    owner, order = owner_order(epoch, world)
    txn = epoch.acc_txn().astype(np.int64) * txn_stride + txn_base
    counts = np.bincount(owner, minlength=world)
    return (epoch.keys[order], epoch.types[order], txn[order].astype(np.int32), counts)


class PartitionedEpoch:
    """One rank's outgoing fragments of one epoch, resident on `device`.
    TPC-C epochs also carry each access's table and operation word.
    position: the origins' batches sequenced txn by txn (origin q's txn j is
    sequence number j * world + q, as DV_COMM_POSITION_ORDER in the engine's
    own drivers) instead of origin after origin."""

    def __init__(self, batch, rank, world, txns_per_rank, device, position=False):
        self.position = bool(position) and world > 1
        self.world, self.txns_per_rank = world, txns_per_rank
        if self.position:
            k, t, x, counts = split_by_owner(batch, rank, world, txn_stride=world)
        else:
            k, t, x, counts = split_by_owner(batch, rank * txns_per_rank, world)
        self.send_counts = [int(c) for c in counts]
        self.keys = torch.from_numpy(k.view(np.int64)).to(device)
        self.types = torch.from_numpy(t).to(device)
        self.txn = torch.from_numpy(x).to(device)
        self.tables = self.args = None
        if getattr(batch, "args", None) is not None:
            _, order = owner_order(batch, world)
            self.tables = torch.from_numpy(batch.tables[order]).to(device)
            self.args = torch.from_numpy(batch.args[order].view(np.int64)).to(device)
        self.n_txn_global = txns_per_rank * world
        self.max_txn_acc = batch.max_txn_acc()


class PartitionedRunner:
    """Runs epochs over `engine`, a CC engine bound to this rank's partition
    (CCEngine on the GPU; a test double on CPU)."""

    LAG = 2  # rounds enqueued ahead of the outcome the host reads

    def __init__(self, engine, world, rank, group=None, device="cuda"):
        self.engine = engine
        self.world, self.rank, self.group = world, rank, group
        self.device = device

    def exchange_counts(self, pe):
        send = torch.tensor(pe.send_counts, dtype=torch.int64, device=self.device)
        recv = torch.empty_like(send)
        dist.all_to_all_single(recv, send, group=self.group)
        return [int(c) for c in recv.cpu().tolist()]

    def exchange(self, pe, recv_counts):
        """All-to-all of the access fragments (keys, types, global txn; TPC-C:
        tables and operation words too)."""
        n = sum(recv_counts)
        out = []
        cols = [(pe.keys, torch.int64), (pe.types, torch.uint8), (pe.txn, torch.int32)]
        if pe.args is not None:
            cols += [(pe.tables, torch.uint8), (pe.args, torch.int64)]
        for src, dt in cols:
            dst = torch.empty(n, dtype=dt, device=self.device)
            dist.all_to_all_single(dst, src, output_split_sizes=recv_counts,
                                   input_split_sizes=pe.send_counts, group=self.group)
            out.append(dst)
        return out

    def run(self, pe, recv_counts=None, commit=None):
        """One partitioned epoch.  Returns (stats of this rank, rounds)."""
        if recv_counts is None:
            recv_counts = self.exchange_counts(pe)
        cols = self.exchange(pe, recv_counts)
        if getattr(pe, "position", False):
            # each origin's fragment holds its txns' accesses in order, ids
            # j * world + q rising: a stable sort by id merges them into the
            # sequence order (the engine's drivers interleave the same way)
            order = torch.sort(cols[2], stable=True).indices
            cols = [c[order] for c in cols]
        n_txn = pe.n_txn_global
        extra = {"tables": cols[3], "args": cols[4]} if len(cols) > 3 else {}
        self.engine.begin_partition(*cols[:3], n_txn, max_txn_acc=pe.max_txn_acc, **extra)
        err = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.engine.errors_local(err)
        dist.all_reduce(err, op=dist.ReduceOp.MAX, group=self.group)
        self.engine.errors_combined(err)
        rounds = 0
        if self.engine.needs_votes:
            verdict = torch.zeros((n_txn + 3) // 4 * 4, dtype=torch.uint8, device=self.device)
            counts = [n_txn]  # counts[k]: list length entering round k (known rounds)
            r = 0
            while counts[-1] > 0:
                # round r's list is no longer than the last one known
                self.engine.round_local(verdict)
                dist.all_reduce(verdict[:counts[-1]], op=dist.ReduceOp.MAX, group=self.group)
                self.engine.round_apply(verdict, wait=False)
                r += 1
                if r >= self.LAG:
                    und = self.engine.round_wait(r - self.LAG)
                    if und >= counts[-1] > 0:  # every round decides the lowest undecided txn
                        raise RuntimeError(f"decision rounds stalled at {und} undecided txns")
                    counts.append(und)
            rounds = len(counts) - 1
        if not getattr(pe, "position", False):
            return self.engine.finish(commit), rounds
        # position-major: the decisions (and TPC-C's o_id) are per sequence
        # number; they go back to origin order, origin q's txn j at q * tpr + j
        tpr, world = pe.txns_per_rank, pe.world
        seq = None if commit is None else torch.zeros_like(commit[:n_txn])
        st = self.engine.finish(seq)
        if commit is not None:
            commit[:n_txn] = seq.view(tpr, world).t().reshape(-1)
        oid = getattr(self.engine, "oid", None)
        if oid is not None:
            self.engine.oid = oid[:n_txn].view(tpr, world).t().reshape(-1).clone()
        return st, rounds


class EnginePartition:
    """Gives CCEngine the partition interface PartitionedRunner drives.  The
    engine is bound to torch's current stream (dv_set_stream), so its kernels,
    the RCCL collectives and torch's own copies are ordered on one stream."""

    def __init__(self, engine):
        self.engine = engine
        self.needs_votes = engine.cc_alg != 10  # CALVIN has no votes
        engine.set_stream(torch.cuda.current_stream().cuda_stream)

    def begin_partition(self, keys, types, txn, n_txn, max_txn_acc=0, tables=None, args=None):
        """TPC-C (args given): dv_tpcc_epoch_begin; the o_id of committed
        NewOrders whose district is on this partition land in self.oid."""
        from .engine import DeviceEpoch
        self._dep = DeviceEpoch.from_tensors(keys, types, txn, n_txn, tables=tables, max_txn_acc=max_txn_acc)
        if args is not None:
            self.oid = torch.zeros(max(1, n_txn), dtype=torch.int64, device=keys.device)
            self._args = args
            self.engine.begin_tpcc(self._dep, args, self.oid)
        else:
            self.engine.begin(self._dep)

    def errors_local(self, word):
        self.engine.errors_local(word)

    def errors_combined(self, word):
        self.engine.errors_combined(word)

    def round_local(self, verdict):
        self.engine.round_local(verdict)

    def round_apply(self, verdict, wait=True):
        return self.engine.round_apply(verdict, wait=wait)

    def round_wait(self, r):
        return self.engine.round_wait(r)

    def finish(self, commit=None):
        return self.engine.finish(commit)


__all__ = ["owner_order", "split_by_owner", "PartitionedEpoch", "PartitionedRunner", "EnginePartition", "Epoch"]
