"""Deneva wire format in and out of the engine (include/dvcc.h, dv_wire_*).

A server node's ingress of its clients' message batches -- the mbufs runcl's
MessageThread sends (transport/msg_thread.cpp:53-111): CL_QRY messages of
YCSBClientQueryMessage / TPCCClientQueryMessage (transport/message.cpp:
451-687, 856-916), or under CALVIN the sequencer's forwarded CL_QRY batches
ended by RDONE -- decoded by libdvcc straight into the host arrays of an
epoch, and the replies (CL_RSP to the clients, CALVIN_ACK to the sequencers)
packed the same way from the epoch's commit bytes.
"""
import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib as L
from .engine import Epoch, _ptr


@dataclass
class WireEpoch(Epoch):
    """An epoch decoded from batches, with what the replies need."""
    args: np.ndarray = None            # TPC-C operation words
    txn_type: np.ndarray = None        # TPC-C: 1 Payment, 2 NewOrder
    owner: np.ndarray = None           # partition of every access
    txn_id: np.ndarray = None          # uint64 [n_txn]
    client_startts: np.ndarray = None  # uint64 [n_txn]
    return_node: np.ndarray = None     # uint32 [n_txn]: client (CALVIN: sequencer)
    batch_id: int = None               # CALVIN
    rdone: int = 0                     # CALVIN: RDONEs taken for batch_id


class WireIngress:
    """dv_wire_open / dv_wire_decode / dv_wire_respond over host buffers of
    max_txn txns and max_acc accesses.  feed(batch) decodes a received batch
    (bytes); whenever the current epoch cannot take the next message (full,
    or a CALVIN message of a later batch) it is closed and queued, and
    decoding goes on into a fresh one.  take() closes the current epoch
    early; ready holds the closed ones."""

    def __init__(self, workload, max_txn, max_acc, node_id=0, node_cnt=1, part_cnt=1, synth_table_size=0,
                 calvin=False, tpcc=None, max_req=0):
        self.cfg = L.WireCfg(workload, 1 if calvin else 0, node_id, node_cnt, part_cnt, max_req, synth_table_size,
                             ctypes.pointer(tpcc) if tpcc is not None else None)
        self._tpcc = tpcc
        self.workload = workload
        self.max_txn, self.max_acc = max_txn, max_acc
        self.ready = []
        self._bufs = self._alloc()
        self.ep = L.WireEpoch()
        self._bind()
        L.check(L.lib().dv_wire_epoch_reset(ctypes.byref(self.ep)), "dv_wire_epoch_reset")

    def _alloc(self):
        tp = self.workload == L.TPCC
        A, T = self.max_acc, self.max_txn
        return dict(keys=np.zeros(A, np.uint64), types=np.zeros(A, np.uint8), txn_begin=np.zeros(T + 1, np.uint32),
                    tables=np.zeros(A, np.uint8) if tp else None, args=np.zeros(A, np.uint64) if tp else None,
                    txn_type=np.zeros(T, np.uint8) if tp else None, owner=np.zeros(A, np.uint8),
                    txn_id=np.zeros(T, np.uint64), client_startts=np.zeros(T, np.uint64),
                    return_node=np.zeros(T, np.uint32))

    def _bind(self):
        self.ep.max_txn, self.ep.max_acc = self.max_txn, self.max_acc
        for k, v in self._bufs.items():
            setattr(self.ep, k, None if v is None else v.ctypes.data)

    def _close(self):
        b, e = self._bufs, self.ep
        n, a = e.n_txn, e.n_acc
        cut = lambda x, m: None if x is None else x[:m].copy()  # noqa: E731
        out = WireEpoch(cut(b["keys"], a), cut(b["types"], a), b["txn_begin"][:n + 1].copy(),
                        cut(b["tables"], a), args=cut(b["args"], a), txn_type=cut(b["txn_type"], n),
                        owner=cut(b["owner"], a), txn_id=cut(b["txn_id"], n),
                        client_startts=cut(b["client_startts"], n), return_node=cut(b["return_node"], n),
                        batch_id=None if e.batch_id == (1 << 64) - 1 else int(e.batch_id), rdone=int(e.rdone))
        L.check(L.lib().dv_wire_epoch_reset(ctypes.byref(e)), "dv_wire_epoch_reset")
        return out

    def feed(self, batch):
        """Decodes one received batch; returns the epochs it closed."""
        buf = np.frombuffer(bytes(batch), dtype=np.uint8)
        cur = L.WireCursor()
        L.check(L.lib().dv_wire_open(ctypes.byref(self.cfg), _ptr(buf), len(buf), ctypes.byref(cur)), "dv_wire_open")
        closed = []
        while True:
            rc = L.lib().dv_wire_decode(ctypes.byref(self.cfg), ctypes.byref(cur), ctypes.byref(self.ep))
            if rc == L.WIRE_MORE:
                closed.append(self._close())
                continue
            L.check(rc, "dv_wire_decode")
            break
        self.ready.extend(closed)
        return closed

    def feed_many(self, batches):
        """Decodes a list of received batches with one call per epoch
        (dv_wire_decode_batches); returns the epochs it closed."""
        if not batches:
            return []
        off = np.zeros(len(batches) + 1, np.uint64)
        off[1:] = np.cumsum([len(b) for b in batches])
        buf = np.frombuffer(b"".join(bytes(b) for b in batches), dtype=np.uint8)
        return self.feed_buffer(buf, off)

    def feed_buffer(self, buf, off):
        """The same over batches already back to back in one uint8 array,
        batch b at buf[off[b]:off[b + 1]]."""
        cur = L.WireCursor()
        nxt = ctypes.c_uint32(0)
        closed = []
        while True:
            rc = L.lib().dv_wire_decode_batches(ctypes.byref(self.cfg), _ptr(buf), _ptr(off), len(off) - 1,
                                                ctypes.byref(cur), ctypes.byref(nxt), ctypes.byref(self.ep))
            if rc == L.WIRE_MORE:
                closed.append(self._close())
                continue
            L.check(rc, "dv_wire_decode_batches")
            break
        self.ready.extend(closed)
        return closed

    def take(self):
        """Closes and returns the epoch being filled."""
        return self._close()

    def _hdr(self):  # Message::mget_size (message.cpp:196-209)
        return 4 + 8 + (8 if self.cfg.calvin else 0) + 8 + 7 * 8

    def respond(self, ep, commit=None):
        """The replies to a decoded epoch as a list of batches (bytes):
        CL_RSP for every committed txn (commit bytes), or under CALVIN a
        CALVIN_ACK for every txn."""
        n = ep.n_txn
        e = L.WireEpoch()
        e.n_txn, e.max_txn = n, n
        e.batch_id = (1 << 64) - 1 if ep.batch_id is None else ep.batch_id
        tid = np.ascontiguousarray(ep.txn_id, np.uint64)
        cst = np.ascontiguousarray(ep.client_startts, np.uint64)
        rn = np.ascontiguousarray(ep.return_node, np.uint32)
        e.txn_id, e.client_startts, e.return_node = tid.ctypes.data, cst.ctypes.data, rn.ctypes.data
        cm = None if commit is None else np.ascontiguousarray(np.asarray(commit)[:n], np.uint8)
        # (a batch holds (MSG_MAX - 12) // message size replies; one partial batch per destination)
        per = (L.WIRE_MSG_MAX - L.WIRE_HDR) // (self._hdr() + (4 if self.cfg.calvin else 8))
        max_b = n // per + len(np.unique(rn)) + 1
        out = np.zeros(max_b * L.WIRE_MSG_MAX, np.uint8)
        off = np.zeros(max_b + 1, np.uint64)
        nb = ctypes.c_uint32()
        L.check(L.lib().dv_wire_respond(ctypes.byref(self.cfg), ctypes.byref(e), _ptr(cm), _ptr(out), len(out),
                                        _ptr(off), max_b, ctypes.byref(nb)), "dv_wire_respond")
        return [out[int(off[b]):int(off[b + 1])].tobytes() for b in range(nb.value)]


def tpcc_gen_queries(p, n_txn, seed, home_part=0):
    """dv_tpcc_gen_queries: the client queries of dv_tpcc_gen (same draws)."""
    q = (L.TpccQuery * max(1, n_txn))()
    L.check(L.lib().dv_tpcc_gen_queries(ctypes.byref(p), seed, home_part, n_txn, q), "dv_tpcc_gen_queries")
    return q
