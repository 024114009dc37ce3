"""Test infrastructure: an encoder / decoder of Deneva's message batches
written from the reference's copy_to_buf field order, independent of the
product's decoder (deneva-plus_amd/csrc/wire.cpp), to check it.

Layout (transport/message.cpp; COPY_BUF = memcpy of sizeof(field), fields back
to back, system/helper.h:163-165; x86-64 sizes):
  batch (mbuf, msg_thread.h:24-62; MessageThread::send_batch,
         msg_thread.cpp:53-73): u32 dest, u32 src, u32 count, messages
  Message::mcopy_to_buf (248-270): u32 rtype, u64 txn_id, [CALVIN u64 batch_id],
         u64 mq_time, 7 x f64 latency
  ClientQueryMessage::copy_to_buf (905-916): u64 client_startts, size_t n, n x u64
  YCSBClientQueryMessage::copy_to_buf (512-526): size_t n, n x ycsb_request
         (u32 acctype, 4 pad, u64 key, char value, 7 pad: ycsb_query.h:35-50)
  TPCCClientQueryMessage::copy_to_buf (657-687): 7 x u64 (txn_type, w_id,
         d_id, c_id, d_w_id, c_w_id, c_d_id), char c_last[16], u64 h_amount,
         bool by_last_name, size_t n, n x Item_no (3 x u64), bool rbk, bool
         remote, u64 ol_cnt, u64 o_entry_d
  DoneMessage (973-977): the header alone
  ClientResponseMessage (944-949): header + u64 client_startts
  AckMessage: header + RC (u32)
Parity unpinned: the reference's transport cannot be built or run here
(SURVEY.md 8c); this restates the source text's field order.
"""
import struct

import numpy as np

CL_QRY, RDONE, CL_RSP, CALVIN_ACK = 3, 19, 20, 24
MSG_MAX = 4096
U64_MAX = (1 << 64) - 1


def header(rtype, txn_id=U64_MAX, batch_id=None, mq_time=0, lat=(0.0,) * 7):
    b = struct.pack("<IQ", rtype, txn_id)
    if batch_id is not None:  # CC_ALG == CALVIN (message.cpp:252-254)
        b += struct.pack("<Q", batch_id)
    return b + struct.pack("<Q", mq_time) + struct.pack("<7d", *lat)


def client_part(client_startts, partitions):
    return struct.pack("<QQ", client_startts, len(partitions)) + b"".join(struct.pack("<Q", p) for p in partitions)


def ycsb_query(reqs, partitions, client_startts=0, txn_id=U64_MAX, batch_id=None, value=0x5A):
    """reqs: [(acctype, key)]; value: ycsb_request::value (never read)."""
    body = struct.pack("<Q", len(reqs)) + b"".join(struct.pack("<I4xQB7x", a, k, value) for a, k in reqs)
    return header(CL_QRY, txn_id, batch_id) + client_part(client_startts, partitions) + body


def tpcc_query(q, client_startts=0, txn_id=U64_MAX, batch_id=None):
    """q: dict of TPCCClientQueryMessage fields; items [(i_id, supply_w, qty)]."""
    items = q.get("items", [])
    body = struct.pack("<7Q", q["txn_type"], q["w_id"], q["d_id"], q.get("c_id", 0), q.get("d_w_id", 0),
                       q.get("c_w_id", 0), q.get("c_d_id", 0))
    body += q.get("c_last", b"").ljust(16, b"\0")[:16]
    body += struct.pack("<Q?", q.get("h_amount", 0), bool(q.get("by_last_name", False)))
    body += struct.pack("<Q", len(items)) + b"".join(struct.pack("<3Q", *it) for it in items)
    body += struct.pack("<??QQ", bool(q.get("rbk", False)), bool(q.get("remote", False)), q.get("ol_cnt", 0),
                        q.get("o_entry_d", 0))
    return header(CL_QRY, txn_id, batch_id) + client_part(client_startts, q.get("parts", [])) + body


def rdone(batch_id):
    return header(RDONE, U64_MAX, batch_id)


def batches(dest, src, msgs, limit=MSG_MAX):
    """MessageThread::run: a message goes into the destination's mbuf; when it
    does not fit, the mbuf is sent first (msg_thread.cpp:90-103)."""
    out, cur = [], []
    size = 12
    for m in msgs:
        if size + len(m) > limit:
            out.append(struct.pack("<III", dest, src, len(cur)) + b"".join(cur))
            cur, size = [], 12
        cur.append(m)
        size += len(m)
    if cur:
        out.append(struct.pack("<III", dest, src, len(cur)) + b"".join(cur))
    return out


def ycsb_epoch_messages(ep, part_cnt=1, client_startts=None, batch_id=None, txn_ids=None):
    """One CL_QRY per txn of an Epoch (keys / types / txn_begin), partitions as
    YCSBQuery's std::set of key_to_part (ascending)."""
    tb = ep.txn_begin
    out = []
    for t in range(ep.n_txn):
        a, b = int(tb[t]), int(tb[t + 1])
        reqs = [(int(ep.types[i]), int(ep.keys[i])) for i in range(a, b)]
        parts = sorted({k % part_cnt for _, k in reqs})
        cst = t if client_startts is None else int(client_startts[t])
        out.append(ycsb_query(reqs, parts, cst, U64_MAX if txn_ids is None else int(txn_ids[t]), batch_id))
    return out


def ycsb_epoch_buffer_np(ep, dest, src, client_startts_base=0):
    """ycsb_epoch_batches_np's batches back to back in one uint8 array and
    their offsets (batch b at buf[off[b]:off[b + 1]]), as a receive queue
    holds them, without a bytes object per batch."""
    bs = ycsb_epoch_batches_np(ep, dest, src, client_startts_base)
    off = np.zeros(len(bs) + 1, np.uint64)
    off[1:] = np.cumsum([len(b) for b in bs])
    return np.frombuffer(b"".join(bs), np.uint8), off


def ycsb_epoch_batches_np(ep, dest, src, client_startts_base=0):
    """The same messages and batches for an epoch of equal-length txns on one
    partition (config D), built with numpy for a million txns: every message
    is the same size, so a batch holds (MSG_MAX - 12) // size of them."""
    R = int(ep.txn_begin[1] - ep.txn_begin[0]) if ep.n_txn else 0
    assert (np.diff(ep.txn_begin.astype(np.int64)) == R).all()
    req = np.dtype([("acc", "<u4"), ("pad", "<u4"), ("key", "<u8"), ("val", "u1"), ("pad2", "u1", (7,))])
    msg = np.dtype([("rtype", "<u4"), ("txn_id", "<u8"), ("mq", "<u8"), ("lat", "<f8", (7,)), ("cst", "<u8"),
                    ("np", "<u8"), ("part", "<u8"), ("nreq", "<u8"), ("req", req, (R,))], align=False)
    n = ep.n_txn
    m = np.zeros(n, dtype=msg)
    m["rtype"] = CL_QRY
    m["txn_id"] = U64_MAX
    m["cst"] = client_startts_base + np.arange(n, dtype=np.uint64)
    m["np"] = 1
    m["part"] = 0
    m["nreq"] = R
    m["req"]["acc"] = ep.types.reshape(n, R)
    m["req"]["key"] = ep.keys.reshape(n, R)
    per = (MSG_MAX - 12) // msg.itemsize
    raw = m.view(np.uint8).reshape(n, msg.itemsize)
    out = []
    for s in range(0, n, per):
        e = min(n, s + per)
        out.append(struct.pack("<III", dest, src, e - s) + raw[s:e].tobytes())
    return out


def parse_batch(batch, calvin=False):
    """(dest, src, [messages as dicts]) of a reply batch (CL_RSP / CALVIN_ACK)."""
    dest, src, cnt = struct.unpack_from("<III", batch, 0)
    off, msgs = 12, []
    for _ in range(cnt):
        rtype, txn_id = struct.unpack_from("<IQ", batch, off)
        off += 12
        m = {"rtype": rtype, "txn_id": txn_id}
        if calvin:
            (m["batch_id"],) = struct.unpack_from("<Q", batch, off)
            off += 8
        m["mq_time"] = struct.unpack_from("<Q", batch, off)[0]
        m["lat"] = struct.unpack_from("<7d", batch, off + 8)
        off += 64
        if rtype == CL_RSP:
            (m["client_startts"],) = struct.unpack_from("<Q", batch, off)
            off += 8
        elif rtype == CALVIN_ACK:
            (m["rc"],) = struct.unpack_from("<I", batch, off)
            off += 4
        else:
            raise ValueError(f"unexpected rtype {rtype}")
        msgs.append(m)
    assert off == len(batch), (off, len(batch))
    return dest, src, msgs
