// wire.cpp -- Deneva's message batches in and out of the engine's host epochs.
//
// Ingress: a batch as runcl's MessageThread sends it (transport/msg_thread.cpp:
// 53-111, mbuf in msg_thread.h:24-62) is decoded message by message straight
// into the epoch's host arrays -- what Message::create_messages (message.cpp:
// 29-50) + copy_from_buf (YCSB 493-510, TPC-C 620-655, ClientQueryMessage
// 889-903, Message header 224-246) + the txn managers' access lists do, without
// a Message object or a per-request allocation.  Egress: the epoch's outcome
// as the replies the reference's server sends (CL_RSP, worker_thread.cpp:152;
// CALVIN_ACK, 127-136), packed into mbufs the same way.
//
// Byte layout (COPY_VAL / COPY_BUF, system/helper.h:155-169: memcpy of
// sizeof(field), fields back to back, no alignment): see include/dvcc.h.  The
// reader below never dereferences a field in place (memcpy out of the byte
// stream), so unaligned offsets are fine.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#include "dvcc.h"

namespace {

constexpr uint64_t kU64Max = ~0ull;
constexpr uint32_t kMaxReq = 128;   // the engine's longest txn (kMaxPos)
constexpr uint64_t kYcsbReq = 24;   // sizeof(ycsb_request) on x86-64

// Message::mget_size (message.cpp:196-209): rtype, txn_id, [batch_id], mq_time, 7 doubles
uint64_t hdr_size(const dv_wire_cfg *c) { return 4 + 8 + (c->calvin ? 8 : 0) + 8 + 7 * 8; }

struct Reader {  // bounds-checked COPY_VAL over [p, end)
    const uint8_t *p, *end;
    bool ok = true;
    template <class T>
    T get() {
        T v{};
        if ((uint64_t)(end - p) < sizeof(T)) {
            ok = false;
            p = end;
            return v;
        }
        std::memcpy(&v, p, sizeof(T));
        p += sizeof(T);
        return v;
    }
    void skip(uint64_t n) {
        if ((uint64_t)(end - p) < n) {
            ok = false;
            p = end;
        } else {
            p += n;
        }
    }
};

struct Writer {  // COPY_BUF into [p, end)
    uint8_t *p;
    template <class T>
    void put(const T &v) {
        std::memcpy(p, &v, sizeof(T));
        p += sizeof(T);
    }
    void zeros(uint64_t n) {
        std::memset(p, 0, n);
        p += n;
    }
};

// one decoded message, checked, before it touches the epoch
struct Msg {
    uint32_t rtype = 0;
    uint64_t txn_id = kU64Max, batch_id = kU64Max, client_startts = 0;
    uint32_t n_acc = 0;
    const uint8_t *reqs = nullptr;  // YCSB: the request records
    dv_tpcc_query tq;               // TPC-C
};

// Message header + ClientQueryMessage part; false if malformed
bool read_client_part(const dv_wire_cfg *c, Reader &r, Msg &m, bool check) {
    m.rtype = r.get<uint32_t>();
    m.txn_id = r.get<uint64_t>();
    if (c->calvin) m.batch_id = r.get<uint64_t>();
    r.skip(8 + 7 * 8);  // mq_time, latency doubles (statistics)
    if (m.rtype == DV_WIRE_RDONE) return r.ok;
    if (m.rtype != DV_WIRE_CL_QRY) return false;  // (clients and sequencers send CL_QRY)
    m.client_startts = r.get<uint64_t>();
    const uint64_t np = r.get<uint64_t>();  // size_t partitions
    if (!r.ok || np > DV_TPCC_MAX_PARTS) return false;
    if (!check) {
        r.skip(np * 8);
        return r.ok;
    }
    for (uint64_t i = 0; i < np; i++) {
        const uint64_t part = r.get<uint64_t>();
        if (part >= c->part_cnt) return false;
    }
    return r.ok;
}

bool read_ycsb(const dv_wire_cfg *c, Reader &r, Msg &m, bool check) {
    const uint64_t n = r.get<uint64_t>();  // size_t requests
    const uint32_t lim = std::min<uint32_t>(c->max_req ? c->max_req : kMaxReq, kMaxReq);
    if (!r.ok || n > lim || (uint64_t)(r.end - r.p) < n * kYcsbReq) return false;
    m.reqs = r.p;
    m.n_acc = (uint32_t)n;
    for (uint64_t i = 0; check && i < n; i++) {
        uint32_t acctype;
        uint64_t key;
        std::memcpy(&acctype, r.p + i * kYcsbReq, 4);
        std::memcpy(&key, r.p + i * kYcsbReq + 8, 8);
        if (acctype > DV_WR || key >= c->synth_table_size) return false;  // RD / WR; assert(key < g_synth_table_size)
    }
    r.skip(n * kYcsbReq);
    return r.ok;
}

bool read_tpcc(Reader &r, Msg &m) {
    dv_tpcc_query &q = m.tq;
    std::memset(&q, 0, sizeof(q));
    q.txn_type = r.get<uint64_t>();
    q.w_id = r.get<uint64_t>();
    q.d_id = r.get<uint64_t>();
    q.c_id = r.get<uint64_t>();
    q.d_w_id = r.get<uint64_t>();
    q.c_w_id = r.get<uint64_t>();
    q.c_d_id = r.get<uint64_t>();
    for (char &ch : q.c_last) ch = (char)r.get<uint8_t>();
    q.h_amount = r.get<uint64_t>();
    q.by_last_name = r.get<uint8_t>() != 0;
    const uint64_t n = r.get<uint64_t>();  // size_t items
    if (!r.ok || n > DV_TPCC_MAX_OL) return false;
    for (uint64_t i = 0; i < n; i++) {
        q.items[i].ol_i_id = r.get<uint64_t>();
        q.items[i].ol_supply_w_id = r.get<uint64_t>();
        q.items[i].ol_quantity = r.get<uint64_t>();
    }
    q.rbk = r.get<uint8_t>() != 0;
    q.remote = r.get<uint8_t>() != 0;
    q.ol_cnt = r.get<uint64_t>();
    q.o_entry_d = r.get<uint64_t>();
    if (!r.ok) return false;
    // the txn manager walks items[0 .. ol_cnt) (new_order_6..9): the list must hold them
    if (q.txn_type == 2 && q.ol_cnt != n) return false;
    if (q.txn_type == 1) q.ol_cnt = 0;  // (a Payment carries no items)
    if (q.txn_type != 1 && q.txn_type != 2) return false;
    m.n_acc = q.txn_type == 1 ? 3 : (uint32_t)(3 + 2 * q.ol_cnt);
    return true;
}

}  // namespace

extern "C" int dv_wire_epoch_reset(dv_wire_epoch *ep) {
    if (!ep || !ep->txn_begin) return DV_ERR_ARG;
    ep->n_txn = 0;
    ep->n_acc = 0;
    ep->rdone = 0;
    ep->batch_id = kU64Max;
    ep->txn_begin[0] = 0;
    return DV_OK;
}

namespace {
// one message at r: header, client part and body, every field checked (the
// TPC-C ones by the access-list expansion into scratch arrays) -- or, for a
// batch dv_wire_open has checked (check false), only parsed
bool read_msg(const dv_wire_cfg *c, Reader &r, Msg &m, bool check = true) {
    if (!read_client_part(c, r, m, check)) return false;
    if (c->calvin ? m.batch_id == kU64Max : m.rtype == DV_WIRE_RDONE) return false;  // (RDONE ends Calvin batches)
    if (m.rtype == DV_WIRE_RDONE) return true;
    if (c->workload != DV_TPCC) return read_ycsb(c, r, m, check);
    if (!read_tpcc(r, m)) return false;
    if (!check) return true;
    uint64_t k[3 + 2 * DV_TPCC_MAX_OL], a[3 + 2 * DV_TPCC_MAX_OL];
    uint8_t ty[3 + 2 * DV_TPCC_MAX_OL], tb[3 + 2 * DV_TPCC_MAX_OL];
    uint32_t beg[2];
    return dv_tpcc_expand(c->tpcc, &m.tq, 1, 3 + 2 * DV_TPCC_MAX_OL, k, ty, tb, a, beg, nullptr, nullptr) == DV_OK;
}

bool cfg_ok(const dv_wire_cfg *c) {
    return c && c->part_cnt && c->node_cnt && (c->workload == DV_YCSB || (c->workload == DV_TPCC && c->tpcc));
}
}  // namespace

extern "C" int dv_wire_open(const dv_wire_cfg *cfg, const uint8_t *batch, uint64_t len, dv_wire_cursor *cur) {
    if (!cfg_ok(cfg) || !cur || !batch || len < DV_WIRE_HDR || len > DV_WIRE_MSG_MAX) return DV_ERR_ARG;
    uint32_t h[3];
    std::memcpy(h, batch, sizeof(h));
    // create_messages' asserts (message.cpp:39-41): addressed here, from another node, not empty
    if (h[0] != cfg->node_id || h[1] == cfg->node_id || h[2] == 0) return DV_ERR_ARG;
    // the whole batch, message by message, before any of it is decoded:
    // exactly `count` well-formed messages filling exactly `len` bytes
    Reader r{batch + DV_WIRE_HDR, batch + len};
    Msg m;
    for (uint32_t i = 0; i < h[2]; i++)
        if (!read_msg(cfg, r, m)) return DV_ERR_ARG;
    if (r.p != batch + len) return DV_ERR_ARG;
    cur->buf = batch;
    cur->len = len;
    cur->off = DV_WIRE_HDR;
    cur->left = h[2];
    cur->src = h[1];
    return DV_OK;
}

extern "C" int dv_wire_decode(const dv_wire_cfg *cfg, dv_wire_cursor *cur, dv_wire_epoch *ep) {
    if (!cfg_ok(cfg) || !cur || !ep || !cur->buf || !ep->keys || !ep->types || !ep->txn_begin) return DV_ERR_ARG;
    const bool tpcc = cfg->workload == DV_TPCC;
    if (tpcc && (!ep->tables || !ep->args)) return DV_ERR_ARG;
    Msg m;
    while (cur->left > 0) {
        Reader r{cur->buf + cur->off, cur->buf + cur->len};
        if (!read_msg(cfg, r, m, false)) return DV_ERR_ARG;  // (checked whole by dv_wire_open)
        if (cfg->calvin && ep->batch_id != kU64Max) {  // the sequencer's batch (sequencer.cpp:207-210)
            if (m.batch_id < ep->batch_id) return DV_ERR_ARG;  // stale
            if (m.batch_id > ep->batch_id) return DV_WIRE_MORE;
        }
        if (m.rtype == DV_WIRE_RDONE) {
            ep->batch_id = m.batch_id;
            ep->rdone++;
        } else {
            if (ep->n_txn >= ep->max_txn || ep->n_acc + m.n_acc > ep->max_acc) {
                if (ep->n_txn == 0) return DV_ERR_ARG;  // (it would never fit)
                return DV_WIRE_MORE;
            }
            const uint32_t t = ep->n_txn;
            const uint64_t a0 = ep->n_acc;
            if (tpcc) {
                // the access list of TPCCTxnManager (fields checked at dv_wire_open)
                const int rc = dv_tpcc_expand(cfg->tpcc, &m.tq, 1, ep->max_acc - a0, ep->keys + a0, ep->types + a0,
                                              ep->tables + a0, ep->args + a0, ep->txn_begin + t,
                                              ep->txn_type ? ep->txn_type + t : nullptr,
                                              ep->owner ? ep->owner + a0 : nullptr);
                ep->txn_begin[t] = (uint32_t)a0;  // (expand numbered from 0)
                if (rc) return DV_ERR_ARG;
            } else {
                for (uint32_t i = 0; i < m.n_acc; i++) {
                    uint32_t acctype;
                    uint64_t key;
                    std::memcpy(&acctype, m.reqs + i * kYcsbReq, 4);
                    std::memcpy(&key, m.reqs + i * kYcsbReq + 8, 8);
                    ep->keys[a0 + i] = key;
                    ep->types[a0 + i] = (uint8_t)acctype;
                    if (ep->owner) ep->owner[a0 + i] = (uint8_t)(key % cfg->part_cnt);  // key_to_part
                }
                if (ep->tables) std::memset(ep->tables + a0, 0, m.n_acc);
            }
            if (cfg->calvin) ep->batch_id = m.batch_id;
            if (ep->txn_id)  // Calvin: the sequencer's id; else WorkerThread::get_next_txn_id for one worker
                ep->txn_id[t] = cfg->calvin ? m.txn_id : cfg->node_id + (uint64_t)cfg->node_cnt * ep->next_txn;
            if (!cfg->calvin) ep->next_txn++;
            if (ep->client_startts) ep->client_startts[t] = m.client_startts;
            if (ep->return_node) ep->return_node[t] = cur->src;
            ep->n_acc = a0 + m.n_acc;
            ep->n_txn = t + 1;
            ep->txn_begin[t + 1] = (uint32_t)ep->n_acc;
        }
        cur->off = (uint64_t)(r.p - cur->buf);
        cur->left--;
    }
    return DV_OK;
}

extern "C" int dv_wire_decode_batches(const dv_wire_cfg *cfg, const uint8_t *buf, const uint64_t *off,
                                      uint32_t n_batches, dv_wire_cursor *cur, uint32_t *next_batch,
                                      dv_wire_epoch *ep) {
    if (!cfg || !buf || !off || !cur || !next_batch || !ep) return DV_ERR_ARG;
    for (;;) {
        if (cur->buf && cur->left > 0) {
            const int rc = dv_wire_decode(cfg, cur, ep);
            if (rc) return rc;  // DV_WIRE_MORE (the cursor holds the rest) or an error
        }
        if (*next_batch >= n_batches) return DV_OK;
        const uint32_t b = *next_batch;
        if (off[b + 1] < off[b]) return DV_ERR_ARG;
        const int rc = dv_wire_open(cfg, buf + off[b], off[b + 1] - off[b], cur);
        if (rc) return rc;  // (*next_batch stays at the refused batch)
        *next_batch = b + 1;
    }
}

extern "C" int dv_wire_respond(const dv_wire_cfg *cfg, const dv_wire_epoch *ep, const uint8_t *commit, uint8_t *out,
                               uint64_t cap, uint64_t *batch_off, uint32_t max_batches, uint32_t *n_batches) {
    if (!cfg || !ep || !out || !batch_off || !n_batches || !ep->txn_id || !ep->return_node) return DV_ERR_ARG;
    if (!cfg->calvin && (!commit || !ep->client_startts)) return DV_ERR_ARG;
    const uint64_t H = hdr_size(cfg);
    // ClientResponseMessage: header + client_startts; AckMessage: header + RC (4 bytes)
    const uint64_t msz = cfg->calvin ? H + 4 : H + 8;
    std::vector<uint32_t> order;
    order.reserve(ep->n_txn);
    for (uint32_t t = 0; t < ep->n_txn; t++)
        if (cfg->calvin || commit[t]) order.push_back(t);
    std::stable_sort(order.begin(), order.end(),
                     [&](uint32_t a, uint32_t b) { return ep->return_node[a] < ep->return_node[b]; });
    const uint32_t per = (uint32_t)((DV_WIRE_MSG_MAX - DV_WIRE_HDR) / msz);
    uint64_t pos = 0;
    uint32_t nb = 0;
    size_t i = 0;
    batch_off[0] = 0;
    while (i < order.size()) {
        const uint32_t dest = ep->return_node[order[i]];
        size_t j = i;
        while (j < order.size() && j - i < per && ep->return_node[order[j]] == dest) j++;
        const uint64_t bytes = DV_WIRE_HDR + (j - i) * msz;
        if (nb >= max_batches || pos + bytes > cap) return DV_ERR_ARG;
        Writer w{out + pos};
        w.put<uint32_t>(dest);
        w.put<uint32_t>(cfg->node_id);
        w.put<uint32_t>((uint32_t)(j - i));
        for (size_t k = i; k < j; k++) {
            const uint32_t t = order[k];
            w.put<uint32_t>(cfg->calvin ? DV_WIRE_CALVIN_ACK : DV_WIRE_CL_RSP);
            w.put<uint64_t>(ep->txn_id[t]);
            if (cfg->calvin) w.put<uint64_t>(ep->batch_id);
            w.zeros(8 + 7 * 8);  // mq_time, latencies
            if (cfg->calvin)
                w.put<uint32_t>(0);  // RC RCOK: a Calvin txn's rc at calvin_wrapup (txn.cpp:287)
            else
                w.put<uint64_t>(ep->client_startts[t]);
        }
        pos += bytes;
        batch_off[++nb] = pos;
        i = j;
    }
    *n_batches = nb;
    return DV_OK;
}
