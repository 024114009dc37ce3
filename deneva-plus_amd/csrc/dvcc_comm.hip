// dvcc_comm.hip -- partitioned epochs driven from the engine over RCCL
// (SURVEY.md 8(b) dv_comm_init, 8(e)).
//
// One process per GPU; rank r owns partition r (PART_CNT == ranks,
// GET_NODE_ID(part) == part, system/global.h:294).  dv_epoch_run_part runs a
// whole epoch from this rank's client batch:
//   1. split the batch by owner rank = key % PART_CNT (YCSBWorkload::
//      key_to_part, benchmarks/ycsb_wl.cpp:69-74) on the device, stably, into
//      16-byte dv_access records;
//   2. one all-to-all of the counts and one all-to-allv of the records -- the
//      RQRY messages of msg_queue / nanomsg (ycsb_txn.cpp:160-175,
//      transport/transport.cpp:224-304).  Records arrive in origin-rank order,
//      which is the global sequence order (epoch, origin node, position) Calvin
//      locks in (work_queue.cpp:105-151);
//   3. NO_WAIT / WAIT_DIE / OCC: decision rounds, each closed by an
//      all-reduce(MAX) of the verdict bytes of the still-undecided txns in list
//      order -- TxnManager::received_response's vote combine (txn.cpp:544-554)
//      for every open txn at once -- queued two rounds ahead of the outcome the
//      host reads, each all-reduce sized by the list length of two rounds
//      earlier (the same number on every rank); CALVIN needs no votes;
//   4. execute the committed accesses on this rank's rows.
// Everything runs on the context's stream, RCCL collectives included.  The
// Python driver (deneva-plus_amd/dvcc/partitioned.py) runs the same protocol
// over torch.distributed.
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

#include "dvcc_common.h"

namespace dvcc {

// ---- owner split: per-block owner counts, then a stable scatter of records
__global__ __launch_bounds__(kBlock) void k_owner_count(const uint64_t *__restrict__ keys, uint64_t n,
                                                        uint32_t P, uint32_t *__restrict__ counts,
                                                        uint32_t nb) {
    __shared__ uint32_t c[kRadix];
    for (uint32_t o = threadIdx.x; o < kRadix; o += kBlock) c[o] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * kTile;
    for (uint32_t j = threadIdx.x; j < (uint32_t)kTile; j += kBlock)
        if (base + j < n) atomicAdd(&c[(uint32_t)(keys[base + j] % P)], 1u);
    __syncthreads();
    for (uint32_t o = threadIdx.x; o < P; o += kBlock) counts[(uint64_t)o * nb + blockIdx.x] = c[o];
}

// counts[o][b] -> exclusive prefix within owner o; tot[o] = owner o's total
__global__ __launch_bounds__(kBlock) void k_owner_scan(uint32_t *__restrict__ counts, uint32_t nb,
                                                       uint32_t *__restrict__ tot) {
    __shared__ uint32_t lds4[4];
    uint32_t *c = counts + (uint64_t)blockIdx.x * nb;
    const uint32_t per = (nb + kBlock - 1) / kBlock;
    const uint32_t lo = threadIdx.x * per, hi = lo + per < nb ? lo + per : nb;
    uint32_t sum = 0;
    for (uint32_t i = lo; i < hi; i++) sum += c[i];
    uint32_t t = 0;
    uint32_t pre = block_excl_scan256(sum, lds4, &t);
    for (uint32_t i = lo; i < hi; i++) {
        const uint32_t v = c[i];
        c[i] = pre;
        pre += v;
    }
    if (threadIdx.x == 0) tot[blockIdx.x] = t;
}

// record i of the batch -> its owner's segment, in batch order (stable: a
// wave walks 64 consecutive records per step, ranks by ballot)
__global__ __launch_bounds__(kBlock) void k_owner_scatter(const uint64_t *__restrict__ keys,
                                                          const uint8_t *__restrict__ types,
                                                          const uint32_t *__restrict__ acc_txn,
                                                          uint64_t n, uint32_t P, uint32_t txn_base,
                                                          const uint32_t *__restrict__ counts,
                                                          const uint32_t *__restrict__ tot, uint32_t nb,
                                                          dv_access *__restrict__ out) {
    __shared__ uint32_t wc[4][kRadix];
    __shared__ uint32_t obase[kRadix];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) {
        uint32_t s = 0;
        for (uint32_t o = 0; o < P; o++) {
            obase[o] = s;
            s += tot[o];
        }
    }
    for (uint32_t o = tid; o < kRadix; o += kBlock) wc[0][o] = wc[1][o] = wc[2][o] = wc[3][o] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * kTile + wave * (64 * kIPT);
    uint32_t own[kIPT], r[kIPT];
    for (int j = 0; j < kIPT; j++) {
        const uint64_t idx = base + j * 64 + lane;
        const bool valid = idx < n;
        const uint32_t o = valid ? (uint32_t)(keys[idx] % P) : 0u;
        const uint64_t peers = match_digit(o, __ballot(valid));
        const uint32_t before = wc[wave][o];
        own[j] = o;
        r[j] = before + mask_rank(peers);
        if (valid && lane == (uint32_t)__builtin_ctzll(peers)) wc[wave][o] = before + (uint32_t)__popcll(peers);
    }
    __syncthreads();
    for (int j = 0; j < kIPT; j++) {
        const uint64_t idx = base + j * 64 + lane;
        if (idx >= n) continue;
        const uint32_t o = own[j];
        uint32_t wpre = 0;
        for (uint32_t w = 0; w < wave; w++) wpre += wc[w][o];
        const uint64_t dst = (uint64_t)obase[o] + counts[(uint64_t)o * nb + blockIdx.x] + wpre + r[j];
        dv_access a;
        a.key = keys[idx];
        a.txn_seq = txn_base + acc_txn[idx];
        a.type = types[idx];
        a.table = 0;
        a.flags = 0;
        out[dst] = a;
    }
}

struct DvComm {
    ncclComm_t comm = nullptr;
    int nranks = 0, rank = 0;
    uint64_t acc_cap = 0;  // capacity of the record / SoA buffers
    uint32_t nb_cap = 0, txn_cap = 0;
    dv_access *send = nullptr, *recv = nullptr;
    uint64_t *keys = nullptr;
    uint8_t *types = nullptr, *tables = nullptr, *verdict = nullptr;
    uint32_t *txn = nullptr, *counts = nullptr, *tot = nullptr, *err = nullptr;
    uint64_t *xcnt = nullptr;  // [2 * nranks]: send counts, received counts
    uint32_t *xmax = nullptr;  // longest txn, all-reduced
};

}  // namespace dvcc

using namespace dvcc;

namespace {

int nccl_fail(ncclResult_t e, const char *what) {
    if (e == ncclSuccess) return DV_OK;
    std::fprintf(stderr, "dvcc: %s failed: %s\n", what, ncclGetErrorString(e));
    return DV_ERR_HIP;
}
int hip_fail2(hipError_t e, const char *what) {
    if (e == hipSuccess) return DV_OK;
    std::fprintf(stderr, "dvcc: %s failed: %s\n", what, hipGetErrorString(e));
    return DV_ERR_HIP;
}
#define CHK(x)                 \
    do {                       \
        int _r = (x);          \
        if (_r) return _r;     \
    } while (0)

template <class T>
int alloc(T **p, uint64_t n) {
    return hip_fail2(hipMalloc(reinterpret_cast<void **>(p), sizeof(T) * (n ? n : 1)), "hipMalloc");
}

void free_bufs(DvComm *m) {
    void *b[] = {m->send, m->recv, m->keys, m->types, m->tables, m->verdict, m->txn,
                 m->counts, m->tot, m->err, m->xcnt, m->xmax};
    for (void *p : b)
        if (p) (void)hipFree(p);
    m->send = m->recv = nullptr;
    m->keys = nullptr;
    m->types = m->tables = m->verdict = nullptr;
    m->txn = m->counts = m->tot = m->err = m->xmax = nullptr;
    m->xcnt = nullptr;
}

int reserve(DvComm *m, uint64_t acc, uint32_t nb, uint32_t txn) {
    if (acc <= m->acc_cap && nb <= m->nb_cap && txn <= m->txn_cap && m->xcnt) return DV_OK;
    free_bufs(m);
    acc = std::max(acc, m->acc_cap);
    nb = std::max(nb, m->nb_cap);
    txn = std::max(txn, m->txn_cap);
    const uint32_t P = (uint32_t)m->nranks;
    CHK(alloc(&m->send, acc));
    CHK(alloc(&m->recv, acc));
    CHK(alloc(&m->keys, acc));
    CHK(alloc(&m->types, acc));
    CHK(alloc(&m->tables, acc));
    CHK(alloc(&m->txn, acc));
    CHK(alloc(&m->verdict, ((uint64_t)txn + 3) & ~3ull));
    CHK(alloc(&m->counts, (uint64_t)P * nb));
    CHK(alloc(&m->tot, P));
    CHK(alloc(&m->err, 1));
    CHK(alloc(&m->xcnt, 2ull * P));
    CHK(alloc(&m->xmax, 1));
    m->acc_cap = acc;
    m->nb_cap = nb;
    m->txn_cap = txn;
    return DV_OK;
}

}  // namespace

void comm_free(DvComm *m) {
    if (!m) return;
    free_bufs(m);
    if (m->comm) (void)ncclCommDestroy(m->comm);
    delete m;
}

extern "C" {

int dv_comm_unique_id(void *id_out) {
    if (!id_out) return DV_ERR_ARG;
    ncclUniqueId id;
    CHK(nccl_fail(ncclGetUniqueId(&id), "ncclGetUniqueId"));
    std::memcpy(id_out, &id, sizeof(id));
    return DV_OK;
}

int dv_comm_init(dv_ctx *c, const void *unique_id, int nranks, int rank) {
    if (!c || !unique_id || nranks < 1 || nranks > kRadix || rank < 0 || rank >= nranks) return DV_ERR_ARG;
    const dv_config &cfg = ctx_config(c);
    if ((int)cfg.part_cnt != nranks || (int)cfg.part_id != rank) return DV_ERR_ARG;  // partition == rank
    CHK(hip_fail2(hipSetDevice(cfg.device), "hipSetDevice"));
    DvComm *&slot = ctx_comm(c);
    comm_free(slot);
    slot = new DvComm();
    slot->nranks = nranks;
    slot->rank = rank;
    ncclUniqueId id;
    std::memcpy(&id, unique_id, sizeof(id));
    int r = nccl_fail(ncclCommInitRank(&slot->comm, nranks, id, rank), "ncclCommInitRank");
    if (r) {
        slot->comm = nullptr;
        comm_free(slot);
        slot = nullptr;
    }
    return r;
}

int dv_epoch_run_part(dv_ctx *c, const dv_epoch_dev *home, uint32_t txns_per_rank, uint8_t *d_commit,
                      dv_stats *st) {
    if (!c || !home || (home->n_acc && (!home->keys || !home->types || !home->acc_txn))) return DV_ERR_ARG;
    DvComm *m = ctx_comm(c);
    if (!m) return DV_ERR_STATE;
    if (home->n_txn > txns_per_rank) return DV_ERR_ARG;
    const dv_config &cfg = ctx_config(c);
    const uint32_t P = (uint32_t)m->nranks;
    const uint64_t n_txn64 = (uint64_t)txns_per_rank * P;
    if (n_txn64 > cfg.max_txn) return DV_ERR_ARG;
    const uint32_t n_txn = (uint32_t)n_txn64;
    hipStream_t s = ctx_stream(c);
    const uint32_t nb = home->n_acc ? (uint32_t)((home->n_acc + kTile - 1) / kTile) : 1;
    CHK(reserve(m, std::max<uint64_t>(home->n_acc, cfg.max_acc), nb, n_txn));

    // 1. split the batch by owner
    if (home->n_acc) {
        k_owner_count<<<nb, kBlock, 0, s>>>(home->keys, home->n_acc, P, m->counts, nb);
        k_owner_scan<<<P, kBlock, 0, s>>>(m->counts, nb, m->tot);
        k_owner_scatter<<<nb, kBlock, 0, s>>>(home->keys, home->types, home->acc_txn, home->n_acc, P,
                                             (uint32_t)m->rank * txns_per_rank, m->counts, m->tot, nb,
                                             m->send);
    } else {
        CHK(hip_fail2(hipMemsetAsync(m->tot, 0, P * sizeof(uint32_t), s), "memset"));
    }
    CHK(hip_fail2(hipGetLastError(), "owner split"));
    // 2. counts, then the records
    std::vector<uint32_t> tot(P);
    CHK(hip_fail2(hipMemcpyAsync(tot.data(), m->tot, P * sizeof(uint32_t), hipMemcpyDeviceToHost, s), "D2H"));
    CHK(hip_fail2(hipStreamSynchronize(s), "sync"));
    std::vector<uint64_t> sendc(P), recvc(P);
    for (uint32_t o = 0; o < P; o++) sendc[o] = tot[o];
    CHK(hip_fail2(hipMemcpyAsync(m->xcnt, sendc.data(), P * 8, hipMemcpyHostToDevice, s), "H2D"));
    CHK(nccl_fail(ncclAllToAll(m->xcnt, m->xcnt + P, 1, ncclUint64, m->comm, s), "ncclAllToAll"));
    // the longest txn anywhere sets the verdict-byte stride on every rank
    const uint32_t mx = home->max_txn_acc ? home->max_txn_acc : kMaxPos;
    CHK(hip_fail2(hipMemcpyAsync(m->xmax, &mx, 4, hipMemcpyHostToDevice, s), "H2D"));
    CHK(nccl_fail(ncclAllReduce(m->xmax, m->xmax, 1, ncclUint32, ncclMax, m->comm, s), "ncclAllReduce"));
    uint32_t gmax = 0;
    CHK(hip_fail2(hipMemcpyAsync(recvc.data(), m->xcnt + P, P * 8, hipMemcpyDeviceToHost, s), "D2H"));
    CHK(hip_fail2(hipMemcpyAsync(&gmax, m->xmax, 4, hipMemcpyDeviceToHost, s), "D2H"));
    CHK(hip_fail2(hipStreamSynchronize(s), "sync"));
    std::vector<size_t> sc(P), sd(P), rc(P), rd(P);
    uint64_t n_recv = 0, so = 0;
    for (uint32_t o = 0; o < P; o++) {
        sc[o] = sendc[o] * sizeof(dv_access);
        sd[o] = so * sizeof(dv_access);
        so += sendc[o];
        rc[o] = recvc[o] * sizeof(dv_access);
        rd[o] = n_recv * sizeof(dv_access);
        n_recv += recvc[o];
    }
    if (n_recv > cfg.max_acc) return DV_ERR_ARG;
    CHK(nccl_fail(ncclAllToAllv(m->send, sc.data(), sd.data(), m->recv, rc.data(), rd.data(), ncclUint8,
                                m->comm, s),
                  "ncclAllToAllv"));
    CHK(hip_fail2(hipMemsetAsync(m->err, 0, 4, s), "memset"));
    launch_split_access(s, m->recv, n_recv, nullptr, n_txn, m->keys, m->types, m->txn, m->tables, m->err);
    CHK(hip_fail2(hipGetLastError(), "unpack"));

    // 3. the partition's epoch: rounds closed by list all-reduces
    dv_epoch_dev ep{};
    ep.keys = m->keys;
    ep.types = m->types;
    ep.acc_txn = m->txn;
    ep.tables = nullptr;
    ep.n_acc = n_recv;
    ep.n_txn = n_txn;
    ep.max_txn_acc = std::min<uint32_t>(gmax, kMaxPos);
    CHK(dv_epoch_begin(c, &ep, nullptr));
    if (cfg.cc_alg != DV_CALVIN) {
        constexpr uint32_t kLag = 2;  // rounds queued ahead of the outcome read
        std::vector<uint32_t> counts{n_txn};  // list length entering each known round
        uint32_t r = 0;
        while (counts.back() > 0) {
            CHK(dv_epoch_round_local(c, m->verdict));
            CHK(nccl_fail(ncclAllReduce(m->verdict, m->verdict, counts.back(), ncclUint8, ncclMax, m->comm, s),
                          "ncclAllReduce"));
            CHK(dv_epoch_round_apply(c, m->verdict, nullptr));
            if (++r >= kLag) {
                uint32_t und = 0;
                CHK(dv_epoch_round_wait(c, r - kLag, &und));
                if (und != 0 && und >= counts.back()) return DV_ERR_STATE;  // every round decides one
                counts.push_back(und);
            }
        }
    }
    // 4. execute and report
    return dv_epoch_finish(c, d_commit, st);
}

}  // extern "C"
