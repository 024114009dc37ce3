// dvcc_runtime.hip -- epoch runtime and C ABI (include/dvcc.h).
//
// Host side of the engine: owns the device, the stream, the HBM row store and
// hash index, and the per-epoch workspace; sequences the kernels of
// dvcc_kernels.hip.  Replaces the per-txn machinery of the reference
// (TxnManager/txn_table/worker loop, system/txn.cpp, txn_table.cpp,
// worker_thread.cpp:183-518) with dense epoch arrays: txn sequence number ==
// array index, one byte of decision state per txn.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <map>
#include <new>
#include <string>
#include <vector>

#include "dvcc_common.h"
#include "dvcc_tpcc.h"

using namespace dvcc;

namespace {

// dv_lanes_order: the execution order of epoch groups over several lanes,
// shared by them (ticket k * n + l is lane l's k-th execution)
struct LaneOrder {
    std::mutex mu;
    std::condition_variable cv;
    uint64_t next = 0;             // the ticket whose execution may be queued now
    hipEvent_t last = nullptr;     // recorded after the previous ticket's execution
    uint64_t fail_at = ~0ull;      // a lane's group failed: this ticket never executes, nor any later one
    uint32_t n = 0;
};

constexpr int kLaneWaitS = 120;  // lane_exec_begin's longest wait for its turn

// dv_epoch_run_device_lanes: up to 8 lanes, each on its share of the CUs
// (measured best: 4, gpurun_out r03_l8 / r03_hq)
constexpr uint32_t kMaxLanes = 8;

struct HostTable {
    bool created = false, loaded = false;
    bool implicit_rows = false;  // direct map with local row == bucket: probes read pkey
    bool dense = false;          // dv_load_ycsb_partition: bucket b holds key b * P + part, every b
    uint64_t cap_rows = 0, n_rows = 0, nbuckets = 0, row_base = 0;
    uint32_t hash_kind = DV_HASH_YCSB;
    IxEntry *ix = nullptr;      // device
    uint32_t *bstart = nullptr; // device (chained only)
    uint32_t *hbits = nullptr;  // device: home-tag bitmap of an implicit-row map (TableDesc::hbits)
    uint32_t htag = kTagWide;
    uint64_t ix_cap = 0;
};

}  // namespace

// per-launch kernel timing of one context (DV_FLAG_KERNEL_PROFILE,
// dv_kernel_times; DV_LAUNCH in dvcc_internal.h)
struct dvcc::KProf {
    struct Pending {
        const char *name;
        hipEvent_t e0, e1;
        bool owned;  // from the pool (else the runtime's own timing events)
    };
    struct Sum {
        uint64_t launches = 0;
        double ms = 0;
    };
    static constexpr size_t kPool = 8192;  // event pairs (a 1M-txn epoch takes ~40)
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pool;
    size_t used = 0;                       // pool pairs handed out and not yet read
    std::vector<Pending> pending;
    std::map<std::string, Sum> sums;
    uint64_t dropped = 0;                  // launches not timed: the pool was spent
    int depth = 0;                         // nested C-ABI entries (KProfScope)
};

struct dv_ctx {
    dv_config cfg{};
    hipStream_t stream = nullptr;      // where work is launched
    hipStream_t own_stream = nullptr;  // created by dv_open
    HostTable tab[kMaxTables];
    uint64_t total_rows = 0;
    uint64_t *f0 = nullptr;    // hot column, global row id
    uint64_t *pkey = nullptr;  // primary key per row (row_t::get_primary_key)
    uint8_t *ktag = nullptr;   // key tag per row (key_tag, dvcc_internal.h)
    // DV_TPCC: the three 8-byte state columns of a row side by side (24 B,
    // row-major: k_tpcc_apply touches all three of a row), f0 = column 0;
    // YCSB: f0 alone (cstride 1)
    uint32_t cstride = 1;
    // decision lanes (dv_open_lane): a lane shares its owner's tables (the
    // arrays above and tab[]'s index arrays are the owner's, never freed
    // here); lanes_open counts the lanes of an owner (its tables are frozen)
    dv_ctx *table_owner = nullptr;
    uint32_t lanes_open = 0;
    uint32_t *d_gate = nullptr;    // 2 words: decision lanes' turn, and (lanes[0]) the executed turns
    uint32_t lane_issued = 0;      // (lanes[0]) turns queued through d_gate[1] so far (run_lanes)
    hipEvent_t lane_ev = nullptr;  // recorded after this context's last queued execution
    // dv_epoch_run_device_lanes runs lane l of n on lane_stream, masked to
    // the CUs i with i % n == l: a lane's asynchronous round launch needs all
    // of its workgroups resident at once, and on the whole chip the other
    // lanes' kernels keep taking the CUs its last workgroups wait for (its
    // workgroups yield, the epochs run again -- 0.69 ms per epoch instead of
    // 0.29 for two lanes, gpurun_out r03_w); lane_g: its workgroups on its share
    hipStream_t lane_stream = nullptr;
    uint32_t lane_n = 0, lane_l = 0, lane_g = 0;
    // dv_lanes_order: this lane's place in the groups' execution order
    std::shared_ptr<LaneOrder> order;
    uint64_t order_k = 0;  // executions of this lane so far

    // TPC-C epoch (dv_tpcc_epoch_run_device): execution scratch, and the
    // operation words / o_id output of this epoch
    uint64_t *tp_dsnap = nullptr;  // per district row: D_NEXT_O_ID before the epoch, then its queue's start
    uint64_t tp_dsnap_cap = 0;
    const uint64_t *tp_args = nullptr;
    uint64_t *tp_oid = nullptr;

    // workspace (capacities from cfg)
    uint64_t *pairs[2] = {nullptr, nullptr};
    uint64_t *el = nullptr;                          // row-queue elements (sorted)
    uint8_t *ew = nullptr;
    uint32_t *counts = nullptr, *digit_tot = nullptr;
    uint64_t *rel[2] = {nullptr, nullptr};           // live accesses, ping-pong
    uint8_t *vb8 = nullptr;                          // per access: verdict, txn-strided
    uint64_t vb8_cap = 0;                            // bytes
    uint32_t slog = 4;                               // log2 of vb8's per-txn stride
    bool el32 = false;                               // 32-bit round elements this epoch
    uint8_t *tlen = nullptr;                         // per txn: accesses here
    uint32_t *acc_row = nullptr;                     // per access: row | wr << 31
    uint32_t *ulist[2] = {nullptr, nullptr};         // undecided txns, ping-pong
    uint32_t *tb_start = nullptr, *tb_end = nullptr; // per txn: its access range
    // the current epoch's txn ranges for every kernel that reads them:
    // tb_start / tb_end, or the epoch's own boundaries (dv_epoch_dev::txn_begin,
    // rs = txn_begin, re = txn_begin + 1: run_prefix_epoch's tb mode)
    const uint32_t *rs = nullptr, *re = nullptr;
    bool tb_mode = false;
    uint64_t *desc = nullptr;                        // look-back tile descriptors
    uint32_t *tile_ctr = nullptr;                    // tile tickets, one per single-pass launch
    uint32_t *abounds = nullptr;                     // asynchronous-round slice carries
    uint32_t *tword = nullptr;                       // asynchronous-round txn fact words
    uint32_t async_g = 0;                            // its workgroups (all co-resident)
    uint32_t *carry_b = nullptr;                     // abort carry-over: block counts (2 x carry_nb)
    uint32_t carry_nb = 0;
    uint32_t *carry_tot = nullptr;                   // its totals (kRefillTot words)
    uint32_t *gc_tb = nullptr;                       // dv_epoch_group_carry: a batch's ranges (2 x max_txn)
    uint32_t *gc_tot = nullptr;                      // ... 3 totals per batch (kMaxGroupBatches)
    DvComm *comm = nullptr;                          // RCCL communicator (dv_comm_init)
    uint32_t round_tag = 0;                          // descriptor tag of the last pass
    uint32_t ticket = 0;                             // next tile_ctr slot
    uint8_t *status = nullptr, *verdict = nullptr;
    Counters *ctr = nullptr;    // device
    Counters *h_ctr = nullptr;  // host-mapped mirror (written by k_ctr_out) = h_mir[0] ...
    Counters *d_hctr = nullptr;                 // ... its device address
    unsigned long long *h_cseq = nullptr, *d_cseq = nullptr;  // its sequence word (after the mirror)
    unsigned long long cseq = 0;                // the last sequence number asked for
    // two mirror slots: pipelined epochs (dv_epoch_run_device_batch) alternate
    Counters *h_mir[2] = {nullptr, nullptr}, *d_mir[2] = {nullptr, nullptr};
    unsigned long long *h_mseq[2] = {nullptr, nullptr}, *d_mseq[2] = {nullptr, nullptr};
    bool clear_gate = false;                    // the next epoch clear is gated on the previous epoch
    // a pipelined epoch whose counter mirror the next epoch's clear writes
    // (pipe_enqueue with defer); mirror_flush writes it if that clear never came
    bool mir_pending = false;
    int mir_slot = 0;
    unsigned long long mir_seq = 0;
    // epoch graphs (graph_decide): a pipelined epoch's decision launches --
    // everything after its clear -- captured once per (epoch buffers, sizes,
    // knobs) and replayed; ws_gen counts the workspace reallocations that
    // would invalidate a captured graph's pointers
    struct EpochGraph {
        uint64_t key[22] = {};
        hipGraphExec_t exec = nullptr;
        uint32_t seen = 0;
        uint64_t used = 0;
    };
    std::vector<EpochGraph> graphs;
    uint64_t graph_clock = 0, ws_gen = 0;
    // dv_tpcc_epoch_begin: the probe resolves the last-name accesses (k_probe<RSV>)
    bool tp_resolve = false;
    uint32_t r0_n = 0;                    // round 0's live accesses (RoundBufs::n0)
    const uint32_t *r0_n_dev = nullptr;   // ... or their count on the device
    uint32_t n_txn_cap_pad = 0;

    // staging for dv_epoch_run (host-buffer entry point)
    dv_access *d_acc = nullptr;
    uint64_t *d_keys = nullptr;
    uint8_t *d_types = nullptr, *d_tables = nullptr, *d_commit = nullptr;
    uint32_t *d_txn = nullptr, *d_grant = nullptr;
    uint32_t *d_tb = nullptr;         // txn_begin
    uint32_t *split_err = nullptr;    // the record check's error bits (begin clears the counters)
    uint64_t *d_args = nullptr, *d_oid = nullptr;  // dv_tpcc_epoch_run staging
    // double-buffered host input (dv_epoch_stage_host / dv_epoch_run_staged):
    // two record slots filled on a copy stream while the context's stream runs
    struct HostSlot {
        dv_access *acc = nullptr;
        uint32_t *tb = nullptr;
        hipEvent_t copied = nullptr;  // the slot's H2D is done
        hipEvent_t drained = nullptr; // the split has read the slot
        uint64_t n_acc = 0;
        uint32_t n_txn = 0, max_len = 0;
        bool csr = false, full = false;
        bool rows = false;  // 4-byte row records (dv_epoch_stage_host_rows)
    } hslot[2];
    hipStream_t copy_stream = nullptr;

    // epoch state
    int phase = 0;  // 0 idle, 1 begun
    uint64_t n_acc = 0;
    bool n_acc_is_bound = false;  // n_acc bounds a device-side count (dv_epoch_dev::n_acc_dev)
    uint32_t n_txn = 0, n_txn_pad = 0;
    int sorted = 0;
    uint32_t rounds = 0, sort_passes = 0;
    uint32_t live_ub = 0;  // host-side upper bound of the next round's live accesses
    uint32_t und_ub = 0;   // host-side upper bound of the undecided-txn list
    RoundPub *h_pub = nullptr;  // host-mapped round progress (single-GPU rounds)
    RoundPub *d_pub = nullptr;  // its device address
    uint32_t rounds_real = 0;   // rounds until every txn was decided
    const uint32_t *err_seed = nullptr;  // dv_epoch_run: the record check's bits, for the next begin
    // asynchronous rounds: a workgroup yields after this many iterations, or
    // this many wall-clock ticks without a decision (dv_set_async_limits)
    uint32_t async_max_iters = 1u << 18;
    uint64_t async_idle_ticks = 0;
    uint64_t wall_khz = 100000;  // hipDeviceAttributeWallClockRate

    // the (sub-)epoch the decision rounds work on: the epoch itself, or one
    // stage of a prefix-kill epoch (the prefix; the survivors, renumbered)
    uint8_t *v_status = nullptr, *v_tlen = nullptr;
    uint32_t v_n_txn = 0;                    // its txns (an upper bound when v_n_txn_dev is set)
    const uint32_t *v_n_txn_dev = nullptr;   // its real txn count, on the device
    uint32_t v_thresh = 0;                   // asynchronous-try threshold (0: async_thresh's rule)

    // prefix-kill epochs (run_prefix_epoch, dvcc_prefix.hip)
    uint32_t prefix_txns = 0;     // dv_set_prefix: prefix size (0: automatic, ~n_txn / 32)
    bool prefix_mode = false;     // the epoch in flight is one
    // the stage's asynchronous launch leaves its statuses in tword, no
    // finalize: the prefix's (k_prefix_mark reads them), the survivors'
    // (k_sub_scatter_back)
    bool prefix_words = false, surv_words = false;
    uint32_t rounds_prefix = 0;   // rounds the prefix took (0: read from the counters, a_rounds)
    uint32_t rep_P = 0;           // replicated epoch in flight over rep_P partitions (epoch_run_replicated)
    const uint32_t *keys32 = nullptr;  // ... its keys as 32-bit row ids
    const RouteOut *route = nullptr;   // epoch groups: committed accesses go to their owners (run_group)
    // epoch groups (RouteOut::defer): the finish waits for its counters after
    // the outcome vote (epoch_finish_complete)
    bool fin_pending = false;
    unsigned long long fin_want = 0;
    uint8_t *fin_commit = nullptr;
    // what a synchronous redo of the prefix needs (dv_epoch_finish, Counters::a_halt)
    uint32_t pf_K = 0, pf_ub_a = 0;
    const uint32_t *pf_n_acc_dev = nullptr;  // the epoch's device-side access count (dv_epoch_dev::n_acc_dev)
    KillKeys pf_kk{};                        // tb mode: the keys k_kill / k_kill_emit probe
    int pf_sorted_a = 0, pf_key_bits = 0;
    uint64_t pf_n_acc = 0;
    uint32_t *row_state = nullptr; // 2 bits per row: the prefix's committed readers / writers
    uint64_t row_state_cap = 0;    // (words)
    uint8_t *b_status = nullptr, *b_tlen = nullptr;  // the survivors' sub-epoch (txn capacity)
    uint32_t *b_map = nullptr;                      // survivor -> txn
    uint32_t *kinfo = nullptr;                      // k_kill_count -> k_kill_emit: one word per txn
    uint32_t *ktsum = nullptr;                      // ... and two counts per tile
    uint64_t *kill_bits = nullptr;                  // one bit per access: killed by the prefix's commits

    // timing
    hipEvent_t ev[32] = {};
    hipEvent_t sev[16] = {};
    hipEvent_t pev[2 * kRoundLog] = {};  // around each decision-round pass
    uint32_t passes = 0;                 // pass launches this epoch
    uint32_t applied = 0;                // partitioned rounds applied this epoch
    uint32_t async_launched = 0;         // asynchronous-round tries this epoch
    bool async_unconfirmed = false;      // the rounds ended in a try nobody waited for
    uint32_t async_hint = 0;             // round the last epoch's asynchronous launch ran at
    float ms_probe = 0, ms_sort = 0, ms_decide = 0, ms_exec = 0;
    KProf kprof;                         // DV_FLAG_KERNEL_PROFILE
};

// ---- per-launch kernel timing (dvcc_internal.h, DV_LAUNCH)
namespace dvcc {
thread_local KProf *tl_kprof = nullptr;
thread_local bool tl_dry = false;
thread_local bool tl_hprof = false;
thread_local double tl_hp_launch_s = 0;
thread_local uint32_t tl_hp_launch_n = 0;

void kprof_events(const char *kernel, hipEvent_t *e0, hipEvent_t *e1) {
    KProf *p = tl_kprof;
    *e0 = *e1 = nullptr;
    if (!p) return;
    if (p->used >= KProf::kPool) {
        p->dropped++;
        return;
    }
    if (p->used == p->pool.size()) {
        hipEvent_t a = nullptr, b = nullptr;
        if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) {
            if (a) (void)hipEventDestroy(a);
            p->dropped++;
            return;
        }
        p->pool.push_back({a, b});
    }
    *e0 = p->pool[p->used].first;
    *e1 = p->pool[p->used].second;
    p->used++;
    p->pending.push_back({kernel, *e0, *e1, true});
}

void kprof_add(const char *kernel, hipEvent_t e0, hipEvent_t e1) {
    if (tl_kprof) tl_kprof->pending.push_back({kernel, e0, e1, false});
}

namespace {
// "(k_round_pass<true, uint64_t, E>)" -> "k_round_pass"
std::string kernel_base(const char *s) {
    std::string out;
    for (; *s; s++) {
        if (*s == '(' || *s == ' ') continue;
        if (*s == '<' || *s == ')') break;
        out += *s;
    }
    return out;
}

// read every pending pair whose stop event has completed (wait: all of them);
// the pool is reused once nothing is pending
void kprof_harvest(KProf *p, bool wait) {
    size_t keep = 0;
    for (size_t i = 0; i < p->pending.size(); i++) {
        KProf::Pending &q = p->pending[i];
        if (wait) (void)hipEventSynchronize(q.e1);
        else if (hipEventQuery(q.e1) != hipSuccess) {
            p->pending[keep++] = q;
            continue;
        }
        float ms = 0;
        if (hipEventElapsedTime(&ms, q.e0, q.e1) == hipSuccess) {
            KProf::Sum &s = p->sums[kernel_base(q.name)];
            s.launches++;
            s.ms += ms;
        }
    }
    p->pending.resize(keep);
    if (keep == 0) p->used = 0;
}
}  // namespace

KProfScope::KProfScope(dv_ctx *c) : prev_(tl_kprof), mine_(nullptr) {
    if (c && (c->cfg.flags & DV_FLAG_KERNEL_PROFILE)) {
        mine_ = &c->kprof;
        mine_->depth++;
        tl_kprof = mine_;
    }
}

KProfScope::~KProfScope() {
    if (mine_ && --mine_->depth == 0) kprof_harvest(mine_, false);
    tl_kprof = prev_;
}
}  // namespace dvcc

namespace {

inline void dfree(void *p) {
    if (p) (void)hipFree(p);
}

int hip_fail(hipError_t e, const char *what) {
    if (e == hipSuccess) return DV_OK;
    std::fprintf(stderr, "dvcc: %s failed: %s\n", what, hipGetErrorString(e));
    return DV_ERR_HIP;
}
#define HIPCHK(x)                                         \
    do {                                                  \
        int _r = hip_fail((x), #x);                       \
        if (_r) return _r;                                \
    } while (0)

template <class T>
int dalloc(T **p, uint64_t count) {
    if (count == 0) count = 1;
    hipError_t e = hipMalloc(reinterpret_cast<void **>(p), sizeof(T) * count);
    if (e != hipSuccess) {
        *p = nullptr;
        std::fprintf(stderr, "dvcc: hipMalloc(%llu B) failed: %s\n",
                     (unsigned long long)(sizeof(T) * count), hipGetErrorString(e));
        return DV_ERR_NOMEM;
    }
    return DV_OK;
}

int bits_for(uint64_t n) {  // bits needed to represent values in [0, n)
    int b = 0;
    while (b < 64 && (1ull << b) < n) b++;
    return b;
}

RoundBufs round_bufs(dv_ctx *c) {
    RoundBufs b;
    b.pairs0 = c->pairs[c->sorted];
    b.rel[0] = c->rel[0];
    b.rel[1] = c->rel[1];
    b.el32 = c->el32;
    b.vb8 = c->vb8;
    b.slog = c->slog;
    b.status = c->v_status;
    b.tlen = c->v_tlen;
    b.ulist[0] = c->ulist[0];
    b.ulist[1] = c->ulist[1];
    b.n_txn_dev = c->v_n_txn_dev;
    b.n0_dev = c->r0_n_dev;
    b.n0 = c->r0_n;
    b.n_txn0 = c->v_n_txn;
    b.desc = c->desc;
    b.tile_ctr = c->tile_ctr;
    b.ctr = c->ctr;
    return b;
}

// c->ev slots of the probe launch's dispatch timestamps (0-5: stage markers)
constexpr int kEvProbe0 = 8, kEvProbe1 = 9;

// Something a captured epoch graph's launch arguments name has moved or
// changed meaning -- a table's index, bucket bitmap, state columns (f0, pkey,
// ktag: dv_create_table grows them), the carry-over's block counts, or the
// look-back tags after a wrap: no graph captured before this replays again
// (ws_gen is part of every graph key).  Lanes share their owner's tables, but
// those are frozen while any lane is open, so the owner's counter covers them.
void graphs_stale(dv_ctx *c) { c->ws_gen++; }

// descriptor tag of the next single-pass launch (tags are kTagBits wide)
uint32_t next_tag(dv_ctx *c) {
    if (++c->round_tag >= (1u << 25)) {
        (void)hipMemsetAsync(c->desc, 0, (size_t)((c->cfg.max_acc + kRTile - 1) / kRTile) * 8,
                             c->stream);
        c->round_tag = 1;
        // a replayed graph writes the tags it was captured with: once the
        // tags come round again, one of them could meet a later non-graph
        // epoch's tag in a stale descriptor
        graphs_stale(c);
    }
    return c->round_tag;
}

// the decision rounds work on the whole epoch
void view_epoch(dv_ctx *c) {
    c->v_status = c->status;
    c->v_tlen = c->tlen;
    c->v_n_txn = c->n_txn;
    c->v_n_txn_dev = nullptr;
    c->v_thresh = 0;
}

// a zeroed tile-ticket counter for the next single-pass launch
uint32_t *next_ticket(dv_ctx *c) {
    if (c->ticket > 0 && c->ticket % kTileCtrs == 0)
        (void)hipMemsetAsync(c->tile_ctr, 0, kTileCtrs * sizeof(uint32_t), c->stream);
    return &c->tile_ctr[c->ticket++ % kTileCtrs];
}

// the stable sort of pairs[0][0, n) by row (n_dev: the count on the device,
// n its upper bound); returns the buffer holding the result.  hist0_done:
// the probe counted the first pass's tile histogram.  (A one-sweep variant --
// digit totals in one launch, one scatter launch per pass with a per-digit
// decoupled look-back -- measured slower here: every tile of these sorts is
// resident at once, so the look-back became a chain of cross-XCD hand-offs,
// 167 us of scatters per config-D epoch against 125 us for the three-launch
// passes.  Round 3 measured it again with a thread per digit walking 16 tiles
// per round trip: 17.6 us per pass + 10.4 us of histogram per sort against
// 19.5 us per three-launch pass, 127 us per epoch against 114; and with every
// predecessor's count summed in one hop (no inclusive prefixes), 21.8 us per
// pass: the hand-offs cost more than the two kernel boundaries they save.)
// Small sorts: one LSD pass, then every bucket sorted inside one workgroup
// (k_bucket_sort, dvcc_internal.h bucket_sort_applies; DV_FLAG_LSD_SORT: off).
bool lsd_only(const dv_ctx *c) { return (c->cfg.flags & DV_FLAG_LSD_SORT) != 0; }
int sort_rows(dv_ctx *c, uint64_t n, int key_bits, hipEvent_t *ev, bool hist0_done, const uint32_t *n_dev) {
    return radix_sort_rows(c->stream, c->pairs, n, key_bits, c->counts, c->digit_tot, ev, hist0_done, n_dev,
                           lsd_only(c));
}
// the sort's timed launches (dv_stats.sort_passes): the scatter of every
// pass, or the one pass's scatter and the bucket launch
uint32_t sort_launches(const dv_ctx *c, uint64_t n, int key_bits, bool hist0_done, bool n_on_dev) {
    if (!lsd_only(c) && bucket_sort_applies(n, key_bits, hist0_done, n_on_dev)) return 2;
    return (uint32_t)radix_passes(key_bits, hist0_done);
}

Tables make_tables(dv_ctx *c) {
    Tables t{};
    t.n = 0;
    for (uint32_t i = 0; i < kMaxTables; i++) {
        const HostTable &h = c->tab[i];
        if (!h.created) continue;
        t.n = i + 1;
        t.t[i].ix = h.ix;
        t.t[i].pkey = h.implicit_rows ? c->pkey + h.row_base : nullptr;
        t.t[i].ktag = h.implicit_rows ? c->ktag + h.row_base : nullptr;
        t.t[i].hbits = h.implicit_rows ? h.hbits : nullptr;
        t.t[i].htag = h.htag;
        t.t[i].dense = h.implicit_rows && h.dense && h.htag < kTagWide ? 1u : 0u;
        t.t[i].bstart = h.bstart;
        t.t[i].nbuckets = h.nbuckets ? h.nbuckets : 1;
        t.t[i].row_base = h.row_base;
        t.t[i].hash_kind = h.hash_kind;
        t.t[i].part_cnt = c->cfg.part_cnt ? c->cfg.part_cnt : 1;
        t.t[i].m_part = div_magic(t.t[i].part_cnt);
        t.t[i].m_nb = div_magic(t.t[i].nbuckets);
        t.t[i].rep_part = (c->rep_P && i == 0) ? c->cfg.part_id : kNoRep;
    }
    return t;
}

// the row ids this epoch's sort keys and row-state bitmap span: the context's
// rows, or in a replicated epoch the global row space (a row id is the key)
uint64_t row_space(const dv_ctx *c) {
    return c->rep_P ? (uint64_t)c->rep_P * c->tab[0].nbuckets : c->total_rows;
}

int err_from_bits(uint32_t b) { return err_code_of(b); }

// idle time after which an asynchronous workgroup yields: the
// whole asynchronous phase of a config-D epoch takes ~130 us
constexpr uint64_t kAsyncIdleUs = 200;

bool timing(dv_ctx *c) { return (c->cfg.flags & DV_FLAG_TIMING) != 0; }
// dispatch timestamps of the scatter and pass launches (hipExtLaunchKernelGGL)
bool ktiming(dv_ctx *c) { return (c->cfg.flags & (DV_FLAG_TIMING | DV_FLAG_KERNEL_TIMING)) != 0; }

void rec(dv_ctx *c, int i) {
    if (timing(c)) (void)hipEventRecord(c->ev[i], c->stream);
}

float elapsed(dv_ctx *c, int a, int b) {
    float ms = 0;
    if (timing(c)) (void)hipEventElapsedTime(&ms, c->ev[a], c->ev[b]);
    return ms;
}

// the counters on the host once everything queued so far has run: the last
// kernel writes them into host-mapped memory and bumps a sequence word the
// host spins on (a blit plus a stream synchronisation cost ~25 us per epoch)
// the counters into mirror slot k behind everything queued so far; returns
// the sequence number mirror_wait waits for
unsigned long long mirror_out(dv_ctx *c, int k) {
    const unsigned long long want = ++c->cseq;
    launch_ctr_out(c->stream, c->ctr, c->d_mir[k], c->d_mseq[k], want);
    return want;
}

int mirror_wait(dv_ctx *c, int k, unsigned long long want) {
    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t i = 0;; i++) {
        if (__atomic_load_n(c->h_mseq[k], __ATOMIC_ACQUIRE) >= want) return DV_OK;
        if ((i & 1023) == 1023) {
            const hipError_t q = hipStreamQuery(c->stream);
            if (q == hipSuccess) {  // drained: the word must be there now
                if (__atomic_load_n(c->h_mseq[k], __ATOMIC_ACQUIRE) >= want) return DV_OK;
                return hip_fail(hipErrorUnknown, "counter mirror");
            }
            if (q != hipErrorNotReady) return hip_fail(q, "stream");
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(120)) return DV_ERR_STATE;
        }
        __builtin_ia32_pause();
    }
}

// a deferred counter mirror that no epoch clear has written yet: now
void mirror_flush(dv_ctx *c) {
    if (!c->mir_pending) return;
    c->mir_pending = false;
    launch_ctr_out(c->stream, c->ctr, c->d_mir[c->mir_slot], c->d_mseq[c->mir_slot], c->mir_seq);
}

int sync_counters(dv_ctx *c) {
    const unsigned long long want = mirror_out(c, 0);
    HIPCHK(hipGetLastError());
    return mirror_wait(c, 0, want);
}

}  // namespace

DvComm *&ctx_comm(dv_ctx *c) { return c->comm; }
hipStream_t ctx_stream(dv_ctx *c) { return c->stream; }
const dv_config &ctx_config(dv_ctx *c) { return c->cfg; }
bool ctx_has_tables(dv_ctx *c) {
    for (const auto &t : c->tab)
        if (t.loaded) return true;
    return false;
}
bool ctx_rep_capable(dv_ctx *c, uint32_t nranks) {
    const HostTable &t = c->tab[0];
    return c->cfg.workload == DV_YCSB && t.loaded && t.implicit_rows && t.hash_kind == DV_HASH_YCSB &&
           (uint64_t)nranks * t.nbuckets <= 0x7FFFFFFFull;
}
bool ctx_group_capable(dv_ctx *c, uint32_t nranks) {
    return ctx_rep_capable(c, nranks) && c->tab[0].dense && c->tab[0].nbuckets < (1ull << 30);
}
uint64_t ctx_table0_rows(dv_ctx *c) { return c->tab[0].nbuckets; }
void ctx_table0_cols(dv_ctx *c, uint64_t **f0, const uint64_t **pkey) {
    *f0 = c->f0 + c->tab[0].row_base;
    *pkey = c->pkey + c->tab[0].row_base;
}
uint32_t *ctx_err_words(dv_ctx *c) { return &c->ctr->err; }
const Counters *ctx_counters(dv_ctx *c) { return c->ctr; }
bool ctx_finish_pending(dv_ctx *c) { return c && c->fin_pending; }

int lane_exec_begin(dv_ctx *c, hipStream_t s) {
    if (!c->order) return DV_OK;
    LaneOrder &o = *c->order;
    const uint64_t t = c->order_k * o.n + c->lane_l;
    std::unique_lock<std::mutex> lk(o.mu);
    // (a lane never run for its turn -- groups not handed round the lanes in
    // order -- ends the order after kLaneWaitS instead of hanging the caller)
    if (!o.cv.wait_for(lk, std::chrono::seconds(kLaneWaitS), [&] { return t >= o.fail_at || o.next == t; }))
        o.fail_at = std::min(o.fail_at, o.next), o.cv.notify_all();
    if (t >= o.fail_at || o.next != t) return DV_ERR_STATE;  // (fail_at itself never executes)
    if (o.last) HIPCHK(hipStreamWaitEvent(s, o.last, 0));
    return DV_OK;
}

void lane_exec_end(dv_ctx *c, hipStream_t s) {
    if (!c->order) return;
    LaneOrder &o = *c->order;
    std::lock_guard<std::mutex> lk(o.mu);
    if (hipEventRecord(c->lane_ev, s) != hipSuccess) o.fail_at = std::min(o.fail_at, o.next + 1);
    o.last = c->lane_ev;
    o.next++;
    c->order_k++;
    o.cv.notify_all();
}

void lane_fail(dv_ctx *c) {
    if (!c->order) return;
    LaneOrder &o = *c->order;
    std::lock_guard<std::mutex> lk(o.mu);
    const uint64_t t = c->order_k * o.n + c->lane_l;  // (the execution this lane did not reach)
    o.fail_at = std::min(o.fail_at, t);
    o.cv.notify_all();
}

extern "C" {

const char *dv_strerror(int code) {
    switch (code) {
    case DV_OK: return "ok";
    case DV_ERR_ARG: return "bad argument or capacity exceeded";
    case DV_ERR_HIP: return "HIP runtime error";
    case DV_ERR_NOMEM: return "device allocation failed";
    case DV_ERR_KEY_NOT_FOUND: return "key does not exist in the index";
    case DV_ERR_DUP_ROW: return "a 2PL/OCC txn accesses the same row twice";
    case DV_ERR_NO_TABLE: return "table not created or not loaded";
    case DV_ERR_STATE: return "call out of order";
    case DV_ERR_NO_DEVICE: return "no HIP device";
    case DV_ERR_TXN_RANGE: return "access names a txn outside the epoch or txns out of order";
    default: return "unknown error";
    }
}

int dv_device_count(int *count) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (count) *count = (e == hipSuccess) ? n : 0;
    return (e == hipSuccess && n > 0) ? DV_OK : DV_ERR_NO_DEVICE;
}

void dv_close(dv_ctx *c) {
    if (!c) return;
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (auto &g : c->graphs)
        if (g.exec) (void)hipGraphExecDestroy(g.exec);
    c->graphs.clear();
    comm_free(c->comm);
    c->comm = nullptr;
    if (c->table_owner) {  // a lane: the tables are its owner's
        if (c->table_owner->lanes_open) c->table_owner->lanes_open--;
        for (auto &t : c->tab) t.ix = nullptr, t.bstart = nullptr, t.hbits = nullptr;
        c->f0 = c->pkey = nullptr;
        c->ktag = nullptr;
    }
    dfree(c->d_gate);
    if (c->lane_ev) (void)hipEventDestroy(c->lane_ev);
    for (auto &t : c->tab) {
        dfree(t.ix);
        dfree(t.bstart);
        dfree(t.hbits);
    }
    void *bufs[] = {c->f0, c->pkey, c->ktag, c->pairs[0], c->pairs[1], c->el, c->ew, c->counts,
                    c->digit_tot, c->rel[0], c->rel[1], c->vb8, c->tlen, c->acc_row,
                    c->ulist[0], c->ulist[1], c->tb_start, c->tb_end, c->desc, c->tile_ctr,
                    c->abounds, c->tword, c->carry_b, c->carry_tot,
                    c->status, c->verdict, c->ctr, c->d_acc, c->d_keys, c->d_types,
                    c->d_tables, c->d_commit, c->d_txn, c->d_grant, c->d_tb, c->split_err,
                    c->d_args, c->d_oid, c->tp_dsnap,
                    c->row_state, c->b_status, c->b_tlen, c->b_map, c->kinfo, c->ktsum, c->kill_bits, c->gc_tb, c->gc_tot,
                    c->hslot[0].acc, c->hslot[0].tb, c->hslot[1].acc, c->hslot[1].tb};
    for (void *b : bufs) dfree(b);
    for (auto &h : c->hslot) {
        if (h.copied) (void)hipEventDestroy(h.copied);
        if (h.drained) (void)hipEventDestroy(h.drained);
    }
    if (c->copy_stream) {
        (void)hipStreamSynchronize(c->copy_stream);
        (void)hipStreamDestroy(c->copy_stream);
    }
    if (c->h_ctr) (void)hipHostFree(c->h_ctr);
    if (c->h_pub) (void)hipHostFree(c->h_pub);
    for (auto &e : c->ev) if (e) (void)hipEventDestroy(e);
    for (auto &e : c->sev) if (e) (void)hipEventDestroy(e);
    for (auto &e : c->pev) if (e) (void)hipEventDestroy(e);
    for (auto &pr : c->kprof.pool) {
        (void)hipEventDestroy(pr.first);
        (void)hipEventDestroy(pr.second);
    }
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    if (c->lane_stream) (void)hipStreamDestroy(c->lane_stream);
    delete c;
}

int dv_open(dv_ctx **out, const dv_config *cfg) {
    if (!out || !cfg) return DV_ERR_ARG;
    *out = nullptr;
    if (cfg->cc_alg != DV_NO_WAIT && cfg->cc_alg != DV_WAIT_DIE && cfg->cc_alg != DV_OCC &&
        cfg->cc_alg != DV_CALVIN)
        return DV_ERR_ARG;
    if (cfg->workload != DV_YCSB && cfg->workload != DV_TPCC) return DV_ERR_ARG;
    if (cfg->max_txn == 0 || cfg->max_txn > kMaxTxn || cfg->max_acc == 0 ||
        cfg->max_acc > kMaxAcc || cfg->part_cnt == 0 || cfg->part_id >= cfg->part_cnt)
        return DV_ERR_ARG;
    int ndev = 0;
    if (dv_device_count(&ndev) != DV_OK || cfg->device < 0 || cfg->device >= ndev)
        return DV_ERR_NO_DEVICE;
    dv_ctx *c = new (std::nothrow) dv_ctx();
    if (!c) return DV_ERR_NOMEM;
    c->cfg = *cfg;
    c->cstride = cfg->workload == DV_TPCC ? 3u : 1u;
    int r = hip_fail(hipSetDevice(cfg->device), "hipSetDevice");
    if (!r) r = hip_fail(hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking), "stream");
    c->stream = c->own_stream;
    const uint64_t A = cfg->max_acc;
    const uint32_t T = cfg->max_txn;
    c->n_txn_cap_pad = (T + 3u) & ~3u;
    const uint32_t nb = nblocks_for(A);
    if (!r) r = dalloc(&c->pairs[0], A);
    if (!r) r = dalloc(&c->pairs[1], A);
    if (!r) r = dalloc(&c->counts, (uint64_t)kRadixMax * nb);
    if (!r) r = dalloc(&c->digit_tot, kRadixMax);
    if (!r) r = dalloc(&c->status, c->n_txn_cap_pad);
    if (!r) r = dalloc(&c->verdict, c->n_txn_cap_pad);
    if (!r) r = dalloc(&c->ctr, 1);
    const uint32_t rnb = (uint32_t)((A + kRTile - 1) / kRTile);  // single-pass tiles
    if (!r) r = dalloc(&c->tb_start, c->n_txn_cap_pad);
    if (!r) r = dalloc(&c->tb_end, c->n_txn_cap_pad);
    if (!r) r = dalloc(&c->desc, rnb);
    if (!r) r = dalloc(&c->tile_ctr, kTileCtrs);
    if (!r) r = dalloc(&c->d_gate, 2);
    if (!r) r = hip_fail(hipEventCreateWithFlags(&c->lane_ev, hipEventDisableTiming), "hipEventCreate");
    if (!r) r = hip_fail(hipMemsetAsync(c->desc, 0, (size_t)rnb * 8, c->stream), "memset");
    if (!r) r = hip_fail(hipMemsetAsync(c->d_gate, 0, 2 * sizeof(uint32_t), c->stream), "memset");
    if (!r && cfg->cc_alg != DV_CALVIN) {
        r = dalloc(&c->rel[0], A);
        if (!r) r = dalloc(&c->rel[1], A);
        if (!r) r = dalloc(&c->tlen, c->n_txn_cap_pad);
        if (!r) r = dalloc(&c->acc_row, A);
        if (!r) r = dalloc(&c->ulist[0], T);
        if (!r) r = dalloc(&c->ulist[1], T);
        if (!r) r = dalloc(&c->abounds, kAsyncGroups);
        if (!r) r = dalloc(&c->tword, c->n_txn_cap_pad);
        if (!r) c->async_g = async_groups(cfg->device);
        int khz = 0;
        if (!r && hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, cfg->device) == hipSuccess && khz > 0)
            c->wall_khz = (uint64_t)khz;
        c->async_idle_ticks = kAsyncIdleUs * c->wall_khz / 1000;
        // verdict bytes: 16 per txn; grown on demand for longer txns (dv_epoch_begin)
        c->vb8_cap = (uint64_t)c->n_txn_cap_pad << 4;
        if (!r) r = dalloc(&c->vb8, c->vb8_cap);
    }
    if (!r && cfg->cc_alg == DV_CALVIN) r = dalloc(&c->el, A);
    if (!r && cfg->cc_alg == DV_CALVIN) r = dalloc(&c->ew, A);
    constexpr size_t kMirBytes = ((sizeof(Counters) + 63) & ~size_t(63)) + 128;  // a mirror slot + its word
    if (!r) r = hip_fail(hipHostMalloc(reinterpret_cast<void **>(&c->h_ctr), 2 * kMirBytes,
                                       hipHostMallocMapped | hipHostMallocCoherent),
                         "hipHostMalloc");
    if (!r) r = hip_fail(hipHostGetDevicePointer(reinterpret_cast<void **>(&c->d_hctr), c->h_ctr, 0),
                         "hipHostGetDevicePointer");
    if (!r) {
        std::memset(c->h_ctr, 0, 2 * kMirBytes);
        const size_t off = (sizeof(Counters) + 63) & ~size_t(63);
        for (int k = 0; k < 2; k++) {
            char *h = reinterpret_cast<char *>(c->h_ctr) + k * kMirBytes;
            char *d = reinterpret_cast<char *>(c->d_hctr) + k * kMirBytes;
            c->h_mir[k] = reinterpret_cast<Counters *>(h);
            c->d_mir[k] = reinterpret_cast<Counters *>(d);
            c->h_mseq[k] = reinterpret_cast<unsigned long long *>(h + off);
            c->d_mseq[k] = reinterpret_cast<unsigned long long *>(d + off);
        }
        c->h_cseq = c->h_mseq[0];
        c->d_cseq = c->d_mseq[0];
    }
    if (!r && cfg->cc_alg != DV_CALVIN) {
        r = hip_fail(hipHostMalloc(reinterpret_cast<void **>(&c->h_pub), sizeof(RoundPub),
                                   hipHostMallocMapped | hipHostMallocCoherent),
                     "hipHostMalloc");
        if (!r) r = hip_fail(hipHostGetDevicePointer(reinterpret_cast<void **>(&c->d_pub), c->h_pub, 0),
                             "hipHostGetDevicePointer");
        if (!r) std::memset(c->h_pub, 0, sizeof(RoundPub));
    }
    if (!r && ktiming(c)) {
        for (auto &e : c->ev) if (!r) r = hip_fail(hipEventCreate(&e), "hipEventCreate");
        for (auto &e : c->sev) if (!r) r = hip_fail(hipEventCreate(&e), "hipEventCreate");
        for (auto &e : c->pev) if (!r) r = hip_fail(hipEventCreate(&e), "hipEventCreate");
    }
    if (!r) r = hip_fail(hipMemsetAsync(c->verdict, 0, c->n_txn_cap_pad, c->stream), "memset");
    if (!r) r = hip_fail(hipStreamSynchronize(c->stream), "sync");
    if (r) {
        dv_close(c);
        return r;
    }
    *out = c;
    return DV_OK;
}

// a decision lane of `owner`: a context of the same configuration whose
// epochs run against the owner's tables (dv_epoch_run_device_lanes); the
// owner's tables are loaded first and stay frozen while lanes are open
int dv_open_lane(dv_ctx *owner, dv_ctx **out) {
    if (!owner || !out) return DV_ERR_ARG;
    *out = nullptr;
    if (owner->table_owner || owner->comm) return DV_ERR_ARG;
    if (owner->phase != 0) return DV_ERR_STATE;
    if (!ctx_has_tables(owner)) return DV_ERR_NO_TABLE;
    dv_ctx *c = nullptr;
    int r = dv_open(&c, &owner->cfg);
    if (r) return r;
    r = hip_fail(hipStreamSynchronize(owner->stream), "sync");
    if (r) {
        dv_close(c);
        return r;
    }
    for (uint32_t i = 0; i < kMaxTables; i++) c->tab[i] = owner->tab[i];
    c->total_rows = owner->total_rows;
    c->f0 = owner->f0;
    c->pkey = owner->pkey;
    c->ktag = owner->ktag;
    c->cstride = owner->cstride;
    c->prefix_txns = owner->prefix_txns;
    c->table_owner = owner;
    owner->lanes_open++;
    *out = c;
    return DV_OK;
}

void *dv_stream(dv_ctx *c) { return c ? (void *)c->stream : nullptr; }
void *dv_own_stream(dv_ctx *c) { return c ? (void *)c->own_stream : nullptr; }

int dv_set_stream(dv_ctx *c, void *stream) {
    if (!c) return DV_ERR_ARG;
    if (c->phase != 0) return DV_ERR_STATE;
    HIPCHK(hipStreamSynchronize(c->stream));
    c->stream = reinterpret_cast<hipStream_t>(stream);
    return DV_OK;
}

}  // extern "C"

namespace {
// the carry-over's block counts for nb blocks and its totals (kRefillTot words)
int carry_bufs(dv_ctx *c, uint32_t nb) {
    if (nb <= c->carry_nb && c->carry_tot) return DV_OK;
    HIPCHK(hipStreamSynchronize(c->stream));
    graphs_stale(c);
    dfree(c->carry_b);
    c->carry_b = nullptr;
    c->carry_nb = 0;
    int r = dalloc(&c->carry_b, 2ull * (nb ? nb : 1));
    if (!r && !c->carry_tot) r = dalloc(&c->carry_tot, kRefillTot);
    if (r) return r;
    c->carry_nb = nb ? nb : 1;
    return DV_OK;
}
}  // namespace

extern "C" {

int dv_epoch_carry(dv_ctx *c, const dv_epoch_dev *ep, uint32_t max_txn, dv_epoch_dev *out) {
    KProfScope kps_(c);
    if (!c || !ep || !out) return DV_ERR_ARG;
    if (c->phase != 0 || c->cfg.cc_alg == DV_CALVIN) return DV_ERR_STATE;
    if (ep->n_txn != c->n_txn || ep->n_acc != c->n_acc) return DV_ERR_STATE;  // not the last epoch
    if (ep->n_acc && (!out->keys || !out->types || !out->acc_txn || (ep->tables && !out->tables)))
        return DV_ERR_ARG;
    HIPCHK(hipSetDevice(c->cfg.device));
    const uint32_t nb = carry_blocks(ep->n_txn);
    int r = carry_bufs(c, nb);
    if (r) return r;
    launch_carry(c->stream, c->status, c->rs, c->re, ep->n_txn, max_txn, ep->keys, ep->types,
                 ep->tables, const_cast<uint64_t *>(out->keys), const_cast<uint8_t *>(out->types),
                 const_cast<uint32_t *>(out->acc_txn),
                 ep->tables ? const_cast<uint8_t *>(out->tables) : nullptr,
                 c->carry_b, c->carry_b + c->carry_nb, c->carry_tot);
    HIPCHK(hipGetLastError());
    uint32_t tot[3] = {0, 0, 0};
    HIPCHK(hipMemcpyAsync(tot, c->carry_tot, sizeof(tot), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    out->n_txn = tot[0];
    out->n_acc = tot[1];
    out->max_txn_acc = ep->max_txn_acc;
    return DV_OK;
}

int dv_epoch_group_carry(dv_ctx *c, const dv_epoch_dev *homes, uint32_t n_homes, uint32_t txns_per_rank,
                         const uint8_t *d_commit, uint32_t max_txn, dv_epoch_dev *outs) {
    KProfScope kps_(c);
    constexpr uint32_t kMaxGroupBatches = 64;
    if (!c || !homes || !d_commit || !outs || !n_homes || n_homes > kMaxGroupBatches) return DV_ERR_ARG;
    if (c->phase != 0) return DV_ERR_STATE;
    if (txns_per_rank > c->cfg.max_txn) return DV_ERR_ARG;
    for (uint32_t e = 0; e < n_homes; e++) {
        const dv_epoch_dev &h = homes[e];
        const dv_epoch_dev &o = outs[e];
        if (h.n_txn > txns_per_rank || (h.n_acc && (!h.keys || !h.types || !h.acc_txn))) return DV_ERR_ARG;
        if (h.n_acc && (!o.keys || !o.types || !o.acc_txn || (h.tables && !o.tables))) return DV_ERR_ARG;
    }
    HIPCHK(hipSetDevice(c->cfg.device));
    int r = carry_bufs(c, carry_blocks(txns_per_rank));
    if (!r && !c->gc_tb) r = dalloc(&c->gc_tb, 2ull * c->cfg.max_txn + 2);
    if (!r && !c->gc_tot) r = dalloc(&c->gc_tot, 3ull * kMaxGroupBatches);
    if (r) return r;
    uint32_t *tbs = c->gc_tb, *tbe = c->gc_tb + c->cfg.max_txn + 1;
    for (uint32_t e = 0; e < n_homes; e++) {
        const dv_epoch_dev &h = homes[e];
        dv_epoch_dev &o = outs[e];
        launch_txn_ranges(c->stream, h.acc_txn, h.n_acc, h.n_txn, tbs, tbe);
        // the commit bytes of this rank's txns of epoch e: 1 committed (== ST_COMMIT), 0 aborted
        launch_carry(c->stream, d_commit + (size_t)e * txns_per_rank, tbs, tbe, h.n_txn, max_txn, h.keys, h.types,
                     h.tables, const_cast<uint64_t *>(o.keys), const_cast<uint8_t *>(o.types),
                     const_cast<uint32_t *>(o.acc_txn), h.tables ? const_cast<uint8_t *>(o.tables) : nullptr,
                     c->carry_b, c->carry_b + c->carry_nb, c->gc_tot + 3 * e);
    }
    HIPCHK(hipGetLastError());
    uint32_t tot[3 * kMaxGroupBatches];
    HIPCHK(hipMemcpyAsync(tot, c->gc_tot, 3ull * n_homes * sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    for (uint32_t e = 0; e < n_homes; e++) {
        outs[e].n_txn = tot[3 * e];
        outs[e].n_acc = tot[3 * e + 1];
        outs[e].max_txn_acc = homes[e].max_txn_acc;
        outs[e].ts = nullptr;
        outs[e].n_acc_dev = nullptr;
    }
    return DV_OK;
}

int dv_set_timing(dv_ctx *c, uint32_t flags) {
    if (!c) return DV_ERR_ARG;
    if (c->phase != 0) return DV_ERR_STATE;
    constexpr uint32_t kBits = DV_FLAG_TIMING | DV_FLAG_KERNEL_TIMING | DV_FLAG_KERNEL_PROFILE;
    if ((c->cfg.flags & DV_FLAG_KERNEL_PROFILE) && !(flags & DV_FLAG_KERNEL_PROFILE)) {
        HIPCHK(hipStreamSynchronize(c->stream));  // the launches still pending are read now
        kprof_harvest(&c->kprof, true);
    }
    c->cfg.flags = (c->cfg.flags & ~kBits) | (flags & kBits);
    if (ktiming(c) && !c->ev[0]) {
        HIPCHK(hipSetDevice(c->cfg.device));
        for (auto &e : c->ev) HIPCHK(hipEventCreate(&e));
        for (auto &e : c->sev) HIPCHK(hipEventCreate(&e));
        for (auto &e : c->pev) HIPCHK(hipEventCreate(&e));
    }
    return DV_OK;
}

int dv_kernel_times(dv_ctx *c, dv_kernel_time *out, uint32_t cap, int reset) {
    if (!c || (cap && !out)) return DV_ERR_ARG;
    if (c->phase != 0) return DV_ERR_STATE;
    HIPCHK(hipSetDevice(c->cfg.device));
    HIPCHK(hipStreamSynchronize(c->stream));
    kprof_harvest(&c->kprof, true);
    uint32_t n = 0;
    for (const auto &kv : c->kprof.sums) {
        if (n < cap) {
            dv_kernel_time &k = out[n];
            std::memset(&k, 0, sizeof(k));
            std::snprintf(k.name, sizeof(k.name), "%s", kv.first.c_str());
            k.launches = kv.second.launches;
            k.ms_total = kv.second.ms;
        }
        n++;
    }
    if (reset) {
        c->kprof.sums.clear();
        c->kprof.dropped = 0;
    }
    return (int)n;
}

namespace {
// one state column of n rows between the host (dense) and the context's
// column array (every cstride-th word), synchronously
hipError_t col_copy(dv_ctx *c, void *dst, const void *src, uint64_t n, hipMemcpyKind kind) {
    const size_t cs = (size_t)c->cstride * 8;
    const bool to_dev = kind == hipMemcpyHostToDevice;
    hipError_t e = c->cstride == 1 ? hipMemcpyAsync(dst, src, n * 8, kind, c->stream)
                                   : hipMemcpy2DAsync(dst, to_dev ? cs : 8, src, to_dev ? 8 : cs, 8, n, kind,
                                                      c->stream);
    return e == hipSuccess ? hipStreamSynchronize(c->stream) : e;
}
}  // namespace

// Workload::init_schema (system/wl.cpp:31-149) + IndexHash::init (index_hash.cpp:22-42)
int dv_create_table(dv_ctx *c, uint32_t table, uint64_t capacity_rows, uint64_t nbuckets,
                    uint32_t hash_kind) {
    if (!c || table >= kMaxTables || capacity_rows == 0 || nbuckets == 0 ||
        (hash_kind != DV_HASH_YCSB && hash_kind != DV_HASH_MOD))
        return DV_ERR_ARG;
    HostTable &t = c->tab[table];
    if (t.created || c->lanes_open || c->table_owner) return DV_ERR_STATE;  // (lanes share frozen tables)
    if (c->total_rows + capacity_rows > kMaxRows) return DV_ERR_ARG;
    HIPCHK(hipSetDevice(c->cfg.device));
    // grow the global hot column / primary-key arrays (load-time only)
    const uint64_t new_total = c->total_rows + capacity_rows;
    const uint64_t cs = c->cstride;  // (TPC-C: 3 state columns per row, row-major)
    uint64_t *nf0 = nullptr, *npk = nullptr;
    uint8_t *ntg = nullptr;
    int r = dalloc(&nf0, new_total * cs);
    if (!r) r = dalloc(&npk, new_total);
    if (!r) r = dalloc(&ntg, new_total);
    if (r) { dfree(nf0); dfree(npk); dfree(ntg); return r; }
    if (c->total_rows) {
        HIPCHK(hipMemcpyAsync(nf0, c->f0, c->total_rows * cs * 8, hipMemcpyDeviceToDevice, c->stream));
        HIPCHK(hipMemcpyAsync(npk, c->pkey, c->total_rows * 8, hipMemcpyDeviceToDevice, c->stream));
        HIPCHK(hipMemcpyAsync(ntg, c->ktag, c->total_rows, hipMemcpyDeviceToDevice, c->stream));
    }
    HIPCHK(hipMemsetAsync(nf0 + c->total_rows * cs, 0, capacity_rows * cs * 8, c->stream));
    HIPCHK(hipMemsetAsync(npk + c->total_rows, 0xFF, capacity_rows * 8, c->stream));
    HIPCHK(hipMemsetAsync(ntg + c->total_rows, kTagWide, capacity_rows, c->stream));  // (no key: pkey decides)
    HIPCHK(hipStreamSynchronize(c->stream));
    graphs_stale(c);
    dfree(c->f0);
    dfree(c->pkey);
    dfree(c->ktag);
    c->f0 = nf0;
    c->pkey = npk;
    c->ktag = ntg;
    t.created = true;
    t.cap_rows = capacity_rows;
    t.row_base = c->total_rows;
    t.nbuckets = nbuckets;
    t.hash_kind = hash_kind;
    c->total_rows = new_total;
    return DV_OK;
}

// The home-tag bitmap of an implicit-row table: one bit per row, set where
// the row's key tag is htag (TableDesc::hbits; htag = kTagWide: none).
int build_home_bits(dv_ctx *c, HostTable &t, uint32_t htag) {
    graphs_stale(c);
    dfree(t.hbits);
    t.hbits = nullptr;
    t.htag = kTagWide;
    if (htag >= kTagWide || !t.implicit_rows || t.nbuckets == 0) return DV_OK;
    int r = dalloc(&t.hbits, (t.nbuckets + 31) / 32);
    if (r) return r;
    launch_home_bits(c->stream, c->ktag + t.row_base, t.nbuckets, htag, t.hbits);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->stream));
    t.htag = htag;
    return DV_OK;
}

// table_t::get_new_row + IndexHash::index_insert for n rows (row i = keys[i]).
// Chains keep BucketHeader::insert_item order (index_hash.cpp:172-201): distinct
// keys in first-insertion order, repeated keys newest first.
int dv_load_table(dv_ctx *c, uint32_t table, const uint64_t *keys, const uint64_t *f0, uint64_t n) {
    if (!c || table >= kMaxTables || (!keys && n)) return DV_ERR_ARG;
    HostTable &t = c->tab[table];
    if (!t.created) return DV_ERR_NO_TABLE;
    if (n > t.cap_rows) return DV_ERR_ARG;
    if (c->lanes_open || c->table_owner) return DV_ERR_STATE;
    HIPCHK(hipSetDevice(c->cfg.device));
    const uint64_t nb = t.nbuckets;
    const uint32_t P = c->cfg.part_cnt;
    auto bucket = [&](uint64_t k) { return t.hash_kind == DV_HASH_YCSB ? (k / P) % nb : k % nb; };
    std::vector<uint32_t> cnt(nb + 1, 0);
    for (uint64_t i = 0; i < n; i++) cnt[bucket(keys[i]) + 1]++;
    bool direct = (n == nb);
    for (uint64_t b = 0; b < nb && direct; b++) direct = cnt[b + 1] == 1;
    for (uint64_t b = 0; b < nb; b++) cnt[b + 1] += cnt[b];
    std::vector<IxEntry> ent(n ? n : 1);
    {
        std::vector<uint32_t> fill(cnt.begin(), cnt.end() - 1);
        for (uint64_t i = 0; i < n; i++) ent[fill[bucket(keys[i])]++] = IxEntry{keys[i], i};
        // within a bucket: group equal keys at the first occurrence, newest first
        for (uint64_t b = 0; b < nb && !direct; b++) {
            const uint32_t lo = cnt[b], hi = cnt[b + 1];
            if (hi - lo < 2) continue;
            std::vector<IxEntry> tmp(ent.begin() + lo, ent.begin() + hi), outv;
            std::vector<bool> used(tmp.size(), false);
            for (size_t a = 0; a < tmp.size(); a++) {
                if (used[a]) continue;
                std::vector<IxEntry> same;
                for (size_t z = a; z < tmp.size(); z++)
                    if (!used[z] && tmp[z].key == tmp[a].key) { same.push_back(tmp[z]); used[z] = true; }
                for (auto it = same.rbegin(); it != same.rend(); ++it) outv.push_back(*it);
            }
            std::copy(outv.begin(), outv.end(), ent.begin() + lo);
        }
    }
    graphs_stale(c);
    dfree(t.ix);
    dfree(t.bstart);
    dfree(t.hbits);
    t.ix = nullptr;
    t.bstart = nullptr;
    t.hbits = nullptr;
    t.htag = kTagWide;
    // keys in bucket order: row b is in bucket b, the pkey column is the index
    bool implicit = direct;
    for (uint64_t b = 0; b < nb && implicit; b++) implicit = ent[cnt[b]].row == b;
    t.implicit_rows = implicit;
    t.dense = false;
    int r = implicit ? DV_OK : dalloc(&t.ix, direct ? nb : (n ? n : 1));
    if (r) return r;
    if (direct && !implicit) {
        std::vector<IxEntry> d(nb);
        for (uint64_t b = 0; b < nb; b++) d[b] = ent[cnt[b]];
        HIPCHK(hipMemcpy(t.ix, d.data(), nb * sizeof(IxEntry), hipMemcpyHostToDevice));
    } else if (!direct) {
        r = dalloc(&t.bstart, nb + 1);
        if (r) return r;
        if (n) HIPCHK(hipMemcpy(t.ix, ent.data(), n * sizeof(IxEntry), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(t.bstart, cnt.data(), (nb + 1) * sizeof(uint32_t), hipMemcpyHostToDevice));
    }
    if (n) {
        if (f0) HIPCHK(col_copy(c, c->f0 + t.row_base * c->cstride, f0, n, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(c->pkey + t.row_base, keys, n * 8, hipMemcpyHostToDevice));
        if (implicit) {  // row i holds keys[i]
            std::vector<uint8_t> tg(n);
            uint64_t hist[256] = {};
            for (uint64_t i = 0; i < n; i++) hist[tg[i] = key_tag(t.hash_kind, nb, P, keys[i])]++;
            HIPCHK(hipMemcpy(c->ktag + t.row_base, tg.data(), n, hipMemcpyHostToDevice));
            uint32_t home = 0;  // the most common tag
            for (uint32_t v = 1; v < kTagWide; v++)
                if (hist[v] > hist[home]) home = v;
            r = build_home_bits(c, t, hist[home] ? home : kTagWide);
            if (r) return r;
        }
    }
    t.n_rows = n;
    t.loaded = true;
    return DV_OK;
}

int dv_load_ycsb_partition(dv_ctx *c, uint64_t rows_per_part) {
    if (!c || rows_per_part == 0) return DV_ERR_ARG;
    if (c->lanes_open || c->table_owner) return DV_ERR_STATE;
    HostTable &t = c->tab[0];
    if (!t.created) {
        int r = dv_create_table(c, 0, rows_per_part, rows_per_part, DV_HASH_YCSB);
        if (r) return r;
    }
    if (t.cap_rows < rows_per_part || t.nbuckets != rows_per_part || t.hash_kind != DV_HASH_YCSB)
        return DV_ERR_ARG;
    HIPCHK(hipSetDevice(c->cfg.device));
    graphs_stale(c);
    dfree(t.ix);
    dfree(t.bstart);
    t.ix = nullptr;
    t.bstart = nullptr;
    t.implicit_rows = true;  // row r holds key r * P + part, in bucket r
    t.dense = true;
    launch_ycsb_load(c->stream, rows_per_part, c->cfg.part_cnt, c->cfg.part_id, c->f0 + t.row_base,
                     c->pkey + t.row_base, c->ktag + t.row_base);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->stream));
    // row r holds key r * P + part: every tag is the partition's
    const int r = build_home_bits(c, t, key_tag(DV_HASH_YCSB, rows_per_part, c->cfg.part_cnt ? c->cfg.part_cnt : 1,
                                                c->cfg.part_id));
    if (r) return r;
    t.n_rows = rows_per_part;
    t.loaded = true;
    return DV_OK;
}

int dv_read_rows(dv_ctx *c, uint32_t table, const uint64_t *keys, uint64_t n, uint64_t *out_f0) {
    if (!c || table >= kMaxTables || (n && (!keys || !out_f0))) return DV_ERR_ARG;
    if (!c->tab[table].loaded) return DV_ERR_NO_TABLE;
    if (!n) return DV_OK;
    HIPCHK(hipSetDevice(c->cfg.device));
    uint64_t *dk = nullptr, *dout = nullptr;
    int r = dalloc(&dk, n);
    if (!r) r = dalloc(&dout, n);
    if (!r) {
        HIPCHK(hipMemsetAsync(c->ctr, 0, sizeof(Counters), c->stream));
        HIPCHK(hipMemcpyAsync(dk, keys, n * 8, hipMemcpyHostToDevice, c->stream));
        launch_gather_rows(c->stream, make_tables(c), table, dk, n, c->f0, c->cstride, dout, c->ctr);
        HIPCHK(hipMemcpyAsync(out_f0, dout, n * 8, hipMemcpyDeviceToHost, c->stream));
        r = sync_counters(c);
        if (!r) r = err_from_bits(c->h_ctr->err);
    }
    dfree(dk);
    dfree(dout);
    return r;
}

int dv_read_table(dv_ctx *c, uint32_t table, uint64_t first_row, uint64_t n, uint64_t *out_f0) {
    if (!c || table >= kMaxTables || (n && !out_f0)) return DV_ERR_ARG;
    const HostTable &t = c->tab[table];
    if (!t.created) return DV_ERR_NO_TABLE;
    if (first_row + n > t.cap_rows) return DV_ERR_ARG;
    if (!n) return DV_OK;
    HIPCHK(hipSetDevice(c->cfg.device));
    HIPCHK(col_copy(c, out_f0, c->f0 + (t.row_base + first_row) * c->cstride, n, hipMemcpyDeviceToHost));
    return DV_OK;
}

// ---------------------------------------------------------------- TPC-C tables
int dv_load_table_cols(dv_ctx *c, uint32_t table, const uint64_t *keys, const uint64_t *col0,
                       const uint64_t *col1, const uint64_t *col2, uint64_t n) {
    if (!c || c->cfg.workload != DV_TPCC) return DV_ERR_ARG;
    int r = dv_load_table(c, table, keys, col0, n);
    if (r || !n) return r;
    const HostTable &t = c->tab[table];
    uint64_t *g = c->f0 + t.row_base * c->cstride;
    if (col1) HIPCHK(col_copy(c, g + 1, col1, n, hipMemcpyHostToDevice));
    if (col2) HIPCHK(col_copy(c, g + 2, col2, n, hipMemcpyHostToDevice));
    return DV_OK;
}

int dv_read_table_col(dv_ctx *c, uint32_t table, uint32_t col, uint64_t first_row, uint64_t n,
                      uint64_t *out) {
    if (!c || col > 2 || (col && c->cfg.workload != DV_TPCC)) return DV_ERR_ARG;
    if (col == 0) return dv_read_table(c, table, first_row, n, out);
    if (table >= kMaxTables || (n && !out)) return DV_ERR_ARG;
    const HostTable &t = c->tab[table];
    if (!t.created) return DV_ERR_NO_TABLE;
    if (first_row + n > t.cap_rows) return DV_ERR_ARG;
    if (!n) return DV_OK;
    HIPCHK(hipSetDevice(c->cfg.device));
    HIPCHK(col_copy(c, out, c->f0 + (t.row_base + first_row) * c->cstride + col, n, hipMemcpyDeviceToHost));
    return DV_OK;
}

// TPCCWorkload::init (tpcc_wl.cpp:95-200): the six tables of this context's
// partition, chained IndexHash tables with one bucket per row (key % rows)
int dv_tpcc_load(dv_ctx *c, const dv_tpcc_params *p, uint64_t seed) {
    if (!c || !p || c->cfg.workload != DV_TPCC || p->part_cnt != c->cfg.part_cnt) return DV_ERR_ARG;
    const uint32_t part = c->cfg.part_id;
    for (uint32_t tb = DV_TPCC_WAREHOUSE; tb <= DV_TPCC_CUST_LAST; tb++) {
        uint64_t n = 0;
        int r = dv_tpcc_table_rows(p, part, tb, &n);
        if (r) return r;
        const uint64_t cap = n ? n : 1;
        std::vector<uint64_t> k(cap), a(cap), b(cap), d(cap);
        r = dv_tpcc_table(p, seed, part, tb, k.data(), a.data(), b.data(), d.data());
        if (!r) r = dv_create_table(c, tb, cap, cap, DV_HASH_MOD);
        if (!r) r = dv_load_table_cols(c, tb, k.data(), a.data(), b.data(), d.data(), n);
        if (r) return r;
    }
    return DV_OK;
}

// ---------------------------------------------------------------- epoch
// Probe + sort + per-row queue construction; for CALVIN also the grant groups
// (the lock thread's whole job for the epoch, calvin_thread.cpp:40-100).
namespace {
bool tb_epoch(const dv_ctx *c, const dv_epoch_dev *ep);

// ---- epoch graphs.  A pipelined epoch's host work is ~15-25 launches (the
// TPC-C window and config B were bound by it: ~3 us of host time per
// launch).  Its decision -- every launch after the epoch's clear -- depends
// on the epoch's buffers, sizes and the context's knobs only, so the second
// time the same (buffers, sizes, knobs) come, the launches are captured into
// a graph (hipStreamBeginCapture right after the clear), and from then on
// replayed with one hipGraphLaunch: the host walks the same enqueue code for
// its state with every launch skipped (tl_dry).  What a replay reuses and
// the kernels must not see stale: the look-back tags baked into the graph --
// the clear of a graph epoch zeroes the descriptors -- and the tile tickets,
// which every clear zeroes.  The clear itself stays a plain launch (its
// gate, mirror slot and sequence differ per epoch).  A capture that fails
// (a call the capture cannot take) runs the decision again uncaptured and
// the key is never captured again; DVCC_NO_GRAPHS=1 turns the graphs off.
extern "C++" {  // (templates, inside the C API's block)
// (prefix-kill epochs take no graphs: their ~25 launches overlap the device
// work under decision lanes -- config D is device-bound.  Measured with every
// prefix epoch replayed (4 distinct epochs over 4 lanes, 100 steps): host
// queueing 89-103 -> 47-49 us per epoch, epoch 0.1608-0.1613 -> 0.1623-0.1642
// ms, profiles/r05_n)
constexpr size_t kMaxGraphs = 24;  // per context
constexpr uint32_t kGraphNever = 0xFFFFFFFFu;
constexpr uint32_t kGraphAfter = 3;  // encounters of a key before its capture
struct GraphRun {
    dv_ctx *c = nullptr;
    dv_ctx::EpochGraph *g = nullptr;
    bool capture = false, began = false;
};
thread_local GraphRun *tl_graph = nullptr;
// DVCC_HOST_PROF: host seconds in graph_decide's replays -- the walk of the
// enqueue code (its clear launch included) and hipGraphLaunch -- and captures
thread_local double tl_hp_walk = 0, tl_hp_glaunch = 0;
thread_local uint32_t tl_hp_replays = 0, tl_hp_captures = 0;

bool graph_active(const dv_ctx *c) {
    const GraphRun *g = tl_graph;
    return g && g->c == c && (g->g->exec || g->capture);
}
uint64_t *graph_desc(dv_ctx *c) { return graph_active(c) ? c->desc : nullptr; }
uint32_t graph_ndesc(dv_ctx *c) {
    return graph_active(c) ? (uint32_t)((c->cfg.max_acc + kRTile - 1) / kRTile) : 0u;
}

// right after an epoch's clear: start the capture, or skip the launches of a replay
void graph_after_clear(dv_ctx *c) {
    GraphRun *g = tl_graph;
    if (!g || g->c != c || g->began) return;
    g->began = true;
    if (g->g->exec) {
        tl_dry = true;
    } else if (g->capture && hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal) != hipSuccess) {
        (void)hipGetLastError();
        g->capture = false;
        g->g->seen = kGraphNever;
    }
}

// decide(): an epoch's queueing from its epoch_setup through its decision
// (the clear first) -- and, under decision lanes, its execution (run_lanes'
// tail); ep / args name its buffers, xk whatever else the launches' arguments
// hold (the tail's commit / o_id outputs and ordering words)
struct GraphKeyX {
    uint64_t w[4] = {0, 0, 0, 0};
};
template <class F>
int graph_decide(dv_ctx *c, const dv_epoch_dev *ep, const void *args, F &&decide, const GraphKeyX &xk = {}) {
    static const bool off = std::getenv("DVCC_NO_GRAPHS") != nullptr;
    if (off || timing(c) || ktiming(c) || (c->cfg.flags & DV_FLAG_KERNEL_PROFILE) || tl_kprof || c->comm ||
        c->rep_P || c->route || tl_graph)
        return decide();
    const uint64_t key[22] = {(uint64_t)ep->keys, (uint64_t)ep->types, (uint64_t)ep->acc_txn, (uint64_t)ep->tables,
                              (uint64_t)ep->txn_begin, (uint64_t)ep->recs32, (uint64_t)ep->ts,
                              (uint64_t)ep->n_acc_dev, ep->n_acc, ep->n_txn | (uint64_t)ep->max_txn_acc << 32,
                              (uint64_t)args, c->async_g | (uint64_t)c->async_max_iters << 32, c->async_idle_ticks,
                              c->cfg.flags | (uint64_t)c->prefix_txns << 32, c->ws_gen, (uint64_t)c->keys32,
                              (uint64_t)c->stream, (uint64_t)c->cfg.max_acc, xk.w[0], xk.w[1], xk.w[2], xk.w[3]};
    dv_ctx::EpochGraph *e = nullptr;
    for (auto &g : c->graphs)
        if (std::equal(key, key + 22, g.key)) e = &g;
    if (!e) {
        if (c->graphs.size() >= kMaxGraphs) {  // (the least recently used goes)
            auto lru = std::min_element(c->graphs.begin(), c->graphs.end(),
                                        [](const dv_ctx::EpochGraph &a, const dv_ctx::EpochGraph &b) {
                                            return a.used < b.used;
                                        });
            if (lru->exec) (void)hipGraphExecDestroy(lru->exec);
            *lru = dv_ctx::EpochGraph{};
            e = &*lru;
        } else {
            c->graphs.emplace_back();
            e = &c->graphs.back();
        }
        std::copy(key, key + 22, e->key);
    }
    e->used = ++c->graph_clock;
    if (e->seen != kGraphNever) e->seen++;
    GraphRun g;
    g.c = c;
    g.g = e;
    // (the first two times run as they are: a short batch pays no capture
    // it will not replay, and the buffers have grown to their sizes)
    g.capture = !e->exec && e->seen >= kGraphAfter && e->seen != kGraphNever;
    tl_graph = &g;
    const auto t0 = std::chrono::steady_clock::now();
    const uint64_t gen0 = c->ws_gen;
    int r = decide();
    tl_graph = nullptr;
    if (tl_dry) {  // a replay: the host state is the epoch's, the launches are the graph's
        tl_dry = false;
        const auto t1 = std::chrono::steady_clock::now();
        if (!r) r = hip_fail(hipGraphLaunch(e->exec, c->stream), "hipGraphLaunch");
        // the look-back tags wrapped during the walk (next_tag): the replay
        // has just written pre-wrap tags into the descriptors, zero them again
        if (!r && c->ws_gen != gen0)
            r = hip_fail(hipMemsetAsync(c->desc, 0, (size_t)((c->cfg.max_acc + kRTile - 1) / kRTile) * 8,
                                        c->stream), "hipMemsetAsync");
        tl_hp_walk += std::chrono::duration<double>(t1 - t0).count();
        tl_hp_glaunch += std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count();
        tl_hp_replays++;
        return r;
    }
    if (!g.capture || !g.began) return r;
    hipGraph_t graph = nullptr;
    const hipError_t ee = hipStreamEndCapture(c->stream, &graph);
    hipGraphExec_t ex = nullptr;
    hipError_t ei = hipErrorUnknown;
    if (!r && ee == hipSuccess && graph) ei = hipGraphInstantiate(&ex, graph, nullptr, nullptr, 0);
    if (graph) (void)hipGraphDestroy(graph);
    if (!r && ee == hipSuccess && ei == hipSuccess) {
        e->exec = ex;
        tl_hp_captures++;
        return hip_fail(hipGraphLaunch(ex, c->stream), "hipGraphLaunch");
    }
    // nothing the capture recorded ran: the decision again, uncaptured (its
    // clear repeats harmlessly -- the previous epoch's read-back was written
    // by the first one, and the gate it set stands)
    (void)hipGetLastError();
    if (ex) (void)hipGraphExecDestroy(ex);
    e->seen = kGraphNever;
    return decide();
}
}  // extern "C++"

// the common start of an epoch: argument checks, the verdict-byte stride,
// the per-epoch host state
int epoch_setup(dv_ctx *c, const dv_epoch_dev *ep) {
    if (ep->n_acc > c->cfg.max_acc || ep->n_txn > c->cfg.max_txn) return DV_ERR_ARG;
    // (epoch groups: no types -- the write bit rides in the 32-bit row ids;
    // no per-access txn ids where the boundaries are every range, tb_epoch)
    if (ep->n_acc && (!ep->keys || (!ep->types && !c->keys32) || (!ep->acc_txn && !tb_epoch(c, ep))))
        return DV_ERR_ARG;
    bool any = false;
    for (auto &t : c->tab) any |= t.loaded;
    if (!any) return DV_ERR_NO_TABLE;
    HIPCHK(hipSetDevice(c->cfg.device));
    const bool calvin = c->cfg.cc_alg == DV_CALVIN;
    if (ep->n_txn > kMaxTxn || ep->max_txn_acc > kMaxPos) return DV_ERR_ARG;
    // a device-side access count: single-GPU YCSB, decision rounds (dvcc.h)
    if (ep->n_acc_dev && (calvin || c->cfg.workload != DV_YCSB || c->rep_P)) return DV_ERR_ARG;
    // verdict-byte stride: 1 << slog >= the longest txn (16 at least)
    uint32_t slog = 7;
    if (!calvin) {
        const uint32_t hint = ep->max_txn_acc ? ep->max_txn_acc : kMaxPos;
        slog = 4;
        while ((1u << slog) < hint) slog++;
        const uint64_t need = (uint64_t)((ep->n_txn + 3u) & ~3u) << slog;
        if (need > c->vb8_cap) {
            HIPCHK(hipStreamSynchronize(c->stream));
            c->ws_gen++;
            dfree(c->vb8);
            c->vb8 = nullptr;
            c->vb8_cap = 0;
            int r = dalloc(&c->vb8, need);
            if (r) return r;
            c->vb8_cap = need;
        }
        c->slog = slog;
        c->el32 = round_el32(ep->n_txn, slog) && !(c->cfg.flags & DV_FLAG_EL64);
    }
    c->n_acc = ep->n_acc;
    c->n_acc_is_bound = ep->n_acc_dev != nullptr;
    c->n_txn = ep->n_txn;
    c->n_txn_pad = (ep->n_txn + 3u) & ~3u;
    c->rounds = 0;
    c->rounds_real = 0;
    c->passes = 0;
    c->applied = 0;
    c->async_launched = 0;
    c->async_unconfirmed = false;
    c->prefix_mode = false;
    c->rounds_prefix = 0;
    c->ms_probe = c->ms_sort = c->ms_decide = c->ms_exec = 0;
    c->rs = c->tb_start;
    c->re = c->tb_end;
    c->tb_mode = false;
    view_epoch(c);
    return DV_OK;
}
}  // namespace

int dv_epoch_begin(dv_ctx *c, const dv_epoch_dev *ep, uint32_t *d_grant) {
    KProfScope kps_(c);
    if (!c || !ep) return DV_ERR_ARG;
    const uint32_t *err_seed = c->err_seed;  // only for the epoch dv_epoch_run staged just now
    c->err_seed = nullptr;
    int r = epoch_setup(c, ep);
    if (r) return r;
    const bool calvin = c->cfg.cc_alg == DV_CALVIN;
    const uint32_t slog = calvin ? 7u : c->slog;  // CALVIN: positions only name access ids
    rec(c, 0);
    // (TPC-C: the o_id outputs zeroed here, the execution writes the committed NewOrders'; a
    // pipelined batch, dv_tpcc_epoch_run_device_batch: gated on the epoch before, whose
    // read-back this clear writes)
    const bool mir = c->mir_pending;
    c->mir_pending = false;
    launch_epoch_clear(c->stream, c->status, c->n_txn, c->n_txn_pad, calvin ? ST_COMMIT : ST_UNDEC,
                       c->tb_start, c->tb_end, calvin ? nullptr : c->tlen, c->tile_ctr, err_seed, c->ctr, nullptr,
                       0, c->clear_gate, mir ? c->d_mir[c->mir_slot] : nullptr,
                       mir ? c->d_mseq[c->mir_slot] : nullptr, mir ? c->mir_seq : 0ull,
                       c->cfg.workload == DV_TPCC ? c->tp_oid : nullptr, graph_desc(c), graph_ndesc(c));
    graph_after_clear(c);
    c->ticket = 0;
    const bool fuse_hist = nblocks_for(ep->n_acc) >= kProbeHistTiles && !ep->n_acc_dev;
    launch_probe(c->stream, make_tables(c), ep->keys, ep->types, ep->acc_txn, ep->tables, ep->n_acc,
                 ep->n_txn, slog, c->pairs[0], c->tb_start, c->tb_end, calvin ? nullptr : c->tlen,
                 calvin ? nullptr : c->acc_row, c->ctr, fuse_hist ? c->counts : nullptr, ep->n_txn,
                 ktiming(c) ? c->ev[kEvProbe0] : nullptr, ktiming(c) ? c->ev[kEvProbe1] : nullptr, c->keys32,
                 c->cfg.cc_alg == DV_WAIT_DIE ? ep->ts : nullptr, ep->n_acc_dev, c->tp_resolve ? c->f0 : nullptr);
    if (c->rep_P && !c->route) {  // replicated epoch: owners' key checks combined before anything depends on
        // them (epoch groups vote on every decider's outcome before anything executes)
        const int re = comm_combine_errors(c);
        if (re) return re;
    }
    rec(c, 1);
    const int key_bits = bits_for(row_space(c));
    c->sort_passes = sort_launches(c, ep->n_acc, key_bits, fuse_hist, ep->n_acc_dev != nullptr);
    c->sorted = sort_rows(c, ep->n_acc, key_bits, ktiming(c) ? c->sev : nullptr, fuse_hist, ep->n_acc_dev);
    if (calvin)  // NO_WAIT / WAIT_DIE / OCC: classified by round 0 itself
        launch_seg_prepare(c->stream, c->pairs[c->sorted], ep->n_acc, 1, c->tb_start, c->el, c->ctr);
    rec(c, 2);
    if (calvin) {
        const uint32_t tag = next_tag(c);
        calvin_grant(c->stream, c->el, ep->n_acc, d_grant, c->ew, c->desc, next_ticket(c), tag, c->ctr);
    } else {
        c->r0_n = (uint32_t)ep->n_acc;  // (round 0's sizes, RoundBufs)
        c->r0_n_dev = ep->n_acc_dev;
        __atomic_store_n(&c->h_pub->ru, 0ull, __ATOMIC_RELEASE);
        __atomic_store_n(&c->h_pub->tl, 0ull, __ATOMIC_RELEASE);
        c->live_ub = (uint32_t)ep->n_acc;
        c->und_ub = ep->n_txn;
    }
    rec(c, 3);
    HIPCHK(hipGetLastError());
    c->phase = 1;
    return DV_OK;
}

namespace {

// enqueue one decision round (scan + push + compaction); partitioned epochs
// then write verdict bytes, single-GPU epochs settle statuses directly
void enqueue_round(dv_ctx *c, uint8_t *d_verdict, bool settle, bool async_words = false) {
    const uint32_t r = c->rounds;
    const uint32_t tag = next_tag(c);
    uint32_t *tc = next_ticket(c);
    const RoundBufs b = round_bufs(c);
    // timing: the pass's own dispatch records its events (hipExtLaunchKernel),
    // no extra packets in the stream
    const bool t = ktiming(c) && c->passes < (uint32_t)kRoundLog;
    round_pass(c->stream, b, r, c->cfg.cc_alg != DV_OCC, c->live_ub, tag,
               (uint32_t)(tc - c->tile_ctr), settle, settle ? c->d_pub : nullptr,
               t ? c->pev[2 * c->passes] : nullptr, t ? c->pev[2 * c->passes + 1] : nullptr);
    c->passes++;
    if (settle && async_words && r == 0)  // round 0 with the asynchronous launch behind it (round0_then_async)
        round_settle(c->stream, b, r, c->v_n_txn, c->und_ub, c->tword, c->abounds, c->async_g);
    else if (settle) round_settle(c->stream, b, r, c->v_n_txn, c->und_ub);
    else list_verdict(c->stream, b, r, c->und_ub, d_verdict);
    c->rounds++;
}

}  // namespace

namespace {

// rounds settled so far (and the undecided count after the last of them)
inline uint32_t pub_round(const dv_ctx *c, uint32_t *und) {
    const unsigned long long ru = __atomic_load_n(&c->h_pub->ru, __ATOMIC_ACQUIRE);
    if (und) *und = (uint32_t)ru;
    return (uint32_t)(ru >> 32);
}

// returns DV_OK, kTailDeclined when the tail launched at round tail_r0
// declined, or an error
constexpr int kTailDeclined = 1;
int wait_published(dv_ctx *c, uint32_t target, uint32_t tail_r0) {
    const auto t0 = std::chrono::steady_clock::now();
    const unsigned long long declined = ((unsigned long long)tail_r0 << 32) | 1u;
    for (uint64_t i = 0;; i++) {
        if (pub_round(c, nullptr) >= target) return DV_OK;
        if (tail_r0 && __atomic_load_n(&c->h_pub->tl, __ATOMIC_ACQUIRE) == declined) return kTailDeclined;
        if ((i & 255) == 255) {
            const hipError_t q = hipStreamQuery(c->stream);
            if (q == hipSuccess) {  // drained: the record must be there now
                if (pub_round(c, nullptr) >= target) return DV_OK;
                if (tail_r0 && __atomic_load_n(&c->h_pub->tl, __ATOMIC_ACQUIRE) == declined)
                    return kTailDeclined;
                return DV_ERR_STATE;
            }
            if (q != hipErrorNotReady) return hip_fail(q, "round stream");
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) return DV_ERR_STATE;
        }
        __builtin_ia32_pause();
    }
}

// Rounds are published by the NEXT round's pass, so kRoundsAhead >= 2 keeps
// the round the host waits for always enqueued.
// Once the published live count and undecided count fit the tail kernel's
// LDS, the remaining rounds run in one single-workgroup launch (round_tail).
}  // namespace

// one decision round on this partition's accesses; writes this partition's
// verdict byte per txn (bit1 abort, bit0 wait) into d_verdict (NULL = internal)
int dv_epoch_round_local(dv_ctx *c, uint8_t *d_verdict) {
    KProfScope kps_(c);
    if (!c || c->phase != 1) return DV_ERR_STATE;
    if (c->cfg.cc_alg == DV_CALVIN) return DV_ERR_STATE;
    enqueue_round(c, d_verdict ? d_verdict : c->verdict, false);
    HIPCHK(hipGetLastError());
    return DV_OK;
}

// apply verdicts combined over all partitions (MAX); returns undecided txns
int dv_epoch_round_apply(dv_ctx *c, const uint8_t *d_verdict, uint32_t *undecided) {
    KProfScope kps_(c);
    if (!c || c->phase != 1 || c->cfg.cc_alg == DV_CALVIN) return DV_ERR_STATE;
    if (c->rounds == 0 || c->applied >= c->rounds) return DV_ERR_STATE;
    const uint32_t tag = next_tag(c);
    list_apply(c->stream, round_bufs(c), c->applied, c->und_ub, d_verdict ? d_verdict : c->verdict, tag,
               next_ticket(c), c->d_pub);
    HIPCHK(hipGetLastError());
    c->applied++;
    if (!undecided) return DV_OK;  // asynchronous: dv_epoch_round_wait reads the outcome
    return dv_epoch_round_wait(c, c->applied - 1, undecided);
}

int dv_epoch_round_wait(dv_ctx *c, uint32_t round, uint32_t *undecided) {
    if (!c || c->phase != 1 || c->cfg.cc_alg == DV_CALVIN || round >= c->applied) return DV_ERR_STATE;
    // the count log keeps the last kPubLog rounds enqueued
    if (c->applied - round > RoundPub::kPubLog) return DV_ERR_STATE;
    int r = wait_published(c, round + 1, 0);
    if (r) {
        (void)hipStreamSynchronize(c->stream);
        c->phase = 0;
        return r;
    }
    const uint32_t seen = pub_round(c, nullptr);
    const uint32_t und = __atomic_load_n(&c->h_pub->und_log[round % RoundPub::kPubLog], __ATOMIC_ACQUIRE);
    const unsigned long long le = __atomic_load_n(&c->h_pub->le, __ATOMIC_ACQUIRE);
    r = err_from_bits((uint32_t)le);
    if (r) {
        (void)hipStreamSynchronize(c->stream);
        c->phase = 0;
        return r;
    }
    // bounds for the rounds enqueued from now on
    c->und_ub = std::min(c->und_ub, und);
    c->live_ub = std::min(c->live_ub, (uint32_t)(le >> 32));
    if (seen > c->rounds_real) c->rounds_real = seen;
    if (undecided) *undecided = und;
    return DV_OK;
}

namespace {
int run_rounds(dv_ctx *c, bool resume);
int redo_prefix(dv_ctx *c);
int redo_survivors(dv_ctx *c);

// the execution of the committed txns and the commit bytes (every execution
// kernel is a no-op for a rejected epoch, input_err, and while the rounds
// are halted, Counters::halt)
// the last of the epoch's decision that enqueue_exec would queue: the
// survivors' decisions back to their txns (a prefix-kill epoch; the epoch's
// own state) -- decision lanes queue it before the wait for the previous
// epoch's execution
void exec_prologue(dv_ctx *c) {
    if (c->prefix_mode)
        launch_sub_scatter_back(c->stream, c->b_map, c->b_status, c->v_n_txn, c->status, c->ctr,
                                c->surv_words ? c->tword : nullptr);
}

// prologue_done: exec_prologue ran (decision lanes)
void enqueue_exec(dv_ctx *c, uint8_t *d_commit, bool prologue_done = false) {
    if (!prologue_done) exec_prologue(c);
    if (c->cfg.workload == DV_TPCC) {
        const HostTable &dt = c->tab[DV_TPCC_DISTRICT];
        TpccExec x{};
        x.pairs = c->pairs[c->sorted];
        x.n = c->n_acc;
        x.status = c->status;
        x.tb_start = c->tb_start;
        x.args = c->tp_args;
        x.cols = c->f0;
        x.oid_direct = c->cfg.cc_alg != DV_CALVIN;
        x.dsnap = c->tp_dsnap;
        x.dist_base = dt.row_base;
        x.dist_rows = dt.created ? dt.cap_rows : 0;
        x.oid = c->tp_oid;
        x.ctr = c->ctr;
        x.n_txn = c->n_txn;
        x.commit_out = d_commit;
        launch_tpcc_exec(c->stream, x);  // (the commit bytes too)
        return;
    } else if (c->route) {  // epoch groups: the owners execute (dvcc_comm.hip), nothing here
        if (c->cfg.cc_alg == DV_CALVIN) {
            launch_route_rowq(c->stream, *c->route, c->pairs[c->sorted], c->el, c->ew, c->n_acc, c->status, c->ctr);
        } else {  // (the commit bytes too)
            launch_route_txn(c->stream, *c->route, c->rs, c->re, c->acc_row, c->n_txn, c->status, c->ctr, d_commit);
            return;
        }
    } else {
        RowMap rm{};  // replicated epoch: global rows -> this partition's
        if (c->rep_P) {
            rm.P = c->rep_P;
            rm.part = c->cfg.part_id;
        }
        if (c->cfg.cc_alg == DV_CALVIN)
            launch_exec(c->stream, c->pairs[c->sorted], c->el, c->ew, c->n_acc, c->status, c->f0, c->pkey, c->ctr,
                        rm);
        else {  // (the commit bytes and count too)
            // (its dense test; only with table 0 the context's one table -- a
            // row of another table takes its key from the pkey column)
            const KillKeys dk = kill_keys(make_tables(c), nullptr, nullptr, nullptr);
            launch_exec_txn(c->stream, c->rs, c->re, c->acc_row, c->n_txn, c->status, c->f0, c->pkey,
                            c->cfg.cc_alg != DV_OCC, c->ctr, rm, d_commit,
                            dk.tabs.n == 1 && dk.dense_lim != 0 && dk.tabs.t[0].rep_part == kNoRep, dk.dense_base);
            return;
        }
    }
    launch_commit_out(c->stream, c->status, c->n_txn, d_commit, c->ctr);
}
}  // namespace

int epoch_finish(dv_ctx *c, uint8_t *d_commit, dv_stats *st);
int finish_tail(dv_ctx *c, uint8_t *d_commit, dv_stats *st, int r);

// ordered lanes (dv_lanes_order) running the per-epoch partitioned drivers
// (dv_epoch_run_part / dv_tpcc_epoch_run_part): the epoch's execution takes
// its turn after the previous epoch's, on whichever lane (the epoch groups
// take theirs in run_group's execution step instead)
int dv_epoch_finish(dv_ctx *c, uint8_t *d_commit, dv_stats *st) {
    const bool ordered = c && c->phase == 1 && c->order && c->comm && !c->route;
    if (ordered) {
        const int r = lane_exec_begin(c, c->stream);
        if (r) {
            c->phase = 0;
            c->prefix_mode = false;
            c->tp_args = c->tp_oid = nullptr;
            return r;
        }
    }
    const int r = epoch_finish(c, d_commit, st);
    if (ordered) {
        if (r)
            lane_fail(c);
        else
            lane_exec_end(c, c->stream);
    }
    return r;
}

int epoch_finish(dv_ctx *c, uint8_t *d_commit, dv_stats *st) {
    KProfScope kps_(c);
    if (!c || c->phase != 1 || c->fin_pending) return DV_ERR_STATE;
    if (c->cfg.workload == DV_TPCC && !c->tp_args) {  // only through dv_tpcc_epoch_begin
        c->phase = 0;
        return DV_ERR_STATE;
    }
    rec(c, 4);
    enqueue_exec(c, d_commit);
    rec(c, 5);
    int r = hip_fail(hipGetLastError(), "execution launch");
    if (!r && c->route && c->route->defer) {
        // epoch groups: the counters are queued for the host now and read
        // after the outcome vote, whose own round trip brings them
        // (epoch_finish_complete; run_group votes again on a halted decider)
        c->fin_want = mirror_out(c, 0);
        r = hip_fail(hipGetLastError(), "counter mirror");
        if (r) return finish_tail(c, d_commit, st, r);  // (the context is free again)
        c->fin_commit = d_commit;
        c->fin_pending = true;
        return DV_OK;
    }
    if (!r) r = sync_counters(c);
    return finish_tail(c, d_commit, st, r);
}

int epoch_finish_complete(dv_ctx *c, dv_stats *st) {
    if (!c || !c->fin_pending) return DV_ERR_STATE;
    c->fin_pending = false;
    const int r = mirror_wait(c, 0, c->fin_want);
    return finish_tail(c, c->fin_commit, st, r);
}

// after the counters reached the host: a halted decision is finished and
// executed again (each redo reads the counters itself), then the outcome
int finish_tail(dv_ctx *c, uint8_t *d_commit, dv_stats *st, int r) {
    const bool calvin = c->cfg.cc_alg == DV_CALVIN;
    if (!r && c->prefix_mode && c->h_ctr->a_halt) {
        // the prefix's rounds halted and nothing behind them ran
        c->async_unconfirmed = false;
        r = redo_prefix(c);
        if (!r) {
            rec(c, 4);
            enqueue_exec(c, d_commit);
            rec(c, 5);
            r = hip_fail(hipGetLastError(), "execution launch");
        }
        if (!r) r = sync_counters(c);
    }
    if (!r && !calvin && c->h_ctr->halt) {
        // the asynchronous rounds yielded (a workgroup waited too long for
        // facts, e.g. while another kernel held CUs): the execution above was
        // a no-op; finish the rounds synchronously, then execute (a stage
        // decided by one launch from round 0 has no round state to resume
        // from: its rounds start again)
        r = hip_fail(hipMemsetAsync(&c->ctr->halt, 0, sizeof(uint32_t), c->stream), "memset");
        c->async_unconfirmed = false;
        if (!r) r = c->prefix_mode && c->surv_words ? redo_survivors(c) : run_rounds(c, true);
        if (!r) {
            rec(c, 4);
            enqueue_exec(c, d_commit);
            rec(c, 5);
            r = hip_fail(hipGetLastError(), "execution launch");
        }
        if (!r) r = sync_counters(c);
    }
    c->phase = 0;
    c->tp_args = nullptr;  // per epoch (dv_tpcc_epoch_begin)
    c->tp_oid = nullptr;
    const bool prefix = c->prefix_mode;
    c->prefix_mode = false;
    if (r) return r;
    r = err_from_bits(c->h_ctr->err | c->h_ctr->peer_err);
    if (r) {
        if (c->h_ctr->err & ERRB_SPIN)
            std::fprintf(stderr, "dvcc: a bounded wait ran out (site %u: 1 look-back, 3 tail)\n",
                         c->h_ctr->spin_site);
        return r;
    }
    if (!calvin && (c->h_ctr->async_r0 || c->h_ctr->async_wr0)) {  // an asynchronous launch decided the rest
        uint32_t left = 0;
        for (const CtrSlot &sl : c->h_ctr->slot) left += sl.undecided;
        if (left) return DV_ERR_STATE;  // cannot happen: every workgroup left decided
        c->rounds_real = c->h_ctr->async_r0 + c->h_ctr->async_iters;
    } else if (c->async_unconfirmed) {
        // the last try found nothing left to decide (a declined one would
        // leave txns undecided: cannot happen, its live count fitted)
        if (c->h_ctr->async_go == 2u) return DV_ERR_STATE;
        uint32_t r_end = 0;  // the passes decided everything: the last round with undecided txns
        for (uint32_t k = 0; k < std::min(c->rounds, (uint32_t)kRoundLog); k++)
            if (c->h_ctr->log_und[k]) r_end = k + 1;
        c->rounds_real = std::max(r_end, 1u);
    }
    c->async_hint = calvin ? c->async_hint : c->h_ctr->async_r0;
    if (st) {
        std::memset(st, 0, sizeof(*st));
        st->n_txn = c->n_txn;
        st->n_acc = c->n_acc;
        uint64_t committed = 0, wcnt = 0, dig = 0;
        for (const CtrSlot &sl : c->h_ctr->slot) {
            committed += sl.committed;
            wcnt += sl.write_cnt;
            dig += sl.read_digest;
        }
        st->committed = committed;
        st->aborted = c->n_txn - committed;
        st->write_cnt = wcnt;
        st->read_digest = dig;
        st->rounds = calvin ? 0 : (c->rounds_real ? c->rounds_real : c->rounds);
        if (prefix) st->rounds += c->rounds_prefix ? c->rounds_prefix : c->h_ctr->a_rounds;  // + the survivors'
        st->sort_passes = c->sort_passes;
        st->async_launches = (uint16_t)std::min(c->async_launched, 0xFFFFu);
        st->async_declined = (uint16_t)std::min(c->h_ctr->async_declined, 0xFFFFu);
        st->async_yields = c->h_ctr->async_yields;
        if (timing(c)) {
            st->ms_probe = elapsed(c, 0, 1);
            st->ms_sort = elapsed(c, 1, 2);
            st->ms_decide = elapsed(c, 2, 4);
            st->ms_exec = elapsed(c, 4, 5);
            st->ms_total = elapsed(c, 0, 5);
        }
        if (ktiming(c)) {
            float s = 0;
            for (uint32_t p = 0; p < c->sort_passes && p < 8; p++) {
                float m = 0;
                (void)hipEventElapsedTime(&m, c->sev[2 * p], c->sev[2 * p + 1]);
                s += m;
            }
            st->ms_scatter = s;
            st->scatter_launches = c->n_acc ? c->sort_passes : 0;
            const uint32_t np = std::min(c->passes, (uint32_t)kRoundLog);
            float sp = 0;
            for (uint32_t p = 0; p < np; p++) {
                float m = 0;
                (void)hipEventElapsedTime(&m, c->pev[2 * p], c->pev[2 * p + 1]);
                sp += m;
            }
            st->pass_launches = np;
            st->ms_pass = sp;
            st->pass_live = c->passes <= (uint32_t)kRoundLog ? c->h_ctr->pass_live : 0;  // (no-op passes add 0)
            if (c->n_acc) (void)hipEventElapsedTime(&st->ms_probe_kernel, c->ev[kEvProbe0], c->ev[kEvProbe1]);
        }
        st->async_live = c->h_ctr->async_live;
        if (c->n_acc_is_bound) st->n_acc = c->h_ctr->n_acc;
        if (prefix) {
            st->prefix_txn = c->pf_K;
            st->prefix_acc = c->h_ctr->a_acc;
            st->surv_txn = c->h_ctr->b_txn;
            st->surv_acc = c->h_ctr->b_acc;
        }
    }
    return DV_OK;
}

namespace {

// Single-GPU decision rounds, pipelined: kRoundsAhead rounds stay queued
// while the host follows the published progress record (no stream sync).
// Each round decides at least the lowest undecided txn, so the undecided
// count strictly falls from one observed round to the next; rounds queued
// past the fixpoint are no-ops.
constexpr uint32_t kRoundsAhead = 2;

// The rounds queued ahead lag the published count by about two rounds, so the
// tail is first tried at kTailTry (the live set shrinks ~2x per round pair
// once it is that small); if it declines, the next try waits for a published
// count that fits outright.
constexpr uint32_t kTailTryFactor = 4;

// The asynchronous launch (round_async) takes over once the published live
// count is at most kAsyncLiveFrac of the epoch's accesses (and fits its
// workgroups); the passes already queued behind it become no-ops.  Launching
// earlier does not pay: every asynchronous iteration re-reads the facts of
// its whole slice, so while the live set is large it costs more than the
// synchronous rounds it replaces (1M-txn zipf-0.9 epoch: 570 us from round
// 1, 240 us from round 3, 153 us from round 5 after 107 us of rounds 3-4).
// The launch is a device-decided try (round_async), so speculative tries
// queued behind passes are possible (kAsyncSpeculate); they lost ~40 us of
// empty launches and no-op passes for ~20 us gained, and are off.
constexpr double kAsyncLiveFrac = 0.5;
constexpr bool kAsyncSpeculate = false;

// Small epochs (TPC-C's 65K txns): the slices are a few elements per thread,
// so an asynchronous iteration is cheap and the launch pays from round 1.
constexpr uint64_t kAsyncSmallAcc = 2u << 20;

uint32_t async_thresh(dv_ctx *c) {
    if (c->v_thresh) return std::min<uint32_t>(c->v_thresh, async_try_limit(c->async_g));
    const uint64_t frac = c->n_acc <= kAsyncSmallAcc ? c->n_acc : (uint64_t)(kAsyncLiveFrac * (double)c->n_acc);
    return (uint32_t)std::min<uint64_t>(frac, async_try_limit(c->async_g));
}

void async_try(dv_ctx *c, uint32_t r0, bool words_done = false, bool words = false) {
    c->async_launched++;
    round_async(c->stream, round_bufs(c), r0, c->cfg.cc_alg != DV_OCC, c->async_g, async_thresh(c),
                c->abounds, c->tword, c->v_n_txn, c->d_pub, c->async_max_iters, c->async_idle_ticks, words_done,
                words);
}

// round 0, then every remaining decision in one asynchronous launch at round
// 1, queued with no host wait; round 0's settle writes the launch's fact and
// carry words (no k_async_words).  words: the statuses stay in the fact
// words for the stage's consumer (no k_round_finalize)
void round0_then_async(dv_ctx *c, bool words = false) {
    c->v_thresh = async_try_limit(c->async_g);
    enqueue_round(c, nullptr, true, true);
    async_try(c, 1, true, words);
    c->async_unconfirmed = true;
}

// Small epochs (a TPC-C epoch, at most kAsyncSmallAcc accesses): round 0,
// then the asynchronous launch from round 1 with no host wait in between --
// its slices are a few elements per thread, so it pays from round 1 on.  A
// declined or yielded try halts execution and dv_epoch_finish resumes the
// synchronous rounds; larger epochs take the pipelined loop.
int decide_epoch(dv_ctx *c) {
    const bool async = c->el32 && c->async_g && !(c->cfg.flags & DV_FLAG_NO_ASYNC);
    if (!async || c->n_acc > kAsyncSmallAcc) return run_rounds(c, false);
    round0_then_async(c);
    return hip_fail(hipGetLastError(), "rounds");
}

// resume: continue after an asynchronous launch that yielded or declined
// (dv_epoch_finish) from the round it started at, without further
// asynchronous tries
int run_rounds(dv_ctx *c, bool resume) {
    if (!resume) __atomic_store_n(&c->h_pub->ru, 0ull, __ATOMIC_RELEASE);
    __atomic_store_n(&c->h_pub->tl, 0ull, __ATOMIC_RELEASE);
    uint32_t prev = c->v_n_txn + 1, seen = resume ? pub_round(c, nullptr) : 0;
    uint32_t tail_r0 = 0;             // round the pending tail launch starts at (0: none)
    const uint32_t cap = tail_cap(c->el32);
    uint32_t tail_limit = kTailTryFactor * cap;  // published live count that triggers a try
    const bool async = !resume && c->el32 && c->async_g && !(c->cfg.flags & DV_FLAG_NO_ASYNC);
    // speculative tries start one round before the previous epoch's launch
    const uint32_t try_from = !kAsyncSpeculate ? ~0u : (c->async_hint > 1 ? c->async_hint - 1 : 1);
    for (;;) {
        while (!tail_r0 && c->rounds < seen + kRoundsAhead + 1) {
            enqueue_round(c, nullptr, true);
            if (async && c->rounds >= try_from) async_try(c, c->rounds);
        }
        int r = hip_fail(hipGetLastError(), "round launch");
        if (!r) r = wait_published(c, seen + 1, tail_r0);
        if (r == kTailDeclined) {
            tail_r0 = 0;
            tail_limit = cap;
            continue;
        }
        if (r) {
            (void)hipStreamSynchronize(c->stream);
            return r;
        }
        uint32_t und = 0;
        seen = pub_round(c, &und);
        const unsigned long long le = __atomic_load_n(&c->h_pub->le, __ATOMIC_ACQUIRE);
        r = err_from_bits((uint32_t)le);
        if (!r && und != 0 && und >= prev) r = DV_ERR_STATE;  // no progress: internal error
        if (r) {
            (void)hipStreamSynchronize(c->stream);
            return r;
        }
        if (und == 0) {  // (after an asynchronous launch: dv_epoch_finish counts its rounds)
            c->rounds_real = seen;
            c->rounds = std::max(c->rounds, seen);
            return DV_OK;
        }
        prev = und;
        c->live_ub = std::min(c->live_ub, (uint32_t)(le >> 32));  // bounds for rounds not yet enqueued
        c->und_ub = und;
        if (async && !tail_r0 && c->live_ub <= async_thresh(c)) {
            // the try behind the last queued pass qualifies: it decides the
            // rest, or finds nothing left (an earlier try ran, or the passes
            // finished).  No wait here: dv_epoch_finish queues the execution
            // behind it and checks the outcome with the counters.
            if (c->rounds < try_from) async_try(c, c->rounds);
            c->async_unconfirmed = true;
            return DV_OK;
        }
        if (!tail_r0 && !(c->cfg.flags & DV_FLAG_NO_TAIL) && c->live_ub <= tail_limit) {
            tail_r0 = c->rounds;
            round_tail(c->stream, round_bufs(c), tail_r0, c->cfg.cc_alg != DV_OCC, c->d_pub);
        }
    }
}

// ---- prefix-kill epochs (dvcc_prefix.hip) ----------------------------------
// Epochs from kPrefixMinTxn txns up; the prefix is ~1/32 of the epoch, at
// least kPrefixMin txns (config D: 32,768 of 1,048,576, whose commits kill
// ~91 % of the later txns).
constexpr uint32_t kPrefixMinTxn = 1u << 17;
constexpr uint32_t kPrefixMin = 4096, kPrefixMax = 1u << 16;

uint32_t prefix_size(const dv_ctx *c, uint32_t n_txn) {
    if (c->prefix_txns) return c->prefix_txns;
    return std::min(kPrefixMax, std::max(kPrefixMin, n_txn / 32));
}

bool prefix_applies(const dv_ctx *c, const dv_epoch_dev *ep) {
    if (c->cfg.cc_alg == DV_CALVIN || c->cfg.workload != DV_YCSB) return false;
    if (c->prefix_txns == ~0u) return false;  // dv_set_prefix: off
    if (ep->n_txn < (c->prefix_txns ? 2 : kPrefixMinTxn)) return false;
    return prefix_size(c, ep->n_txn) < ep->n_txn;
}

// A small YCSB epoch that queues without a host wait too: CALVIN (the grant
// scan and the execution are all launches), or NO_WAIT / WAIT_DIE / OCC whose
// rounds are round 0 plus one asynchronous launch (decide_epoch, at most
// kAsyncSmallAcc accesses and 32-bit round elements) -- so the pipelined batch
// and the decision lanes take it like a prefix-kill epoch (config B: 65,536
// CALVIN txns per epoch ran one synchronous epoch at a time before).
bool small_pipelined(const dv_ctx *c, const dv_epoch_dev *ep) {
    if (c->cfg.workload != DV_YCSB || ep->n_acc_dev || prefix_applies(c, ep)) return false;
    if (c->cfg.cc_alg == DV_CALVIN) return true;
    if (ep->n_acc > kAsyncSmallAcc || !c->async_g || (c->cfg.flags & DV_FLAG_NO_ASYNC) || !ep->n_txn) return false;
    uint32_t slog = 4;  // (epoch_setup's verdict-byte stride)
    const uint32_t hint = ep->max_txn_acc ? ep->max_txn_acc : kMaxPos;
    while ((1u << slog) < hint) slog++;
    return round_el32(ep->n_txn, slog) && !(c->cfg.flags & DV_FLAG_EL64);
}

// ... queued: begin (probe, sort; CALVIN's grant scan), then the rounds
int small_enqueue(dv_ctx *c, const dv_epoch_dev *ep) {
    int r = dv_epoch_begin(c, ep, nullptr);
    if (!r && c->cfg.cc_alg != DV_CALVIN && c->n_txn) {
        r = decide_epoch(c);
        if (r) c->phase = 0;
    }
    return r;
}

// tb mode: a prefix-kill epoch whose own txn boundaries are every kernel's
// ranges (k_probe_tb probes the prefix alone, the kill pass the rest).  Not
// for a replicated epoch whose owners' key checks must be combined before
// the kill (run_part); epoch groups (route) vote on the decider's outcome
// instead, and hand their 32-bit rows over as the 4-byte records.
bool tb_epoch(const dv_ctx *c, const dv_epoch_dev *ep) {
    // (a device-side access count: the closed loop's tb-form epochs, loop_tb)
    return prefix_applies(c, ep) && ep->txn_begin && (!ep->n_acc_dev || ep->recs32) && !ep->tables &&
           (!c->keys32 || ep->recs32) && (!c->rep_P || c->route) && (ep->keys || ep->recs32);
}

// The rounds of one stage: round 0, then every remaining decision in one
// asynchronous launch (stages are small: a declined or yielded try halts and
// the stage is decided again synchronously), or the pipelined loop when
// asynchronous rounds are off.  words (a prefix-kill stage): the launch leaves
// the statuses in the fact words and *words = true -- its consumer
// (k_prefix_mark, k_sub_scatter_back) reads them, no k_round_finalize.
int stage_rounds(dv_ctx *c, const uint32_t *n_acc_dev, uint32_t n_acc_ub, bool *words = nullptr) {
    if (words) *words = false;
    c->rounds = 0;
    c->rounds_real = 0;
    c->async_unconfirmed = false;
    c->el32 = round_el32(c->v_n_txn, c->slog) && !(c->cfg.flags & DV_FLAG_EL64);
    c->live_ub = n_acc_ub;
    c->und_ub = c->v_n_txn;
    c->r0_n = n_acc_ub;  // (round 0's sizes, RoundBufs)
    c->r0_n_dev = n_acc_dev;
    __atomic_store_n(&c->h_pub->ru, 0ull, __ATOMIC_RELEASE);
    __atomic_store_n(&c->h_pub->tl, 0ull, __ATOMIC_RELEASE);
    const bool async = c->el32 && c->async_g && !(c->cfg.flags & DV_FLAG_NO_ASYNC);
    if (!async) return run_rounds(c, false);
    if (words) *words = true;
    round0_then_async(c, words != nullptr);  // (v_thresh: whatever fits the workgroups)
    return hip_fail(hipGetLastError(), "stage rounds");
}

// Behind the prefix's rounds, with no host wait: the kill of the later txns
// that conflict with the prefix's commits, the survivors' sub-epoch (sort
// keys into pairs[0], the prefix is done with it), its sort and rounds.  Every
// kernel here is a no-op while the prefix's rounds are halted (k_prefix_mark
// then sets Counters::a_halt and dv_epoch_finish redoes the prefix).
int enqueue_survivors(dv_ctx *c) {
    const bool nowait = c->cfg.cc_alg != DV_OCC;
    const uint64_t rs_words = row_state_words(row_space(c));
    const uint32_t K = c->pf_K;
    launch_prefix_mark(c->stream, c->status, c->rs, c->re, c->acc_row, K, c->row_state, rs_words, nowait,
                       c->ctr, c->prefix_words ? c->tword : nullptr);
    launch_kill_compact(c->stream, c->rs, c->re, c->acc_row, c->pf_n_acc, c->pf_n_acc_dev, K, c->n_txn,
                        c->row_state, rs_words, nowait, c->kill_bits,
                        nowait ? c->kill_bits + kill_words(c->cfg.max_acc) : nullptr, c->status, c->b_map, c->b_status,
                        c->b_tlen,
                        c->pairs[0], c->kinfo, c->ktsum, c->ctr, c->tb_mode ? &c->pf_kk : nullptr);
    // the survivors: renumbered 0..S-1, counts on the device
    c->sorted = sort_rows(c, c->pf_n_acc, c->pf_key_bits, nullptr, false, &c->ctr->b_acc);
    c->v_status = c->b_status;
    c->v_tlen = c->b_tlen;
    c->v_n_txn = c->n_txn - K;
    c->v_n_txn_dev = &c->ctr->b_txn;
    return stage_rounds(c, &c->ctr->b_acc, (uint32_t)c->pf_n_acc, &c->surv_words);
}

// The survivors' asynchronous launch yielded or declined: nothing behind it
// executed, and with no finalize their status bytes hold only round 0's
// decisions, so their rounds run again from round 0, synchronously (the
// greedy's fixpoint is the same).
int redo_survivors(dv_ctx *c) {
    const uint32_t flags = c->cfg.flags;
    c->cfg.flags |= DV_FLAG_NO_ASYNC;
    int r = stage_rounds(c, &c->ctr->b_acc, (uint32_t)c->pf_n_acc, &c->surv_words);
    c->cfg.flags = flags;
    return r;
}

// The prefix's rounds halted (an asynchronous try yielded or declined) and
// nothing behind them ran: decide the prefix again from scratch with the
// synchronous rounds (its partial decisions are discarded; the greedy's
// fixpoint is the same), then queue the survivors' stage again.
int redo_prefix(dv_ctx *c) {
    HIPCHK(hipMemsetAsync(&c->ctr->halt, 0, sizeof(uint32_t), c->stream));
    HIPCHK(hipMemsetAsync(&c->ctr->a_halt, 0, sizeof(uint32_t), c->stream));
    HIPCHK(hipMemsetAsync(c->status, ST_UNDEC, c->pf_K, c->stream));
    c->sorted = c->pf_sorted_a;
    c->v_status = c->status;
    c->v_tlen = c->tlen;
    c->v_n_txn = c->pf_K;
    c->v_n_txn_dev = nullptr;
    c->v_thresh = 0;
    const uint32_t flags = c->cfg.flags;
    c->cfg.flags |= DV_FLAG_NO_ASYNC;
    int r = stage_rounds(c, &c->ctr->a_acc, c->pf_ub_a, &c->prefix_words);
    c->cfg.flags = flags;
    if (r) return r;
    c->rounds_prefix = c->rounds_real ? c->rounds_real : c->rounds;
    return enqueue_survivors(c);
}

// Probe -> prefix: sort + rounds -> kill + compaction -> survivors: sort +
// rounds; dv_epoch_finish then maps the survivors' decisions back and
// executes.  Only the prefix and the survivors are ever sorted.
int run_prefix_epoch(dv_ctx *c, const dv_epoch_dev *ep) {
    const uint32_t *err_seed = c->err_seed;
    c->err_seed = nullptr;
    int r = epoch_setup(c, ep);
    if (r) return r;
    const uint32_t K = prefix_size(c, ep->n_txn);
    const uint32_t T = c->cfg.max_txn;
    const uint64_t rs_words = row_state_words(row_space(c));
    if (!c->row_state || c->row_state_cap < rs_words) {
        HIPCHK(hipStreamSynchronize(c->stream));
        c->ws_gen++;
        dfree(c->row_state);
        c->row_state = nullptr;
        c->row_state_cap = 0;
        r = dalloc(&c->row_state, rs_words);
        if (r) return r;
        c->row_state_cap = rs_words;
    }
    if (!c->b_status) {
        c->ws_gen++;
        r = dalloc(&c->b_status, (T + 3u) & ~3u);
        if (!r) r = dalloc(&c->b_tlen, (T + 3u) & ~3u);
        if (!r) r = dalloc(&c->b_map, T);
        if (!r) r = dalloc(&c->kill_bits, 2 * kill_words(c->cfg.max_acc));  // kill bits, then skip bits
        if (!r) r = dalloc(&c->kinfo, T);
        if (!r) r = dalloc(&c->ktsum, 2ull * kill_tiles(T) + 2);
        if (r) return r;
    }
    const int key_bits = bits_for(row_space(c));
    // (the prefix's sort: its count is on the device)
    c->sort_passes = sort_launches(c, ep->n_acc, key_bits, false, true);
    c->prefix_mode = true;
    c->prefix_words = c->surv_words = false;
    // tb mode: the epoch's own txn boundaries are every kernel's ranges, the
    // prefix alone is probed here and the rest by the kill pass (k_probe_tb)
    c->tb_mode = tb_epoch(c, ep);
    if (c->tb_mode) {
        c->rs = ep->txn_begin;
        c->re = ep->txn_begin + 1;
        c->pf_kk = kill_keys(make_tables(c), ep->keys, ep->types, ep->recs32);
    }
    rec(c, 0);
    const bool mir = c->mir_pending;  // (the previous pipelined epoch's read-back rides on this clear)
    c->mir_pending = false;
    launch_epoch_clear(c->stream, c->status, c->n_txn, c->n_txn_pad, ST_UNDEC, c->tb_mode ? nullptr : c->tb_start,
                       c->tb_mode ? nullptr : c->tb_end, c->tb_mode ? nullptr : c->tlen, c->tile_ctr, err_seed, c->ctr,
                       c->row_state, rs_words, c->clear_gate,
                       mir ? c->d_mir[c->mir_slot] : nullptr, mir ? c->d_mseq[c->mir_slot] : nullptr,
                       mir ? c->mir_seq : 0ull, nullptr, graph_desc(c), graph_ndesc(c));
    graph_after_clear(c);
    c->ticket = 0;
    if (c->tb_mode)
        launch_probe_tb(c->stream, make_tables(c), ep->keys, ep->types, ep->recs32, ep->txn_begin, ep->n_acc,
                        ep->n_txn, K,
                        c->slog, c->pairs[0], c->tlen, c->acc_row, c->ctr,
                        c->cfg.cc_alg == DV_WAIT_DIE ? ep->ts : nullptr, ktiming(c) ? c->ev[kEvProbe0] : nullptr,
                        ktiming(c) ? c->ev[kEvProbe1] : nullptr, ep->n_acc_dev);
    else
        launch_probe(c->stream, make_tables(c), ep->keys, ep->types, ep->acc_txn, ep->tables, ep->n_acc, ep->n_txn,
                     c->slog, c->pairs[0], c->tb_start, c->tb_end, c->tlen, c->acc_row, c->ctr, nullptr, K,
                     ktiming(c) ? c->ev[kEvProbe0] : nullptr, ktiming(c) ? c->ev[kEvProbe1] : nullptr, c->keys32,
                     c->cfg.cc_alg == DV_WAIT_DIE ? ep->ts : nullptr, ep->n_acc_dev);
    if (c->rep_P && !c->route) {  // replicated epoch: owners' key checks combined before anything depends on
        // them (epoch groups vote on every decider's outcome before anything executes)
        r = comm_combine_errors(c);
        if (r) return r;
    }
    rec(c, 1);
    // the prefix: txns [0, K), the first ctr->a_acc accesses
    const uint32_t ub_a = (uint32_t)std::min<uint64_t>(ep->n_acc, (uint64_t)K * (ep->max_txn_acc ? ep->max_txn_acc
                                                                                                    : kMaxPos));
    c->sorted = sort_rows(c, ub_a, key_bits, ktiming(c) ? c->sev : nullptr, false, &c->ctr->a_acc);
    rec(c, 2);
    c->v_status = c->status;
    c->v_tlen = c->tlen;
    c->v_n_txn = K;
    c->v_n_txn_dev = nullptr;
    c->phase = 1;
    c->pf_K = K;
    c->pf_ub_a = ub_a;
    c->pf_sorted_a = c->sorted;
    c->pf_key_bits = key_bits;
    c->pf_n_acc = ep->n_acc;
    c->pf_n_acc_dev = ep->n_acc_dev;
    r = stage_rounds(c, &c->ctr->a_acc, ub_a, &c->prefix_words);
    // the prefix's rounds ran synchronously (no asynchronous try): their count
    // is known here; else k_prefix_mark records it (Counters::a_rounds)
    c->rounds_prefix = c->async_unconfirmed ? 0u : (c->rounds_real ? c->rounds_real : c->rounds);
    if (!r) r = enqueue_survivors(c);
    if (r) {
        (void)hipStreamSynchronize(c->stream);
        c->phase = 0;
        c->prefix_mode = false;
    }
    return r;
}

}  // namespace

int dv_set_prefix(dv_ctx *c, uint32_t prefix_txns) {
    if (!c) return DV_ERR_ARG;
    if (c->phase != 0) return DV_ERR_STATE;
    c->prefix_txns = prefix_txns;
    return DV_OK;
}

int dv_epoch_run_device(dv_ctx *c, const dv_epoch_dev *ep, uint8_t *d_commit, uint32_t *d_grant,
                        dv_stats *st) {
    KProfScope kps_(c);
    if (c && ep && prefix_applies(c, ep)) {
        HIPCHK(hipSetDevice(c->cfg.device));
        const int r = run_prefix_epoch(c, ep);
        if (r) return r;
        return dv_epoch_finish(c, d_commit, st);
    }
    int r = dv_epoch_begin(c, ep, d_grant);
    if (r) return r;
    if (c->cfg.cc_alg != DV_CALVIN && c->n_txn) {
        r = decide_epoch(c);
        if (r) { c->phase = 0; return r; }
    }
    return dv_epoch_finish(c, d_commit, st);
}


}  // extern "C"

namespace {

// What a pipelined epoch's statistics need of the host state it was queued
// with (the next epoch's queueing overwrites the context's copy).
struct EpochSnap {
    uint64_t n_acc = 0;
    uint32_t n_txn = 0, rounds = 0, rounds_real = 0, rounds_prefix = 0, async_launched = 0, sort_passes = 0;
    uint32_t prefix_txn = 0;
    bool async_unconfirmed = false, n_acc_is_bound = false;
    unsigned long long seq = 0;
    int slot = 0;
};

// a prefix-kill epoch queued through its execution, commit bytes and counter
// mirror (slot), with no host wait; gate: the epoch before it is still unread;
// defer: another pipelined epoch is queued right behind it, whose clear
// writes this one's mirror (one launch fewer per epoch)
template <class Decide>
int pipe_enqueue(dv_ctx *c, Decide &&decide, uint8_t *d_commit, bool gate, int slot, EpochSnap &sn, bool defer) {
    c->clear_gate = gate;
    int r = decide();
    c->clear_gate = false;
    if (r) {
        mirror_flush(c);  // (the previous epoch's read-back, when this one never reached its clear)
        return r;
    }
    enqueue_exec(c, d_commit);
    r = hip_fail(hipGetLastError(), "execution launch");
    sn.n_acc = c->n_acc;
    sn.n_txn = c->n_txn;
    sn.rounds = c->rounds;
    sn.rounds_real = c->rounds_real;
    sn.rounds_prefix = c->rounds_prefix;
    sn.async_launched = c->async_launched;
    sn.sort_passes = c->sort_passes;
    sn.prefix_txn = c->pf_K;
    sn.n_acc_is_bound = c->n_acc_is_bound;
    sn.async_unconfirmed = c->async_unconfirmed;
    sn.slot = slot;
    if (defer && !r) {
        sn.seq = ++c->cseq;
        c->mir_pending = true;
        c->mir_slot = slot;
        c->mir_seq = sn.seq;
    } else {
        sn.seq = mirror_out(c, slot);
    }
    c->phase = 0;
    c->prefix_mode = false;
    c->tp_args = c->tp_oid = nullptr;
    if (!r) r = hip_fail(hipGetLastError(), "counter mirror");
    return r;
}

// wait for a pipelined epoch's counters; *halted: its rounds halted (or the
// epoch before it did), nothing of it executed -- the caller runs it again
int pipe_complete(dv_ctx *c, const EpochSnap &sn, dv_stats *st, bool *halted) {
    *halted = false;
    int r = mirror_wait(c, sn.slot, sn.seq);
    if (r) return r;
    const Counters *hc = c->h_mir[sn.slot];
    r = err_from_bits(hc->err | hc->peer_err);
    if (r) return r;
    if (hc->halt || hc->a_halt) {
        *halted = true;
        return DV_OK;
    }
    uint32_t rounds_real = sn.rounds_real;
    if (hc->async_r0 || hc->async_wr0) {
        uint32_t left = 0;
        for (const CtrSlot &sl : hc->slot) left += sl.undecided;
        if (left) return DV_ERR_STATE;
        rounds_real = hc->async_r0 + hc->async_iters;
    } else if (sn.async_unconfirmed) {
        if (hc->async_go == 2u) return DV_ERR_STATE;
        uint32_t r_end = 0;
        for (uint32_t k = 0; k < std::min(sn.rounds, (uint32_t)kRoundLog); k++)
            if (hc->log_und[k]) r_end = k + 1;
        rounds_real = std::max(r_end, 1u);
    }
    c->async_hint = hc->async_r0;
    if (st) {
        std::memset(st, 0, sizeof(*st));
        st->n_txn = sn.n_txn;
        st->n_acc = sn.n_acc;
        uint64_t committed = 0, wcnt = 0, dig = 0;
        for (const CtrSlot &sl : hc->slot) {
            committed += sl.committed;
            wcnt += sl.write_cnt;
            dig += sl.read_digest;
        }
        st->committed = committed;
        st->aborted = sn.n_txn - committed;
        st->write_cnt = wcnt;
        st->read_digest = dig;
        st->rounds = (rounds_real ? rounds_real : sn.rounds) + (sn.rounds_prefix ? sn.rounds_prefix : hc->a_rounds);
        st->sort_passes = sn.sort_passes;
        st->async_launches = (uint16_t)std::min(sn.async_launched, 0xFFFFu);
        st->async_declined = (uint16_t)std::min(hc->async_declined, 0xFFFFu);
        st->async_yields = hc->async_yields;
        st->async_live = hc->async_live;
        if (sn.n_acc_is_bound) st->n_acc = hc->n_acc;
        st->prefix_txn = sn.prefix_txn;
        st->prefix_acc = hc->a_acc;
        st->surv_txn = hc->b_txn;
        st->surv_acc = hc->b_acc;
    }
    return DV_OK;
}

// after a halted pipelined epoch: the stream drained, halts cleared, then the
// epochs run again one at a time (decisions depend only on an epoch's own
// accesses, and neither touched the tables)
int pipe_redo(dv_ctx *c) {
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipMemsetAsync(&c->ctr->halt, 0, sizeof(uint32_t), c->stream));
    HIPCHK(hipMemsetAsync(&c->ctr->a_halt, 0, sizeof(uint32_t), c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return DV_OK;
}

// Pipelined epochs: epoch k+1 is queued (gated on epoch k) before epoch k
// is read back.  pipelined(k): epoch k can be queued that way; enqueue(k):
// queues its decision (the clear honours clear_gate / mir_pending); run(k,
// st): runs it synchronously (an epoch that cannot be pipelined, or one to
// redo after a halt).
template <class Commit, class Pipelined, class Enqueue, class Run>
int run_batch(dv_ctx *c, uint32_t n, dv_stats *sts, Commit &&commit_of, Pipelined &&pipelined, Enqueue &&enqueue,
              Run &&run) {
    EpochSnap snap[2];
    int64_t pend = -1;  // the epoch queued but not yet read back
    auto stats_of = [&](uint32_t k) { return sts ? &sts[k] : nullptr; };
    // the pending epoch: read back; if it halted, it runs again, and so does
    // `next` (queued behind it, gated) when given
    auto settle = [&](int64_t next) -> int {
        bool halted = false;
        int r = pipe_complete(c, snap[pend & 1], stats_of((uint32_t)pend), &halted);
        if (r) {
            (void)hipStreamSynchronize(c->stream);
            return r;
        }
        if (!halted) return DV_OK;
        c->mir_pending = false;  // (`next`'s read-back: it runs again below)
        r = pipe_redo(c);
        if (!r) r = run((uint32_t)pend, stats_of((uint32_t)pend));
        if (!r && next >= 0) r = run((uint32_t)next, stats_of((uint32_t)next));
        return r ? r : 1;  // 1: `next` ran already
    };
    auto fail = [&](int r) {  // (no read-back is waited for after an error)
        c->mir_pending = false;
        return r;
    };
    for (uint32_t k = 0; k < n; k++) {
        if (!pipelined(k)) {
            if (pend >= 0) {
                const int r = settle(-1);
                if (r < 0) return fail(r);
                pend = -1;
            }
            const int r = run(k, stats_of(k));
            if (r) return fail(r);
            continue;
        }
        // the next epoch's clear writes this one's read-back when it is queued right behind
        const bool defer = k + 1 < n && pipelined(k + 1);
        int r = pipe_enqueue(c, [&] { return enqueue(k); }, commit_of(k), pend >= 0, (int)(k & 1), snap[k & 1],
                             defer);
        if (r) {
            (void)hipStreamSynchronize(c->stream);
            if (pend >= 0) {  // (its read-back, for the statistics; the error is returned either way)
                bool halted = false;
                (void)pipe_complete(c, snap[pend & 1], stats_of((uint32_t)pend), &halted);
            }
            return fail(r);
        }
        if (pend >= 0) {
            r = settle((int64_t)k);
            if (r < 0) return fail(r);
            if (r == 1) {
                pend = -1;
                continue;
            }
        }
        pend = k;
    }
    if (pend >= 0) {
        const int r = settle(-1);
        if (r < 0) return fail(r);
    }
    return DV_OK;
}

}  // namespace

extern "C" {

int dv_epoch_run_device_batch(dv_ctx *c, const dv_epoch_dev *eps, uint32_t n, uint8_t *const *d_commits,
                              dv_stats *sts) {
    KProfScope kps_(c);
    if (!c || (n && !eps)) return DV_ERR_ARG;
    if (c->phase != 0) return DV_ERR_STATE;
    HIPCHK(hipSetDevice(c->cfg.device));
    auto commit_of = [&](uint32_t k) { return d_commits ? d_commits[k] : nullptr; };
    return run_batch(
        c, n, sts, commit_of,
        [&](uint32_t k) {
            return (prefix_applies(c, &eps[k]) || small_pipelined(c, &eps[k])) && !timing(c) && !ktiming(c) &&
                   !c->rep_P;
        },
        [&](uint32_t k) {
            if (prefix_applies(c, &eps[k])) return run_prefix_epoch(c, &eps[k]);
            return graph_decide(c, &eps[k], nullptr, [&] { return small_enqueue(c, &eps[k]); });
        },
        [&](uint32_t k, dv_stats *st) { return dv_epoch_run_device(c, &eps[k], commit_of(k), nullptr, st); });
}

int dv_tpcc_epoch_run_device_batch(dv_ctx *c, const dv_epoch_dev *eps, const uint64_t *const *d_args, uint32_t n,
                                   uint8_t *const *d_commits, uint64_t *const *d_oids, dv_stats *sts) {
    KProfScope kps_(c);
    if (!c || (n && (!eps || !d_args)) || c->cfg.workload != DV_TPCC) return DV_ERR_ARG;
    if (c->phase != 0) return DV_ERR_STATE;
    HIPCHK(hipSetDevice(c->cfg.device));
    auto commit_of = [&](uint32_t k) { return d_commits ? d_commits[k] : nullptr; };
    auto oid_of = [&](uint32_t k) { return d_oids ? d_oids[k] : nullptr; };
    return run_batch(
        c, n, sts, commit_of, [&](uint32_t) { return !timing(c) && !ktiming(c); },
        [&](uint32_t k) {
            return graph_decide(c, &eps[k], d_args[k], [&] {
                int r = dv_tpcc_epoch_begin(c, &eps[k], d_args[k], oid_of(k));
                if (!r && c->cfg.cc_alg != DV_CALVIN && c->n_txn) {
                    r = decide_epoch(c);
                    if (r) {
                        c->phase = 0;
                        c->tp_args = c->tp_oid = nullptr;
                    }
                }
                return r;
            });
        },
        [&](uint32_t k, dv_stats *st) {
            return dv_tpcc_epoch_run_device(c, &eps[k], d_args[k], commit_of(k), oid_of(k), st);
        });
}

}  // extern "C"

namespace {

// the lanes of one call: non-null, distinct, one owner's tables, one device,
// one CC algorithm and workload
int check_lanes(dv_ctx *const *lanes, uint32_t n_lanes) {
    if (!lanes || n_lanes == 0 || n_lanes > kMaxLanes) return DV_ERR_ARG;
    dv_ctx *const c0 = lanes[0];
    for (uint32_t l = 0; l < n_lanes; l++) {
        dv_ctx *c = lanes[l];
        if (!c) return DV_ERR_ARG;
        if (c->phase != 0) return DV_ERR_STATE;
        const dv_ctx *own = c->table_owner ? c->table_owner : c;
        const dv_ctx *own0 = c0->table_owner ? c0->table_owner : c0;
        if (own != own0 || c->cfg.device != c0->cfg.device || c->cfg.cc_alg != c0->cfg.cc_alg ||
            c->cfg.workload != c0->cfg.workload)
            return DV_ERR_ARG;
        for (uint32_t m = 0; m < l; m++)
            if (lanes[m] == c) return DV_ERR_ARG;
    }
    return DV_OK;
}

// each lane's CU-masked stream (lane l of n: the CUs i with i % n == l) and
// its asynchronous launch's workgroups on that share
int lane_streams(dv_ctx *const *lanes, uint32_t n_lanes) {
    int cus = 0;
    HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, lanes[0]->cfg.device));
    for (uint32_t l = 0; l < n_lanes; l++) {
        dv_ctx *c = lanes[l];
        if (c->lane_stream && c->lane_n == n_lanes && c->lane_l == l) continue;
        if (c->lane_stream) (void)hipStreamDestroy(c->lane_stream);
        c->lane_stream = nullptr;
        std::vector<uint32_t> mask((cus + 31) / 32, 0u);
        uint32_t mine = 0;
        for (int i = 0; i < cus; i++)
            if ((uint32_t)i % n_lanes == l) mask[i / 32] |= 1u << (i % 32), mine++;
        HIPCHK(hipExtStreamCreateWithCUMask(&c->lane_stream, (uint32_t)mask.size(), mask.data()));
        c->lane_n = n_lanes;
        c->lane_l = l;
        // (3/4 of what the share holds: with all of it, three lanes' launches
        // never found their workgroups co-resident -- the CU mask's bits do
        // not split every way evenly -- 2.7 ms per epoch; with 3/4, 0.29)
#ifndef DVCC_LANE_G_EIGHTHS
#define DVCC_LANE_G_EIGHTHS 6  // (the asynchronous launch's share of a lane's workgroups, in eighths)
#endif
        c->lane_g = std::max(1u, (uint32_t)((uint64_t)c->async_g * mine * DVCC_LANE_G_EIGHTHS / 8 / (uint32_t)cus));
    }
    return DV_OK;
}

// Ordered lanes with communicators (dv_lanes_order at N > 1): every lane's
// collectives go to its own stream, and RCCL kernels wait for their peers, so
// two lanes' streams must never feed one hardware queue -- two collectives
// queued in opposite orders on two GPUs would wait for each other for ever.
// A CU mask is a property of the hardware queue, so a CU-masked stream gets
// a queue of its own (measured, tools/micro/queue_share.hip: with
// GPU_MAX_HW_QUEUES 4, plain streams 0 and 7 share one, CU-masked streams
// never).  The order does not rest on that observation alone: for every pair
// of lane streams a bounded probe checks it -- a kernel on lane a spins (at
// most ~50 ms) until a kernel queued after it on lane b sets a word, which
// only happens if b's kernel runs beside a's, i.e. on another queue.
__global__ void k_queue_probe_wait(uint32_t *flag, uint32_t *seen) {
    if (threadIdx.x != 0) return;
    const uint64_t t0 = wall_clock64();
    uint32_t v = 0;
    while ((v = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0u &&
           wall_clock64() - t0 < 5000000ull)  // ~50 ms at the 100 MHz constant clock
        __builtin_amdgcn_s_sleep(4);
    *seen = v;
}
__global__ void k_queue_probe_set(uint32_t *flag) {
    if (threadIdx.x == 0) __hip_atomic_store(flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

int lanes_own_queues(dv_ctx *const *lanes, uint32_t n_lanes) {
    uint32_t *d = nullptr;
    HIPCHK(hipMalloc(&d, 2 * sizeof(uint32_t)));
    int r = DV_OK;
    for (uint32_t a = 0; a < n_lanes && !r; a++)
        for (uint32_t b = 0; b < n_lanes && !r; b++) {
            if (a == b) continue;
            uint32_t seen = 0;
            hipStream_t sa = lanes[a]->lane_stream, sb = lanes[b]->lane_stream;
            if (hipMemsetAsync(d, 0, 2 * sizeof(uint32_t), sa) != hipSuccess ||
                hipStreamSynchronize(sa) != hipSuccess) { r = DV_ERR_HIP; break; }
            hipLaunchKernelGGL(k_queue_probe_wait, dim3(1), dim3(64), 0, sa, d, d + 1);
            hipLaunchKernelGGL(k_queue_probe_set, dim3(1), dim3(64), 0, sb, d);
            if (hipStreamSynchronize(sa) != hipSuccess || hipStreamSynchronize(sb) != hipSuccess ||
                hipMemcpy(&seen, d + 1, sizeof(seen), hipMemcpyDeviceToHost) != hipSuccess)
                r = DV_ERR_HIP;
            else if (!seen)
                r = DV_ERR_STATE;  // lanes a and b share a hardware queue: no ordered lanes with collectives
        }
    (void)hipFree(d);
    return r;
}

// while a lanes call runs each lane works on its masked stream, ordered after
// the caller's stream at the start, and the caller's after it at the end
// nothing queued on s is unfinished (a "not ready" answer is not left
// behind as the thread's last error)
bool stream_idle(hipStream_t s) {
    const hipError_t q = hipStreamQuery(s);
    if (q == hipErrorNotReady && hipPeekAtLastError() == hipErrorNotReady) (void)hipGetLastError();
    return q == hipSuccess;
}

struct OnLaneStreams {
    dv_ctx *const *ls;
    uint32_t n;
    hipStream_t saved[kMaxLanes];
    uint32_t saved_g[kMaxLanes];
    // (a stream with nothing unfinished needs no event: what it ran is
    // visible to every later launch -- the common case at both ends of a
    // pipelined call, whose event pairs cost the host ~10 us per lane)
    OnLaneStreams(dv_ctx *const *l, uint32_t m) : ls(l), n(m) {
        for (uint32_t i = 0; i < n; i++) {
            saved[i] = ls[i]->stream;
            saved_g[i] = ls[i]->async_g;
            if (!stream_idle(ls[i]->stream)) {
                (void)hipEventRecord(ls[i]->lane_ev, ls[i]->stream);
                (void)hipStreamWaitEvent(ls[i]->lane_stream, ls[i]->lane_ev, 0);
            }
            ls[i]->stream = ls[i]->lane_stream;
            ls[i]->async_g = ls[i]->lane_g;
        }
    }
    ~OnLaneStreams() {
        for (uint32_t i = 0; i < n; i++) {
            if (!stream_idle(ls[i]->stream)) {
                (void)hipEventRecord(ls[i]->lane_ev, ls[i]->stream);
                (void)hipStreamWaitEvent(saved[i], ls[i]->lane_ev, 0);
            }
            ls[i]->stream = saved[i];
            ls[i]->async_g = saved_g[i];
        }
    }
};

// Decision lanes: epoch k is decided on lanes[k % n_lanes] (each lane its own
// stream and workspace), so one lane's rounds overlap another's; executions
// stay in epoch order -- epoch k's waits for epoch k-1's post (k_lane_wait /
// k_lane_post: a device word, not an event across the lanes' streams) and
// starts halted when k-1 halted or failed.  The host reads epochs back oldest first; a halted
// one is run again with every epoch queued behind it, synchronously and in
// order, as run_batch does on one stream.  pipelined(k): epoch k can be
// queued that way; decide(c, k, tail): queues its decision on lane c, then
// tail() -- the execution in epoch order -- inside the epoch's graph when it
// replays one (graph_decide with lanes_key); after(c, k): queues what follows the execution on the lane (a
// closed loop's refill; it runs before the next epoch's execution, on any
// lane, is queued, and is a no-op when the epoch halted); run(k, st): runs
// it synchronously on its lane.
// the graph key words of a lanes epoch's execution (run_lanes' tail): its
// outputs and the lanes' shared order word (lanes[0]'s); the lane's own turn
// word is its context's
GraphKeyX lanes_key(dv_ctx *const *lanes, uint32_t n_lanes, const void *commit, const void *oid) {
    GraphKeyX x;
    x.w[0] = (uint64_t)commit;
    x.w[1] = (uint64_t)oid;
    x.w[2] = (uint64_t)lanes[0];
    x.w[3] = n_lanes | 1ull << 32;
    return x;
}

template <class Commit, class Pipelined, class Decide, class After, class Run>
int run_lanes(dv_ctx *const *lanes, uint32_t n_lanes, uint32_t n, dv_stats *sts, Commit &&commit_of,
              Pipelined &&pipelined, Decide &&decide, After &&after, Run &&run) {
    const auto t_enter = std::chrono::steady_clock::now();
    HIPCHK(hipSetDevice(lanes[0]->cfg.device));
    int r0 = lane_streams(lanes, n_lanes);
    if (r0) return r0;
    // DVCC_HOST_PROF: the host time from the last read-back to the return
    // (the lane streams handed back below), printed on the way out
    struct ExitProf {
        bool on = false;
        std::chrono::steady_clock::time_point t0;
        ~ExitProf() {
            if (on)
                std::fprintf(stderr, "dvcc host: %.1f us from the last read-back to the return\n",
                             std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() * 1e6);
        }
    } exit_prof_;
    const auto t_streams = std::chrono::steady_clock::now();
    OnLaneStreams on_lanes_(lanes, n_lanes);
    const double us_streams = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_streams).count() * 1e6;
    auto stats_of = [&](uint32_t k) { return sts ? &sts[k] : nullptr; };
    auto lane_of = [&](uint32_t k) { return lanes[k % n_lanes]; };
    struct Pend {
        uint32_t k;
        EpochSnap sn;
    };
    // queued and unread epochs, oldest first; each lane holds at most two
    // (its two mirror slots)
    const uint32_t window = 2 * n_lanes - 1;
    Pend ring[2 * kMaxLanes];
    uint32_t head = 0, count = 0;
    uint32_t lane_slot[kMaxLanes] = {};
    dv_ctx *prev = nullptr;  // the lane of the last queued epoch (nullptr: nothing queued is unfinished)
    // the executions' order words (k_lane_wait / k_lane_post): each lane's
    // turn (its d_gate[0]) and the shared count of executed turns (lanes[0]'s
    // d_gate[1]), set at the start of every run of pipelined epochs (the
    // call's, and after a synchronous run), while nothing queued is
    // unfinished: the turns count on from every turn ever issued through that
    // word, from the run's first lane, each written on its own lane's stream,
    // and the count is set to where they start on the first lane's stream --
    // no older post can match a turn of this run (none reached past the
    // issued count), so no host wait
    uint32_t *const done_w = lanes[0]->d_gate + 1;
    auto order_init = [&](uint32_t k0) -> int {
        const uint32_t base = lanes[0]->lane_issued & 0x7FFFFFFFu;
        for (uint32_t i = 0; i < n_lanes; i++) {
            dv_ctx *l = lanes[(k0 + i) % n_lanes];
            HIPCHK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(l->d_gate), base + i, 1, l->stream));
        }
        HIPCHK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(done_w), base << 1, 1, lanes[k0 % n_lanes]->stream));
        return DV_OK;
    };
    auto drain = [&] {
        for (uint32_t l = 0; l < n_lanes; l++) (void)hipStreamSynchronize(lanes[l]->stream);
    };
    auto run_sync = [&](uint32_t k) { return run(k, stats_of(k)); };
    // DVCC_HOST_PROF=1: the host's time queueing epochs vs waiting for their
    // read-backs, to stderr (is the host or the device the bound?)
    static const bool hprof = std::getenv("DVCC_HOST_PROF") != nullptr;
    using hclock = std::chrono::steady_clock;
    double t_queue = 0, t_wait = 0, t_decide = 0;
    tl_hp_walk = tl_hp_glaunch = 0;
    tl_hp_replays = tl_hp_captures = 0;
    tl_hprof = hprof;
    tl_hp_launch_s = 0;
    tl_hp_launch_n = 0;
    const auto t_all = hclock::now();
    // read back the oldest queued epoch; a halted one and all behind it run again
    auto settle = [&]() -> int {
        Pend &p = ring[head];
        bool halted = false;
        int r = pipe_complete(lane_of(p.k), p.sn, stats_of(p.k), &halted);
        if (r) {
            drain();
            return r;
        }
        head = (head + 1) % (2 * kMaxLanes);
        count--;
        if (!halted) return DV_OK;
        drain();
        for (uint32_t l = 0; l < n_lanes; l++) {
            r = pipe_redo(lanes[l]);
            if (r) return r;
        }
        r = run_sync(p.k);
        for (; !r && count; count--, head = (head + 1) % (2 * kMaxLanes)) r = run_sync(ring[head].k);
        count = 0;
        prev = nullptr;
        return r;
    };
    for (uint32_t k = 0; k < n; k++) {
        dv_ctx *c = lane_of(k);
        if (!prev && pipelined(k)) {  // (every lane idle: nothing queued is unfinished)
            const int r = order_init(k);
            if (r) return r;
        }
        if (!pipelined(k)) {
            while (count) {
                const int r = settle();
                if (r) return r;
            }
            const int r = run_sync(k);
            if (r) return r;
            prev = nullptr;
            continue;
        }
        {
            const auto tw = hclock::now();
            while (count >= window) {
                const int r = settle();
                if (r) return r;
            }
            t_wait += std::chrono::duration<double>(hclock::now() - tw).count();
        }
        const auto tq = hclock::now();
        const uint32_t l = k % n_lanes;
        const int slot = (int)(lane_slot[l]++ & 1u);
        Pend &p = ring[(head + count) % (2 * kMaxLanes)];
        p.k = k;
        // the execution in epoch order, on the device: wait for the previous
        // epoch's post (its gate halts this one), execute (and refill), post
        // -- queued by decide() behind the decision, inside its graph when it
        // replays one; the counter read-back after it, off that chain
        auto tail = [&]() -> int {
            exec_prologue(c);
            launch_lane_wait(c->stream, c->d_gate, done_w, c->ctr);
            enqueue_exec(c, commit_of(k), true);
            int rt = hip_fail(hipGetLastError(), "execution launch");
            if (!rt) rt = after(c, k);
            if (!rt) launch_lane_post(c->stream, c->d_gate, done_w, n_lanes, c->ctr);
            return rt;
        };
        const auto td = hclock::now();
        int r = decide(c, k, tail);
        // (this epoch's turn, counted whether or not its post was queued:
        // a count past the posts is safe, one short of them is not)
        lanes[0]->lane_issued++;
        t_decide += std::chrono::duration<double>(hclock::now() - td).count();
        if (!r) {
            EpochSnap &sn = p.sn;
            sn.n_acc = c->n_acc;
            sn.n_txn = c->n_txn;
            sn.rounds = c->rounds;
            sn.rounds_real = c->rounds_real;
            sn.rounds_prefix = c->rounds_prefix;
            sn.async_launched = c->async_launched;
            sn.sort_passes = c->sort_passes;
            sn.prefix_txn = c->pf_K;
            sn.n_acc_is_bound = c->n_acc_is_bound;
            sn.async_unconfirmed = c->async_unconfirmed;
            sn.slot = slot;
            sn.seq = mirror_out(c, slot);
            r = hip_fail(hipGetLastError(), "lane post");
        }
        c->phase = 0;
        c->prefix_mode = false;
        c->tp_args = c->tp_oid = nullptr;
        if (r) {
            drain();
            while (count) {  // (the read-backs, for the statistics; the error is returned either way)
                bool halted = false;
                (void)pipe_complete(lane_of(ring[head].k), ring[head].sn, stats_of(ring[head].k), &halted);
                head = (head + 1) % (2 * kMaxLanes);
                count--;
            }
            return r;
        }
        count++;
        prev = c;
        t_queue += std::chrono::duration<double>(hclock::now() - tq).count();
    }
    const auto tw = hclock::now();
    while (count) {
        const int r = settle();
        if (r) return r;
    }
    t_wait += std::chrono::duration<double>(hclock::now() - tw).count();
    if (hprof) {
        exit_prof_.on = true;
        exit_prof_.t0 = hclock::now();
    }
    if (hprof && n)
        std::fprintf(stderr, "dvcc host: %u epochs over %u lanes, %.1f us per epoch: queueing %.1f (decision %.1f), "
                     "waiting %.1f; %.1f us of set-up before the first epoch (%.1f handing over the streams)\n",
                     n, n_lanes, std::chrono::duration<double>(hclock::now() - t_all).count() * 1e6 / n,
                     t_queue * 1e6 / n, t_decide * 1e6 / n, t_wait * 1e6 / n,
                     std::chrono::duration<double>(t_all - t_enter).count() * 1e6, us_streams);
    tl_hprof = false;
    if (hprof && n)
        std::fprintf(stderr, "dvcc host: %.1f kernel launches per epoch, %.2f us of host time each (%.1f us per "
                     "epoch)\n", (double)tl_hp_launch_n / n, tl_hp_launch_n ? tl_hp_launch_s * 1e6 / tl_hp_launch_n : 0.0,
                     tl_hp_launch_s * 1e6 / n);
    if (hprof && tl_hp_replays)
        std::fprintf(stderr, "dvcc host: %u graph replays (%u captures): walk %.1f us, hipGraphLaunch %.1f us each\n",
                     tl_hp_replays, tl_hp_captures, tl_hp_walk * 1e6 / tl_hp_replays,
                     tl_hp_glaunch * 1e6 / tl_hp_replays);
    return DV_OK;
}

}  // namespace

extern "C" {

int dv_epoch_run_device_lanes(dv_ctx *const *lanes, uint32_t n_lanes, const dv_epoch_dev *eps, uint32_t n,
                              uint8_t *const *d_commits, dv_stats *sts) {
    int r = check_lanes(lanes, n_lanes);
    if (r) return r;
    if (n && !eps) return DV_ERR_ARG;
    if (lanes[0]->cfg.workload != DV_YCSB) return DV_ERR_ARG;
    if (n_lanes == 1) return dv_epoch_run_device_batch(lanes[0], eps, n, d_commits, sts);
    auto commit_of = [&](uint32_t k) { return d_commits ? d_commits[k] : nullptr; };
    return run_lanes(
        lanes, n_lanes, n, sts, commit_of,
        [&](uint32_t k) {
            dv_ctx *c = lanes[k % n_lanes];
            return (prefix_applies(c, &eps[k]) || small_pipelined(c, &eps[k])) && !timing(c) && !ktiming(c) &&
                   !c->rep_P && !c->comm;
        },
        [&](dv_ctx *c, uint32_t k, auto &tail) {
            if (prefix_applies(c, &eps[k])) {
                const int r = run_prefix_epoch(c, &eps[k]);
                return r ? r : tail();
            }
            return graph_decide(
                c, &eps[k], nullptr,
                [&] {
                    const int r = small_enqueue(c, &eps[k]);
                    return r ? r : tail();
                },
                lanes_key(lanes, n_lanes, commit_of(k), nullptr));
        },
        [](dv_ctx *, uint32_t) { return 0; },
        [&](uint32_t k, dv_stats *st) {
            return dv_epoch_run_device(lanes[k % n_lanes], &eps[k], commit_of(k), nullptr, st);
        });
}

int dv_lanes_order(dv_ctx *const *lanes, uint32_t n_lanes) {
    int r = check_lanes(lanes, n_lanes);
    if (r) return r;
    HIPCHK(hipSetDevice(lanes[0]->cfg.device));
    for (uint32_t l = 0; l < n_lanes; l++) HIPCHK(hipStreamSynchronize(lanes[l]->stream));
    if (n_lanes == 1) {  // (back on its own stream, no order)
        dv_ctx *c = lanes[0];
        if (c->order) {
            c->stream = c->own_stream;
            c->async_g = async_groups(c->cfg.device);
            c->order.reset();
        }
        return DV_OK;
    }
    for (uint32_t l = 0; l < n_lanes; l++)
        if (lanes[l]->order) return DV_ERR_STATE;  // (already ordered: dv_lanes_order(&lane, 1) first)
    r = lane_streams(lanes, n_lanes);
    if (r) return r;
    bool comm = false;
    for (uint32_t l = 0; l < n_lanes; l++) comm |= lanes[l]->comm != nullptr;
    if (comm) {  // (collectives on every lane: each lane stream on a hardware queue of its own)
        r = lanes_own_queues(lanes, n_lanes);
        if (r) return r;
    }
    auto o = std::make_shared<LaneOrder>();
    o->n = n_lanes;
    for (uint32_t l = 0; l < n_lanes; l++) {
        dv_ctx *c = lanes[l];
        c->stream = c->lane_stream;
        c->async_g = c->lane_g;
        c->order = o;
        c->order_k = 0;
    }
    return DV_OK;
}

int dv_tpcc_epoch_run_device_lanes(dv_ctx *const *lanes, uint32_t n_lanes, const dv_epoch_dev *eps,
                                   const uint64_t *const *d_args, uint32_t n, uint8_t *const *d_commits,
                                   uint64_t *const *d_oids, dv_stats *sts) {
    int r = check_lanes(lanes, n_lanes);
    if (r) return r;
    if (n && (!eps || !d_args)) return DV_ERR_ARG;
    if (lanes[0]->cfg.workload != DV_TPCC) return DV_ERR_ARG;
    if (n_lanes == 1) return dv_tpcc_epoch_run_device_batch(lanes[0], eps, d_args, n, d_commits, d_oids, sts);
    auto commit_of = [&](uint32_t k) { return d_commits ? d_commits[k] : nullptr; };
    auto oid_of = [&](uint32_t k) { return d_oids ? d_oids[k] : nullptr; };
    return run_lanes(
        lanes, n_lanes, n, sts, commit_of,
        [&](uint32_t k) {
            dv_ctx *c = lanes[k % n_lanes];
            return !timing(c) && !ktiming(c) && !c->comm;
        },
        [&](dv_ctx *c, uint32_t k, auto &tail) {
            return graph_decide(
                c, &eps[k], d_args[k],
                [&] {
                    int rr = dv_tpcc_epoch_begin(c, &eps[k], d_args[k], oid_of(k));
                    if (!rr && c->cfg.cc_alg != DV_CALVIN && c->n_txn) rr = decide_epoch(c);
                    return rr ? rr : tail();
                },
                lanes_key(lanes, n_lanes, commit_of(k), oid_of(k)));
        },
        [](dv_ctx *, uint32_t) { return 0; },
        [&](uint32_t k, dv_stats *st) {
            return dv_tpcc_epoch_run_device(lanes[k % n_lanes], &eps[k], d_args[k], commit_of(k), oid_of(k), st);
        });
}

}  // extern "C"

namespace {

// The closed loop's epochs in tb form: every buffer carries 4-byte records and
// txn boundaries (dv_epoch_dev::recs32, txn_begin), the pool records, and no
// table bytes.  The refill then writes that form -- 4 B per access and 4 per
// txn -- and, only when the epochs do not take the prefix-kill path (whose tb
// mode reads nothing else: k_probe_tb probes the prefix, the kill pass the
// later keys), also keys / types / txn ids (8 + 1 + 4 B).
struct LoopForm {
    bool tb = false, old = true;
};
LoopForm loop_form(const dv_ctx *c, const dv_epoch_dev *pool, const dv_epoch_dev *bufs, uint32_t n_bufs,
                   uint32_t n_txn) {
    LoopForm f;
    if (std::getenv("DVCC_LOOP_NO_TB") || !pool->recs32 || pool->tables) return f;
    for (uint32_t b = 0; b < n_bufs; b++)
        if (!bufs[b].recs32 || !bufs[b].txn_begin) return f;
    dv_epoch_dev d = bufs[0];
    d.n_txn = n_txn;
    d.tables = nullptr;
    f.tb = true;
    f.old = !tb_epoch(c, &d);
    return f;
}

// the closed loop's next epoch (launch_refill) into `out`: prev's aborted txns
// (prev: the epoch the context decided last, prev_buf: its buffer; NULL: none,
// all fresh), then fresh ones from the pool, in the forms f names
void enqueue_refill(dv_ctx *c, const dv_epoch_dev *prev, const dv_epoch_dev *prev_buf, const dv_epoch_dev *pool,
                    const uint32_t *pool_begin, uint32_t *cursor, uint32_t n_out, const dv_epoch_dev &out,
                    LoopForm f = {}) {
    launch_refill(c->stream, c->status, c->rs, c->re, prev ? prev->n_txn : 0u,
                  prev && f.old ? prev->keys : nullptr, prev && f.old ? prev->types : nullptr,
                  prev && f.old ? prev->tables : nullptr, pool->keys, pool->types, pool->tables, pool->acc_txn,
                  pool_begin, pool->n_txn, cursor, n_out, (uint64_t)n_out * pool->max_txn_acc,
                  f.old ? const_cast<uint64_t *>(out.keys) : nullptr, const_cast<uint8_t *>(out.types),
                  const_cast<uint32_t *>(out.acc_txn), const_cast<uint8_t *>(out.tables),
                  const_cast<uint32_t *>(out.n_acc_dev), c->carry_b, c->carry_b + c->carry_nb, c->carry_tot,
                  prev ? c->ctr : nullptr, f.tb && prev_buf ? prev_buf->recs32 : nullptr,
                  f.tb ? pool->recs32 : nullptr, f.tb ? const_cast<uint32_t *>(out.recs32) : nullptr,
                  f.tb ? const_cast<uint32_t *>(out.txn_begin) : nullptr);
}

}  // namespace

extern "C" {

int dv_epoch_run_closed_loop(dv_ctx *c, const dv_epoch_dev *pool, const uint32_t *pool_begin, uint32_t *cursor,
                             uint32_t n_txn, dv_epoch_dev *bufs, uint64_t buf_cap, uint32_t n_epochs,
                             int resume, uint8_t *const *d_commits, dv_stats *sts) {
    KProfScope kps_(c);
    if (!c || !pool || !pool_begin || !cursor || !bufs || !n_txn) return DV_ERR_ARG;
    if (c->phase != 0) return DV_ERR_STATE;
    if (c->cfg.cc_alg == DV_CALVIN || c->cfg.workload != DV_YCSB || c->comm) return DV_ERR_STATE;
    const uint64_t bound = (uint64_t)n_txn * pool->max_txn_acc;
    if (!pool->max_txn_acc || n_txn > pool->n_txn || n_txn > c->cfg.max_txn || bound > buf_cap ||
        bound > c->cfg.max_acc || !pool->keys || !pool->types || !pool->acc_txn)
        return DV_ERR_ARG;
    for (int b = 0; b < 2; b++)
        if (!bufs[b].keys || !bufs[b].types || !bufs[b].acc_txn || !bufs[b].n_acc_dev ||
            (pool->tables && !bufs[b].tables))
            return DV_ERR_ARG;
    HIPCHK(hipSetDevice(c->cfg.device));
    int r = carry_bufs(c, carry_blocks(n_txn));
    if (r) return r;
    const LoopForm form = loop_form(c, pool, bufs, 2, n_txn);
    // epoch k's descriptor: buffer k & 1, its access count on the device
    auto desc = [&](uint32_t k) {
        dv_epoch_dev d = bufs[k & 1];
        if (form.old) d.txn_begin = d.recs32 = nullptr;  // (the engine reads the old form)
        d.tables = pool->tables ? bufs[k & 1].tables : nullptr;
        d.n_txn = n_txn;
        d.n_acc = bound;
        d.max_txn_acc = pool->max_txn_acc;
        d.ts = nullptr;  // (sequence order: carried txns first keep their priority)
        return d;
    };
    auto commit_of = [&](uint32_t k) { return d_commits ? d_commits[k] : nullptr; };
    auto stats_of = [&](uint32_t k) { return sts ? &sts[k] : nullptr; };
    auto fail = [&](int e) {
        c->mir_pending = false;
        (void)hipStreamSynchronize(c->stream);
        return e;
    };
    if (!resume) enqueue_refill(c, nullptr, nullptr, pool, pool_begin, cursor, n_txn, bufs[0], form);
    const dv_epoch_dev d0 = desc(0);
    const bool pipelined = prefix_applies(c, &d0) && !timing(c) && !ktiming(c) && !c->rep_P;
    EpochSnap snap[2];
    int64_t pend = -1;
    // epoch k run synchronously, then its refill
    auto run_one = [&](uint32_t k) {
        const dv_epoch_dev d = desc(k);
        int e = dv_epoch_run_device(c, &d, commit_of(k), nullptr, stats_of(k));
        if (!e) {
            enqueue_refill(c, &d, &bufs[k & 1], pool, pool_begin, cursor, n_txn, bufs[(k + 1) & 1], form);
            e = hip_fail(hipGetLastError(), "refill");
        }
        return e;
    };
    for (uint32_t k = 0; k < n_epochs; k++) {
        if (!pipelined) {
            r = run_one(k);
            if (r) return fail(r);
            continue;
        }
        const dv_epoch_dev d = desc(k);
        r = pipe_enqueue(c, [&] { return run_prefix_epoch(c, &d); }, commit_of(k), pend >= 0, (int)(k & 1),
                         snap[k & 1], k + 1 < n_epochs);
        if (!r) {
            // behind the execution: epoch k + 1 from epoch k's final statuses (a
            // no-op when k halted -- the host redoes both below)
            enqueue_refill(c, &d, &bufs[k & 1], pool, pool_begin, cursor, n_txn, bufs[(k + 1) & 1], form);
            r = hip_fail(hipGetLastError(), "refill");
        }
        if (r) {
            (void)hipStreamSynchronize(c->stream);
            if (pend >= 0) {
                bool halted = false;
                (void)pipe_complete(c, snap[pend & 1], stats_of((uint32_t)pend), &halted);
            }
            return fail(r);
        }
        if (pend >= 0) {
            bool halted = false;
            r = pipe_complete(c, snap[pend & 1], stats_of((uint32_t)pend), &halted);
            if (r) return fail(r);
            if (halted) {
                // epoch pend halted: epoch k started halted and neither refill
                // ran.  Decide pend again synchronously, refill from it, and
                // queue epoch k again.
                c->mir_pending = false;
                r = pipe_redo(c);
                if (!r) r = run_one((uint32_t)pend);
                if (r) return fail(r);
                pend = -1;
                k--;  // (k = pend + 1 again)
                continue;
            }
        }
        pend = k;
    }
    if (pend >= 0) {
        bool halted = false;
        r = pipe_complete(c, snap[pend & 1], stats_of((uint32_t)pend), &halted);
        if (r) return fail(r);
        if (halted) {
            r = pipe_redo(c);
            if (!r) r = run_one((uint32_t)pend);
            if (r) return fail(r);
        }
    }
    HIPCHK(hipStreamSynchronize(c->stream));  // (the next epoch's refill: the caller may read it)
    return DV_OK;
}

// The closed loop over decision lanes: epoch k on lanes[k % L]; each lane
// keeps its own pair of epoch buffers (bufs[2l], bufs[2l + 1]) and its epochs
// form a closed loop of their own -- epoch k + L is epoch k's aborted txns,
// then fresh pool txns -- while the shared pool cursor advances in epoch
// order (refill k is queued behind execution k, which waits for execution
// k - 1 and the refill behind it).  The epochs are those of one sequence in
// which an aborted txn returns L epochs later (the reference's retry after a
// penalty, abort_queue.cpp:26-82, with a penalty of L epochs).
int dv_epoch_run_closed_loop_lanes(dv_ctx *const *lanes, uint32_t n_lanes, const dv_epoch_dev *pool,
                                   const uint32_t *pool_begin, uint32_t *cursor, uint32_t n_txn, dv_epoch_dev *bufs,
                                   uint64_t buf_cap, uint32_t n_epochs, int resume, uint8_t *const *d_commits,
                                   dv_stats *sts) {
    int r = check_lanes(lanes, n_lanes);
    if (r) return r;
    if (n_lanes == 1)
        return dv_epoch_run_closed_loop(lanes[0], pool, pool_begin, cursor, n_txn, bufs, buf_cap, n_epochs, resume,
                                        d_commits, sts);
    if (!pool || !pool_begin || !cursor || !bufs || !n_txn) return DV_ERR_ARG;
    dv_ctx *const c0 = lanes[0];
    if (c0->cfg.cc_alg == DV_CALVIN || c0->cfg.workload != DV_YCSB) return DV_ERR_STATE;
    const uint64_t bound = (uint64_t)n_txn * pool->max_txn_acc;
    if (!pool->max_txn_acc || n_txn > pool->n_txn || n_txn > c0->cfg.max_txn || bound > buf_cap ||
        bound > c0->cfg.max_acc || !pool->keys || !pool->types || !pool->acc_txn)
        return DV_ERR_ARG;
    for (uint32_t b = 0; b < 2 * n_lanes; b++)
        if (!bufs[b].keys || !bufs[b].types || !bufs[b].acc_txn || !bufs[b].n_acc_dev ||
            (pool->tables && !bufs[b].tables))
            return DV_ERR_ARG;
    for (uint32_t l = 0; l < n_lanes; l++)
        if (lanes[l]->comm) return DV_ERR_STATE;
    HIPCHK(hipSetDevice(c0->cfg.device));
    for (uint32_t l = 0; l < n_lanes; l++) {
        r = carry_bufs(lanes[l], carry_blocks(n_txn));
        if (r) return r;
    }
    const LoopForm form = loop_form(c0, pool, bufs, 2 * n_lanes, n_txn);
    // lane l's j-th epoch of this call (global k = j * L + l) sits in buffer
    // 2l + (j & 1); its refill writes 2l + ((j + 1) & 1)
    auto buf_of = [&](uint32_t k, uint32_t ahead) { return &bufs[2 * (k % n_lanes) + (((k / n_lanes) + ahead) & 1)]; };
    auto desc = [&](uint32_t k) {
        dv_epoch_dev d = *buf_of(k, 0);
        if (form.old) d.txn_begin = d.recs32 = nullptr;  // (the engine reads the old form)
        d.tables = pool->tables ? d.tables : nullptr;
        d.n_txn = n_txn;
        d.n_acc = bound;
        d.max_txn_acc = pool->max_txn_acc;
        d.ts = nullptr;
        return d;
    };
    auto commit_of = [&](uint32_t k) { return d_commits ? d_commits[k] : nullptr; };
    if (!resume)  // each lane's first epoch: fresh txns, drawn in lane order
        for (uint32_t l = 0; l < n_lanes; l++) {
            dv_ctx *c = lanes[l];
            enqueue_refill(c, nullptr, nullptr, pool, pool_begin, cursor, n_txn, *buf_of(l, 0), form);
            HIPCHK(hipGetLastError());
            HIPCHK(hipStreamSynchronize(c->stream));
        }
    const dv_epoch_dev d0 = desc(0);
    const bool pipelined = prefix_applies(c0, &d0) && !timing(c0) && !ktiming(c0);
    r = run_lanes(
        lanes, n_lanes, n_epochs, sts, commit_of, [&](uint32_t) { return pipelined; },
        [&](dv_ctx *c, uint32_t k, auto &tail) {
            const dv_epoch_dev d = desc(k);
            const int e = run_prefix_epoch(c, &d);
            return e ? e : tail();
        },
        [&](dv_ctx *c, uint32_t k) {  // (behind the execution; a no-op when k halted)
            const dv_epoch_dev d = desc(k);
            enqueue_refill(c, &d, buf_of(k, 0), pool, pool_begin, cursor, n_txn, *buf_of(k, 1), form);
            return hip_fail(hipGetLastError(), "refill");
        },
        [&](uint32_t k, dv_stats *st) {  // (synchronous, refill included: the next refill, on
                                         // another lane, draws from the cursor after it)
            dv_ctx *c = lanes[k % n_lanes];
            const dv_epoch_dev d = desc(k);
            int e = dv_epoch_run_device(c, &d, commit_of(k), nullptr, st);
            if (!e) {
                enqueue_refill(c, &d, buf_of(k, 0), pool, pool_begin, cursor, n_txn, *buf_of(k, 1), form);
                e = hip_fail(hipGetLastError(), "refill");
            }
            if (!e) e = hip_fail(hipStreamSynchronize(c->stream), "sync");
            return e;
        });
    for (uint32_t l = 0; l < n_lanes; l++) (void)hipStreamSynchronize(lanes[l]->stream);
    return r;
}

}  // extern "C"

// A replicated epoch (dv_epoch_run_part): the whole epoch's accesses, the
// global txn order, on this rank; every key's row id is the key, keys of this
// partition are checked against its index and the error bits combined over
// the ranks after the probe, all txns are decided here, and only this
// partition's rows execute.  Every rank computes the same decisions.
bool group_tb_epoch(const dv_ctx *c, const dv_epoch_dev *ep) {
    return prefix_applies(c, ep) && ep->txn_begin && ep->recs32 && !ep->n_acc_dev && !ep->tables;
}

int epoch_run_replicated(dv_ctx *c, const dv_epoch_dev *ep, const uint32_t *keys32, uint32_t nranks,
                         uint8_t *d_commit, dv_stats *st, const RouteOut *route) {
    if (!c || !ep || nranks == 0) return DV_ERR_ARG;
    c->rep_P = nranks;
    c->keys32 = keys32;
    c->route = route;
    const int r = dv_epoch_run_device(c, ep, d_commit, nullptr, st);
    if (c->fin_pending) return r;  // (the route stays set for epoch_replicated_complete's redo)
    c->rep_P = 0;
    c->keys32 = nullptr;
    c->route = nullptr;
    return r;
}

int epoch_replicated_complete(dv_ctx *c, dv_stats *st) {
    if (!c || !c->fin_pending) return DV_ERR_STATE;
    const int r = epoch_finish_complete(c, st);
    c->rep_P = 0;
    c->keys32 = nullptr;
    c->route = nullptr;
    return r;
}

extern "C" {

// TPC-C epochs: the last-name lookups resolve into a scratch copy of the
// epoch, which then runs the generic path; dv_epoch_finish executes the
// committed txns' TPC-C operations (dvcc_tpcc.hip).
int dv_tpcc_epoch_begin(dv_ctx *c, const dv_epoch_dev *ep, const uint64_t *d_args, uint64_t *d_oid) {
    KProfScope kps_(c);
    if (!c || !ep || (ep->n_acc && (!d_args || !ep->tables)) || c->cfg.workload != DV_TPCC) return DV_ERR_ARG;
    if (ep->n_acc > c->cfg.max_acc || ep->n_txn > c->cfg.max_txn) return DV_ERR_ARG;
    HIPCHK(hipSetDevice(c->cfg.device));
    int r = DV_OK;
    const HostTable &dt = c->tab[DV_TPCC_DISTRICT];
    const uint64_t drows = dt.created ? dt.cap_rows : 1;
    if (c->tp_dsnap_cap < drows) {
        c->ws_gen++;
        dfree(c->tp_dsnap);
        c->tp_dsnap = nullptr;
        r = dalloc(&c->tp_dsnap, 2 * drows);  // (snapshots, then the queue starts: k_tpcc_oid)
        if (r) return r;
        c->tp_dsnap_cap = drows;
    }
    // no host wait: the probe of dv_epoch_begin resolves the last names in
    // place, and one without customers resolves to key ~0, which it then
    // reports as DV_ERR_KEY_NOT_FOUND
    static const uint64_t kNoArgs = 0;
    c->tp_args = d_args ? d_args : &kNoArgs;  // an empty partition still finishes
    c->tp_oid = d_oid;
    c->tp_resolve = true;
    r = dv_epoch_begin(c, ep, nullptr);
    c->tp_resolve = false;
    if (r) c->tp_args = c->tp_oid = nullptr;
    return r;
}

int dv_tpcc_epoch_run_device(dv_ctx *c, const dv_epoch_dev *ep, const uint64_t *d_args, uint8_t *d_commit,
                             uint64_t *d_oid, dv_stats *st) {
    KProfScope kps_(c);
    int r = dv_tpcc_epoch_begin(c, ep, d_args, d_oid);
    if (r) return r;
    if (c->cfg.cc_alg != DV_CALVIN && c->n_txn) {
        r = decide_epoch(c);
        if (r) { c->phase = 0; c->tp_args = nullptr; c->tp_oid = nullptr; return r; }
    }
    return dv_epoch_finish(c, d_commit, st);
}

int dv_set_async_limits(dv_ctx *c, uint32_t max_iters, uint32_t idle_us) {
    if (!c) return DV_ERR_ARG;
    if (c->phase != 0) return DV_ERR_STATE;
    c->async_max_iters = max_iters ? max_iters : (1u << 18);
    c->async_idle_ticks = (uint64_t)(idle_us ? idle_us : kAsyncIdleUs) * c->wall_khz / 1000;
    return DV_OK;
}

// partitioned epochs: every partition must learn of an input error found on
// any of them before the rounds, so that all leave at the same collective
int dv_epoch_errors_local(dv_ctx *c, uint32_t *d_word) {
    KProfScope kps_(c);
    if (!c || !d_word) return DV_ERR_ARG;
    if (c->phase != 1) return DV_ERR_STATE;
    HIPCHK(hipMemcpyAsync(d_word, &c->ctr->err, sizeof(uint32_t), hipMemcpyDeviceToDevice, c->stream));
    return DV_OK;
}

int dv_epoch_errors_combined(dv_ctx *c, const uint32_t *d_word) {
    KProfScope kps_(c);
    if (!c || !d_word) return DV_ERR_ARG;
    if (c->phase != 1) return DV_ERR_STATE;
    HIPCHK(hipMemcpyAsync(&c->ctr->peer_err, d_word, sizeof(uint32_t), hipMemcpyDeviceToDevice, c->stream));
    return DV_OK;
}

int dv_round_log(dv_ctx *c, uint32_t *live, uint32_t *undecided, uint32_t cap) {
    if (!c || !c->h_ctr) return 0;
    uint32_t n = c->rounds < (uint32_t)kRoundLog ? c->rounds : (uint32_t)kRoundLog;
    if (n > cap) n = cap;
    for (uint32_t r = 0; r < n; r++) {
        if (live) live[r] = c->h_ctr->log_live[r];
        if (undecided) undecided[r] = c->h_ctr->log_und[r];
    }
    return (int)n;
}

}  // extern "C"

namespace {
// host buffers -> the context's device epoch (H2D of the 16-B records, then
// split into SoA on the device, checked against txn_begin there)
// the host side of an epoch from host records: capacity and the CSR form
// (txn_begin: monotone, ends at n_acc; its longest txn bounds the verdict
// bytes).  One branch-free pass, so it vectorises (a 1M-txn epoch: ~0.3 ms).
int check_host_epoch(const dv_ctx *c, const dv_access *acc, uint64_t n_acc, const uint32_t *txn_begin,
                     uint32_t n_txn, uint32_t *max_len) {
    if (!c || (n_acc && !acc)) return DV_ERR_ARG;
    if (n_acc > c->cfg.max_acc || n_txn > c->cfg.max_txn) return DV_ERR_ARG;
    *max_len = 0;
    if (!txn_begin) return DV_OK;  // records only: their txn_seq order is checked by the probe
    if (txn_begin[0] != 0 || txn_begin[n_txn] != n_acc) return DV_ERR_ARG;
    uint32_t mx = 0, bad = 0;
    for (uint32_t t = 0; t < n_txn; t++) {
        const uint32_t d = txn_begin[t + 1] - txn_begin[t];
        bad |= (uint32_t)(txn_begin[t + 1] < txn_begin[t]);
        mx = d > mx ? d : mx;
    }
    if (bad || mx > kMaxPos) return DV_ERR_ARG;
    *max_len = mx;
    return DV_OK;
}

int alloc_host_staging(dv_ctx *c) {
    if (c->d_acc) return DV_OK;
    const uint64_t A = c->cfg.max_acc;
    int r = dalloc(&c->d_acc, A);
    if (!r) r = dalloc(&c->d_keys, A);
    if (!r) r = dalloc(&c->d_types, A);
    if (!r) r = dalloc(&c->d_tables, A);
    if (!r) r = dalloc(&c->d_txn, A);
    if (!r) r = dalloc(&c->d_commit, c->cfg.max_txn);
    if (!r && c->cfg.cc_alg == DV_CALVIN) r = dalloc(&c->d_grant, A);
    if (!r) r = dalloc(&c->d_tb, (uint64_t)c->cfg.max_txn + 1);
    if (!r) r = dalloc(&c->split_err, 1);
    return r;
}

// device records (d_acc, and d_tb for the CSR form) -> the epoch's arrays,
// on the context's stream
void split_records(dv_ctx *c, const dv_access *d_acc, uint64_t n_acc, const uint32_t *d_tb, uint32_t n_txn,
                   uint32_t max_len, dv_epoch_dev *ep) {
    if (n_acc) {
        (void)hipMemsetAsync(c->split_err, 0, sizeof(uint32_t), c->stream);
        launch_split_access(c->stream, d_acc, n_acc, d_tb, n_txn, c->d_keys, c->d_types, c->d_txn, c->d_tables,
                            c->split_err);
        c->err_seed = c->split_err;  // the epoch starts with the record check's verdict (input_err)
    }
    *ep = dv_epoch_dev{};
    ep->keys = c->d_keys;
    ep->types = c->d_types;
    ep->acc_txn = c->d_txn;
    ep->tables = c->d_tables;
    ep->n_acc = n_acc;
    ep->n_txn = n_txn;
    ep->max_txn_acc = max_len;
}

int stage_host_epoch(dv_ctx *c, const dv_access *acc, uint64_t n_acc, const uint32_t *txn_begin,
                     uint32_t n_txn, dv_epoch_dev *ep) {
    uint32_t max_len = 0;
    int r = check_host_epoch(c, acc, n_acc, txn_begin, n_txn, &max_len);
    if (r) return r;
    HIPCHK(hipSetDevice(c->cfg.device));
    r = alloc_host_staging(c);
    if (r) return r;
    if (n_acc) {
        HIPCHK(hipMemcpyAsync(c->d_acc, acc, n_acc * sizeof(dv_access), hipMemcpyHostToDevice, c->stream));
        if (txn_begin)
            HIPCHK(hipMemcpyAsync(c->d_tb, txn_begin, ((size_t)n_txn + 1) * sizeof(uint32_t),
                                  hipMemcpyHostToDevice, c->stream));
    }
    split_records(c, c->d_acc, n_acc, txn_begin ? c->d_tb : nullptr, n_txn, max_len, ep);
    return DV_OK;
}

}  // namespace

extern "C" {

int dv_epoch_run(dv_ctx *c, const dv_access *acc, uint64_t n_acc, const uint32_t *txn_begin,
                 uint32_t n_txn, const uint64_t *ts, uint8_t *out_commit, uint32_t *out_grant,
                 dv_stats *st) {
    KProfScope kps_(c);
    if (!c || !out_commit) return DV_ERR_ARG;
    // WAIT_DIE: decisions follow sequence order, which equals timestamp order
    // when ts rises with it (TS_CAS, manager.cpp:52-57, taken in sequence
    // order; a retried txn keeps its ts and is sequenced first,
    // worker_thread.cpp:478-480).  Otherwise the reference would make txns
    // wait (row_lock.cpp:119-147): not supported, rejected.  NO_WAIT and
    // CALVIN never read ts; OCC's start_ts only feeds the history check,
    // which is empty under central validation.
    if (ts && c->cfg.cc_alg == DV_WAIT_DIE)
        for (uint32_t t = 1; t < n_txn; t++)
            if (ts[t] <= ts[t - 1]) return DV_ERR_ARG;
    dv_epoch_dev ep;
    int r = stage_host_epoch(c, acc, n_acc, txn_begin, n_txn, &ep);
    if (r) return r;
    const bool calvin = c->cfg.cc_alg == DV_CALVIN;
    r = dv_epoch_run_device(c, &ep, c->d_commit, (calvin && out_grant) ? c->d_grant : nullptr, st);
    if (r) return r;
    if (n_txn)
        HIPCHK(hipMemcpyAsync(out_commit, c->d_commit, n_txn, hipMemcpyDeviceToHost, c->stream));
    if (calvin && out_grant && n_acc)
        HIPCHK(hipMemcpyAsync(out_grant, c->d_grant, n_acc * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return DV_OK;
}

// Double-buffered host input: the H2D copy of the next
// epoch's records runs on a copy stream while the current epoch decides.
}  // extern "C"

namespace {
// queue the H2D of a slot's records (bytes per record: rec) on the copy stream
int stage_slot(dv_ctx *c, int slot, const void *recs, size_t rec, uint64_t n_acc, const uint32_t *txn_begin,
               uint32_t n_txn, uint32_t max_len, bool rows) {
    HIPCHK(hipSetDevice(c->cfg.device));
    int r = alloc_host_staging(c);
    if (r) return r;
    auto &h = c->hslot[slot];
    if (!c->copy_stream) HIPCHK(hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
    if (!h.acc) {
        r = dalloc(&h.acc, c->cfg.max_acc);
        if (!r) r = dalloc(&h.tb, (uint64_t)c->cfg.max_txn + 1);
        if (!r) r = hip_fail(hipEventCreateWithFlags(&h.copied, hipEventDisableTiming), "event");
        if (!r) r = hip_fail(hipEventCreateWithFlags(&h.drained, hipEventDisableTiming), "event");
        if (r) return r;
        HIPCHK(hipEventRecord(h.drained, c->stream));
    }
    // the slot's previous epoch has been split out of it
    HIPCHK(hipStreamWaitEvent(c->copy_stream, h.drained, 0));
    if (n_acc) {
        HIPCHK(hipMemcpyAsync(h.acc, recs, n_acc * rec, hipMemcpyHostToDevice, c->copy_stream));
        if (txn_begin)
            HIPCHK(hipMemcpyAsync(h.tb, txn_begin, ((size_t)n_txn + 1) * sizeof(uint32_t), hipMemcpyHostToDevice,
                                  c->copy_stream));
    }
    HIPCHK(hipEventRecord(h.copied, c->copy_stream));
    h.n_acc = n_acc;
    h.n_txn = n_txn;
    h.max_len = max_len;
    h.csr = txn_begin != nullptr;
    h.rows = rows;
    h.full = true;
    return DV_OK;
}
}  // namespace

extern "C" {

int dv_epoch_stage_host_rows(dv_ctx *c, int slot, const uint32_t *row_wr, uint64_t n_acc,
                             const uint32_t *txn_begin, uint32_t n_txn) {
    KProfScope kps_(c);
    if (!c || slot < 0 || slot > 1 || !txn_begin) return DV_ERR_ARG;
    uint32_t max_len = 0;
    int r = check_host_epoch(c, reinterpret_cast<const dv_access *>(row_wr), n_acc, txn_begin, n_txn, &max_len);
    if (r) return r;
    return stage_slot(c, slot, row_wr, sizeof(uint32_t), n_acc, txn_begin, n_txn, max_len, true);
}

int dv_epoch_stage_host(dv_ctx *c, int slot, const dv_access *acc, uint64_t n_acc, const uint32_t *txn_begin,
                        uint32_t n_txn) {
    KProfScope kps_(c);
    if (!c || slot < 0 || slot > 1) return DV_ERR_ARG;
    uint32_t max_len = 0;
    int r = check_host_epoch(c, acc, n_acc, txn_begin, n_txn, &max_len);
    if (r) return r;
    return stage_slot(c, slot, acc, sizeof(dv_access), n_acc, txn_begin, n_txn, max_len, false);
}

int dv_epoch_run_staged(dv_ctx *c, int slot, const uint64_t *ts, uint8_t *out_commit, uint32_t *out_grant,
                        dv_stats *st) {
    KProfScope kps_(c);
    if (!c || slot < 0 || slot > 1 || !out_commit) return DV_ERR_ARG;
    auto &h = c->hslot[slot];
    if (!h.full) return DV_ERR_STATE;
    if (ts && c->cfg.cc_alg == DV_WAIT_DIE)  // as dv_epoch_run
        for (uint32_t t = 1; t < h.n_txn; t++)
            if (ts[t] <= ts[t - 1]) return DV_ERR_ARG;
    HIPCHK(hipSetDevice(c->cfg.device));
    h.full = false;
    HIPCHK(hipStreamWaitEvent(c->stream, h.copied, 0));
    dv_epoch_dev ep;
    if (h.rows) {
        launch_split_rows(c->stream, reinterpret_cast<const uint32_t *>(h.acc), h.n_acc, h.tb, h.n_txn, c->d_keys,
                          c->d_types, c->d_txn, c->d_tables);
        ep = dv_epoch_dev{};
        ep.keys = c->d_keys;
        ep.types = c->d_types;
        ep.acc_txn = c->d_txn;
        ep.tables = c->d_tables;
        ep.n_acc = h.n_acc;
        ep.n_txn = h.n_txn;
        ep.max_txn_acc = h.max_len;
    } else {
        split_records(c, h.acc, h.n_acc, h.csr ? h.tb : nullptr, h.n_txn, h.max_len, &ep);
    }
    HIPCHK(hipEventRecord(h.drained, c->stream));
    const bool calvin = c->cfg.cc_alg == DV_CALVIN;
    int r = dv_epoch_run_device(c, &ep, c->d_commit, (calvin && out_grant) ? c->d_grant : nullptr, st);
    if (r) return r;
    if (h.n_txn)
        HIPCHK(hipMemcpyAsync(out_commit, c->d_commit, h.n_txn, hipMemcpyDeviceToHost, c->stream));
    if (calvin && out_grant && h.n_acc)
        HIPCHK(hipMemcpyAsync(out_grant, c->d_grant, h.n_acc * 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return DV_OK;
}

int dv_tpcc_epoch_run(dv_ctx *c, const dv_access *acc, uint64_t n_acc, const uint32_t *txn_begin,
                      uint32_t n_txn, const uint64_t *args, uint8_t *out_commit, uint64_t *out_oid,
                      dv_stats *st) {
    KProfScope kps_(c);
    if (!out_commit || (n_acc && !args)) return DV_ERR_ARG;
    dv_epoch_dev ep;
    int r = stage_host_epoch(c, acc, n_acc, txn_begin, n_txn, &ep);
    if (r) return r;
    if (!c->d_args) {
        r = dalloc(&c->d_args, c->cfg.max_acc);
        if (!r) r = dalloc(&c->d_oid, c->cfg.max_txn);
        if (r) return r;
    }
    if (n_acc) HIPCHK(hipMemcpyAsync(c->d_args, args, n_acc * 8, hipMemcpyHostToDevice, c->stream));
    r = dv_tpcc_epoch_run_device(c, &ep, c->d_args, c->d_commit, c->d_oid, st);
    if (r) return r;
    if (n_txn) {
        HIPCHK(hipMemcpyAsync(out_commit, c->d_commit, n_txn, hipMemcpyDeviceToHost, c->stream));
        if (out_oid) HIPCHK(hipMemcpyAsync(out_oid, c->d_oid, (size_t)n_txn * 8, hipMemcpyDeviceToHost, c->stream));
    }
    HIPCHK(hipStreamSynchronize(c->stream));
    return DV_OK;
}

}  // extern "C"
