// dvcc_internal.h -- shared declarations between the epoch runtime and the
// gfx950 kernels.  Not part of the public ABI (see include/dvcc.h).
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <chrono>

#include "dvcc.h"

namespace dvcc {

// ---- per-launch kernel timing (dv_kernel_times, DV_FLAG_KERNEL_PROFILE).
// Every launch of the engine goes through DV_LAUNCH.  While the profile of
// the context a C-ABI entry works for is on, that entry points tl_kprof at it
// (this host thread only), and each launch is dispatched with its own start
// and stop timestamps (hipExtLaunchKernelGGL events: no marker packets in the
// stream); the entry reads them once its work has completed.
struct KProf;
extern thread_local KProf *tl_kprof;
// epoch graphs (dvcc_runtime.hip): while a captured epoch is replayed, the
// host walks the same enqueue code for its state with every launch skipped
extern thread_local bool tl_dry;
// DVCC_HOST_PROF (run_lanes): host time inside the launch calls themselves
extern thread_local bool tl_hprof;
extern thread_local double tl_hp_launch_s;
extern thread_local uint32_t tl_hp_launch_n;
struct HpTimer {
    bool on;
    std::chrono::steady_clock::time_point t0;
    HpTimer() : on(tl_hprof) {
        if (on) t0 = std::chrono::steady_clock::now();
    }
    ~HpTimer() {
        if (!on) return;
        tl_hp_launch_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        tl_hp_launch_n++;
    }
};
// a fresh event pair for one launch of `kernel` (both null when the pool is spent)
void kprof_events(const char *kernel, hipEvent_t *e0, hipEvent_t *e1);
// events the caller owns and records itself (the probe / scatter / pass
// timing of dv_stats): the profile reads them too
void kprof_add(const char *kernel, hipEvent_t e0, hipEvent_t e1);
// every C-ABI entry that queues work opens one: points tl_kprof at the
// context's profile while DV_FLAG_KERNEL_PROFILE is set, and when the
// outermost scope closes reads the timestamps of the launches that completed
class KProfScope {
  public:
    explicit KProfScope(dv_ctx *c);
    ~KProfScope();
    KProfScope(const KProfScope &) = delete;
    KProfScope &operator=(const KProfScope &) = delete;

  private:
    KProf *prev_, *mine_;
};
#define DV_LAUNCH(kernel, grid, block, shm, stream, ...)                                                     \
    do {                                                                                                     \
        if (::dvcc::tl_dry) break;                                                                           \
        hipEvent_t dv_e0_ = nullptr, dv_e1_ = nullptr;                                                       \
        if (::dvcc::tl_kprof) ::dvcc::kprof_events(#kernel, &dv_e0_, &dv_e1_);                              \
        ::dvcc::HpTimer dv_hp_;                                                                              \
        hipExtLaunchKernelGGL(kernel, dim3(grid), dim3(block), shm, stream, dv_e0_, dv_e1_, 0, __VA_ARGS__); \
    } while (0)
// the same with the caller's own events (may be null)
#define DV_LAUNCH_EV(kernel, grid, block, shm, stream, ev0, ev1, ...)                                        \
    do {                                                                                                     \
        if (::dvcc::tl_dry) break;                                                                           \
        hipEvent_t dv_e0_ = (ev0), dv_e1_ = (ev1);                                                           \
        if (::dvcc::tl_kprof) {                                                                              \
            if (dv_e0_ && dv_e1_) ::dvcc::kprof_add(#kernel, dv_e0_, dv_e1_);                                \
            else ::dvcc::kprof_events(#kernel, &dv_e0_, &dv_e1_);                                            \
        }                                                                                                    \
        ::dvcc::HpTimer dv_hp_;                                                                              \
        hipExtLaunchKernelGGL(kernel, dim3(grid), dim3(block), shm, stream, dv_e0_, dv_e1_, 0, __VA_ARGS__); \
    } while (0)

constexpr int kBlock = 256;           // 4 waves of 64
constexpr int kIPT = 16;              // items per thread in the radix kernels
constexpr int kTile = kBlock * kIPT;  // 4096 keys per radix workgroup
constexpr int kRadixBits = 8;
constexpr int kRadix = 1 << kRadixBits;
constexpr int kMaxTables = 8;

// per-txn decision state (one byte per txn)
enum : uint8_t { ST_UNDEC = 0, ST_COMMIT = 1, ST_ABORT = 2 };
// partition verdict bits (combined across partitions by element-wise MAX)
enum : uint8_t { V_WAIT = 1, V_ABORT = 2 };

// sort key of an access: row << 32 | txn << 8 | pos << 1 | wr
//   pos = position of the access among its txn's accesses in this partition
constexpr uint32_t kMaxTxn = 1u << 24;
constexpr uint32_t kMaxPos = 1u << 7;
constexpr uint64_t kMaxAcc = 1ull << 28;
__host__ __device__ inline uint64_t pair_pack(uint64_t row, uint32_t txn, uint32_t pos, uint32_t wr) {
    return (row << 32) | ((uint64_t)txn << 8) | ((uint64_t)pos << 1) | wr;
}
__host__ __device__ inline uint32_t pair_row(uint64_t p) { return (uint32_t)(p >> 32); }
__host__ __device__ inline uint32_t pair_txn(uint64_t p) { return (uint32_t)(p >> 8) & 0xFFFFFFu; }
__host__ __device__ inline uint32_t pair_pos(uint64_t p) { return (uint32_t)(p >> 1) & 0x7Fu; }

// row-queue element (row order): txn << 32 | id << 4 | flags
//   id: Calvin -- the access id (index into the epoch's access arrays);
//       decision rounds -- the access's position in its txn (verdict byte
//       vb8[txn << slog | pos]).
//   head: first access of a row queue; dup: repeat access of the same txn to
//   the same row; bnd: Calvin grant-group boundary; done: decision rounds --
//   the access is already OK.
constexpr uint64_t EL_WR = 1u, EL_HEAD = 2u, EL_DUP = 4u, EL_BND = 8u, EL_DONE = 8u;
__host__ __device__ inline uint32_t el_txn(uint64_t e) { return (uint32_t)(e >> 32); }
__host__ __device__ inline uint32_t el_acc(uint64_t e) { return (uint32_t)(e >> 4) & 0x0FFFFFFFu; }
__host__ __device__ inline uint32_t el_pos(uint64_t e) { return (uint32_t)(e >> 4) & (kMaxPos - 1); }
__host__ __device__ inline uint64_t el_pack(uint32_t txn, uint32_t acc, uint64_t flags) {
    return ((uint64_t)txn << 32) | ((uint64_t)acc << 4) | flags;
}
// row of an access for the txn-major execution: row | wr << 31
constexpr uint32_t AR_WR = 0x80000000u;
constexpr uint64_t kMaxRows = 0x7FFFFFFFull;

// device counters block (zeroed per epoch).  Sums that every workgroup adds
// to go to one of kSlots line-separated slots (slot = block % kSlots): one
// device-scope atomic word saturates at ~88 adds/us (MI355X_MICROARCH.md,
// "dequeue"), so 4096 blocks on one word would cost ~50 us.  The host adds
// the slots up.
constexpr int kRoundLog = 64;
#ifndef DVCC_SLOTS
#define DVCC_SLOTS 32
#endif
constexpr int kSlots = DVCC_SLOTS;
struct alignas(128) CtrSlot {
    unsigned long long read_digest;
    unsigned long long write_cnt;
    uint32_t committed;
    uint32_t undecided;   // partitioned rounds: txns still undecided after apply
};
struct Counters {
    uint32_t err;         // ERRB_* bits of every failure seen
    uint32_t peer_err;    // partitioned epochs: the input-error bits of every partition (MAX-combined)
    uint32_t halt;        // 1: the asynchronous rounds yielded undecided txns; execution waits for the
                          // synchronous rounds the host resumes (dv_epoch_finish)
    uint32_t async_go;        // the last asynchronous try: 1 ran, 2 declined, 0 nothing to do
    uint32_t async_iters;     // most iterations any asynchronous workgroup ran
    uint32_t async_r0;        // round the accepted asynchronous launch started at (0: none)
    uint32_t async_declined;  // asynchronous tries that found the live set too large
    uint32_t async_yields;    // asynchronous launches whose workgroups yielded (no more tries this epoch)
    uint32_t calvin_dups;     // CALVIN: some txn touches a row twice (k_calvin_dup_fix)
    uint32_t async_block;     // the rounds of this (sub-)epoch take no further asynchronous tries
    uint32_t a_acc;           // prefix-kill: accesses of the prefix txns
    uint32_t b_txn, b_acc;    // prefix-kill: surviving txns after the prefix, their accesses
    uint32_t a_halt;          // prefix-kill: the prefix's rounds halted (yield / decline), nothing after ran
    uint32_t a_rounds;        // prefix-kill: rounds the prefix's decisions took (k_prefix_mark)
    uint32_t async_wr0;       // an accepted asynchronous launch from this round left its statuses in the
                              // fact words, no finalize (a prefix-kill stage: k_prefix_mark /
                              // k_sub_scatter_back read them)
    uint32_t n_acc;           // the accesses the probe read (the real count of a device-built epoch)
    unsigned long long pass_live;  // live accesses every k_round_pass of the epoch read, summed
    unsigned long long async_live; // live accesses entering every asynchronous launch that ran, summed
    uint32_t spin_site;       // with ERRB_SPIN: 1 look-back, 2 asynchronous rounds, 3 tail (max seen)
    uint32_t async_done;      // workgroups of the asynchronous launch that finished (its last one finalizes;
                              // reset by it)
    uint32_t nlive[2];    // live accesses of the current / next decision round
    uint32_t nund[2];     // undecided-txn list lengths (single-GPU settle)
    uint32_t log_live[kRoundLog];  // per round: live accesses entering it
    uint32_t log_und[kRoundLog];   // per round: undecided txns before it
    CtrSlot slot[kSlots];
};
__device__ inline CtrSlot &my_slot(Counters *ctr) { return ctr->slot[blockIdx.x & (kSlots - 1)]; }

struct IxEntry {
    uint64_t key;
    uint64_t row;
};

struct TableDesc {
    // Direct maps whose bucket b holds local row b (the YCSB loader, and
    // dv_load_table when the keys arrive in bucket order) keep no entry array:
    // slot b's key is that row's primary key, so a probe reads 8 bytes of the
    // pkey column instead of a 16-byte {key, row} entry (config D: a 134 MB
    // probe target instead of 268 MB).
    const uint64_t *pkey;     // implicit-row direct map: pkey of local rows [0, nbuckets)
    // ... and its key tags (key_tag below), one byte per row: the probe reads
    // the tag, and the pkey word only behind the kTagWide sentinel
    const uint8_t *ktag;
    // ... and one bit per row of "the tag is htag", the tag almost every row
    // of a partition's table carries (YCSB: q = 0, the partition id): a probe
    // whose key has that tag reads the bit (config D: a 2 MB target that stays
    // in L2) instead of the byte; nullptr = no such bitmap
    const uint32_t *hbits;
    uint32_t htag;
    // ... and for a dense map (dv_load_ycsb_partition: bucket b holds the key
    // of tag htag, for every b) the key set is known: a key is there iff its
    // tag is htag -- no gather at all (ycsb_wl.cpp:173-186 loads every key)
    uint32_t dense;
    const IxEntry *ix;        // index entries (direct: [nbuckets]; chained: sorted by bucket)
    const uint32_t *bstart;   // chained: [nbuckets+1] bucket starts; nullptr = direct map
    uint64_t nbuckets;
    uint64_t row_base;        // global row id of local row 0
    uint32_t hash_kind;       // DV_HASH_*
    uint32_t part_cnt;
    uint64_t m_part, m_nb;    // div_magic of part_cnt / nbuckets (key_split)
    // replicated epochs (dv_epoch_run_part, "replicated sequencing"): every
    // partition's keys probe here -- rep_part is this context's partition, its
    // own keys are checked against the local direct map, the others are
    // range-checked only (their owner checks them), and every key's row is the
    // key itself (the global row space); kNoRep otherwise
    uint32_t rep_part;
};
constexpr uint32_t kNoRep = 0xFFFFFFFFu;

// replicated epochs: a global row (= key) -> this partition's local row, or
// false for another partition's row (execution touches own rows only)
struct RowMap {
    uint32_t P = 0, part = 0;  // P == 0: rows are local already
};
__device__ __forceinline__ bool own_row(const RowMap &m, uint64_t &row) {
    if (m.P == 0) return true;
    if (row % m.P != m.part) return false;
    row /= m.P;
    return true;
}

// Key tag of an implicit-row direct map.  A bucket's keys differ only in
// what the bucket function drops: with DV_HASH_YCSB, b = (k / P) % nb, a key
// is (q, b, lo) with q = k / P / nb and lo = k % P; with DV_HASH_MOD,
// b = k % nb, it is (q, b).  So q * P + lo (P = 1 for MOD) names the key
// within its bucket exactly; a loaded row stores it in one byte when it is
// below kTagWide (YCSB's loader: q = 0, the tag is the partition id), else
// kTagWide, and a probe compares tags -- equal tags below kTagWide mean equal
// keys, unequal ones a missing key -- reading the 8-byte pkey only for
// kTagWide.  Config D's probe target shrinks from 134 MB to 16.8 MB.
constexpr uint32_t kTagWide = 255;
__host__ __device__ inline uint8_t key_tag(uint32_t hash_kind, uint64_t nbuckets, uint32_t part_cnt, uint64_t key) {
    const uint64_t P = hash_kind == DV_HASH_YCSB ? part_cnt : 1u;
    const uint64_t q = key / P / nbuckets;
    if (q >= kTagWide) return (uint8_t)kTagWide;
    const uint64_t code = q * P + key % P;
    return (uint8_t)(code < kTagWide ? code : kTagWide);
}
// n / d and n % d for every 64-bit n without a division: m = div_magic(d) =
// floor((2^64 - 1) / d) puts mulhi(n, m) within 2 below the quotient
__host__ __device__ inline uint64_t div_magic(uint64_t d) { return d ? ~0ull / d : 0ull; }
__device__ __forceinline__ uint64_t divmod_magic(uint64_t n, uint64_t d, uint64_t m, uint64_t &r) {
    uint64_t q = __umul64hi(n, m);
    r = n - q * d;
    if (r >= d) { q++; r -= d; }
    if (r >= d) { q++; r -= d; }
    return q;
}
// the bucket of `key` and its key tag (key_tag) in one pass
__device__ __forceinline__ uint64_t key_split(const TableDesc &t, uint64_t key, uint32_t &tag) {
    uint64_t lo = 0, bk = 0, q;
    if (t.hash_kind == DV_HASH_YCSB) {
        const uint64_t q1 = divmod_magic(key, t.part_cnt, t.m_part, lo);
        q = divmod_magic(q1, t.nbuckets, t.m_nb, bk);
        const uint64_t code = q * t.part_cnt + lo;
        tag = q >= kTagWide || code >= kTagWide ? kTagWide : (uint32_t)code;
    } else {
        q = divmod_magic(key, t.nbuckets, t.m_nb, bk);
        tag = q >= kTagWide ? kTagWide : (uint32_t)q;
    }
    return bk;
}
// implicit-row direct map: does bucket bk hold the key of tag `tag`?
__device__ inline bool direct_holds(const TableDesc &t, uint64_t bk, uint32_t tag, uint64_t key) {
    if (t.dense) return tag == t.htag;
    if (t.hbits != nullptr && tag == t.htag) return (t.hbits[bk >> 5] >> (bk & 31)) & 1u;
    const uint32_t tg = t.ktag[bk];
    return tg != kTagWide ? tg == tag : t.pkey[bk] == key;
}

struct Tables {
    TableDesc t[kMaxTables];
    uint32_t n;
};

// error bits recorded by kernels
enum : uint32_t {
    ERRB_KEY = 1, ERRB_DUP = 2, ERRB_TXN = 4, ERRB_TABLE = 8, ERRB_SPIN = 16, ERRB_BIG = 32,
    ERRB_TS = 64  // WAIT_DIE timestamps that do not rise strictly in sequence order
};
// errors in the epoch's input, all found by the probe (or the host-record
// check before it): once one is set -- on this partition or, for partitioned
// epochs, on any (Counters::peer_err) -- the decision rounds are no-ops and
// no execution kernel touches the tables, so a rejected epoch leaves them as
// they were
constexpr uint32_t ERRB_INPUT = ERRB_KEY | ERRB_DUP | ERRB_TXN | ERRB_TABLE | ERRB_BIG | ERRB_TS;
__device__ __forceinline__ uint32_t input_err(const Counters *ctr) {
    return (ctr->err | ctr->peer_err) & ERRB_INPUT;
}
// the return code of an epoch whose counters hold error bits b (the host's
// epoch finish, and the epoch groups' outcome record on the device)
__host__ __device__ inline int err_code_of(uint32_t b) {
    if (b & ERRB_TABLE) return DV_ERR_NO_TABLE;
    if (b & ERRB_KEY) return DV_ERR_KEY_NOT_FOUND;
    if (b & ERRB_TXN) return DV_ERR_TXN_RANGE;
    if (b & (ERRB_BIG | ERRB_TS)) return DV_ERR_ARG;  // a txn longer than max_txn_acc; WAIT_DIE ts not rising
    if (b & ERRB_DUP) return DV_ERR_DUP_ROW;
    if (b & ERRB_SPIN) return DV_ERR_HIP;
    return DV_OK;
}

// ---- probe / queues (dvcc_kernels.hip)
// counts (optional): the first radix pass's per-tile digit counts (k_radix_hist
// layout); worth it from kProbeHistTiles sort tiles up (below that a block per
// tile leaves CUs idle)
constexpr uint32_t kProbeHistTiles = 1024;
// pairs: sort keys; tb_start/tb_end: each txn's access range; tlen (optional):
// its access count; acc_row (optional): row | wr << 31 per access.  An access
// at position >= 1 << slog in its txn is an error (ERRB_BIG).  pair_limit <
// n_txn: sort keys only for txns < pair_limit (the epoch's first accesses),
// their count stored in ctr->a_acc (prefix-kill epochs).
void launch_probe(hipStream_t s, const Tables &tabs, const uint64_t *keys, const uint8_t *types,
                  const uint32_t *acc_txn, const uint8_t *tables, uint64_t n_acc, uint32_t n_txn,
                  uint32_t slog, uint64_t *pairs, uint32_t *tb_start, uint32_t *tb_end,
                  uint8_t *tlen, uint32_t *acc_row, Counters *ctr, uint32_t *counts, uint32_t pair_limit,
                  hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr, const uint32_t *keys32 = nullptr,
                  const uint64_t *ts = nullptr, const uint32_t *n_dev = nullptr,
                  const uint64_t *rsv_cols = nullptr);  // (TPC-C: last names resolved, tpcc_last_name_key)

// prefix-kill epochs with their txn boundaries (dv_epoch_dev::txn_begin):
// every txn's range checked, the prefix's txns [0, K) probed (acc_row, tlen,
// sort keys; ctr->a_acc = txn_begin[K]); the later accesses are probed by
// k_kill (launch_kill_compact with keys)
void launch_probe_tb(hipStream_t s, const Tables &tabs, const uint64_t *keys, const uint8_t *types,
                     const uint32_t *recs, const uint32_t *txn_begin, uint64_t n_acc, uint32_t n_txn, uint32_t K,
                     uint32_t slog, uint64_t *pairs, uint8_t *tlen, uint32_t *acc_row, Counters *ctr,
                     const uint64_t *ts, hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr, const uint32_t *n_acc_dev = nullptr);

// stable LSD radix sort of pairs on bits [32, 32 + key_bits); returns the index
// (0/1) of the buffer holding the result.  counts: >= kRadix * nblocks(n),
// digit_tot: kRadix.  scatter_ev (optional): 2 events per pass for timing.
// n_dev (optional): the real count on the device, n an upper bound.
// digit width of radix_sort_rows: 8 bits, or 9-10 when that saves a pass
// (never when the probe counted the first 8-bit histogram)
constexpr int kRadixMaxBits = 10;
constexpr int kRadixMax = 1 << kRadixMaxBits;  // counts: kRadixMax x sort tiles, digit_tot: kRadixMax
inline int radix_digit_bits(int key_bits, bool hist0_done) {
    const int p8 = (key_bits + kRadixBits - 1) / kRadixBits;
    if (hist0_done || p8 < 2) return kRadixBits;
    const int w = (key_bits + p8 - 2) / (p8 - 1);  // one pass fewer
    return w <= kRadixMaxBits ? w : kRadixBits;
}
inline int radix_passes(int key_bits, bool hist0_done) {
    const int w = radix_digit_bits(key_bits, hist0_done);
    return (key_bits + w - 1) / w;
}
// Small sorts (a prefix-kill stage, a TPC-C or Calvin epoch: at most
// kBucketMaxN keys, or a count on the device) take ONE stable pass on the top
// kBucketLoBits(key_bits) bits of a hash of the row, h = row * kRowHashMul mod
// 2^key_bits (a bijection), and then sort every bucket by h's remaining bits
// inside one workgroup (k_bucket_sort: a 14-bit local index beside them in a
// 32-bit LDS tag, so at most kBucketHiMax of them) -- 4 launches instead of 9
// for 24-bit rows.  The order is the row queues' (rows grouped, each queue in
// sequence order), rows ordered by h: nothing on the path needs rows in
// ascending order.
constexpr int kBucketHiMax = 18;
constexpr uint32_t kRowHashMul = 0x9E3779B1u;  // odd: x -> x * mul mod 2^b is a bijection
constexpr uint64_t kBucketMaxN = 2u << 20;
inline int kBucketLoBits(int key_bits) { return key_bits - kBucketHiMax > kRadixBits ? key_bits - kBucketHiMax : kRadixBits; }
inline bool bucket_sort_applies(uint64_t n, int key_bits, bool hist0_done, bool n_on_dev) {
    return key_bits > kRadixBits && key_bits <= kRadixMaxBits + kBucketHiMax && !hist0_done &&
           (n_on_dev || n <= kBucketMaxN);
}
// lsd_only: the plain LSD passes whatever the size (DV_FLAG_LSD_SORT)
int radix_sort_rows(hipStream_t s, uint64_t *pairs[2], uint64_t n, int key_bits, uint32_t *counts,
                    uint32_t *digit_tot, hipEvent_t *scatter_ev, bool hist0_done, const uint32_t *n_dev,
                    bool lsd_only = false);

void launch_seg_prepare(hipStream_t s, const uint64_t *pairs, uint64_t n, int calvin,
                        const uint32_t *tb_start, uint64_t *el, Counters *ctr);

// Calvin grant groups: one single-pass segmented scan over the row queues
void calvin_grant(hipStream_t s, const uint64_t *el, uint64_t n, uint32_t *grant_out, uint8_t *ew,
                  uint64_t *desc, uint32_t *tile_ctr, uint32_t tag, Counters *ctr);

// decision rounds (dvcc_rounds.hip): vb8 = per-access verdict (1 = permanently
// OK, 2 = aborts its txn) at vb8[txn << slog | pos]; tlen[txn] = the txn's
// accesses on this partition.
constexpr uint32_t kTileCtrs = 1024;  // tile tickets, reset every kTileCtrs passes
struct RoundBufs {
    const uint64_t *pairs0;  // round-0 input: the row-sorted pairs
    void *rel[2];            // live elements (32- or 64-bit), ping-pong
    bool el32;               // 32-bit round elements (round_el32)
    uint8_t *vb8;            // per access, txn-strided
    uint32_t slog;           // log2 of the per-txn stride of vb8
    uint8_t *status;         // per txn
    const uint8_t *tlen;     // per txn
    uint32_t *ulist[2];      // undecided txns, ping-pong (single-GPU settle)
    const uint32_t *n_txn_dev;  // (optional) the real txn count, n_txn an upper bound (sub-epochs)
    // round 0's sizes (set per (sub-)epoch by the runtime): live accesses (n0_dev on the device,
    // else n0) and txns (n_txn_dev, else n_txn0)
    const uint32_t *n0_dev;
    uint32_t n0, n_txn0;
    uint64_t *desc;
    uint32_t *tile_ctr;
    Counters *ctr;
};
// Host-mapped progress record: the pass of round r (r >= 1) publishes the
// outcome of round r - 1 so the host can follow the rounds without
// synchronising the stream.  Each word is one 64-bit store, so round and
// undecided count are always consistent; nlive may lag (still an upper bound).
struct RoundPub {
    unsigned long long ru;  // rounds settled << 32 | undecided txns
    unsigned long long le;  // live accesses << 32 | error bits
    unsigned long long tl;  // r0 << 32 | code: the tail launched at round r0 but the
                            // live set did not fit (1; the rounds resume from r0);
                            // the asynchronous try at r0 declined (2), yielded
                            // (3) -- both halt execution until the host resumes
                            // the rounds -- decided the rest (4), or found
                            // nothing left to decide (5)
    // partitioned rounds: undecided txns after round r, at [r % kPubLog]
    // (written before ru publishes r + 1), so every rank reads the count of
    // the same round however far its stream has run ahead
    static constexpr uint32_t kPubLog = 64;
    unsigned int und_log[kPubLog];
    unsigned long long ai;  // iterations of the last asynchronous launch that ran (r0 << 32 | iters)
};
// the rounds of one (sub-)epoch begin: round 0's counts (n_acc_dev /
// b.n_txn_dev, when given, hold the real ones), its verdict bytes cleared, the
// asynchronous-try state reset
// round 0 needs no launch of its own: its pass reads the sizes (RoundBufs n0*)
// and resets the round counters, and writes every access's verdict byte
// settle = single GPU (the following settle compacts the undecided list; a
// pass whose round starts with no undecided txn is a no-op)
// ev0/ev1 (optional): recorded by the pass's own dispatch (hipExtLaunchKernel)
void round_pass(hipStream_t s, const RoundBufs &b, uint32_t round, int nowait, uint32_t ub_in,
                uint32_t tag, uint32_t ticket, bool settle, RoundPub *pub, hipEvent_t ev0,
                hipEvent_t ev1);
// single GPU: settle statuses from the verdicts, walking the undecided-txn
// list (ub = upper bound of its length)
// tword / carry / G: round 0 with an asynchronous launch at round 1 behind it
// (round_async with words_done): the settle writes its fact and carry words
void round_settle(hipStream_t s, const RoundBufs &b, uint32_t round, uint32_t n_txn, uint32_t ub,
                  uint32_t *tword = nullptr, uint32_t *carry = nullptr, uint32_t G = 0);
// partitioned: this partition's verdict byte (bit1 abort, bit0 wait) for every
// entry of round `round`'s undecided list, in list order (ub: bound of the
// list length); then apply the MAX-combined bytes, compact the list for the
// next round (same order on every rank) and publish (round + 1, its length)
void list_verdict(hipStream_t s, const RoundBufs &b, uint32_t round, uint32_t ub, uint8_t *verdict);
void list_apply(hipStream_t s, const RoundBufs &b, uint32_t round, uint32_t ub, const uint8_t *verdict,
                uint32_t tag, uint32_t *tile_ctr, RoundPub *pub);
// single GPU: all remaining rounds from round r0 >= 1 in one single-workgroup
// launch; publishes the final round and 0 undecided (0xFFFFFFFF on failure)
// through pub, or declines (pub->tl) and does nothing when the live accesses
// or undecided txns entering round r0 exceed tail_cap()
constexpr int kTailThreads = 1024;
void round_tail(hipStream_t s, const RoundBufs &b, uint32_t r0, int nowait, RoundPub *pub);
uint32_t tail_cap(bool el32);  // live accesses the tail holds in LDS
// single GPU, 32-bit elements: every remaining decision from round r0 >= 1 in
// one multi-workgroup launch without grid barriers, then the status bytes of
// every txn (undecided leftovers -- an error -- counted in the slots'
// `undecided`); carry: kAsyncGroups words of scratch.  The launch is a try,
// decided on the device: it runs when some txn is undecided, no earlier try
// ran, and the live accesses entering round r0 are at most `thresh` (and fit
// its workgroups, async_try_limit()); then it zeroes round r0's undecided
// count, so the passes queued behind it are no-ops that publish "0
// undecided".  A try that finds the live set too large changes nothing and
// publishes pub->tl = r0 << 32 | 2 (declined); the rounds go on.
constexpr uint32_t kAsyncGroups = 512;
// tword: one 32-bit fact word per txn (scratch, n_txn words).  A workgroup
// yields after max_iters iterations or idle_ticks wall-clock ticks without a
// decision; if any did, the finalize sets Counters::halt and publishes
// pub->tl = r0 << 32 | 3 instead of closing the rounds (the host resumes them).
// words: no finalize -- the statuses stay in tword for the stage's consumer
// (k_prefix_mark, k_sub_scatter_back), which also checks nothing is left
// undecided; the launch does the finalize's yield / decline bookkeeping
void round_async(hipStream_t s, const RoundBufs &b, uint32_t r0, int nowait, uint32_t G, uint32_t thresh,
                 uint32_t *carry, uint32_t *tword, uint32_t n_txn, RoundPub *pub, uint32_t max_iters,
                 uint64_t idle_ticks, bool words_done = false, bool words = false);
uint32_t async_groups(int device);  // co-resident workgroups (<= kAsyncGroups; 0: unusable)
// a txn's fact word (status | OK accesses << 8 | accesses << 16) -> its status
__device__ __forceinline__ uint8_t word_status(uint32_t w) {
    const uint32_t s = w & 0xFFu;
    if (s != ST_UNDEC) return (uint8_t)s;
    return ((w >> 8) & 0xFFu) == (w >> 16) ? (uint8_t)ST_COMMIT : (uint8_t)ST_UNDEC;
}
uint32_t async_try_limit(uint32_t G);
// round elements ((txn << slog | pos) << 3 | flags) fit 32 bits
bool round_el32(uint32_t n_txn, uint32_t slog);

// ---- epoch groups (dvcc_comm.hip run_group): the deciding rank routes its
// epoch's committed accesses to their owners instead of executing them.  A
// record is {local row | wr << 31 | "sees an earlier write" << 30, global
// txn}; owner = global row % P, local row = global row / P (YCSB, key % P).
// Records of one owner are contiguous (owner-major, offsets from per-block
// counts); their order inside an owner's segment is free, since one epoch's
// execution on a row does not depend on it (2PL: a written row has one
// committed txn; OCC and Calvin: reads run before writes and carry what they
// see).
constexpr uint32_t kRouteBlocks = 1024;  // (a multiple of kBlock: k_route_scan)
constexpr uint32_t RT_WR = 0x80000000u, RT_SEESW = 0x40000000u;
struct RouteOut {
    uint2 *rec;     // records, owner-major
    uint32_t *blk;  // [P][kRouteBlocks] records per owner per block (then their exclusive prefix)
    uint32_t *tot;  // [P] records per owner
    uint32_t P;
    // the epoch group's outcome record (step 4 of run_group), written by the
    // owner scan when the txn walk routes (null: the host launches
    // k_route_words); *wrote (host) is set when that scan was queued
    uint64_t *orec = nullptr;
    const uint32_t *bad = nullptr;         // a refused batch: the group fails as DV_ERR_ARG
    unsigned long long *xacc = nullptr;    // the execution's digest slots, zeroed for step 6
    uint64_t cap = 0;                      // receive capacity
    const Counters *ctr = nullptr;         // committed count: the slots' sum
    bool *wrote = nullptr;
    bool defer = false;                    // the decider's counter read waits for the outcome vote
};
// NO_WAIT / WAIT_DIE / OCC: the committed txns' accesses (txn-major acc_row),
// and the commit bytes and count in the same pass (k_commit_out's work)
void launch_route_txn(hipStream_t s, const RouteOut &ro, const uint32_t *tb_start, const uint32_t *tb_end,
                      const uint32_t *acc_row, uint32_t n_txn, const uint8_t *status, Counters *ctr,
                      uint8_t *d_commit);
// CALVIN: every access, in row order (sorted pairs, queue elements, "an
// earlier write precedes" flags)
void launch_route_rowq(hipStream_t s, const RouteOut &ro, const uint64_t *pairs, const uint64_t *el,
                       const uint8_t *ew, uint64_t n, const uint8_t *status, Counters *ctr);

// ---- runtime accessors for the RCCL driver (dvcc_comm.hip)
struct DvComm;  // defined in dvcc_comm.hip
}  // namespace dvcc
dvcc::DvComm *&ctx_comm(dv_ctx *c);
hipStream_t ctx_stream(dv_ctx *c);
const dv_config &ctx_config(dv_ctx *c);
bool ctx_has_tables(dv_ctx *c);  // some table is loaded (dv_epoch_begin's precondition)
// replicated epochs (dvcc_comm.hip run_part): table 0 is a loaded YCSB
// implicit-row map whose global row space (nranks x buckets) fits 31 bits
bool ctx_rep_capable(dv_ctx *c, uint32_t nranks);
// epoch groups: ... and the map is dense (dv_load_ycsb_partition: every key
// b * nranks + rank below the row space exists), so a range check is the
// owner's key check
bool ctx_group_capable(dv_ctx *c, uint32_t nranks);
void ctx_table0_cols(dv_ctx *c, uint64_t **f0, const uint64_t **pkey);  // table 0's local rows
uint64_t ctx_table0_rows(dv_ctx *c);  // ... their count (buckets of its direct map)
uint32_t *ctx_err_words(dv_ctx *c);  // &Counters::err (peer_err follows)
const dvcc::Counters *ctx_counters(dv_ctx *c);
// ordered lanes (dv_lanes_order): an execution of an epoch group on lane c
// waits for its turn -- the previous group's execution, on whichever lane,
// queued (host) and finished (its event, device) -- and hands the turn on
// after it is queued; a lane whose group failed ends the order there (every
// later group returns DV_ERR_STATE instead of waiting; earlier ones still
// execute).  No-ops on a context without an order.
int lane_exec_begin(dv_ctx *c, hipStream_t s);
void lane_exec_end(dv_ctx *c, hipStream_t s);
void lane_fail(dv_ctx *c);
// the whole epoch on this rank, its own rows executed (dvcc_runtime.hip)
// keys32: the epoch's keys as 32-bit row ids (ep->keys is then ignored)
// route (epoch groups): committed accesses routed to their owners, nothing
// executes here
// an epoch group's decider epoch (32-bit rows as recs32, txn_begin) takes the
// tb mode of run_prefix_epoch: its per-access txn ids are then never read
bool group_tb_epoch(const dv_ctx *c, const dv_epoch_dev *ep);
int epoch_run_replicated(dv_ctx *c, const dv_epoch_dev *ep, const uint32_t *keys32, uint32_t nranks,
                         uint8_t *d_commit, dv_stats *st, const dvcc::RouteOut *route = nullptr);
// RouteOut::defer: epoch_run_replicated returned with its counters still on
// the way (ctx_finish_pending); this reads them and finishes the decision
// (a halted one is finished and routed again)
int epoch_replicated_complete(dv_ctx *c, dv_stats *st);
bool ctx_finish_pending(dv_ctx *c);
int comm_combine_errors(dv_ctx *c);  // dvcc_comm.hip
void comm_free(dvcc::DvComm *m);
namespace dvcc {

// abort carry-over (dvcc_carry.hip): the accesses of the txns whose status is
// not committed, in sequence order and renumbered from 0, capped at max_txn
// txns, into o*; tot (3 words, device) = carried txns, their accesses, and the
// carried txns before the cap.  bt/ba: carry_blocks(n_txn) words each.
uint32_t carry_blocks(uint32_t n_txn);
void launch_carry(hipStream_t s, const uint8_t *status, const uint32_t *tb_start, const uint32_t *tb_end,
                  uint32_t n_txn, uint32_t max_txn, const uint64_t *keys, const uint8_t *types,
                  const uint8_t *tables, uint64_t *okeys, uint8_t *otypes, uint32_t *otxn,
                  uint8_t *otables, uint32_t *bt, uint32_t *ba, uint32_t *tot);

// per-txn access ranges of a batch from its acc_txn (dv_epoch_group_carry)
void launch_txn_ranges(hipStream_t s, const uint32_t *acc_txn, uint64_t n, uint32_t n_txn, uint32_t *tbs,
                       uint32_t *tbe);

// the closed loop (dv_epoch_refill): the aborted txns of the decided epoch
// (status, access ranges, its keys / types / tables) carried first, capped
// at n_out, then n_out - C fresh txns of the pool (pkeys ... ptb, pool_n txns)
// from *cursor on (advanced, wrapping), into o*; *n_acc_dev = the accesses
// written.  fresh_bound: a bound on the fresh accesses (grid size).  A halted
// or rejected epoch (Counters; NULL for the loop's first epoch, n_txn 0) makes
// every kernel a no-op.  tot: kRefillTot words.  tb form (orecs, otb): the
// next epoch as 4-byte records (recs: the previous epoch's, precs: the
// pool's) and its txn boundaries otb[0..n_out]; okeys NULL: only that form
// (o{keys,types,txn,tables} are not written).
constexpr uint32_t kRefillTot = 6;
void launch_refill(hipStream_t s, const uint8_t *status, const uint32_t *tb_start, const uint32_t *tb_end,
                   uint32_t n_txn, const uint64_t *keys, const uint8_t *types, const uint8_t *tables,
                   const uint64_t *pkeys, const uint8_t *ptypes, const uint8_t *ptables, const uint32_t *ptxn,
                   const uint32_t *ptb, uint32_t pool_n, uint32_t *cursor, uint32_t n_out, uint64_t fresh_bound,
                   uint64_t *okeys, uint8_t *otypes, uint32_t *otxn, uint8_t *otables, uint32_t *n_acc_dev,
                   uint32_t *bt, uint32_t *ba, uint32_t *tot, const Counters *ctr, const uint32_t *recs = nullptr,
                   const uint32_t *precs = nullptr, uint32_t *orecs = nullptr, uint32_t *otb = nullptr);

// ---- prefix-kill epochs (dvcc_prefix.hip)
// the row-state bitmap (2 bits per row): its 32-bit words for `rows` rows;
// launch_prefix_mark clears it and marks the committed prefix txns' rows
uint64_t row_state_words(uint64_t rows);
// words (the prefix's asynchronous launch left its statuses there, no
// finalize): the prefix's statuses are read from its fact words and written
// to status
void launch_prefix_mark(hipStream_t s, uint8_t *status, const uint32_t *tb_start, const uint32_t *tb_end,
                        const uint32_t *acc_row, uint32_t K, uint32_t *row_state, uint64_t rs_words, int nowait,
                        Counters *ctr, const uint32_t *words);
uint32_t kill_tiles(uint32_t n_after);  // look-back tiles of k_kill_compact (descriptors per array)
// k_kill (every access after the prefix's against the row state, one bit
// per access into kill_bits[kill_words(n_acc)]; NO_WAIT / WAIT_DIE, skip_bits
// non-null: one more per access, a read of a row only read by the prefix's
// commits, which the survivors' sub-epoch leaves out) and k_kill_count /
// k_kill_emit (killed txns aborted, the survivors' sub-epoch)
uint64_t kill_words(uint64_t n_acc);
// kk (an epoch with its txn boundaries, launch_probe_tb): the accesses after
// the prefix were not probed -- k_kill probes their keys itself (a missing key:
// ERRB_KEY, the epoch rejected) and k_kill_emit the survivors' (their acc_row
// words, for the execution, and their sort keys)
struct KillKeys {
    Tables tabs;
    const uint64_t *keys;
    const uint8_t *types;
    const uint32_t *recs;  // (optional) the same as 4-byte records, key | write << 31 (dv_epoch_dev::recs32)
    // table 0 a dense map (dv_load_ycsb_partition; every partition's, for a
    // replicated epoch): a key is there iff key < dense_lim, its row key +
    // dense_base -- the kill and emit passes then instantiate only that
    // compare (kk_row), not the general probe; 0 = probe
    uint64_t dense_lim, dense_base;
};
inline KillKeys kill_keys(const Tables &t, const uint64_t *keys, const uint8_t *types, const uint32_t *recs) {
    KillKeys k{t, keys, types, recs, 0, 0};
    if (t.n == 0) return k;
    const TableDesc &d = t.t[0];
    if (d.rep_part != kNoRep) {  // (probe_row's replicated dense branch)
        if (d.dense && d.htag == d.rep_part) k.dense_lim = d.nbuckets * d.part_cnt;
    } else if (d.dense && d.part_cnt == 1 && d.htag == 0) {  // (its one-partition dense branch)
        k.dense_lim = d.nbuckets;
        k.dense_base = d.row_base;
    }
    return k;
}
// access a of a KillKeys epoch: its key and write bit
__device__ __forceinline__ uint64_t kk_key(const KillKeys &kk, uint64_t a, uint32_t &wr) {
    if (kk.recs) {
        const uint32_t r = kk.recs[a];
        wr = r >> 31;
        return r & 0x7FFFFFFFu;
    }
    wr = kk.types[a] == DV_WR ? 1u : 0u;
    return kk.keys[a];
}
// (n_acc_dev: the epoch's real access count when n_acc is a bound, else null)
void launch_kill_compact(hipStream_t s, const uint32_t *tb_start, const uint32_t *tb_end, const uint32_t *acc_row,
                         uint64_t n_acc, const uint32_t *n_acc_dev, uint32_t K, uint32_t n_txn,
                         const uint32_t *row_state, uint64_t rs_words,
                         int nowait,
                         uint64_t *kill_bits, uint64_t *skip_bits, uint8_t *status, uint32_t *map,
                         uint8_t *status_b, uint8_t *tlen_b, uint64_t *pairs_b, uint32_t *info, uint32_t *tsum,
                         Counters *ctr, const KillKeys *kk = nullptr);
// (info: one word per txn after the prefix; tsum: 2 x kill_tiles words)
// words (the survivors' asynchronous launch left their statuses there): their
// statuses from the fact words, else from status_b
void launch_sub_scatter_back(hipStream_t s, const uint32_t *map, const uint8_t *status_b, uint32_t ub,
                             uint8_t *status, Counters *ctr, const uint32_t *words);

// per-epoch reset: counters (err = *err_seed when given), tile tickets,
// status (value; padding aborted), access ranges and counts; with hctr, the
// counters as they stand first go to that host mirror and *hseq = seq (the
// previous pipelined epoch's read-back, launch_ctr_out folded in)
void launch_epoch_clear(hipStream_t s, uint8_t *status, uint32_t n_txn, uint32_t n_txn_pad4, uint8_t value,
                        uint32_t *tb_start, uint32_t *tb_end, uint8_t *tlen, uint32_t *tile_ctr,
                        const uint32_t *err_seed, Counters *ctr, uint32_t *zero = nullptr,
                        uint64_t zero_words = 0, bool gate = false, Counters *hctr = nullptr,
                        unsigned long long *hseq = nullptr, unsigned long long seq = 0,
                        uint64_t *txn_zero8 = nullptr,  // (one 8-byte word per txn zeroed: TPC-C o_ids)
                        uint64_t *desc = nullptr, uint32_t n_desc = 0);  // (descriptors zeroed: epoch graphs)
// the counters into their host-mapped mirror hctr, then *hseq = seq (device
// pointers of host-mapped memory)
void launch_ctr_out(hipStream_t s, const Counters *ctr, Counters *hctr, unsigned long long *hseq,
                    unsigned long long seq);
// decision lanes (dv_epoch_run_device_lanes): before an epoch's execution,
// wait until *done >> 1 reaches this lane's *turn (halt if the gate bit is
// set, or after 1 s without it); after it, *done = (turn + 1) << 1 | (it
// halted or failed) and *turn += n_lanes
void launch_lane_post(hipStream_t s, uint32_t *turn, uint32_t *done, uint32_t n_lanes, const Counters *ctr);
void launch_lane_wait(hipStream_t s, const uint32_t *turn, const uint32_t *done, Counters *ctr);
// Calvin: in row order over the sorted queues
void launch_exec(hipStream_t s, const uint64_t *pairs, const uint64_t *el, const uint8_t *ew,
                 uint64_t n, const uint8_t *status, uint64_t *f0, const uint64_t *pkey,
                 Counters *ctr, RowMap rm = RowMap{});
// NO_WAIT / WAIT_DIE / OCC: in txn order over the committed txns, with the
// commit bytes into d_commit (may be NULL) and the committed count, as
// launch_commit_out would.  pk_dense: the rows are a dense one-partition YCSB
// map whose row r holds key r - pk_base (k_ycsb_load), so a read's primary
// key comes from its row instead of a second random line of the pkey column
void launch_exec_txn(hipStream_t s, const uint32_t *tb_start, const uint32_t *tb_end,
                     const uint32_t *acc_row, uint32_t n_txn, const uint8_t *status, uint64_t *f0,
                     const uint64_t *pkey, bool fused, Counters *ctr, RowMap rm, uint8_t *d_commit,
                     bool pk_dense = false, uint64_t pk_base = 0);
void launch_commit_out(hipStream_t s, const uint8_t *status, uint32_t n_txn, uint8_t *d_commit,
                       Counters *ctr);
void launch_ycsb_load(hipStream_t s, uint64_t rows, uint32_t part_cnt, uint32_t part_id,
                      uint64_t *f0, uint64_t *pkey, uint8_t *ktag);
// bits[w] bit j = (ktag[32 w + j] == htag), rows [0, n)
void launch_home_bits(hipStream_t s, const uint8_t *ktag, uint64_t n, uint32_t htag, uint32_t *bits);
// (f0[row * cstride]: TPC-C contexts keep their three state columns row-major)
void launch_gather_rows(hipStream_t s, const Tables &tabs, uint32_t table, const uint64_t *keys,
                        uint64_t n, const uint64_t *f0, uint32_t cstride, uint64_t *out, Counters *ctr);
// 4-byte row records (row | write << 31) + CSR txn_begin -> the epoch's arrays (table 0)
void launch_split_rows(hipStream_t s, const uint32_t *rw, uint64_t n, const uint32_t *tb, uint32_t n_txn,
                       uint64_t *keys, uint8_t *types, uint32_t *acc_txn, uint8_t *tables);
void launch_split_access(hipStream_t s, const dv_access *acc, uint64_t n, const uint32_t *tb, uint32_t n_txn,
                         uint64_t *keys, uint8_t *types, uint32_t *acc_txn, uint8_t *tables, uint32_t *err);

__host__ __device__ inline uint32_t nblocks_for(uint64_t n) { return (uint32_t)((n + kTile - 1) / kTile); }

}  // namespace dvcc
