// dvcc_rounds.hip -- decision rounds for NO_WAIT / WAIT_DIE / OCC (gfx950).
//
// Under the E-schedule txn i commits iff no EARLIER COMMITTED
// txn conflicts with it:
//   NO_WAIT / WAIT_DIE: they share a row and one of the two accesses is a write
//     (Row_lock::lock_get conflict -> Abort, concurrency_control/row_lock.cpp:69,86-90;
//     WAIT_DIE never waits because owners are always older, row_lock.cpp:101-118)
//   OCC: the earlier txn's write set meets this txn's read or write set
//     (OptCC::central_validate active-set check + test_valid, occ.cpp:185-199, 319-327)
// -- a greedy, sequence-ordered independent set.  Each round evaluates every
// live access against the row queue in front of it with one segmented OR-scan:
//   a blocker is committed         -> the access (so its txn) aborts
//   a blocker is still undecided   -> wait
//   no non-aborted blocker         -> the access is OK, permanently
// A txn commits once all its accesses are OK.  The lowest undecided txn always
// decides, so rounds terminate; zipf 0.9 epochs of 1M txns take ~20.
//
// Layout.  A round element is one access in row order,
//     e = ((txn << slog | pos) << 3) | done << 2 | head << 1 | wr
// with pos = its position in the txn: e >> 3 indexes the access's verdict byte
// vb8[txn << slog | pos], and a txn reads its 1 << slog verdict bytes with one
// 16-byte load per 16 accesses.  Elements are 32-bit when the txn, position
// and flag bits fit (1M txns of <= 16 accesses: 27 bits), else 64-bit.  An
// access reads its txn's status byte (1 B per txn: L2-resident); aborts go
// straight to that byte, OKs to the verdict byte -- plain loads and stores,
// no atomics.  Each pass compacts away what the next round does not need,
// stages tiles through LDS for coalesced loads and stores, and is a single
// launch (decoupled look-back scan, dvcc_common.h).  Round 0 reads the
// row-sorted pairs directly.  Once the live set fits in LDS, one
// single-workgroup launch runs every remaining round (k_round_tail).
#include <hip/hip_ext.h>

#include "dvcc_common.h"

namespace dvcc {

namespace {

// scan value bits (OR): 1 committed / 2 undecided (any access), 4 committed /
// 8 undecided (WR accesses), 16 = the access is kept for the next round
constexpr uint32_t B_CA = 1u, B_UA = 2u, B_CW = 4u, B_UW = 8u, B_KEEP = 16u;
constexpr uint32_t kCarryHead = 1u << 31;  // carry word: the slice holds a queue head
constexpr uint32_t kCarryInit = B_UA | B_UW | B_KEEP | kCarryHead;  // "undecided blockers in front"
constexpr uint8_t VB_OK = 1, VB_ABORT = 2;
constexpr uint32_t F_WR = 1u, F_HEAD = 2u, F_DONE = 4u;

template <class E>
__device__ __forceinline__ uint32_t r_txn(E e, uint32_t slog) {
    return (uint32_t)(e >> (slog + 3));
}

// per-element scan value (without B_KEEP) from its txn's status: aborted
// txns block nobody
template <class E>
__device__ __forceinline__ uint32_t elem_value(E e, uint8_t s, int nowait) {
    const bool wr = (e & F_WR) != 0;
    if (s == ST_COMMIT) return (nowait ? B_CA : 0u) | (wr ? B_CW : 0u);
    if (s == ST_UNDEC) return (nowait ? B_UA : 0u) | (wr ? B_UW : 0u);
    return 0u;
}

// verdict of a live access of an undecided txn from the OR of the scan values
// in front of it in its row queue.  An abort is a final fact about the whole
// txn, so it goes straight to the txn's status byte (readers of that byte in
// this same pass may or may not see it yet -- either view is a true fact, and
// the greedy outcome is unique); an OK is recorded per access for the settle.
// ALL (round 0): every access's verdict byte is written, 0 where not OK, so
// the bytes need no clearing before the epoch
template <bool ALL = false, class E>
__device__ __forceinline__ E decide_elem(E e, uint32_t excl, int nowait, uint8_t *__restrict__ vb8,
                                         uint32_t slog, uint8_t *status) {
    if (e & F_DONE) return e;
    // NO_WAIT/WAIT_DIE: a WR conflicts with any earlier access, a RD with
    // earlier WRs; OCC: any access with earlier committed writes
    const uint32_t sel = (nowait && (e & F_WR)) ? (excl & (B_CA | B_UA)) : ((excl >> 2) & (B_CA | B_UA));
    if (sel & B_CA) {
        status[r_txn(e, slog)] = ST_ABORT;  // Abort (row_lock.cpp:86-90 / occ.cpp:219-234)
        if (ALL) vb8[e >> 3] = 0;
    } else if (!(sel & B_UA)) {
        vb8[e >> 3] = VB_OK;  // granted / validated: permanently OK
        e |= F_DONE;
    } else if (ALL) {
        vb8[e >> 3] = 0;
    }
    return e;
}

// reverse segmented OR (right to left; f = a queue ends inside the span,
// v = some element of the span's first queue piece still needs a verdict)
struct RAgg {
    uint32_t f, v;
};
__device__ __forceinline__ RAgg rcomb(RAgg near, RAgg far) {
    return RAgg{near.f | far.f, near.f ? near.v : (near.v | far.v)};
}

// ---- wave scans from ballots (no LDS traffic).  The scan fields are a few
//      bits wide (a head flag, the 5-bit status OR, a per-thread count below
//      2^CB), so each bit of a field is one ballot and a lane's prefix over a
//      run of lanes is masks and popcounts of the ballots -- VALU and SALU
//      work only, where the shuffle ladders (ds_bpermute) were ~20 dependent
//      LDS round trips per iteration of the asynchronous rounds.
__device__ __forceinline__ uint64_t lanes_before(uint32_t lane) { return (1ull << lane) - 1ull; }
__device__ __forceinline__ uint64_t lanes_after(uint32_t lane) { return lane >= 63u ? 0ull : (~0ull << (lane + 1u)); }
constexpr int bits_for(int n) { return n < 2 ? 1 : 1 + bits_for(n >> 1); }  // bits of a count 0..n

template <int CB>  // Agg values: f 0/1, v below 32, c below 2^CB
struct WaveScan {
    uint64_t H, V[5], C[CB];
    __device__ __forceinline__ explicit WaveScan(Agg p) {
        H = __ballot(p.f != 0u);
#pragma unroll
        for (int b = 0; b < 5; b++) V[b] = __ballot((p.v >> b) & 1u);
#pragma unroll
        for (int b = 0; b < CB; b++) C[b] = __ballot((p.c >> b) & 1u);
    }
    // OpPlain over the lanes of m, a run of lanes starting at lane 0
    __device__ __forceinline__ Agg over(uint64_t m) const {
        const uint64_t hm = H & m;
        const uint64_t from = hm ? ~((1ull << (63 - __clzll((long long)hm))) - 1ull) : ~0ull;  // the last head on
        const uint64_t R = m & from;
        uint32_t v = 0, c = 0;
#pragma unroll
        for (int b = 0; b < 5; b++) v |= (V[b] & R) ? (1u << b) : 0u;
#pragma unroll
        for (int b = 0; b < CB; b++) c += (uint32_t)__popcll(C[b] & m) << b;
        return Agg{hm != 0 ? 1u : 0u, v, c};
    }
};

// the OR of a 5-bit field over the wave
__device__ __forceinline__ uint32_t wave_or5(uint32_t x) {
    uint32_t v = 0;
#pragma unroll
    for (int b = 0; b < 5; b++) v |= __ballot((x >> b) & 1u) ? (1u << b) : 0u;
    return v;
}

// reverse OR (rcomb) over the lanes of m, a run of lanes ending at lane 63,
// from the ballots of f and v
__device__ __forceinline__ RAgg rover(uint64_t F, uint64_t Vb, uint64_t m) {
    const uint64_t fm = F & m;
    const uint64_t upto = fm ? ((2ull << __builtin_ctzll(fm)) - 1ull) : ~0ull;  // through the first cut
    return RAgg{fm != 0 ? 1u : 0u, (Vb & m & upto) != 0 ? 1u : 0u};
}

// the keep bits of a thread's IPT elements from r, "a needy element follows
// my last one in its queue"
template <int IPT, class M>
__device__ __forceinline__ M keep_from(int cnt, M nhm, M needy, M blk, uint32_t r) {
    M keep = 0;
#pragma unroll
    for (int j = IPT - 1; j >= 0; j--) {
        if (j < cnt) {
            const uint32_t after = ((nhm >> j) & 1u) ? 0u : r;
            const uint32_t nd = (uint32_t)(needy >> j) & 1u;
            keep |= (M)(((uint32_t)(blk >> j) & 1u) & (nd | after)) << j;
            r = after | nd;
        }
    }
    return keep;
}

// a thread's reverse aggregate: f = a queue ends inside its elements, v = an
// element of its first queue piece is needy (a thread past the end is
// transparent, so what follows reaches the last element)
template <class M>
__device__ __forceinline__ RAgg thread_rev(int cnt, M nhm, M needy) {
    constexpr int kBits = 8 * (int)sizeof(M);
    const M valid = cnt >= kBits ? ~(M)0 : (((M)1 << cnt) - 1);
    RAgg x{0u, 0u};
    if (cnt > 0) {
        const M cuts = nhm & valid;
        x.f = cuts != 0;
        const int c0 = sizeof(M) == 8 ? __builtin_ctzll((uint64_t)cuts) : __builtin_ctz((uint32_t)cuts);
        const M upto = cuts ? (c0 + 1 >= kBits ? ~(M)0 : (((M)2 << c0) - 1)) : valid;
        x.v = (needy & upto) != 0;
    }
    return x;
}

// Which elements survive into the next round: an element of an undecided
// txn that still waits (needy), and a potential blocker (committed or
// undecided txn) followed in its queue by a needy element.  Each thread holds
// IPT consecutive elements; nhm bit j = the element after j starts a queue.
// `far` describes what follows the last thread's chunk.  Returns keep bits.
template <int IPT, int WAVES, class M = uint32_t>
__device__ __forceinline__ M keep_bits(int cnt, M nhm, M needy, M blk, RAgg *rw, RAgg far, uint32_t lane,
                                       uint32_t wave) {
    const RAgg x = thread_rev<M>(cnt, nhm, needy);
    const uint64_t F = __ballot(x.f != 0u), Vb = __ballot(x.v != 0u);
    if (lane == 0) rw[wave] = rover(F, Vb, ~0ull);   // the wave's aggregate
    const RAgg ex_r = rover(F, Vb, lanes_after(lane));  // the lanes after mine
    __syncthreads();
    for (int w = WAVES - 1; w > (int)wave; w--) far = rcomb(rw[w], far);
    return keep_from<IPT, M>(cnt, nhm, needy, blk, rcomb(ex_r, far).v);
}

// ... the same for a chunk one wave holds alone (no workgroup barrier)
template <int IPT, class M = uint32_t>
__device__ __forceinline__ M keep_bits_wave(int cnt, M nhm, M needy, M blk, RAgg far, uint32_t lane) {
    const RAgg x = thread_rev<M>(cnt, nhm, needy);
    const uint64_t F = __ballot(x.f != 0u), Vb = __ballot(x.v != 0u);
    return keep_from<IPT, M>(cnt, nhm, needy, blk, rcomb(rover(F, Vb, lanes_after(lane)), far).v);
}

}  // namespace

// ---- one tile of a decision round (single-pass OpPlain scan: v = status
//      bits OR-ed along the row queue, c = kept accesses -> compaction offset)
// Tile geometry follows the input width: 1024 threads x 16 32-bit elements,
// or 512 threads x 16 64-bit elements (round 0's pairs, or 64-bit elements);
// 16 elements per thread, the LDS image padded one slot per 16.  Large tiles
// keep the look-back short: the tiles dispatched together all publish their
// aggregates at about the same time and each walks back to the nearest
// inclusive prefix, 64 descriptors per step (config D: 16K/8K-element tiles
// took 2.5 % less epoch time than 8K/4K, 4K/4K took 3 % more).
template <class EIn>
#ifndef DVCC_ROUND_IPT
#define DVCC_ROUND_IPT 16
#endif
#ifndef DVCC_ROUND_T64
#define DVCC_ROUND_T64 1024
#endif
// 64-bit elements (round 0 over the sorted pairs): 4 per thread, 4,096-element
// tiles -- a prefix-kill stage's 328K / 563K pairs in 80 / 138 workgroups
// instead of 40 / 69 (round 0 18.9 -> 16.2 us at config D; 16 per thread 18.9,
// 256 threads x 16 21.3; profiles/r04_rt2); 1,024 threads x 4 instead of
// 512 x 8: 16.5 -> 15.5 us (profiles/r05_aj)
#ifndef DVCC_ROUND_IPT64
#define DVCC_ROUND_IPT64 4
#endif
struct Geo {
    static constexpr int kThreads = sizeof(EIn) == 4 ? 1024 : DVCC_ROUND_T64;
    static constexpr int kMinWaves = sizeof(EIn) == 4 ? 4 : 3;  // per SIMD: <= 128 / 168 VGPRs
    static constexpr int kWaves = kThreads / 64;
    static constexpr int kIPT = sizeof(EIn) == 4 ? DVCC_ROUND_IPT : DVCC_ROUND_IPT64;
    static constexpr uint32_t kTile = kThreads * kIPT;
    // the look-back descriptors are sized for kRTile-element tiles (dvcc_common.h)
    static_assert(kTile >= (uint32_t)kRTile, "round tiles at least kRTile elements");
};
__device__ __forceinline__ uint32_t pad16(uint32_t j) { return j + (j >> 4); }

template <class EIn>
struct TileLds {
    EIn el[Geo<EIn>::kTile + Geo<EIn>::kTile / 16];  // input tile, then the compacted output
    EIn next;
    uint64_t prev;
    Agg wt[Geo<EIn>::kWaves];
    RAgg rw[Geo<EIn>::kWaves];
    Agg pre;        // .v: the OR value in front of the tile
    uint32_t tot;
    uint32_t gpos;  // the tile's output offset (count prefix)
};

// coalesced 16-byte loads of [base, base + tile_n) into the padded LDS image
template <class EIn>
__device__ __forceinline__ void load_tile(const EIn *__restrict__ src, uint32_t base, uint32_t tile_n,
                                          uint32_t n, EIn *s, EIn *s_next, EIn past_end) {
    constexpr int V = 16 / sizeof(EIn);
    constexpr int T = Geo<EIn>::kThreads;
    const uint32_t tid = threadIdx.x;
#pragma unroll
    for (int q = 0; q < Geo<EIn>::kIPT / V; q++) {
        const uint32_t j = (q * T + tid) * V;
        if (j + V <= tile_n) {
            if constexpr (V == 2) {
                const ulonglong2 x = *reinterpret_cast<const ulonglong2 *>(src + base + j);
                s[pad16(j)] = x.x;
                s[pad16(j + 1)] = x.y;
            } else {
                const uint4 x = *reinterpret_cast<const uint4 *>(src + base + j);
                s[pad16(j)] = x.x;
                s[pad16(j + 1)] = x.y;
                s[pad16(j + 2)] = x.z;
                s[pad16(j + 3)] = x.w;
            }
        } else {
            for (int k = 0; k < V; k++)
                if (j + k < tile_n) s[pad16(j + k)] = src[base + j + k];
        }
    }
    if (tid == 0) *s_next = base + tile_n < n ? src[base + tile_n] : past_end;
}

// Round 0 reads the row-sorted pairs (row << 32 | txn << 8 | pos << 1 | wr)
// directly: queue heads and repeats come from the row of the neighbouring
// pair, and every txn is undecided (no status gather).  Later rounds read the
// compacted elements of the previous round.
template <bool FIRST, class EIn, class E>
__device__ __forceinline__ void round_tile(TileLds<EIn> &sh, uint32_t tile, uint32_t n, uint32_t ntiles,
                                           const EIn *__restrict__ el_in, E *__restrict__ el_out,
                                           uint32_t *__restrict__ n_out, uint8_t *status,
                                           uint8_t *__restrict__ vb8, uint32_t slog, int nowait,
                                           uint64_t *desc, uint32_t tag, uint32_t *und_reset,
                                           Counters *ctr);

// the undecided count the following settle (single GPU: list length) or apply
// (partitioned: slot sums) recounts
__device__ __forceinline__ void reset_und(uint32_t *und_reset, Counters *ctr) {
    if (und_reset) *und_reset = 0;
    else for (int k = 0; k < kSlots; k++) ctr->slot[k].undecided = 0;
}

template <bool FIRST, class EIn, class E>
__device__ __forceinline__ void round_tile(TileLds<EIn> &sh, uint32_t tile, uint32_t n, uint32_t ntiles,
                                           const EIn *__restrict__ el_in, E *__restrict__ el_out,
                                           uint32_t *__restrict__ n_out, uint8_t *status,
                                           uint8_t *__restrict__ vb8, uint32_t slog, int nowait,
                                           uint64_t *desc, uint32_t tag, uint32_t *und_reset,
                                           Counters *ctr) {
    using G = Geo<EIn>;
    constexpr int IPT = G::kIPT;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t base = tile * G::kTile;
    const uint32_t tile_n = n - base < G::kTile ? n - base : G::kTile;
    load_tile<EIn>(el_in, base, tile_n, n, sh.el, &sh.next, FIRST ? (EIn)~0ull : (EIn)F_HEAD);
    if (FIRST && tid == 0) sh.prev = base > 0 ? (uint64_t)el_in[base - 1] : ~0ull;
    __syncthreads();

    const uint32_t first = tid * IPT;
    const int cnt = first >= tile_n ? 0 : (tile_n - first < (uint32_t)IPT ? (int)(tile_n - first) : IPT);
    E e[IPT];
    uint32_t v[IPT];
    uint32_t nhm = 0;  // bit j: the element after e[j] starts a new queue
    uint32_t tmask = 0;  // bit j: a repeat access of its txn to the row (transparent)
    if constexpr (FIRST) {
        uint64_t pp = first == 0 ? sh.prev : (uint64_t)sh.el[pad16(first - 1)];
        const uint64_t pn = first + IPT < tile_n ? (uint64_t)sh.el[pad16(first + IPT)] : (uint64_t)sh.next;
        uint64_t p[IPT];
#pragma unroll
        for (int j = 0; j < IPT; j++) p[j] = j < cnt ? (uint64_t)sh.el[pad16(first + j)] : ~0ull;
#pragma unroll
        for (int j = 0; j < IPT; j++) {
            e[j] = (E)F_HEAD;
            if (j < cnt) {
                const bool head = pair_row(pp) != pair_row(p[j]);
                const uint64_t q = j + 1 < cnt ? p[j + 1] : (cnt < IPT ? ~0ull : pn);
                // A txn that touches one row several times (same row and txn:
                // adjacent in row order).  The repeats are transparent -- OK
                // at once, no value in the scan, dropped -- and the group's
                // first access stands for all of them with the OR of their
                // types: OCC puts the row in the txn's write set if any access
                // writes it (occ.cpp:296-317; a txn never validates against
                // itself, 185-199).  NO_WAIT / WAIT_DIE re-lock the row through
                // get_row (txn.cpp:790-803), which conflicts with the txn's own
                // lock unless both are shared (row_lock.cpp:69): NO_WAIT aborts
                // (86-90); WAIT_DIE, whose reference asserts here
                // (row_lock.cpp:106), is given the same outcome -- a txn cannot
                // wait for itself, so it dies (hazard H9).
                const bool rep = !head && pair_txn(pp) == pair_txn(p[j]);
                uint32_t wr = (uint32_t)(p[j] & 1u);
                const uint64_t id = ((uint64_t)pair_txn(p[j]) << slog) | pair_pos(p[j]);
                if (rep) {
                    tmask |= 1u << j;
                    vb8[id] = VB_OK;
                    if (nowait && ((p[j] | pp) & 1u)) status[pair_txn(p[j])] = ST_ABORT;
                } else if ((q >> 8) == (p[j] >> 8)) {  // the first of a group: OR of its types
                    for (uint32_t k = base + first + j + 1; k < n && !wr; k++) {
                        const uint64_t x = (uint64_t)el_in[k];
                        if ((x >> 8) != (p[j] >> 8)) break;
                        wr |= (uint32_t)(x & 1u);
                    }
                }
                e[j] = (E)((id << 3) | (head ? F_HEAD : 0u) | (rep ? F_DONE : 0u) | wr);
                nhm |= (pair_row(q) != pair_row(p[j]) ? 1u : 0u) << j;
                pp = p[j];
            }
        }
    } else {
        // branch-free: first + j < kTile, so the padded index stays inside the image
#pragma unroll
        for (int j = 0; j < IPT; j++) {
            const E x = (E)sh.el[pad16(first + j)];
            e[j] = j < cnt ? x : (E)F_HEAD;
        }
        const E nxt = first + IPT < tile_n ? (E)sh.el[pad16(first + IPT)] : (E)sh.next;
#pragma unroll
        for (int j = 0; j < IPT; j++) {
            const bool nh = j + 1 < cnt ? (e[j + 1] & F_HEAD) != 0
                                        : (cnt < IPT ? true : (nxt & F_HEAD) != 0);
            nhm |= (nh ? 1u : 0u) << j;
        }
    }
    // branch-free over all IPT slots (a padding slot reads txn 0's status and
    // is masked out), so the compiler keeps e[] and v[] in plain registers
    uint32_t umask = 0, needy = 0, blk = 0;
#pragma unroll
    for (int j = 0; j < IPT; j++) {
        const bool valid = j < cnt;
        const uint8_t s0 = FIRST ? (uint8_t)ST_UNDEC : status[r_txn(e[j], slog)];
        const uint8_t s = valid ? s0 : (uint8_t)ST_ABORT;
        umask |= (s == ST_UNDEC ? 1u : 0u) << j;
        needy |= (s == ST_UNDEC && !(e[j] & F_DONE) ? 1u : 0u) << j;
        const bool single = (e[j] & F_HEAD) && ((nhm >> j) & 1u);
        const bool transparent = FIRST && ((tmask >> j) & 1u);
        blk |= (s != ST_ABORT && !single && !transparent ? 1u : 0u) << j;
        v[j] = transparent ? 0u : elem_value(e[j], s, nowait);
    }
    // round 0: every element is needy; later: a queue running past the tile's
    // end is assumed to be followed by a needy element
    const uint32_t keep = FIRST ? blk
                                : keep_bits<IPT, G::kWaves>(cnt, nhm, needy, blk, sh.rw, RAgg{1u, 1u},
                                                            lane, wave);
    Agg a{0u, 0u, 0u};
#pragma unroll
    for (int j = 0; j < IPT; j++) {
        v[j] |= ((keep >> j) & 1u) ? B_KEEP : 0u;
        const Agg x{(uint32_t)((e[j] & F_HEAD) != 0), v[j], (keep >> j) & 1u};
        if (j < cnt) a = OpPlain::comb(a, x);
    }
    const WaveScan<bits_for(IPT)> ws(a);
    if (lane == 63) sh.wt[wave] = ws.over(~0ull);
    __syncthreads();
    // The decisions need only the OR in front of the tile (a walk back to the
    // nearest tile holding a head); the output offset needs the full count
    // prefix.  Wave 0 fetches the first, releases the other waves to decide,
    // then walks on for the second while they work.
    Agg bagg{0u, 0u, 0u};
    if (wave == 0) {
        bagg = sh.wt[0];
        for (int w = 1; w < G::kWaves; w++) bagg = OpPlain::comb(bagg, sh.wt[w]);
        const Agg pre = look_back<OpPlain, true>(desc, tile, tag, bagg, lane, ctr);
        if (lane == 0) {
            sh.pre = Agg{pre.f, pre.v, 0u};
            sh.tot = bagg.c;
            if (tile == 0) reset_und(und_reset, ctr);  // re-counted by this round's settle / apply
        }
    }
    __syncthreads();
    if (wave == 0) {
        const uint32_t gpos = look_back<OpPlain>(desc, tile, tag, bagg, lane, ctr).c;
        if (lane == 0) sh.gpos = gpos;
    }
    Agg wpre{0u, 0u, 0u};  // this wave's prefix within the tile
    for (uint32_t w = 0; w < wave; w++) wpre = OpPlain::comb(wpre, sh.wt[w]);
    const Agg lex = ws.over(lanes_before(lane));
    uint32_t lpos = wpre.c + lex.c;                                   // block-local slot
    uint32_t run = OpPlain::comb(OpPlain::comb(sh.pre, wpre), lex).v;  // OR since queue head
    E *s_out = reinterpret_cast<E *>(sh.el);  // every lane holds its elements: reuse the tile
    // padding slots have umask and keep bits clear: no branch on cnt needed
#pragma unroll
    for (int j = 0; j < IPT; j++) {
        E ej = e[j];
        const uint32_t vj = v[j];
        const bool head = (ej & F_HEAD) != 0;
        const uint32_t excl = head ? 0u : run;
        if ((umask >> j) & 1u) ej = decide_elem<FIRST>(ej, excl, nowait, vb8, slog, status);
        if (vj & B_KEEP) s_out[lpos++] = (E)((ej & ~(E)F_HEAD) | ((excl & B_KEEP) ? 0u : F_HEAD));
        run = head ? vj : (run | vj);
    }
    __syncthreads();
    // coalesced write-out of the compacted tile
    const uint32_t tot = sh.tot, gpos = sh.gpos;
    for (uint32_t k = tid; k < tot; k += G::kThreads) el_out[gpos + k] = s_out[k];
    if (tile == ntiles - 1 && tid == 0) *n_out = gpos + tot;
    __syncthreads();  // the LDS tile is free again
}

// one decision round, one launch; tiles are taken by ticket so that a tile
// only ever waits on tiles already running
template <bool FIRST, class EIn, class E>
__global__ __launch_bounds__(Geo<EIn>::kThreads, Geo<EIn>::kMinWaves) void k_round_pass(
    const EIn *__restrict__ el_in, const uint32_t *__restrict__ n_in, E *__restrict__ el_out,
    uint32_t *__restrict__ n_out, uint8_t *status, uint8_t *__restrict__ vb8, uint32_t slog,
    int nowait, uint64_t *desc, uint32_t *tile_ctr, uint32_t tag, uint32_t *und_reset,
    const uint32_t *und_in, uint32_t round, RoundPub *pub, Counters *ctr, const uint32_t *n0_dev, uint32_t n0,
    const uint32_t *n_txn_dev, uint32_t n_txn0) {
    __shared__ TileLds<EIn> sh;
    __shared__ uint32_t s_tile;
    // round 0 reads its sizes from the arguments and starts the rounds' counts
    const uint32_t n_live = FIRST ? (n0_dev ? *n0_dev : n0) : *n_in;
    const uint32_t und = FIRST || !und_in ? 1u : *und_in;
    if (FIRST && blockIdx.x == 0 && threadIdx.x == 0) {
        ctr->nlive[0] = n_live;
        ctr->nund[0] = n_txn_dev ? *n_txn_dev : n_txn0;  // partitioned rounds: round 0's list is every txn
        // a (sub-)epoch's rounds start with no asynchronous try behind them
        // (halt stays: the epoch clear zeroes it, and a prefix-kill epoch's
        // survivor stage must keep the prefix's halt, k_prefix_mark)
        ctr->async_go = 0;
        ctr->async_r0 = 0;
        ctr->async_wr0 = 0;
        ctr->async_iters = 0;
        ctr->async_block = 0;
    }
    // nothing left to decide, or a rejected epoch: no-op
    const uint32_t n = und && !input_err(ctr) ? n_live : 0u;
    const uint32_t ntiles = (n + Geo<EIn>::kTile - 1) / Geo<EIn>::kTile;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (round < (uint32_t)kRoundLog && (und || round == 0)) {
            ctr->log_live[round] = n_live;
            ctr->log_und[round] = und_in ? und : 0u;
        }
        if (n) ctr->pass_live += n;  // (one pass at a time: the stream orders them)
    }
    // one thread publishes the outcome of the previous round to the host
    const bool publisher = pub && threadIdx.x == 0 && blockIdx.x == (ntiles ? ntiles - 1 : 0);
    if (blockIdx.x >= ntiles) {  // spare blocks of a stale upper bound: no ticket
        if (ntiles == 0 && blockIdx.x == 0 && threadIdx.x == 0) { *n_out = 0; reset_und(und_reset, ctr); }
    } else {
        if (threadIdx.x == 0) s_tile = atomicAdd(tile_ctr, 1u);
        __syncthreads();
        round_tile<FIRST, EIn, E>(sh, s_tile, n, ntiles, el_in, el_out, n_out, status, vb8, slog,
                                  nowait, desc, tag, und_reset, ctr);
    }
    if (publisher) {
        __hip_atomic_store(&pub->le, ((unsigned long long)n_live << 32) | ctr->err | ctr->peer_err,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&pub->ru, ((unsigned long long)round << 32) | und, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// ---- per-txn settle (single GPU): new status from its accesses' verdicts
// The verdict bytes of txn t are vb8[t << slog, (t << slog) + len): one
// 16-byte load per 16 accesses (slog >= 4).
__device__ __forceinline__ uint8_t txn_verdict(const uint8_t *__restrict__ v, uint32_t len, uint32_t *n_ok = nullptr) {
    uint32_t any_abort = 0, all_ok = 1, ok = 0;
    for (uint32_t w = 0; w < len; w += 16) {
        const uint4 x4 = *reinterpret_cast<const uint4 *>(v + w);
        const uint32_t x[4] = {x4.x, x4.y, x4.z, x4.w};
#pragma unroll
        for (uint32_t q = 0; q < 4; q++) {
            const int nb = (int)len - (int)(w + 4 * q);
            const uint32_t m = nb >= 4 ? 0xFFFFFFFFu : (nb <= 0 ? 0u : (1u << (8 * nb)) - 1u);
            any_abort |= x[q] & 0x02020202u & m;
            all_ok &= (x[q] & m) == (0x01010101u & m);
            if (n_ok) ok += __popc(x[q] & 0x01010101u & m);
        }
    }
    if (n_ok) *n_ok = ok;
    return any_abort ? V_ABORT : (all_ok ? 0 : V_WAIT);
}

// Walks the undecided-txn list (round 0: every txn) and writes the survivors
// to the other list: each block takes kSettleChunk consecutive entries,
// compacts its survivors in LDS and reserves space with ONE atomic.
#ifndef DVCC_SETTLE_IPT
#define DVCC_SETTLE_IPT 1  // (txns per thread: 1 took the settle from 8.3-8.9 to 5.9-6.1 us at config D, profiles/r05_af)
#endif
constexpr uint32_t kSettleIPT = DVCC_SETTLE_IPT, kSettleChunk = kBlock * kSettleIPT;

// tword (round 0 with an asynchronous launch behind it): also the txn's fact
// word for k_round_async, as k_async_words would write it from the settled
// state -- status | OK verdicts << 8 | accesses << 16
__device__ __forceinline__ bool settle_txn(uint8_t *__restrict__ status, const uint8_t *__restrict__ vb8,
                                           uint32_t slog, const uint8_t *__restrict__ tlen,
                                           uint32_t t, uint32_t *__restrict__ tword = nullptr) {
    const uint8_t s0 = status[t];
    if (s0 != ST_UNDEC) {  // aborted by the pass
        if (tword) tword[t] = s0 | ((uint32_t)tlen[t] << 16);
        return false;
    }
    const uint32_t len = tlen[t];
    uint32_t ok = 0;
    const uint8_t v = txn_verdict(vb8 + ((size_t)t << slog), len, tword ? &ok : nullptr);
    const uint8_t s = (v & V_ABORT) ? ST_ABORT : (!(v & V_WAIT) ? ST_COMMIT : ST_UNDEC);
    if (s != ST_UNDEC) status[t] = s;
    if (tword) tword[t] = s | ((s == ST_UNDEC ? ok : 0u) << 8) | (len << 16);
    return s == ST_UNDEC;
}

struct SettleLds {
    uint32_t keep[kSettleChunk];
    uint32_t cnt, base;
};

// entries [lo, lo + kSettleChunk) of the list (FIRST: txn ids themselves)
template <bool FIRST>
__device__ __forceinline__ void settle_chunk(SettleLds &sh, uint32_t lo, uint32_t n,
                                             uint8_t *__restrict__ status,
                                             const uint8_t *__restrict__ vb8, uint32_t slog,
                                             const uint8_t *__restrict__ tlen,
                                             const uint32_t *__restrict__ list_in,
                                             uint32_t *__restrict__ list_out,
                                             uint32_t *__restrict__ n_out,
                                             uint32_t *__restrict__ tword = nullptr) {
    if (threadIdx.x == 0) sh.cnt = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
#pragma unroll
    for (uint32_t k = 0; k < kSettleIPT; k++) {
        const uint32_t i = lo + k * kBlock + threadIdx.x;
        uint32_t t = 0;
        bool keep = false;
        if (i < n) {
            t = FIRST ? i : list_in[i];
            keep = settle_txn(status, vb8, slog, tlen, t, tword);
        }
        const uint64_t m = __ballot(keep);
        uint32_t wb = 0;
        if (lane == 0 && m) wb = atomicAdd(&sh.cnt, (uint32_t)__builtin_popcountll(m));
        wb = __shfl(wb, 0, 64);
        if (keep) sh.keep[wb + mask_rank(m)] = t;
    }
    __syncthreads();
    const uint32_t cnt = sh.cnt;
    if (threadIdx.x == 0 && cnt) sh.base = atomicAdd(n_out, cnt);
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < cnt; k += kBlock) list_out[sh.base + k] = sh.keep[k];
    __syncthreads();  // the LDS chunk is free again
}

template <bool FIRST>
__global__ __launch_bounds__(kBlock) void k_round_settle(
    uint8_t *__restrict__ status, const uint8_t *__restrict__ vb8, uint32_t slog,
    const uint8_t *__restrict__ tlen, const uint32_t *__restrict__ list_in,
    const uint32_t *__restrict__ n_in, uint32_t n_txn, uint32_t *__restrict__ list_out,
    uint32_t *__restrict__ n_out, uint32_t *__restrict__ tword, uint32_t *__restrict__ carry, uint32_t G) {
    __shared__ SettleLds sh;
    // round 0: every txn of the (sub-)epoch (its real count from the round-0 pass)
    const uint32_t n = n_in ? *n_in : n_txn;
    const uint32_t lo = blockIdx.x * kSettleChunk;
    if (lo >= n) return;
    // (the asynchronous launch's carry words start pessimistic, k_async_words)
    if (carry && blockIdx.x == 0)
        for (uint32_t g = threadIdx.x; g < G; g += kBlock) carry[g] = kCarryInit;
    settle_chunk<FIRST>(sh, lo, n, status, vb8, slog, tlen, list_in, list_out, n_out, tword);
}

// ---- partitioned rounds over the undecided-txn list -----------------------
// Every partition holds the same statuses after each apply, so the list of
// undecided txns (ascending, compacted by a deterministic scan) is the same
// on every rank: verdict bytes travel for list entries only, in list order,
// and the all-reduce shrinks with the undecided set (1M txns: 1 MB in round
// 0, a few KB by the tail) instead of n_txn bytes every round.
// list = nullptr: round 0, the list is every txn.
__global__ __launch_bounds__(kBlock) void k_list_verdict(const uint32_t *__restrict__ list,
                                                         const uint32_t *__restrict__ n_list,
                                                         const uint8_t *__restrict__ status,
                                                         const uint8_t *__restrict__ vb8, uint32_t slog,
                                                         const uint8_t *__restrict__ tlen,
                                                         uint8_t *__restrict__ verdict) {
    const uint32_t U = *n_list;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < U; i += gridDim.x * blockDim.x) {
        const uint32_t t = list ? list[i] : i;
        const uint8_t s = status[t];
        // a local abort (this round's pass) is final everywhere; an undecided
        // txn reports its local accesses' verdict
        verdict[i] = s == ST_ABORT ? (uint8_t)V_ABORT
                                   : (s == ST_UNDEC ? txn_verdict(vb8 + ((size_t)t << slog), tlen[t]) : 0);
    }
}

// apply the MAX-combined verdicts, compact the list (order kept: decoupled
// look-back over kRTile-entry tiles) and publish the undecided count
__global__ __launch_bounds__(kBlock) void k_list_apply(
    const uint32_t *__restrict__ list, const uint32_t *__restrict__ n_list,
    const uint8_t *__restrict__ verdict, uint8_t *__restrict__ status, uint32_t *__restrict__ list_out,
    uint32_t *__restrict__ n_out, const uint32_t *__restrict__ n_live_next, uint64_t *desc,
    uint32_t *tile_ctr, uint32_t tag, uint32_t round, RoundPub *pub, Counters *ctr) {
    __shared__ Agg wt[4];
    __shared__ Agg s_pre;
    __shared__ uint32_t s_tile;
    const uint32_t U = *n_list;
    const uint32_t ntiles = (U + kRTile - 1) / kRTile;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (blockIdx.x >= ntiles) {
        if (ntiles == 0 && blockIdx.x == 0 && tid == 0) {
            *n_out = 0;
            if (pub) {
                __hip_atomic_store(&pub->und_log[round % RoundPub::kPubLog], 0u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
                __threadfence_system();
                __hip_atomic_store(&pub->le, ((unsigned long long)*n_live_next << 32) | ctr->err | ctr->peer_err,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(&pub->ru, (unsigned long long)(round + 1) << 32, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
        return;
    }
    if (tid == 0) s_tile = atomicAdd(tile_ctr, 1u);
    __syncthreads();
    const uint32_t tile = s_tile, base = tile * kRTile;
    // kRIPT consecutive entries per thread
    uint32_t keepm = 0, tl[kRIPT];
    const uint32_t first = base + tid * kRIPT;
#pragma unroll
    for (int j = 0; j < kRIPT; j++) {
        const uint32_t i = first + j;
        tl[j] = 0;
        if (i < U) {
            const uint32_t t = list ? list[i] : i;
            tl[j] = t;
            const uint8_t v = verdict[i];
            if (status[t] == ST_UNDEC) {
                if (v & V_ABORT) status[t] = ST_ABORT;
                else if (!(v & V_WAIT)) status[t] = ST_COMMIT;
                else keepm |= 1u << j;
            }
        }
    }
    const Agg inc = wave_incl<OpPlain>(Agg{0u, 0u, (uint32_t)__builtin_popcount(keepm)}, lane);
    if (lane == 63) wt[wave] = inc;
    __syncthreads();
    if (wave == 0) {
        Agg bagg = wt[0];
        for (int w = 1; w < 4; w++) bagg = OpPlain::comb(bagg, wt[w]);
        const Agg pre = look_back<OpPlain>(desc, tile, tag, bagg, lane, ctr);
        if (lane == 0) s_pre = pre;
    }
    __syncthreads();
    uint32_t pos = s_pre.c;
    for (uint32_t w = 0; w < wave; w++) pos += wt[w].c;
    pos += wave_excl_from_incl<OpPlain>(inc, lane).c;
#pragma unroll
    for (int j = 0; j < kRIPT; j++)
        if ((keepm >> j) & 1u) list_out[pos++] = tl[j];
    if (tile == ntiles - 1 && tid == 0) {
        uint32_t tot = s_pre.c;
        for (int w = 0; w < 4; w++) tot += wt[w].c;
        *n_out = tot;
        if (pub) {
            __hip_atomic_store(&pub->und_log[round % RoundPub::kPubLog], tot, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
            __threadfence_system();
            __hip_atomic_store(&pub->le, ((unsigned long long)*n_live_next << 32) | ctr->err | ctr->peer_err,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&pub->ru, ((unsigned long long)(round + 1) << 32) | tot, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}


// ---- the tail: every remaining round in ONE single-workgroup launch --------
// Once the live set fits in LDS, a pass + settle pair costs two launches and
// ~20 us of latency for a few thousand elements.  k_round_tail runs the same
// round -- status gather, reverse (dead-element) and forward segmented scans,
// decisions, compaction, settle -- on one CU with __syncthreads as the only
// barrier, until no txn is undecided.  The lowest undecided txn decides in
// every round, so the loop ends; a round without progress is an error.
template <class E>
struct TailGeo {
    static constexpr int kIPT = sizeof(E) == 4 ? 16 : 12;
    static constexpr uint32_t kCap = (uint32_t)kTailThreads * kIPT;  // 16384 / 12288
};
constexpr int kTailWaves = kTailThreads / 64;

template <class E>
struct TailLds {
    E el[TailGeo<E>::kCap];
    uint32_t ul[TailGeo<E>::kCap];
    Agg wt[kTailWaves];
    RAgg rw[kTailWaves];
    uint32_t ucnt;
};

template <class E>
__global__ __launch_bounds__(kTailThreads) void k_round_tail(RoundBufs b, uint32_t r0, int nowait,
                                                             RoundPub *pub) {
    constexpr int IPT = TailGeo<E>::kIPT;
    __shared__ TailLds<E> sh;
    Counters *ctr = b.ctr;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t slog = b.slog;
    uint32_t n = ctr->nlive[r0 & 1];
    uint32_t U = ctr->nund[r0 & 1];
    uint32_t round = r0;
    bool ok = r0 > 0 && n <= TailGeo<E>::kCap && U <= TailGeo<E>::kCap && !input_err(ctr);
    if (!ok) {  // decline: the host resumes the multi-workgroup rounds at r0
        if (tid == 0 && pub)
            __hip_atomic_store(&pub->tl, ((unsigned long long)r0 << 32) | 1u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    {
        const E *src = reinterpret_cast<const E *>(b.rel[(r0 - 1) & 1]);
        const uint32_t *lsrc = b.ulist[r0 & 1];
        for (uint32_t i = tid; i < n; i += kTailThreads) sh.el[i] = src[i];
        for (uint32_t i = tid; i < U; i += kTailThreads) sh.ul[i] = lsrc[i];
    }
    __syncthreads();
    while (ok && U > 0) {
        if (tid == 0 && round < (uint32_t)kRoundLog) {
            ctr->log_live[round] = n;
            ctr->log_und[round] = U;
        }
        // ---- pass: my chunk of k consecutive elements
        const uint32_t k = (n + kTailThreads - 1) / kTailThreads;
        const uint32_t first = tid * k;
        const int cnt = first >= n ? 0 : (int)(n - first < k ? n - first : k);
        E e[IPT];
        uint32_t v[IPT];
#pragma unroll
        for (int j = 0; j < IPT; j++) e[j] = j < cnt ? sh.el[first + j] : (E)F_HEAD;
        const E nxt = first + (uint32_t)cnt < n ? sh.el[first + cnt] : (E)F_HEAD;
        uint32_t nhm = 0, umask = 0, needy = 0, blk = 0;
#pragma unroll
        for (int j = 0; j < IPT; j++) {
            v[j] = 0;
            if (j < cnt) {
                const bool nh = j + 1 < cnt ? (e[j + 1] & F_HEAD) != 0 : (nxt & F_HEAD) != 0;
                nhm |= (nh ? 1u : 0u) << j;
                const uint8_t s = b.status[r_txn(e[j], slog)];
                umask |= (s == ST_UNDEC ? 1u : 0u) << j;
                needy |= (s == ST_UNDEC && !(e[j] & F_DONE) ? 1u : 0u) << j;
                const bool single = (e[j] & F_HEAD) && nh;
                blk |= (s != ST_ABORT && !single ? 1u : 0u) << j;
                v[j] = elem_value(e[j], s, nowait);
            }
        }
        // the whole live set is here: nothing follows the end
        const uint32_t keep = keep_bits<IPT, kTailWaves>(cnt, nhm, needy, blk, sh.rw, RAgg{1u, 0u},
                                                         lane, wave);
        Agg a{0u, 0u, 0u};
#pragma unroll
        for (int j = 0; j < IPT; j++) {
            if (j < cnt) {
                if ((keep >> j) & 1u) v[j] |= B_KEEP;
                a = OpPlain::comb(a, Agg{(uint32_t)((e[j] & F_HEAD) != 0), v[j], (keep >> j) & 1u});
            }
        }
        const Agg inc = wave_incl<OpPlain>(a, lane);
        if (lane == 63) sh.wt[wave] = inc;
        __syncthreads();
        Agg wpre{0u, 0u, 0u}, total{0u, 0u, 0u};
        for (int w = 0; w < kTailWaves; w++) {
            if (w < (int)wave) wpre = OpPlain::comb(wpre, sh.wt[w]);
            total = OpPlain::comb(total, sh.wt[w]);
        }
        const Agg lex = wave_excl_from_incl<OpPlain>(inc, lane);
        const Agg pre = OpPlain::comb(wpre, lex);
        uint32_t lpos = pre.c, run = pre.v;
        // every thread read its elements before the first barrier: write in place
#pragma unroll
        for (int j = 0; j < IPT; j++) {
            if (j < cnt) {
                E ej = e[j];
                const bool head = (ej & F_HEAD) != 0;
                const uint32_t excl = head ? 0u : run;
                if ((umask >> j) & 1u) ej = decide_elem(ej, excl, nowait, b.vb8, slog, b.status);
                if (v[j] & B_KEEP)
                    sh.el[lpos++] = (E)((ej & ~(E)F_HEAD) | ((excl & B_KEEP) ? 0u : F_HEAD));
                run = head ? v[j] : (run | v[j]);
            }
        }
        if (tid == 0) sh.ucnt = 0;
        __syncthreads();  // verdict and status stores are visible to the workgroup
        // ---- settle: the undecided list, compacted in place
        uint32_t tl[IPT];
        uint32_t km = 0;
#pragma unroll
        for (int q = 0; q < IPT; q++) {
            const uint32_t i = q * kTailThreads + tid;
            tl[q] = 0;
            if (i < U) {
                tl[q] = sh.ul[i];
                km |= (settle_txn(b.status, b.vb8, slog, b.tlen, tl[q]) ? 1u : 0u) << q;
            }
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < IPT; q++) {
            const bool kp = (km >> q) & 1u;
            const uint64_t m = __ballot(kp);
            uint32_t wb = 0;
            if (lane == 0 && m) wb = atomicAdd(&sh.ucnt, (uint32_t)__builtin_popcountll(m));
            wb = __shfl(wb, 0, 64);
            if (kp) sh.ul[wb + mask_rank(m)] = tl[q];
        }
        __syncthreads();
        const uint32_t U2 = sh.ucnt;
        round++;
        if (U2 >= U) {  // the lowest undecided txn must have decided
            if (tid == 0) {
                set_err(ctr, ERRB_SPIN);
                atomicMax(&ctr->spin_site, 3u);
            }
            ok = false;
        }
        U = U2;
        n = total.c;
        __syncthreads();  // sh.ucnt is reset by the next round
    }
    if (tid == 0 && pub) {
        __hip_atomic_store(&pub->le, ((unsigned long long)n << 32) | ctr->err, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&pub->ru, ((unsigned long long)round << 32) | (ok ? U : 0xFFFFFFFFu),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// ---- asynchronous rounds: every remaining decision in one multi-workgroup
//      launch, without grid barriers
// Once the live set fits the workgroups' LDS, each workgroup takes an equal
// contiguous slice of the row-ordered elements and iterates on its own: read
// the status of its elements' txns, scan its queues, decide, publish the
// facts, compact.  A txn's status is a monotone fact (undecided, then
// committed or aborted), so any mix of fresh and stale reads of the facts
// other workgroups publish yields only true decisions, and the greedy's
// fixpoint is unique: the outcome equals the round-synchronous one.  A txn's
// facts are one 32-bit word -- status | OK count << 8 | accesses << 16 -- set
// with device-scope atomics and read with agent-scope atomic loads, so they
// cross CUs and XCDs inside the launch and one load tells committed (count ==
// accesses), aborted or undecided.
// A row queue may run across slices (a zipf-hot row spans dozens): each
// workgroup publishes, every iteration, its carry word -- the OR of the scan
// values after its last queue head (the whole slice if it holds no head) and
// a has-head bit.  A workgroup whose first queue runs in takes the value in
// front of it by walking the carries back, 64 at a time, to the nearest slice
// holding a head: a fact reaches the far end of a long queue in one
// iteration, not one slice per iteration.  Carries are built from monotone
// facts and start fully pessimistic (with a head, so walks stop there), so a
// stale carry only delays decisions.  The slice's last element is never
// dropped while its queue runs on, so a carry always describes that queue.
// A workgroup leaves once no element of an undecided txn remains in its slice
// and its carry no longer holds an undecided blocker.  That needs every
// workgroup resident at once: a workgroup waiting for facts only a
// non-resident one can produce (a co-running kernel holding CUs) would never
// learn them.  So a workgroup also leaves -- yields -- after `idle` wall-clock
// ticks without deciding anything, or after `max_iters` iterations: the facts
// it published stay true, the finalize turns them into status bytes and halts
// execution (Counters::halt), and the host resumes the synchronous rounds from
// the element array the launch started from (dv_epoch_finish).  Facts are
// monotone, so that array plus the newer statuses is a valid round state.
#ifndef DVCC_ASYNC_SLEEP
#define DVCC_ASYNC_SLEEP 8  // back-off (x 64 cycles) of a workgroup whose iteration decided nothing
#endif
// 1,024-thread workgroups, one per CU: half the slices of 512-thread ones, so
// a queue crosses fewer slice boundaries and a fact fewer workgroups, while
// the ballot scans take the extra waves for little (config D, one context:
// 37.3-39.2 against 42.2-42.4 us per launch; 512-thread ones two per CU, and
// 256-thread ones four, 44.6-45.6 -- profiles/r05_aw)
constexpr int kAsyncThreads = 1024;
constexpr int kAsyncWaves = kAsyncThreads / 64;
// 28 elements per thread (128 VGPRs, one workgroup per CU): 7.3M live
// accesses chip-wide.  Measured on a 1M-txn zipf-0.9 epoch, the launch pays
// off once the live set has halved: from round 1 (9.2M live) it took 570 us,
// more than the synchronous rounds it replaces -- every iteration re-reads
// the facts of every live access, and while the queues are long a slice
// iterates many times per round's worth of progress.
#ifndef DVCC_ASYNC_IPT
#define DVCC_ASYNC_IPT 28
#endif
constexpr int kAsyncIPT = DVCC_ASYNC_IPT;
constexpr uint32_t kAsyncCap = (uint32_t)kAsyncThreads * kAsyncIPT;  // elements per workgroup

constexpr uint32_t TW_OK = 1u << 8;  // one more access OK

#ifdef DVCC_ASYNC_STAMPS
// measurement builds only (tools/exp_variant.sh ... -DDVCC_ASYNC_STAMPS): per
// workgroup of k_round_async, summed over launches, thread 0's wall-clock
// ticks (100 MHz) -- [0] launches, [1] iterations, [2] ticks in the loop,
// [3] iteration start -> facts loaded, [4] -> carry walk done, [5] -> end of
// the iteration's work (decide, compact, publish, barriers), [6] back-off,
// [7] iterations that decided something; read by dv_debug_async_stamps
__device__ unsigned long long g_async_stamps[kAsyncGroups * 8];
// per launch: [0] launches, [1] the sum over launches of the most iterations
// any of its workgroups ran, [2] the sum of its workgroups' mean iterations
// (x 1024), [3] the last-workgroup ticket (reset per launch)
__device__ unsigned long long g_async_launch[4];
__device__ unsigned int g_async_lsum;
#endif
// the status fact of txn t
__device__ __forceinline__ uint8_t fact_status(const uint32_t *tword, uint32_t t) {
    return word_status(__hip_atomic_load(tword + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// the try's verdict from its inputs, which no kernel of the try changes:
// 1 run, 2 declined (the live set exceeds thresh or does not fit the
// workgroups -- equal slices, the largest holds ceil(n / G)), 0 nothing to
// do (no txn undecided, or an earlier try ran)
__device__ __forceinline__ uint32_t async_gate(const Counters *ctr, uint32_t r0, uint32_t G,
                                               uint32_t thresh) {
    if (ctr->async_r0 != 0 || ctr->async_block != 0 || ctr->nund[r0 & 1] == 0 || input_err(ctr)) return 0u;
    const uint32_t n_all = ctr->nlive[r0 & 1];
    return n_all <= thresh && ((uint64_t)n_all + G - 1) / G <= kAsyncCap ? 1u : 2u;
}

// the words from the synchronous rounds' state (status byte, OK verdict
// bytes), and every carry word pessimistic
__global__ __launch_bounds__(kBlock) void k_async_words(const uint8_t *__restrict__ status,
                                                        const uint8_t *__restrict__ vb8, uint32_t slog,
                                                        const uint8_t *__restrict__ tlen, uint32_t n_txn,
                                                        uint32_t *__restrict__ tword,
                                                        uint32_t *__restrict__ carry, uint32_t G,
                                                        uint32_t thresh, uint32_t r0,
                                                        const uint32_t *__restrict__ n_txn_dev,
                                                        const Counters *__restrict__ ctr) {
    if (async_gate(ctr, r0, G, thresh) != 1u) return;
    if (n_txn_dev && *n_txn_dev < n_txn) n_txn = *n_txn_dev;
    const uint32_t i0 = blockIdx.x * blockDim.x + threadIdx.x;
    for (uint32_t g = i0; g < G; g += gridDim.x * blockDim.x) carry[g] = kCarryInit;
    for (uint32_t t = i0; t < n_txn; t += gridDim.x * blockDim.x) {
        const uint32_t len = tlen[t];
        uint32_t ok = 0;
        const uint8_t s = status[t];
        if (s == ST_UNDEC) {
            for (uint32_t w = 0; w < len; w += 16) {
                const uint4 x4 = *reinterpret_cast<const uint4 *>(vb8 + ((size_t)t << slog) + w);
                const uint32_t x[4] = {x4.x, x4.y, x4.z, x4.w};
#pragma unroll
                for (uint32_t q = 0; q < 4; q++) {
                    const int nb = (int)len - (int)(w + 4 * q);
                    const uint32_t m = nb >= 4 ? 0xFFFFFFFFu : (nb <= 0 ? 0u : (1u << (8 * nb)) - 1u);
                    ok += __popc(x[q] & 0x01010101u & m);
                }
            }
        }
        tword[t] = s | (ok << 8) | (len << 16);
    }
}

// per-element scan value from the element and its txn's status bits
__device__ __forceinline__ uint32_t async_value(uint32_t e, bool undec, bool abort, int nowait) {
    if (abort) return 0u;
    const bool wr = (e & F_WR) != 0;
    return undec ? ((nowait ? B_UA : 0u) | (wr ? B_UW : 0u)) : ((nowait ? B_CA : 0u) | (wr ? B_CW : 0u));
}

// The iteration loop of one workgroup, for slices of at most kAsyncThreads *
// IPT elements: the kernel instantiates it for small slices too (IPT 4: a
// prefix-kill stage's live set, a few elements per thread), where the wide
// instantiation's fully unrolled 28-element loops cost a config-D epoch 38 us.
template <int IPT>
__device__ __forceinline__ void async_slices(const RoundBufs &b, const uint32_t *src, uint32_t n_all,
                                             uint32_t *tword, uint32_t *carry, int nowait, uint32_t max_iters,
                                             uint64_t idle, uint32_t *sel, RAgg *rw, Agg *wt, uint32_t *s_needy,
                                             uint32_t *s_moved, uint32_t &s_cin, uint32_t &s_quit, bool words) {
    using M = uint32_t;  // per-thread element bit masks
    Counters *ctr = b.ctr;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t slog = b.slog, g = blockIdx.x, G = gridDim.x;
    const uint32_t lo = (uint32_t)((uint64_t)g * n_all / G), hi = (uint32_t)((uint64_t)(g + 1) * n_all / G);
    uint32_t n = hi - lo;
    // does a queue run in from the previous slice / out into the next one?
    const bool cont_in = lo > 0 && lo < n_all && !(src[lo] & F_HEAD);
    const bool cont_out = hi < n_all && !(src[hi] & F_HEAD);
    {  // (the slice's loads all in flight before the first LDS store)
        uint32_t v[IPT];
#pragma unroll
        for (int j = 0; j < IPT; j++) {
            const uint32_t i = (uint32_t)j * kAsyncThreads + tid;
            v[j] = i < n ? src[lo + i] : 0u;
        }
#pragma unroll
        for (int j = 0; j < IPT; j++) {
            const uint32_t i = (uint32_t)j * kAsyncThreads + tid;
            if (i < n) sel[i] = v[j] & ~(i == 0 && cont_in ? F_HEAD : 0u);
        }
    }
    if (tid == 0) {
        s_needy[0] = s_needy[1] = s_moved[0] = s_moved[1] = 0;
        s_quit = 0;
    }
    __syncthreads();
    uint32_t it = 0;
    bool yielded = true;                  // cleared when the slice has nothing left to learn
    uint64_t last_move = wall_clock64();  // thread 0's: the last iteration that decided something
#ifdef DVCC_ASYNC_STAMPS
    uint64_t st_facts = 0, st_carry = 0, st_work = 0, st_sleep = 0, st_moved = 0, st_ti = 0, st_tf = 0;
    const uint64_t st_begin = wall_clock64();
#endif
    for (; it < max_iters; it++) {
        const uint32_t p = it & 1u;
#ifdef DVCC_ASYNC_STAMPS
        st_ti = wall_clock64();
#endif
        // the value in front of the slice: carries back to the nearest head,
        // read by wave 0; the first 64 carry words are loaded here, before
        // the facts, and resolved after them (one round trip for both)
        const bool look = cont_in && wave == 0;
        uint32_t cw = 0u;
        if (look) {
            const int64_t j = (int64_t)g - 1 - (int64_t)lane;
            cw = j >= 0 ? __hip_atomic_load(carry + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                        : kCarryHead;  // (slice 0 starts with a head)
        }
        const uint32_t k = (n + kAsyncThreads - 1) / kAsyncThreads;
        const uint32_t first = tid * k;
        const int cnt = first >= n ? 0 : (int)(n - first < k ? n - first : k);
        uint32_t e[IPT];
#pragma unroll
        for (int j = 0; j < IPT; j++) e[j] = j < cnt ? sel[first + j] : F_HEAD;
        const uint32_t nxt = first + (uint32_t)cnt < n ? sel[first + cnt] : (cont_out ? 0u : F_HEAD);
        M nhm = 0, umask = 0, amask = 0, needy = 0, blk = 0;
#pragma unroll
        for (int j = 0; j < IPT; j++) {
            if (j < cnt) {
                const bool nh = j + 1 < cnt ? (e[j + 1] & F_HEAD) != 0 : (nxt & F_HEAD) != 0;
                nhm |= (M)(nh ? 1u : 0u) << j;
                const uint8_t s = fact_status(tword, r_txn(e[j], slog));
                umask |= (M)(s == ST_UNDEC ? 1u : 0u) << j;
                amask |= (M)(s == ST_ABORT ? 1u : 0u) << j;
                needy |= (M)(s == ST_UNDEC && !(e[j] & F_DONE) ? 1u : 0u) << j;
                const bool single = (e[j] & F_HEAD) && nh;
                blk |= (M)(s != ST_ABORT && !single ? 1u : 0u) << j;
            }
        }
#ifdef DVCC_ASYNC_STAMPS
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        st_tf = wall_clock64();
        st_facts += st_tf - st_ti;
#endif
        if (look) {  // (taken from LDS after keep_bits' barrier)
            uint32_t acc = 0;
            for (int64_t j0 = (int64_t)g - 1;; j0 -= 64) {
                const uint64_t hm = __ballot((cw & kCarryHead) != 0);
                const uint32_t stop = hm ? (uint32_t)__builtin_ctzll(hm) : 64u;
                acc |= wave_or5(lane <= stop ? (cw & ~kCarryHead) : 0u);
                if (hm) break;
                const int64_t j = j0 - 64 - (int64_t)lane;
                cw = j >= 0 ? __hip_atomic_load(carry + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                            : kCarryHead;
            }
            if (lane == 0) s_cin = acc;
        }
#ifdef DVCC_ASYNC_STAMPS
        {
            const uint64_t tc = wall_clock64();
            st_carry += tc - st_tf;
            st_tf = tc;
        }
#endif
        // a queue running into the next slice is assumed to be followed by a
        // needy element there; each wave decides its keep bits alone (no
        // barrier), assuming the same past its own last element unless it
        // holds the slice's end -- a few blockers kept one iteration longer
        const bool wave_end = (64u * wave + 64u) * k >= n;
        M keep = keep_bits_wave<IPT, M>(cnt, nhm, needy, blk,
                                        RAgg{1u, wave_end ? (cont_out ? 1u : 0u) : 1u}, lane);
        // ... and the slice's last element anchors that queue here: it is kept
        // whatever its txn, so the carry is always the OR of that queue (were
        // the queue's elements all dropped, the last head would be an
        // earlier queue's)
        if (cont_out && cnt > 0 && first + (uint32_t)cnt == n) keep |= (M)1 << (cnt - 1);
        if (needy) atomicAdd(&s_needy[p], (uint32_t)__popcll(needy));
        Agg a{0u, 0u, 0u};
#pragma unroll
        for (int j = 0; j < IPT; j++) {
            if (j < cnt) {
                const uint32_t kj = (uint32_t)(keep >> j) & 1u;
                const uint32_t vj = async_value(e[j], (umask >> j) & 1u, (amask >> j) & 1u, nowait) |
                                    (kj ? B_KEEP : 0u);
                a = OpPlain::comb(a, Agg{(uint32_t)((e[j] & F_HEAD) != 0), vj, kj});
            }
        }
        const WaveScan<bits_for(IPT)> ws(a);
        if (lane == 63) wt[wave] = ws.over(~0ull);
        __syncthreads();
        // (every thread is past its reads of slot p ^ 1, the previous
        // iteration's; and thread 0's quit flag of that iteration is read here)
        if (s_quit) break;
        if (tid == 0) { s_needy[p ^ 1u] = 0; s_moved[p ^ 1u] = 0; }
        const uint32_t cin = cont_in ? s_cin : 0u;
        // wpre: the carry is in front of the slice; own: the slice alone
        Agg wpre{0u, cin, 0u}, own{0u, 0u, 0u};
        for (int w = 0; w < kAsyncWaves; w++) {
            if (w < (int)wave) wpre = OpPlain::comb(wpre, wt[w]);
            own = OpPlain::comb(own, wt[w]);
        }
        const Agg pre = OpPlain::comb(wpre, ws.over(lanes_before(lane)));
        uint32_t lpos = pre.c, run = pre.v, moved = 0;
#pragma unroll
        for (int j = 0; j < IPT; j++) {
            if (j < cnt) {
                uint32_t ej = e[j];
                const bool head = (ej & F_HEAD) != 0;
                const uint32_t excl = head ? 0u : run;
                const uint32_t kj = (uint32_t)(keep >> j) & 1u;
                const uint32_t vj = async_value(ej, (umask >> j) & 1u, (amask >> j) & 1u, nowait) |
                                    (kj ? B_KEEP : 0u);
                if (((umask >> j) & 1u) && !(ej & F_DONE)) {
                    const uint32_t sl = (nowait && (ej & F_WR)) ? (excl & (B_CA | B_UA))
                                                                : ((excl >> 2) & (B_CA | B_UA));
                    if (sl & B_CA) {  // Abort (row_lock.cpp:86-90 / occ.cpp:219-234)
                        atomicOr(tword + r_txn(ej, slog), (uint32_t)ST_ABORT);
                        moved = 1;
                    } else if (!(sl & B_UA)) {  // permanently OK
                        atomicAdd(tword + r_txn(ej, slog), TW_OK);
                        ej |= F_DONE;
                        moved = 1;
                    }
                }
                // the slice's first element never becomes a head when a queue
                // runs in: what is in front of it arrives through the carry
                if (kj) sel[lpos++] = (ej & ~F_HEAD) | ((excl & B_KEEP) ? 0u : F_HEAD);
                run = head ? vj : (run | vj);
            }
        }
        if (moved) s_moved[p] = 1;
        // the carry word: the OR since the slice's last head (or over all of
        // it) and whether it holds a head; later slices walk back to it
        const uint32_t cout = own.v | (own.f ? kCarryHead : 0u);
        if (cont_out && tid == 0)
            __hip_atomic_store(carry + g, cout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        n = own.c;
        __syncthreads();
        if (s_needy[p] == 0 && (!cont_out || !(cout & (B_UA | B_UW)))) {  // nothing left to learn
            yielded = false;
            break;
        }
        // nothing decided here: the facts this slice waits for come from other
        // workgroups -- back off before reading them again, and yield once
        // they have not come for `idle` ticks (their producer may not be
        // resident).  Thread 0's clock decides for the workgroup; every
        // thread reads its flag after the next iteration's barrier.
        if (tid == 0) {
            const uint64_t now = wall_clock64();
            if (s_moved[p]) last_move = now;
            s_quit = now - last_move > idle;
        }
#ifdef DVCC_ASYNC_STAMPS
        {
            const uint64_t tw = wall_clock64();
            st_work += tw - st_tf;
            st_moved += s_moved[p] ? 1u : 0u;
            st_tf = tw;
        }
#endif
        if (DVCC_ASYNC_SLEEP && !s_moved[p]) __builtin_amdgcn_s_sleep(DVCC_ASYNC_SLEEP);
#ifdef DVCC_ASYNC_STAMPS
        st_sleep += wall_clock64() - st_tf;
#endif
    }
#ifdef DVCC_ASYNC_STAMPS
    if (tid == 0) {
        unsigned long long *w = g_async_stamps + (size_t)g * 8;
        atomicAdd(w + 0, 1ull);
        atomicAdd(w + 1, (unsigned long long)it + (it < max_iters ? 1u : 0u));
        atomicAdd(w + 2, (unsigned long long)(wall_clock64() - st_begin));
        atomicAdd(w + 3, (unsigned long long)st_facts);
        atomicAdd(w + 4, (unsigned long long)st_carry);
        atomicAdd(w + 5, (unsigned long long)st_work);
        atomicAdd(w + 6, (unsigned long long)st_sleep);
        atomicAdd(w + 7, (unsigned long long)st_moved);
        // the launch's mean against its maximum: the last workgroup to get
        // here adds the launch's record (every other's atomicMax is older)
        const unsigned int done_it = it + (it < max_iters ? 1u : 0u);
        atomicMax(&ctr->async_iters, it);
        atomicAdd(&g_async_lsum, done_it);
        __threadfence();
        if (atomicAdd(&g_async_launch[3], 1ull) == (unsigned long long)G - 1) {
            __threadfence();
            const unsigned int sum = atomicExch(&g_async_lsum, 0u);
            atomicAdd(&g_async_launch[0], 1ull);
            atomicAdd(&g_async_launch[1], (unsigned long long)atomicAdd(&ctr->async_iters, 0u) + 1ull);
            atomicAdd(&g_async_launch[2], (unsigned long long)sum * 1024ull / G);
            g_async_launch[3] = 0;
        }
    }
#endif
    if (tid == 0) {
        // the finalize (or, with the statuses left in the words, dv_epoch_finish)
        // hands the rest to the synchronous rounds; one yield counted per launch
        if (yielded && atomicExch(&ctr->halt, 1u) == 0u && words) {
            atomicAdd(&ctr->async_yields, 1u);
            ctr->async_block = 1u;
        }
        atomicMax(&ctr->async_iters, it);
    }
}

// narrower instantiations for small live sets (measured at config D: 1 / 4 /
// 28 elements per thread 0.565 ms per epoch, 4 / 28 0.574-0.585, 28 alone 0.615)
constexpr int kAsyncIPTTiny = 1, kAsyncIPTSmall = 4;

// after the asynchronous rounds: the status bytes from the words and the
// count of txns left undecided (an error).  The outcome goes to pub->tl
// (r0 << 32 | code, RoundPub).  A declined launch changed nothing; like a
// yielded one it halts execution (Counters::halt) and blocks further tries, and
// the host resumes the synchronous rounds at r0.
__device__ __forceinline__ void publish_try(RoundPub *pub, uint32_t r0, uint32_t code) {
    if (pub)
        __hip_atomic_store(&pub->tl, ((unsigned long long)r0 << 32) | code, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}

// fin (small epochs, words == 0): the launch's last workgroup does
// k_round_finalize's work itself -- one launch fewer per epoch, for epochs
// whose txns one workgroup writes back in a few passes (kFinTxns)
constexpr uint32_t kFinTxns = 16384;
__device__ void finalize_go(uint8_t *__restrict__ status, const uint32_t *__restrict__ tword, uint32_t n_txn,
                            uint32_t r0, RoundPub *pub, const uint32_t *__restrict__ n_txn_dev, Counters *ctr) {
    __shared__ uint32_t s_und;
    const bool yielded = __hip_atomic_load(&ctr->halt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
    if (threadIdx.x == 0) {
        s_und = 0;
        if (yielded) {
            ctr->async_yields++;
            ctr->async_block = 1u;
            publish_try(pub, r0, 3u);
        } else {
            ctr->async_r0 = r0;
            ctr->nund[r0 & 1] = 0;
            if (pub)
                __hip_atomic_store(&pub->ai, ((unsigned long long)r0 << 32) | ctr->async_iters, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
            publish_try(pub, r0, 4u);
        }
    }
    if (n_txn_dev && *n_txn_dev < n_txn) n_txn = *n_txn_dev;
    uint32_t und = 0;
    constexpr uint32_t kU = 8;  // (a thread's word loads in flight together)
    for (uint32_t t0 = 0; t0 < n_txn; t0 += kU * blockDim.x) {
        uint32_t w[kU];
#pragma unroll
        for (uint32_t u = 0; u < kU; u++) {
            const uint32_t t = t0 + u * blockDim.x + threadIdx.x;
            w[u] = t < n_txn ? __hip_atomic_load(tword + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
        }
#pragma unroll
        for (uint32_t u = 0; u < kU; u++) {
            const uint32_t t = t0 + u * blockDim.x + threadIdx.x;
            if (t < n_txn) {
                const uint8_t st = word_status(w[u]);
                status[t] = st;
                und += st == ST_UNDEC ? 1u : 0u;
            }
        }
    }
    __syncthreads();
    if (und) atomicAdd(&s_und, und);
    __syncthreads();
    if (threadIdx.x == 0 && s_und && !yielded) atomicAdd(&my_slot(ctr).undecided, s_und);
}

// words: no finalize follows (a prefix-kill stage: k_prefix_mark /
// k_sub_scatter_back read the statuses from the words); the launch then does
// the finalize's bookkeeping itself -- a declined try halts, a yield halts
// (async_slices), an accepted one records its first round (async_wr0)
__global__ __launch_bounds__(kAsyncThreads, 4) void k_round_async(RoundBufs b, const uint32_t *src,
                                                               uint32_t r0, uint32_t thresh,
                                                               uint32_t *tword, uint32_t *carry,
                                                               int nowait, uint32_t max_iters,
                                                               uint64_t idle, int words, int fin, uint32_t n_txn,
                                                               RoundPub *pub) {
    __shared__ uint32_t sel[kAsyncCap];
    __shared__ RAgg rw[kAsyncWaves];
    __shared__ Agg wt[kAsyncWaves];
    // per-iteration counters, double-buffered by iteration parity: slot p is
    // reset during the iteration before it is used, after every thread has
    // read it for the iteration before that
    __shared__ uint32_t s_needy[2], s_moved[2], s_cin, s_quit;
    Counters *ctr = b.ctr;
    const uint32_t G = gridDim.x;
    const uint32_t go = async_gate(ctr, r0, G, thresh);
    const uint32_t n_all = ctr->nlive[r0 & 1];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        ctr->async_go = go;  // for the finalize (its inputs change there)
        if (go == 1u) ctr->async_live += n_all;
        if (words && go == 1u) ctr->async_wr0 = r0;
        if ((words || fin) && go == 2u) {
            ctr->async_declined++;
            ctr->async_block = 1u;
            ctr->halt = 1u;
        }
        if (fin) publish_try(pub, r0, go == 2u ? 2u : 5u);
    }
    if (go != 1u) return;  // declined or nothing to do: the synchronous rounds go on
    const uint64_t per = ((uint64_t)n_all + G - 1) / G;  // the largest slice (uniform)
    if (per <= (uint64_t)kAsyncThreads * kAsyncIPTTiny)
        async_slices<kAsyncIPTTiny>(b, src, n_all, tword, carry, nowait, max_iters, idle, sel, rw, wt, s_needy,
                                    s_moved, s_cin, s_quit, words != 0);
    else if (per <= (uint64_t)kAsyncThreads * kAsyncIPTSmall)
        async_slices<kAsyncIPTSmall>(b, src, n_all, tword, carry, nowait, max_iters, idle, sel, rw, wt, s_needy,
                                     s_moved, s_cin, s_quit, words != 0);
    else
        async_slices<kAsyncIPT>(b, src, n_all, tword, carry, nowait, max_iters, idle, sel, rw, wt, s_needy,
                                s_moved, s_cin, s_quit, words != 0);
    if (fin) {  // the last workgroup to finish finalizes (every other's facts are published)
        __shared__ uint32_t s_last;
        __syncthreads();
        if (threadIdx.x == 0) {
            __threadfence();
            s_last = atomicAdd(&ctr->async_done, 1u) == G - 1u ? 1u : 0u;
        }
        __syncthreads();
        if (s_last) {
            __threadfence();
            finalize_go(b.status, tword, n_txn, r0, pub, b.n_txn_dev, ctr);
            if (threadIdx.x == 0) ctr->async_done = 0;
        }
    }
}

__global__ __launch_bounds__(kBlock) void k_round_finalize(uint8_t *__restrict__ status,
                                                           const uint32_t *__restrict__ tword,
                                                           uint32_t n_txn, uint32_t r0, RoundPub *pub,
                                                           const uint32_t *__restrict__ n_txn_dev,
                                                           Counters *ctr) {
    const uint32_t go = ctr->async_go;
    if (go != 1u) {
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            if (go == 2u) {
                ctr->async_declined++;
                ctr->async_block = 1u;
                ctr->halt = 1u;
            }
            publish_try(pub, r0, go == 2u ? 2u : 5u);
        }
        return;
    }
    const bool yielded = ctr->halt != 0;  // some workgroup left undecided txns behind
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (yielded) {
            // no further tries in these rounds; the round state of r0 stays as
            // it was (nund, the element array), so the host's synchronous
            // rounds resume from it with these statuses
            ctr->async_yields++;
            ctr->async_block = 1u;
            publish_try(pub, r0, 3u);
        } else {
            ctr->async_r0 = r0;
            ctr->nund[r0 & 1] = 0;  // the passes queued behind the try are no-ops
            if (pub)
                __hip_atomic_store(&pub->ai, ((unsigned long long)r0 << 32) | ctr->async_iters,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            publish_try(pub, r0, 4u);
        }
    }
    if (n_txn_dev && *n_txn_dev < n_txn) n_txn = *n_txn_dev;
    uint32_t und = 0;
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < n_txn; t += gridDim.x * blockDim.x) {
        const uint8_t s = word_status(tword[t]);
        status[t] = s;
        und += s == ST_UNDEC ? 1u : 0u;
    }
    if (und && !yielded) atomicAdd(&my_slot(ctr).undecided, und);
}


// ------------------------------------------------------------- launchers
static uint32_t txn_grid(uint32_t n_txn) {
    uint32_t g = (n_txn + kBlock - 1) / kBlock;
    return g < 1 ? 1 : (g > 1024 ? 1024 : g);
}

bool round_el32(uint32_t n_txn, uint32_t slog) {
    uint32_t tb = 0;
    while (tb < 32 && (1ull << tb) < (uint64_t)n_txn) tb++;
    return tb + slog + 3 <= 32;
}

uint32_t tail_cap(bool el32) { return el32 ? TailGeo<uint32_t>::kCap : TailGeo<uint64_t>::kCap; }

template <class E>
static void round_pass_t(hipStream_t s, const RoundBufs &b, uint32_t round, int nowait, uint32_t ub_in,
                         uint32_t tag, uint32_t ticket, bool settle, RoundPub *pub, hipEvent_t ev0,
                         hipEvent_t ev1) {
    E *out = reinterpret_cast<E *>(b.rel[round & 1]);
    const uint32_t *n_in = &b.ctr->nlive[round & 1];
    uint32_t *n_out = &b.ctr->nlive[(round + 1) & 1];
    uint32_t *tc = &b.tile_ctr[ticket % kTileCtrs];
    uint32_t *und = settle ? &b.ctr->nund[(round + 1) & 1] : nullptr;
    // the pass is a no-op once no txn is undecided: single GPU, the settle's
    // list; partitioned, the list the applies keep
    const uint32_t *und_in = !settle || round > 0 ? &b.ctr->nund[round & 1] : nullptr;
    if (round == 0) {
        using G = Geo<uint64_t>;
        const uint32_t nb = ub_in ? (ub_in + G::kTile - 1) / G::kTile : 1;
        DV_LAUNCH_EV((k_round_pass<true, uint64_t, E>), nb, G::kThreads, 0, s, ev0, ev1, b.pairs0, n_in, out, n_out, b.status, b.vb8, b.slog, nowait,
                              b.desc, tc, tag, und, (const uint32_t *)nullptr, round,
                              (RoundPub *)nullptr, b.ctr, b.n0_dev, b.n0, b.n_txn_dev, b.n_txn0);
    } else {
        using G = Geo<E>;
        const uint32_t nb = ub_in ? (ub_in + G::kTile - 1) / G::kTile : 1;
        DV_LAUNCH_EV((k_round_pass<false, E, E>), nb, G::kThreads, 0, s, ev0, ev1,
                              reinterpret_cast<const E *>(b.rel[(round - 1) & 1]), n_in, out, n_out,
                              b.status, b.vb8, b.slog, nowait, b.desc, tc, tag, und, und_in, round,
                              pub, b.ctr, (const uint32_t *)nullptr, 0u, (const uint32_t *)nullptr, 0u);
    }
}

void round_pass(hipStream_t s, const RoundBufs &b, uint32_t round, int nowait, uint32_t ub_in,
                uint32_t tag, uint32_t ticket, bool settle, RoundPub *pub, hipEvent_t ev0,
                hipEvent_t ev1) {
    if (b.el32) round_pass_t<uint32_t>(s, b, round, nowait, ub_in, tag, ticket, settle, pub, ev0, ev1);
    else round_pass_t<uint64_t>(s, b, round, nowait, ub_in, tag, ticket, settle, pub, ev0, ev1);
}

void round_tail(hipStream_t s, const RoundBufs &b, uint32_t r0, int nowait, RoundPub *pub) {
    if (b.el32) DV_LAUNCH((k_round_tail<uint32_t>), 1, kTailThreads, 0, s, b, r0, nowait, pub);
    else DV_LAUNCH((k_round_tail<uint64_t>), 1, kTailThreads, 0, s, b, r0, nowait, pub);
}

void round_async(hipStream_t s, const RoundBufs &b, uint32_t r0, int nowait, uint32_t G, uint32_t thresh,
                 uint32_t *carry, uint32_t *tword, uint32_t n_txn, RoundPub *pub, uint32_t max_iters,
                 uint64_t idle_ticks, bool words_done, bool words) {
    const uint32_t *src = reinterpret_cast<const uint32_t *>(b.rel[(r0 - 1) & 1]);
    if (!words_done)  // (else round 0's settle wrote them: round_settle with tword)
        DV_LAUNCH(k_async_words, txn_grid(n_txn > G ? n_txn : G), kBlock, 0, s, b.status, b.vb8, b.slog, b.tlen,
                                                                    n_txn, tword, carry, G, thresh, r0,
                                                                    b.n_txn_dev, b.ctr);
    const bool fin = !words && n_txn <= kFinTxns;  // (the last workgroup finalizes)
    DV_LAUNCH(k_round_async, G, kAsyncThreads, 0, s, b, src, r0, thresh, tword, carry, nowait, max_iters, idle_ticks,
              words ? 1 : 0, fin ? 1 : 0, n_txn, pub);
    if (!words && !fin)
        DV_LAUNCH(k_round_finalize, txn_grid(n_txn), kBlock, 0, s, b.status, tword, n_txn, r0, pub, b.n_txn_dev,
                  b.ctr);
}

// Every workgroup of the asynchronous launch must be resident at once (one
// may wait for facts only another produces): at most what the occupancy
// calculator admits on every CU of the device.
uint32_t async_groups(int device) {
    int cus = 0, per = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_round_async, kAsyncThreads, 0) !=
            hipSuccess)
        return 0;
    const uint64_t g = (uint64_t)cus * (uint64_t)per;
    return (uint32_t)(g < kAsyncGroups ? g : kAsyncGroups);
}

uint32_t async_try_limit(uint32_t G) { return G * kAsyncCap; }

#ifdef DVCC_ASYNC_STAMPS
// measurement builds: the stamps (kAsyncGroups x 8 words) copied out and reset
extern "C" int dv_debug_async_stamps(uint64_t *out, uint32_t n) {
    if (!out || n > kAsyncGroups * 8) return DV_ERR_ARG;
    if (hipDeviceSynchronize() != hipSuccess) return DV_ERR_HIP;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_async_stamps), n * 8) != hipSuccess) return DV_ERR_HIP;
    static const unsigned long long zero[kAsyncGroups * 8] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_async_stamps), zero, sizeof(zero)) != hipSuccess) return DV_ERR_HIP;
    return DV_OK;
}
// ... and the per-launch record (4 words), reset
extern "C" int dv_debug_async_launches(uint64_t *out) {
    if (!out) return DV_ERR_ARG;
    if (hipDeviceSynchronize() != hipSuccess) return DV_ERR_HIP;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_async_launch), 4 * 8) != hipSuccess) return DV_ERR_HIP;
    static const unsigned long long zero[4] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_async_launch), zero, sizeof(zero)) != hipSuccess) return DV_ERR_HIP;
    return DV_OK;
}
#endif

void round_settle(hipStream_t s, const RoundBufs &b, uint32_t round, uint32_t n_txn, uint32_t ub, uint32_t *tword,
                  uint32_t *carry, uint32_t G) {
    const uint32_t n = round == 0 ? n_txn : (ub < n_txn ? ub : n_txn);
    const uint32_t nb = n ? (n + kSettleChunk - 1) / kSettleChunk : 1;
    uint32_t *n_out = &b.ctr->nund[(round + 1) & 1];
    if (round == 0)
        DV_LAUNCH((k_round_settle<true>), nb, kBlock, 0, s, b.status, b.vb8, b.slog, b.tlen, nullptr, &b.ctr->nund[0],
                                                   n_txn, b.ulist[1], n_out, tword, carry, G);
    else
        DV_LAUNCH((k_round_settle<false>), nb, kBlock, 0, s, b.status, b.vb8, b.slog, b.tlen,
                                                    b.ulist[round & 1], &b.ctr->nund[round & 1],
                                                    n_txn, b.ulist[(round + 1) & 1], n_out, nullptr, nullptr, 0u);
}

void list_verdict(hipStream_t s, const RoundBufs &b, uint32_t round, uint32_t ub, uint8_t *verdict) {
    const uint32_t *list = round == 0 ? nullptr : b.ulist[round & 1];
    DV_LAUNCH(k_list_verdict, txn_grid(ub), kBlock, 0, s, list, &b.ctr->nund[round & 1], b.status, b.vb8,
                                                  b.slog, b.tlen, verdict);
}

void list_apply(hipStream_t s, const RoundBufs &b, uint32_t round, uint32_t ub, const uint8_t *verdict,
                uint32_t tag, uint32_t *tile_ctr, RoundPub *pub) {
    const uint32_t *list = round == 0 ? nullptr : b.ulist[round & 1];
    const uint32_t nb = ub ? (ub + kRTile - 1) / kRTile : 1;
    DV_LAUNCH(k_list_apply, nb, kBlock, 0, s, list, &b.ctr->nund[round & 1], verdict, b.status,
                                       b.ulist[(round + 1) & 1], &b.ctr->nund[(round + 1) & 1],
                                       &b.ctr->nlive[(round + 1) & 1], b.desc, tile_ctr, tag, round, pub,
                                       b.ctr);
}

}  // namespace dvcc
