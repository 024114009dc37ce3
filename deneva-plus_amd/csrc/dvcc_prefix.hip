// dvcc_prefix.hip -- prefix-kill decisions for large single-GPU epochs (gfx950).
//
// The E-schedule's decisions are the sequence-ordered greedy:
// txn i commits iff no earlier COMMITTED txn conflicts with it.  Restricted to
// a prefix T_0..T_{K-1} of the epoch it is the same greedy, so the prefix can
// be decided on its own.  After that, a later txn that conflicts with a
// committed prefix txn aborts, whatever else happens -- and at zipf 0.9 the
// prefix's commits hold the hot rows: deciding the first 16K txns of a
// 1M-txn config-D epoch kills ~91 % of the rest.  The survivors' fate
// depends only on each other (a killed txn blocks nobody), so they form a
// sub-epoch decided by the same rounds, over ~9 % of the accesses.  The
// runtime (dvcc_runtime.hip, run_prefix_epoch) therefore runs
//     probe (sort keys for the prefix only) -> sort + rounds on the prefix ->
//     k_prefix_mark -> k_kill -> k_kill_compact ->
//     sort + rounds on the survivors -> k_sub_scatter_back -> execution,
// instead of sorting and scanning every access of the epoch round after round.
//
// Row state of the prefix's committed txns: a bitmap of 2 bits per row of the
// context (16 rows per 32-bit word; config D's 16.8M rows take 4 MiB, one
// XCD's L2), cleared before every prefix epoch:
//   bit 1  a committed txn writes the row
//   bit 0  (NO_WAIT / WAIT_DIE) a committed txn reads it
// A later access conflicts with it exactly as Row_lock::lock_get's
// conflict_lock would with the committed owners (row_lock.cpp:69, 86-90): a
// write meets either bit, a read meets bit 1; OCC's central validation
// (occ.cpp:185-199) kills any access to a row an earlier committed txn writes.
// NO_WAIT / WAIT_DIE: every surviving access to a row in state 01 (read by a
// committed prefix txn, written by none) reads it -- a write there is killed
// -- so it conflicts with no other survivor and blocks none: the survivors'
// sub-epoch leaves such accesses out (k_kill's skip bits), their txns wait
// only for the rest.  At config D these are the hot rows' readers, about
// half of the survivors' accesses.
#include <algorithm>

#include "dvcc_common.h"

namespace dvcc {

namespace {
#ifndef DVCC_KILL_IPT
#define DVCC_KILL_IPT 2  // (4: k_kill_count 8.1 / k_kill_emit 19.5 us; 2: 6.5 / 18.2; 1: 7.7 / 27.8 -- profiles/r05_ah)
#endif
constexpr int kKillIPT = DVCC_KILL_IPT;                 // txns per thread in k_kill_compact
constexpr uint32_t kKillTile = kBlock * kKillIPT;       // txns per tile
constexpr uint32_t RS_RD = 1u, RS_WR = 2u;

__device__ __forceinline__ uint32_t row_bits(const uint32_t *rs, uint32_t row) {
    return (rs[row >> 4] >> ((row & 15u) * 2u)) & 3u;
}
}  // namespace

// k_kill's LDS copies, so that a later access gathers a bitmap word from L2
// only when it must -- 10.3M gathers at config D were bound by the L2's
// request rate (26 of k_kill's 39 us):
//   the bitmap words of rows [0, kHotRows): zipf's hot rows are the small
//     keys, so over half of the accesses (top 64K of 16.8M rows) read LDS;
//   a one-hash Bloom filter (kBloomBits) of the marked rows from kHotRows on,
//     kept right after the bitmap and cleared with it: a cold access to a row
//     no committed prefix txn touched reads LDS only.
// 16 KiB of hot words + 128 KiB of filter: a filter twice as large took
// k_kill from 28.0 to 25.3 us at config D (fewer false positives, each an L2
// gather; 2^16 or 2^17 hot rows beside it, the same), and a filter half as
// large cost 1.8 us more (tools/kstat_ab.sh).
#ifndef DVCC_HOT_LOG
#define DVCC_HOT_LOG 16
#endif
#ifndef DVCC_BLOOM_LOG
#define DVCC_BLOOM_LOG 20
#endif
constexpr uint32_t kHotRows = 1u << DVCC_HOT_LOG, kHotWords = kHotRows / 16;
constexpr uint32_t kBloomBits = 1u << DVCC_BLOOM_LOG, kBloomWords = kBloomBits / 32;
// k_kill stages both in LDS: gfx950 gives a workgroup 160 KiB (a target with
// less, e.g. gfx942's 64 KiB, needs smaller DVCC_HOT_LOG / DVCC_BLOOM_LOG)
static_assert((kHotWords + kBloomWords) * sizeof(uint32_t) <= 160u * 1024u,
              "k_kill's hot row words + Bloom filter exceed gfx950's 160 KiB of LDS per workgroup");
__device__ __forceinline__ uint32_t bloom_bit(uint32_t row) { return (row * 0x9E3779B1u) >> (32 - DVCC_BLOOM_LOG); }

// (a multiple of 4 words: k_epoch_clear zeroes it in 16-byte stores)
uint64_t row_state_words(uint64_t rows) { return (((rows + 15) / 16 + 3) & ~3ull) + kBloomWords; }

// the rows of the committed prefix txns into the bitmap; lane per txn, its
// accesses from the probe's txn-major acc_row.  The hot rows [0, kHotRows)
// -- which many committed readers share -- are ORed into an LDS copy of
// their bitmap words first, then each nonzero word into the bitmap with one
// atomic per block (one device-scope atomic per access on a shared word ran
// at ~88 per us); other rows go straight to the bitmap and the Bloom filter.
#ifndef DVCC_MARK_BLOCK
#define DVCC_MARK_BLOCK 512  // (threads per block: 1024 9.0 us, 512 6.9, 256 9.2 -- profiles/r05_ah)
#endif
constexpr int kMarkBlock = DVCC_MARK_BLOCK;  // (16 KiB of LDS per block)
__global__ __launch_bounds__(kMarkBlock) void k_prefix_mark(uint8_t *__restrict__ status,
                                                            const uint32_t *__restrict__ tb_start,
                                                            const uint32_t *__restrict__ tb_end,
                                                            const uint32_t *__restrict__ acc_row, uint32_t K,
                                                            uint32_t *__restrict__ row_state, uint64_t state_words,
                                                            uint32_t *__restrict__ bloom, int nowait,
                                                            Counters *__restrict__ ctr,
                                                            const uint32_t *__restrict__ words) {
    __shared__ uint32_t s_hot[kHotWords];
    if (input_err(ctr)) return;
    // queued behind the prefix's rounds with no host wait: when they halted
    // (a yielded or declined asynchronous try) nothing after this runs -- the
    // kill, the compaction, the survivors' stage and the execution all read
    // halt -- and dv_epoch_finish decides the prefix again synchronously
    if (ctr->halt) {
        if (blockIdx.x == 0 && threadIdx.x == 0) ctr->a_halt = 1u;
        return;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // (round 0, then the asynchronous iterations)
        const uint32_t r0 = ctr->async_wr0 ? ctr->async_wr0 : ctr->async_r0;
        ctr->a_rounds = r0 ? r0 + ctr->async_iters : 1u;
    }
    for (uint32_t i = threadIdx.x; i < kHotWords; i += kMarkBlock) s_hot[i] = 0;
    __syncthreads();
    uint32_t und = 0;
    for (uint32_t t = blockIdx.x * kMarkBlock + threadIdx.x; t < K; t += gridDim.x * kMarkBlock) {
        if (words) {  // the asynchronous launch's statuses: the status bytes from the fact words
            const uint8_t st = word_status(words[t]);
            status[t] = st;
            und += st == ST_UNDEC ? 1u : 0u;
            if (st != ST_COMMIT) continue;
        } else if (status[t] != ST_COMMIT) {
            continue;
        }
        // (a chunk's row words loaded before any of its atomics)
        constexpr uint32_t kMU = 8;
        for (uint32_t a0 = tb_start[t], e = tb_end[t]; a0 < e; a0 += kMU) {
            uint32_t arw[kMU];
#pragma unroll
            for (uint32_t u = 0; u < kMU; u++) arw[u] = a0 + u < e ? acc_row[a0 + u] : 0u;
#pragma unroll
            for (uint32_t u = 0; u < kMU; u++) {
                if (a0 + u >= e) continue;
                const uint32_t ar = arw[u];
                const uint32_t row = ar & ~AR_WR;
                const uint32_t bit = (ar & AR_WR) ? RS_WR : (nowait ? RS_RD : 0u);
                if (!bit) continue;
                if (row < kHotRows) {
                    atomicOr(&s_hot[row >> 4], bit << ((row & 15u) * 2u));
                } else {
                    atomicOr(&row_state[row >> 4], bit << ((row & 15u) * 2u));
                    const uint32_t h = bloom_bit(row);
                    atomicOr(&bloom[h >> 5], 1u << (h & 31u));
                }
            }
        }
    }
    if (und) {  // cannot happen: the asynchronous launch decided every txn or yielded (halt)
        set_err(ctr, ERRB_SPIN);
        atomicMax(&ctr->spin_site, 2u);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < kHotWords && i < state_words; i += kMarkBlock) {
        const uint32_t w = s_hot[i];
        if (w) atomicOr(&row_state[i], w);
    }
}

// Every access after the prefix's (index >= ctr->a_acc) against the row
// state, one bit per access: 64 consecutive accesses per wave step, the
// txn-major acc_row streamed (4 B per access), one bitmap word gathered per
// access, and the wave's verdicts stored as one ballot word -- k_kill_compact
// then ORs each txn's range of bits.  (The conflict rule is the one in the
// header comment; the txn id of an access is never needed here.)
#ifndef DVCC_KILL_WORDS
#define DVCC_KILL_WORDS 8
#endif
constexpr int kKillWords = DVCC_KILL_WORDS;  // ballot words per wave per step (loads in flight)
constexpr int kKillBlock = 1024;  // one block per CU (144 KiB of LDS): 16 waves to stream with
// KEYS (an epoch with its txn boundaries, launch_probe_tb): the later
// accesses were never probed -- their rows come from their keys here (the
// dense YCSB map: arithmetic only), 9 bytes read per access instead of the
// probe's 17 plus this pass's 4; a missing key rejects the epoch (ERRB_KEY)
template <int KEYS>  // 0: acc_row; 1: keys, probed; 2: keys of a dense map (KillKeys::dense_lim)
__global__ __launch_bounds__(kKillBlock) void k_kill(const uint32_t *__restrict__ acc_row, uint64_t n,
                                                 const uint32_t *__restrict__ n_dev,
                                                 const uint32_t *__restrict__ row_state, uint64_t state_words,
                                                 const uint32_t *__restrict__ bloom, int nowait,
                                                 uint64_t *__restrict__ kill_bits, uint64_t *__restrict__ skip_bits,
                                                 Counters *__restrict__ ctr, KillKeys kk) {
    __shared__ __align__(16) uint32_t s_lds[kHotWords + kBloomWords];
    uint32_t *const s_hot = s_lds, *const s_bloom = s_lds + kHotWords;
    if (input_err(ctr) || ctr->halt) return;
    if (n_dev && (uint64_t)*n_dev < n) n = *n_dev;  // (rows past the real count were never probed)
    {
        // the 144 KiB in 16-byte loads, all of a thread's in flight before its
        // first LDS store (a load-store loop waited out one L2 round trip per
        // 4 KiB); the bitmap part and the filter are multiples of 4 words
        constexpr uint32_t kH4 = kHotWords / 4, kAll4 = (kHotWords + kBloomWords) / 4;
        static_assert(kAll4 % kKillBlock == 0, "k_kill's LDS fill: whole 16-byte steps per thread");
        constexpr uint32_t kSteps = kAll4 / kKillBlock;
        const uint32_t sw4 = (uint32_t)(state_words / 4 < kH4 ? state_words / 4 : kH4);
        const uint4 *hot4 = reinterpret_cast<const uint4 *>(row_state);
        const uint4 *blm4 = reinterpret_cast<const uint4 *>(bloom);
        uint4 v[kSteps];
#pragma unroll
        for (uint32_t k = 0; k < kSteps; k++) {
            const uint32_t i = k * kKillBlock + threadIdx.x;
            v[k] = i < kH4 ? (i < sw4 ? hot4[i] : make_uint4(0u, 0u, 0u, 0u)) : blm4[i - kH4];
        }
        uint4 *dst = reinterpret_cast<uint4 *>(s_lds);
#pragma unroll
        for (uint32_t k = 0; k < kSteps; k++) dst[k * kKillBlock + threadIdx.x] = v[k];
    }
    __syncthreads();
    const uint64_t first = ctr->a_acc;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t w0 = first >> 6, nw = (n + 63) >> 6;
    const uint64_t waves = (uint64_t)gridDim.x * (kKillBlock / 64);
    const uint64_t wstep = waves * kKillWords;
    // the state words of a step's accesses -- LDS (hot rows; the filter) or, a
    // filter hit, the bitmap word from L2, all of the step's gathers in flight
    // together -- then the verdicts
    auto states = [&](const uint32_t *ar, uint32_t *sw) {
#pragma unroll
        for (int q = 0; q < kKillWords; q++) {
            sw[q] = 0;
            if (ar[q] != ~0u) {
                const uint32_t row = ar[q] & ~AR_WR;
                if (row < kHotRows) {
                    sw[q] = s_hot[row >> 4];
                } else {
                    const uint32_t h = bloom_bit(row);
                    if ((s_bloom[h >> 5] >> (h & 31u)) & 1u) sw[q] = row_state[row >> 4];  // maybe marked
                }
            }
        }
    };
    auto verdicts = [&](uint64_t w, const uint32_t *ar, const uint32_t *sw) {
#pragma unroll
        for (int q = 0; q < kKillWords; q++) {
            bool kill = false, skip = false;
            if (ar[q] != ~0u) {
                const uint32_t row = ar[q] & ~AR_WR;
                const uint32_t st = (sw[q] >> ((row & 15u) * 2u)) & 3u;
                kill = (st & RS_WR) || (nowait && st && (ar[q] & AR_WR));
                skip = st == RS_RD && !(ar[q] & AR_WR);  // (nowait only: skip_bits is null for OCC)
            }
            const uint64_t m = __ballot(kill), sm = __ballot(skip);
            if (lane == 0 && w + q < nw) {
                kill_bits[w + q] = m;
                if (skip_bits) skip_bits[w + q] = sm;
            }
        }
    };
    const uint64_t wbeg = w0 + ((uint64_t)blockIdx.x * (kKillBlock / 64) + (threadIdx.x >> 6)) * kKillWords;
    if (KEYS == 0 || (KEYS == 2 && kk.recs)) {
        // one 4-byte word per access (acc_row, or the dense map's records):
        // software-pipelined -- the next step's words are loaded behind this
        // step's gathers, so the stream's latency overlaps the verdicts
        const uint32_t *src = KEYS == 0 ? acc_row : kk.recs;
        uint32_t nxt[kKillWords];
        auto load = [&](uint64_t w) {
#pragma unroll
            for (int q = 0; q < kKillWords; q++) {
                const uint64_t i = ((w + q) << 6) + lane;
                nxt[q] = w < nw && i >= first && i < n ? src[i] : ~0u;
            }
        };
        load(wbeg);
        for (uint64_t w = wbeg; w < nw; w += wstep) {
            uint32_t ar[kKillWords], sw[kKillWords];
#pragma unroll
            for (int q = 0; q < kKillWords; q++) {
                ar[q] = nxt[q];
                if constexpr (KEYS == 2) {  // key | wr << 31 -> row | AR_WR (a missing key rejects the epoch)
                    const uint64_t i = ((w + q) << 6) + lane;
                    if (i >= first && i < n) {
                        const uint32_t key = nxt[q] & 0x7FFFFFFFu;
                        if (key < kk.dense_lim) {
                            ar[q] = (uint32_t)(key + kk.dense_base) | (nxt[q] & AR_WR);
                        } else {
                            set_err(ctr, ERRB_KEY);
                            ar[q] = ~0u;
                        }
                    } else {
                        ar[q] = ~0u;
                    }
                }
            }
            states(ar, sw);
            load(w + wstep);
            verdicts(w, ar, sw);
        }
        return;
    }
    for (uint64_t w = wbeg; w < nw; w += wstep) {
        uint32_t ar[kKillWords], sw[kKillWords];
        if constexpr (KEYS != 0) {
            uint64_t key[kKillWords];
            uint32_t wr[kKillWords];
            bool in[kKillWords];
#pragma unroll
            for (int q = 0; q < kKillWords; q++) {
                const uint64_t i = ((w + q) << 6) + lane;
                in[q] = i >= first && i < n;
                wr[q] = 0;
                key[q] = in[q] ? kk_key(kk, i, wr[q]) : 0ull;
            }
#pragma unroll
            for (int q = 0; q < kKillWords; q++) {
                uint64_t row = 0;
                ar[q] = ~0u;
                if (in[q] && kk_row<KEYS == 2>(kk, key[q], row, ctr))
                    ar[q] = (uint32_t)row | (wr[q] ? AR_WR : 0u);
            }
        }
        states(ar, sw);
        verdicts(w, ar, sw);
    }
}

// any kill bit in accesses [a0, a1): the first and last words loaded
// unconditionally (a txn spans at most 3 words), so the callers' unrolled
// loops keep every txn's loads in flight together
__device__ __forceinline__ bool range_killed(const uint64_t *__restrict__ kill_bits, uint32_t a0, uint32_t a1) {
    if (a0 >= a1) return false;
    const uint32_t wlo = a0 >> 6, whi = (a1 - 1) >> 6;
    uint64_t lo = kill_bits[wlo], hi = kill_bits[whi];
    lo &= ~0ull << (a0 & 63);
    hi &= ~0ull >> (63 - ((a1 - 1) & 63));
    if (wlo == whi) return (lo & hi) != 0;
    bool k = (lo | hi) != 0;
    for (uint32_t w = wlo + 1; w < whi; w++) k |= kill_bits[w] != 0;
    return k;
}

// set bits of `bits` in [a0, a1)
__device__ __forceinline__ uint32_t range_count(const uint64_t *__restrict__ bits, uint32_t a0, uint32_t a1) {
    if (a0 >= a1) return 0u;
    const uint32_t wlo = a0 >> 6, whi = (a1 - 1) >> 6;
    uint64_t lo = bits[wlo] & (~0ull << (a0 & 63));
    const uint64_t hmask = ~0ull >> (63 - ((a1 - 1) & 63));
    if (wlo == whi) return (uint32_t)__popcll(lo & hmask);
    uint32_t c = (uint32_t)__popcll(lo) + (uint32_t)__popcll(bits[whi] & hmask);
    for (uint32_t w = wlo + 1; w < whi; w++) c += (uint32_t)__popcll(bits[w]);
    return c;
}

// the index of the r-th access from a0 on whose skip bit is clear (the
// caller knows there is one)
__device__ __forceinline__ uint32_t nth_kept(const uint64_t *__restrict__ skip, uint32_t a0, uint32_t r) {
    uint32_t w = a0 >> 6;
    uint64_t m = ~skip[w] & (~0ull << (a0 & 63));
    for (uint32_t c = (uint32_t)__popcll(m); r >= c; c = (uint32_t)__popcll(m)) {
        r -= c;
        m = ~skip[++w];
    }
    for (; r; r--) m &= m - 1;
    return (w << 6) + (uint32_t)__builtin_ctzll(m);
}

// Txns [K, n_txn) after k_kill: a txn with a kill bit in its access range
// aborts (status byte), the others -- survivors -- are renumbered
// 0..S-1 in sequence order -- map[sub] = txn, tlen_b[sub] = its accesses
// without the skipped ones (skip_bits: NO_WAIT / WAIT_DIE, header) -- and
// their sort keys written densely in that order, pairs_b = row << 32 |
// sub << 8 | pos << 1 | wr, pos numbering the txn's accesses left in.  Two
// launches over tiles of kKillTile txns:
//   k_kill_count: the tile's txns checked block-strided (coalesced access
//     ranges and status stores, every txn's kill words in flight together),
//     one info word per txn (survivor: its length | 1 << 31) and the tile's
//     survivor and access counts;
//   k_kill_emit: each tile sums the counts of the tiles before it (plain
//     loads behind the kernel boundary), ranks its survivors, lists them in
//     LDS and writes their accesses with the whole block, one access per
//     thread.  The last tile publishes S and the access count (b_txn, b_acc).
// (One launch with decoupled look-backs for the tile offsets took 33 us at
// config D: the look-backs' cross-CU hand-offs cost more than the boundary.)
__global__ __launch_bounds__(kBlock) void k_kill_count(const uint32_t *__restrict__ tb_start,
                                                       const uint32_t *__restrict__ tb_end, uint32_t K,
                                                       uint32_t n_txn, const uint64_t *__restrict__ kill_bits,
                                                       const uint64_t *__restrict__ skip_bits,
                                                       uint8_t *__restrict__ status, uint32_t *__restrict__ info,
                                                       uint32_t *__restrict__ tsum, const Counters *ctr) {
    __shared__ uint32_t lds4[4];
    const uint32_t m = n_txn > K ? n_txn - K : 0u;
    const uint32_t ntiles = (m + kKillTile - 1) / kKillTile;
    if (blockIdx.x >= ntiles || input_err(ctr) || ctr->halt) return;
    const uint32_t tid = threadIdx.x;
    const uint32_t t_lo = K + blockIdx.x * kKillTile;
    uint32_t a0[kKillIPT], a1[kKillIPT];
#pragma unroll
    for (int j = 0; j < kKillIPT; j++) {
        const uint32_t t = t_lo + j * kBlock + tid;
        a0[j] = t < n_txn ? tb_start[t] : 0u;
        a1[j] = t < n_txn ? tb_end[t] : 0u;
    }
    uint32_t cnt = 0, acc = 0;
#pragma unroll
    for (int j = 0; j < kKillIPT; j++) {
        const uint32_t t = t_lo + j * kBlock + tid;
        if (t >= n_txn) continue;
        // a committed prefix txn holds one of its rows
        const bool killed = range_killed(kill_bits, a0[j], a1[j]);
        if (killed) status[t] = ST_ABORT;
        const uint32_t len = killed ? 0u : a1[j] - a0[j] - (skip_bits ? range_count(skip_bits, a0[j], a1[j]) : 0u);
        info[t - K] = killed ? 0u : len | 0x80000000u;
        cnt += killed ? 0u : 1u;
        acc += len;
    }
    uint32_t tc = 0, ta = 0;
    (void)block_excl_scan256(cnt, lds4, &tc);
    (void)block_excl_scan256(acc, lds4, &ta);
    if (tid == 0) {
        tsum[2 * blockIdx.x] = tc;
        tsum[2 * blockIdx.x + 1] = ta;
    }
}

// KEYS (launch_probe_tb epochs): the survivors' accesses were never probed --
// their rows come from their keys here: their sort keys, and acc_row for every
// access of a survivor (the execution's, the skipped reads' included)
template <int KEYS>  // as k_kill
__global__ __launch_bounds__(kBlock) void k_kill_emit(
    const uint32_t *__restrict__ tb_start, const uint32_t *__restrict__ tb_end, uint32_t *__restrict__ acc_row,
    uint32_t K, uint32_t n_txn,
    const uint64_t *__restrict__ skip_bits, const uint32_t *__restrict__ info, const uint32_t *__restrict__ tsum,
    uint32_t *__restrict__ map,
    uint8_t *__restrict__ status_b, uint8_t *__restrict__ tlen_b, uint64_t *__restrict__ pairs_b, Counters *ctr,
    KillKeys kk, const uint32_t *__restrict__ row_state, int nowait) {
    __shared__ Agg wt_c[kBlock / 64], wt_a[kBlock / 64], wt_f[kBlock / 64];
    __shared__ uint32_t s_sub0, s_ab0, s_nsurv, s_nacc, s_nfull;
    __shared__ uint32_t l_a0[kKillTile], l_pre[kKillTile + 1];  // per survivor: first access, access prefix
    __shared__ uint32_t l_st[kKillTile], l_len[kKillTile];      // per tile txn: first access, info word
    // KEYS: per tile txn its end; per survivor the prefix of its whole length
    // and its skipped accesses (bit j: access j reads a row only committed
    // prefix readers hold, k_kill's skip rule)
    __shared__ uint32_t l_end[KEYS ? kKillTile : 1], l_fpre[KEYS ? kKillTile + 1 : 1];
    __shared__ uint32_t l_skip[KEYS ? kKillTile : 1];
    const uint32_t m = n_txn > K ? n_txn - K : 0u;
    const uint32_t ntiles = (m + kKillTile - 1) / kKillTile;
    if (blockIdx.x >= ntiles || input_err(ctr) || ctr->halt) return;  // (b_txn = b_acc = 0 from the epoch clear)
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t tile = blockIdx.x;
    const uint32_t t_lo = K + tile * kKillTile;
#pragma unroll
    for (int j = 0; j < kKillIPT; j++) {
        const uint32_t t = t_lo + j * kBlock + tid;
        l_st[j * kBlock + tid] = t < n_txn ? tb_start[t] : 0u;
        l_len[j * kBlock + tid] = t < n_txn ? info[t - K] : 0u;
        if constexpr (KEYS) l_end[j * kBlock + tid] = t < n_txn ? tb_end[t] : 0u;
    }
    if (wave < 2) {  // the tiles before this one: wave 0 survivors, wave 1 their accesses
        uint32_t sum = 0;
        // (8 loads per lane in flight at once: a late tile sums ~1,000 earlier ones)
        for (uint32_t q0 = 0; q0 < tile; q0 += 8 * 64) {
            uint32_t v[8];
#pragma unroll
            for (uint32_t u = 0; u < 8; u++) {
                const uint32_t q = q0 + u * 64 + lane;
                v[u] = q < tile ? tsum[2 * q + wave] : 0u;
            }
#pragma unroll
            for (uint32_t u = 0; u < 8; u++) sum += v[u];
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off, 64);
        if (lane == 0) {
            (wave == 0 ? s_sub0 : s_ab0) = sum;
            if (tile == ntiles - 1) (wave == 0 ? ctr->b_txn : ctr->b_acc) = sum + tsum[2 * tile + wave];
        }
    }
    __syncthreads();
    const uint32_t first = t_lo + tid * kKillIPT;
    uint32_t surv = 0, cnt = 0, acc = 0, full = 0;
    uint32_t a0s[kKillIPT], lens[kKillIPT], fls[kKillIPT];
#pragma unroll
    for (int j = 0; j < kKillIPT; j++) {
        const uint32_t w = l_len[tid * kKillIPT + j];
        a0s[j] = l_st[tid * kKillIPT + j];
        lens[j] = w & 0x7FFFFFFFu;
        fls[j] = KEYS ? l_end[tid * kKillIPT + j] - a0s[j] : 0u;
        if (!w) continue;
        surv |= 1u << j;
        cnt++;
        acc += lens[j];
        full += fls[j];
    }
    const Agg inc_c = wave_incl<OpPlain>(Agg{0u, 0u, cnt}, lane);
    const Agg inc_a = wave_incl<OpPlain>(Agg{0u, 0u, acc}, lane);
    const Agg inc_f = KEYS ? wave_incl<OpPlain>(Agg{0u, 0u, full}, lane) : Agg{0u, 0u, 0u};
    if (lane == 63) {
        wt_c[wave] = inc_c;
        wt_a[wave] = inc_a;
        wt_f[wave] = inc_f;
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t c = 0, a = 0, f = 0;
        for (int w = 0; w < kBlock / 64; w++) {
            c += wt_c[w].c;
            a += wt_a[w].c;
            f += wt_f[w].c;
        }
        s_nsurv = c;
        s_nacc = a;
        s_nfull = f;
    }
    // this thread's survivors: their slots in the tile's list
    uint32_t ls = 0, la = 0, lf = 0;
    for (uint32_t w = 0; w < wave; w++) {
        ls += wt_c[w].c;
        la += wt_a[w].c;
        lf += wt_f[w].c;
    }
    ls += wave_excl_from_incl<OpPlain>(inc_c, lane).c;
    la += wave_excl_from_incl<OpPlain>(inc_a, lane).c;
    if constexpr (KEYS) lf += wave_excl_from_incl<OpPlain>(inc_f, lane).c;
    __syncthreads();
    const uint32_t sub0 = s_sub0;
#pragma unroll
    for (int j = 0; j < kKillIPT; j++) {
        if (!((surv >> j) & 1u)) continue;
        const uint32_t sub = sub0 + ls;
        map[sub] = first + j;
        tlen_b[sub] = (uint8_t)lens[j];
        status_b[sub] = ST_UNDEC;
        l_a0[ls] = a0s[j];
        l_pre[ls] = la;
        if constexpr (KEYS) {
            l_fpre[ls] = lf;
            l_skip[ls] = 0;
        }
        la += lens[j];
        lf += fls[j];
        ls++;
    }
    if (tid == 0) {
        l_pre[s_nsurv] = s_nacc;
        if constexpr (KEYS) l_fpre[s_nsurv] = s_nfull;
    }
    __syncthreads();
    if constexpr (KEYS) {
        // every access of every survivor, one per thread: its acc_row word for
        // the execution (the skipped reads' included), the key probed here
        constexpr uint32_t kU = 4;
        const uint32_t ns = s_nsurv, nf = s_nfull;
        for (uint32_t g0 = 0; g0 < nf; g0 += kBlock * kU) {
            uint32_t a[kU], wr[kU];
            uint64_t key[kU];
#pragma unroll
            for (uint32_t u = 0; u < kU; u++) {
                const uint32_t g = g0 + u * kBlock + tid;
                uint32_t lo = 0, hi = ns;  // largest k with l_fpre[k] <= g
                while (hi - lo > 1) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (l_fpre[mid] <= g) lo = mid;
                    else hi = mid;
                }
                a[u] = l_a0[lo] + (g - l_fpre[lo]);
                wr[u] = 0;
                key[u] = g < nf ? kk_key(kk, a[u], wr[u]) : 0ull;
            }
            uint32_t rows[kU];
#pragma unroll
            for (uint32_t u = 0; u < kU; u++) {
                uint64_t row = 0;
                if (g0 + u * kBlock + tid < nf)
                    kk_row<KEYS == 2>(kk, key[u], row, ctr);  // (the kill found every key)
                rows[u] = (uint32_t)row;
            }
#pragma unroll
            for (uint32_t u = 0; u < kU; u++) {
                const uint32_t g = g0 + u * kBlock + tid;
                if (g >= nf) continue;
                acc_row[a[u]] = rows[u] | (wr[u] ? AR_WR : 0u);
                // the skip rule: k_kill's bit for this access (one 64-bit word
                // per 64 consecutive accesses), not a second gather of the row
                // state's random word
#ifdef DVCC_EMIT_ROW_STATE
                const bool skip = nowait && !wr[u] && row_bits(row_state, rows[u]) == RS_RD;
#else
                const bool skip = skip_bits && ((skip_bits[a[u] >> 6] >> (a[u] & 63u)) & 1ull) != 0;
#endif
                if (skip) {
                    uint32_t lo = 0, hi = ns;
                    while (hi - lo > 1) {
                        const uint32_t mid = (lo + hi) >> 1;
                        if (l_fpre[mid] <= g) lo = mid;
                        else hi = mid;
                    }
                    // (one word holds a survivor of <= 32 accesses; a longer
                    // one takes its kept accesses from k_kill's skip_bits)
                    if (l_fpre[lo + 1] - l_fpre[lo] <= 32u) atomicOr(&l_skip[lo], 1u << (g - l_fpre[lo]));
                }
            }
        }
        __syncthreads();
    }
    // the survivors' sort keys: one access per thread, its survivor found by
    // binary search over the access prefix
    // (kCompactU accesses per thread per step: their row gathers in flight together)
    constexpr uint32_t kCompactU = 4;
    const uint32_t ns = s_nsurv, na = s_nacc, ab0 = s_ab0;
    for (uint32_t g0 = 0; g0 < na; g0 += kBlock * kCompactU) {
        uint32_t sv[kCompactU], qv[kCompactU], ar[kCompactU];
#pragma unroll
        for (uint32_t u = 0; u < kCompactU; u++) {
            const uint32_t g = g0 + u * kBlock + tid;
            uint32_t lo = 0, hi = ns;  // largest k with l_pre[k] <= g
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (l_pre[mid] <= g) lo = mid;
                else hi = mid;
            }
            sv[u] = lo;
            qv[u] = g - l_pre[lo];
            uint32_t a = 0;
            if (g < na) {
                if constexpr (KEYS) {  // the qv-th access of the survivor whose skip bit is clear
                    if (l_fpre[lo + 1] - l_fpre[lo] <= 32u) {
                        uint32_t kept = ~l_skip[lo];
                        for (uint32_t r = qv[u]; r; r--) kept &= kept - 1;
                        a = l_a0[lo] + (uint32_t)__builtin_ctz(kept);
                    } else {  // (longer than one skip word: k_kill's bits, the same rule)
                        a = skip_bits ? nth_kept(skip_bits, l_a0[lo], qv[u]) : l_a0[lo] + qv[u];
                    }
                } else {
                    a = skip_bits ? nth_kept(skip_bits, l_a0[lo], qv[u]) : l_a0[lo] + qv[u];
                }
            }
            if constexpr (KEYS) {  // (the row from the key: this block's acc_row stores may not be visible yet)
                uint64_t row = 0;
                uint32_t w = 0;
                if (g < na) kk_row<KEYS == 2>(kk, kk_key(kk, a, w), row, ctr);
                ar[u] = g < na ? (uint32_t)row | (w ? AR_WR : 0u) : 0u;
            } else {
                ar[u] = g < na ? acc_row[a] : 0u;
            }
        }
#pragma unroll
        for (uint32_t u = 0; u < kCompactU; u++) {
            const uint32_t g = g0 + u * kBlock + tid;
            if (g < na) pairs_b[ab0 + g] = pair_pack(ar[u] & ~AR_WR, sub0 + sv[u], qv[u], ar[u] >> 31);
        }
    }
}

// the survivors' decisions back to their txns (after the survivors' rounds;
// a no-op while they are halted, Counters::halt)
__global__ __launch_bounds__(kBlock) void k_sub_scatter_back(const uint32_t *__restrict__ map,
                                                             const uint8_t *__restrict__ status_b,
                                                             uint8_t *__restrict__ status, Counters *ctr,
                                                             const uint32_t *__restrict__ words) {
    if (input_err(ctr) || ctr->halt) return;
    const uint32_t S = ctr->b_txn;
    uint32_t und = 0;
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < S; i += gridDim.x * kBlock) {
        const uint8_t st = words ? word_status(words[i]) : status_b[i];
        status[map[i]] = st;
        und += st == ST_UNDEC ? 1u : 0u;
    }
    if (und) {  // cannot happen: the launch decided every txn or yielded (halt)
        set_err(ctr, ERRB_SPIN);
        atomicMax(&ctr->spin_site, 2u);
    }
}

namespace {
uint32_t grid_of(uint64_t n, uint32_t cap) {
    const uint64_t g = (n + kBlock - 1) / kBlock;
    return (uint32_t)(g < 1 ? 1 : (g > cap ? cap : g));
}
}  // namespace

void launch_prefix_mark(hipStream_t s, uint8_t *status, const uint32_t *tb_start, const uint32_t *tb_end,
                        const uint32_t *acc_row, uint32_t K, uint32_t *row_state, uint64_t rs_words, int nowait,
                        Counters *ctr, const uint32_t *words) {
    // (the bitmap and the Bloom filter after it were zeroed by k_epoch_clear)
    const uint32_t g = std::max<uint32_t>(1, std::min<uint32_t>((K + kMarkBlock - 1) / kMarkBlock, 64));
    DV_LAUNCH(k_prefix_mark, g, kMarkBlock, 0, s, status, tb_start, tb_end, acc_row, K, row_state, rs_words - kBloomWords,
                                           row_state + (rs_words - kBloomWords), nowait, ctr, words);
}

uint32_t kill_tiles(uint32_t n_after) { return (n_after + kKillTile - 1) / kKillTile; }

uint64_t kill_words(uint64_t n_acc) { return (n_acc + 63) / 64 + 1; }

void launch_kill_compact(hipStream_t s, const uint32_t *tb_start, const uint32_t *tb_end, const uint32_t *acc_row,
                         uint64_t n_acc, const uint32_t *n_acc_dev, uint32_t K, uint32_t n_txn,
                         const uint32_t *row_state, uint64_t rs_words,
                         int nowait,
                         uint64_t *kill_bits, uint64_t *skip_bits, uint8_t *status, uint32_t *map,
                         uint8_t *status_b, uint8_t *tlen_b, uint64_t *pairs_b, uint32_t *info, uint32_t *tsum,
                         Counters *ctr, const KillKeys *kk) {
    const uint32_t nt = kill_tiles(n_txn > K ? n_txn - K : 0u);
    if (!nt) return;
    const uint64_t nw = (n_acc + 63) / 64;
    const KillKeys k0 = kk ? *kk : KillKeys{};
    uint32_t *ar = const_cast<uint32_t *>(acc_row);  // (k_kill_emit writes the survivors' with keys)
    // (144 KiB of LDS per block: one per CU, each loads the hot words and the filter once)
    const uint32_t kg = grid_of(nw * 64 / kKillWords / 4 + 1, 256);
    if (kk && k0.dense_lim)
        DV_LAUNCH(k_kill<2>, kg, kKillBlock, 0, s, acc_row, n_acc, n_acc_dev, row_state, rs_words - kBloomWords,
                  row_state + (rs_words - kBloomWords), nowait, kill_bits, skip_bits, ctr, k0);
    else if (kk)
        DV_LAUNCH(k_kill<1>, kg, kKillBlock, 0, s, acc_row, n_acc, n_acc_dev, row_state, rs_words - kBloomWords,
                  row_state + (rs_words - kBloomWords), nowait, kill_bits, skip_bits, ctr, k0);
    else
        DV_LAUNCH(k_kill<0>, kg, kKillBlock, 0, s, acc_row, n_acc, n_acc_dev, row_state, rs_words - kBloomWords,
                  row_state + (rs_words - kBloomWords), nowait, kill_bits, skip_bits, ctr, k0);
    DV_LAUNCH(k_kill_count, nt, kBlock, 0, s, tb_start, tb_end, K, n_txn, (const uint64_t *)kill_bits,
              (const uint64_t *)skip_bits, status, info, tsum, ctr);
    if (kk && k0.dense_lim)
        DV_LAUNCH(k_kill_emit<2>, nt, kBlock, 0, s, tb_start, tb_end, ar, K, n_txn, (const uint64_t *)skip_bits,
                  info, tsum, map, status_b, tlen_b, pairs_b, ctr, k0, row_state, nowait);
    else if (kk)
        DV_LAUNCH(k_kill_emit<1>, nt, kBlock, 0, s, tb_start, tb_end, ar, K, n_txn, (const uint64_t *)skip_bits,
                  info, tsum, map, status_b, tlen_b, pairs_b, ctr, k0, row_state, nowait);
    else
        DV_LAUNCH(k_kill_emit<0>, nt, kBlock, 0, s, tb_start, tb_end, ar, K, n_txn, (const uint64_t *)skip_bits,
                  info, tsum, map, status_b, tlen_b, pairs_b, ctr, k0, row_state, nowait);
}

void launch_sub_scatter_back(hipStream_t s, const uint32_t *map, const uint8_t *status_b, uint32_t ub,
                             uint8_t *status, Counters *ctr, const uint32_t *words) {
    if (!ub) return;
    DV_LAUNCH(k_sub_scatter_back, grid_of(ub, 2048), kBlock, 0, s, map, status_b, status, ctr, words);
}

}  // namespace dvcc
