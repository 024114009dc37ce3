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
// Layout: a round element is one access (txn << 32 | access << 4 | flags) in
// row order.  An access reads its txn's status byte (1 B per txn: L2-resident)
// and writes its own verdict byte vb8[access]; a txn then reads its contiguous
// access range [tb_start, tb_end) -- plain loads and stores, no atomics.
// The round pass compacts away accesses of aborted txns and accesses alone in
// their row queue, stages tiles through LDS for coalesced loads and stores, and
// is a single launch (decoupled look-back scan, below).
#include "dvcc_common.h"

namespace dvcc {

namespace {

// scan value bits (OR): 1 committed / 2 undecided (any access), 4 committed /
// 8 undecided (WR accesses), 16 = the access is kept for the next round
constexpr uint32_t B_CA = 1u, B_UA = 2u, B_CW = 4u, B_UW = 8u, B_KEEP = 16u;
constexpr uint8_t VB_OK = 1, VB_ABORT = 2;

// per-element scan value from its txn's status; an access alone in its row
// queue and the accesses of aborted txns are not kept
__device__ __forceinline__ uint32_t elem_value(uint64_t e, bool next_head, uint8_t s, int nowait) {
    const bool single = (e & EL_HEAD) && next_head;
    const bool wr = (e & EL_WR) != 0;
    if (s == ST_COMMIT) return (nowait ? B_CA : 0u) | (wr ? B_CW : 0u) | (single ? 0u : B_KEEP);
    if (s == ST_UNDEC) return (nowait ? B_UA : 0u) | (wr ? B_UW : 0u) | (single ? 0u : B_KEEP);
    return 0u;
}

// verdict of a live access of an undecided txn from the OR of the scan values
// in front of it in its row queue
__device__ __forceinline__ uint64_t decide_elem(uint64_t e, uint32_t excl, int nowait,
                                                uint8_t *__restrict__ vb8) {
    if (e & EL_DONE) return e;
    // NO_WAIT/WAIT_DIE: a WR conflicts with any earlier access, a RD with
    // earlier WRs; OCC: any access with earlier committed writes
    const uint32_t sel = (nowait && (e & EL_WR)) ? (excl & (B_CA | B_UA)) : ((excl >> 2) & (B_CA | B_UA));
    if (sel & B_CA) {
#ifndef DVCC_EXP_NO_VB
        vb8[el_acc(e)] = VB_ABORT;  // Abort (row_lock.cpp:86-90 / occ.cpp:219-234)
#endif
    } else if (!(sel & B_UA)) {
#ifndef DVCC_EXP_NO_VB
        vb8[el_acc(e)] = VB_OK;     // granted / validated: permanently OK
#endif
        e |= EL_DONE;
    }
    return e;
}

}  // namespace

// ---- one tile of a decision round (single-pass OpPlain scan: v = status
//      bits OR-ed along the row queue, c = kept accesses -> compaction offset)
struct TileLds {
    uint64_t el[kRTile + kRTile / kRIPT];  // input tile, then the compacted output
    uint64_t next;
    Agg wt[4];
    Agg pre;
    uint32_t tot;
};

template <bool FIRST>
__device__ __forceinline__ void round_tile(TileLds &sh, uint32_t tile, uint32_t n, uint32_t ntiles,
                                           const uint64_t *__restrict__ el_in,
                                           uint64_t *__restrict__ el_out, uint32_t *__restrict__ n_out,
                                           const uint8_t *__restrict__ status,
                                           uint8_t *__restrict__ vb8, int nowait, uint64_t *desc,
                                           uint32_t tag, uint32_t *und_reset, Counters *ctr) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t base = tile * kRTile;
    const uint32_t tile_n = n - base < (uint32_t)kRTile ? n - base : (uint32_t)kRTile;
    load_tile64(el_in, base, tile_n, n, sh.el, &sh.next);
    __syncthreads();

    const uint32_t first = tid * kRIPT;
    const int cnt = first >= tile_n ? 0 : (tile_n - first < (uint32_t)kRIPT ? (int)(tile_n - first) : kRIPT);
    uint64_t e[kRIPT];
    uint32_t v[kRIPT];
#pragma unroll
    for (int j = 0; j < kRIPT; j++) e[j] = j < cnt ? sh.el[rpad(first + j)] : (uint64_t)EL_HEAD;
    const uint64_t nxt = first + kRIPT < tile_n ? sh.el[rpad(first + kRIPT)] : sh.next;
    uint64_t *s_out = sh.el;  // reused for the output once every lane holds its elements
    Agg a{0u, 0u, 0u};
    uint32_t umask = 0;
#pragma unroll
    for (int j = 0; j < kRIPT; j++) {
        v[j] = 0;
        if (j < cnt) {
            const bool nh = j + 1 < cnt ? (e[j + 1] & EL_HEAD) != 0
                                        : (cnt < kRIPT ? true : (nxt & EL_HEAD) != 0);
#ifdef DVCC_EXP_NO_GATHER
            const uint8_t s = (uint8_t)ST_UNDEC;
#else
            const uint8_t s = FIRST ? (uint8_t)ST_UNDEC : status[el_txn(e[j])];
#endif
            umask |= (s == ST_UNDEC ? 1u : 0u) << j;
            v[j] = elem_value(e[j], nh, s, nowait);
            a = OpPlain::comb(a, Agg{(uint32_t)((e[j] & EL_HEAD) != 0), v[j],
                                     (v[j] & B_KEEP) ? 1u : 0u});
        }
    }
    const Agg inc = wave_incl<OpPlain>(a, lane);
    if (lane == 63) sh.wt[wave] = inc;
    __syncthreads();
    if (wave == 0) {
        Agg bagg = sh.wt[0];
        for (int w = 1; w < 4; w++) bagg = OpPlain::comb(bagg, sh.wt[w]);
#ifdef DVCC_EXP_NO_LOOKBACK
        const Agg pre{0u, 0u, tile * (uint32_t)kRTile};
#else
        const Agg pre = look_back<OpPlain>(desc, tile, tag, bagg, lane, ctr);
#endif
        if (lane == 0) {
            sh.pre = pre;
            sh.tot = bagg.c;
            if (tile == 0) *und_reset = 0;  // re-counted by this round's settle
        }
    }
    __syncthreads();
    Agg wpre{0u, 0u, 0u};  // this wave's prefix within the tile
    for (uint32_t w = 0; w < wave; w++) wpre = OpPlain::comb(wpre, sh.wt[w]);
    const Agg lex = wave_excl_from_incl<OpPlain>(inc, lane);
    uint32_t lpos = wpre.c + lex.c;                                   // block-local slot
    uint32_t run = OpPlain::comb(OpPlain::comb(sh.pre, wpre), lex).v;  // OR since queue head
#pragma unroll
    for (int j = 0; j < kRIPT; j++) {
        if (j < cnt) {
            uint64_t ej = e[j];
            const uint32_t vj = v[j];
            const bool head = (ej & EL_HEAD) != 0;
            const uint32_t excl = head ? 0u : run;
            if ((umask >> j) & 1u) ej = decide_elem(ej, excl, nowait, vb8);
            if (vj & B_KEEP)
                s_out[lpos++] = (ej & ~(uint64_t)EL_HEAD) | ((excl & B_KEEP) ? 0u : EL_HEAD);
            run = head ? vj : (run | vj);
        }
    }
    __syncthreads();
    // coalesced write-out of the compacted tile
    const uint32_t tot = sh.tot, gpos = sh.pre.c;
    for (uint32_t k = tid; k < tot; k += kBlock) el_out[gpos + k] = s_out[k];
    if (tile == ntiles - 1 && tid == 0) *n_out = gpos + tot;
    __syncthreads();  // the LDS tile is free again
}

// one decision round, one launch; tiles are taken by ticket so that a tile
// only ever waits on tiles already running
template <bool FIRST>
__global__ __launch_bounds__(kBlock) void k_round_pass(
    const uint64_t *__restrict__ el_in, const uint32_t *__restrict__ n_in,
    uint64_t *__restrict__ el_out, uint32_t *__restrict__ n_out, const uint8_t *__restrict__ status,
    uint8_t *__restrict__ vb8, int nowait, uint64_t *desc, uint32_t *tile_ctr, uint32_t tag,
    uint32_t *und_reset, const uint32_t *und_in, uint32_t round, RoundPub *pub, Counters *ctr) {
    __shared__ TileLds sh;
    __shared__ uint32_t s_tile;
    const uint32_t n_live = *n_in;
    const uint32_t und = und_in ? *und_in : 1u;
    const uint32_t n = und ? n_live : 0u;  // nothing left to decide: no-op
    const uint32_t ntiles = (n + kRTile - 1) / kRTile;
    // one thread publishes the outcome of the previous round to the host
    const bool publisher = pub && threadIdx.x == 0 && blockIdx.x == (ntiles ? ntiles - 1 : 0);
    if (blockIdx.x >= ntiles) {  // spare blocks of a stale upper bound: no ticket
        if (ntiles == 0 && blockIdx.x == 0 && threadIdx.x == 0) { *n_out = 0; *und_reset = 0; }
    } else {
        if (threadIdx.x == 0) s_tile = atomicAdd(tile_ctr, 1u);
        __syncthreads();
        round_tile<FIRST>(sh, s_tile, n, ntiles, el_in, el_out, n_out, status, vb8, nowait, desc, tag,
                          und_reset, ctr);
    }
    if (publisher) {
        __hip_atomic_store(&pub->le, ((unsigned long long)n_live << 32) | ctr->err, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&pub->ru, ((unsigned long long)round << 32) | und, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// ---- per-txn settle (single GPU): new status from its accesses' verdicts
__device__ __forceinline__ uint8_t txn_verdict(const uint8_t *__restrict__ vb8, uint32_t a0, uint32_t a1) {
    uint32_t any_abort = 0, all_ok = 1;
    for (uint32_t w = a0 & ~3u; w < a1; w += 4) {  // aligned dwords over [a0, a1)
        const uint32_t x = *reinterpret_cast<const uint32_t *>(vb8 + w);
#pragma unroll
        for (uint32_t b = 0; b < 4; b++) {
            if (w + b < a0 || w + b >= a1) continue;
            const uint32_t vb = (x >> (8 * b)) & 0xFFu;
            any_abort |= vb == VB_ABORT;
            all_ok &= vb == VB_OK;
        }
    }
    return any_abort ? V_ABORT : (all_ok ? 0 : V_WAIT);
}

__device__ __forceinline__ void block_count(uint32_t und, Counters *ctr) {
    __shared__ uint32_t part[4];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) und += __shfl_down(und, off, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = und;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t t = part[0] + part[1] + part[2] + part[3];
        if (t) atomicAdd(&ctr->undecided, t);
    }
}

// Walks the undecided-txn list (round 0: every txn) and writes the survivors
// to the other list: each block takes kSettleChunk consecutive entries,
// compacts its survivors in LDS and reserves space with ONE atomic.
constexpr uint32_t kSettleIPT = 4, kSettleChunk = kBlock * kSettleIPT;

__device__ __forceinline__ bool settle_txn(uint8_t *__restrict__ status, const uint8_t *__restrict__ vb8,
                                           const uint32_t *__restrict__ tb_start,
                                           const uint32_t *__restrict__ tb_end, uint32_t t) {
    const uint8_t v = txn_verdict(vb8, tb_start[t], tb_end[t]);
    if (v & V_ABORT) status[t] = ST_ABORT;
    else if (!(v & V_WAIT)) status[t] = ST_COMMIT;
    return (v & (V_ABORT | V_WAIT)) == V_WAIT;
}

struct SettleLds {
    uint32_t keep[kSettleChunk];
    uint32_t cnt, base;
};

// entries [lo, lo + kSettleChunk) of the list (FIRST: txn ids themselves)
template <bool FIRST>
__device__ __forceinline__ void settle_chunk(SettleLds &sh, uint32_t lo, uint32_t n,
                                             uint8_t *__restrict__ status,
                                             const uint8_t *__restrict__ vb8,
                                             const uint32_t *__restrict__ tb_start,
                                             const uint32_t *__restrict__ tb_end,
                                             const uint32_t *__restrict__ list_in,
                                             uint32_t *__restrict__ list_out,
                                             uint32_t *__restrict__ n_out) {
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
            keep = settle_txn(status, vb8, tb_start, tb_end, t);
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
    uint8_t *__restrict__ status, const uint8_t *__restrict__ vb8,
    const uint32_t *__restrict__ tb_start, const uint32_t *__restrict__ tb_end,
    const uint32_t *__restrict__ list_in, const uint32_t *__restrict__ n_in, uint32_t n_txn,
    uint32_t *__restrict__ list_out, uint32_t *__restrict__ n_out) {
    __shared__ SettleLds sh;
    const uint32_t n = FIRST ? n_txn : *n_in;
    const uint32_t lo = blockIdx.x * kSettleChunk;
    if (lo >= n) return;
    settle_chunk<FIRST>(sh, lo, n, status, vb8, tb_start, tb_end, list_in, list_out, n_out);
}

// ---- partitioned: this partition's verdict byte per txn (bit1 abort, bit0
//      wait), combined across partitions by an element-wise MAX
__global__ __launch_bounds__(kBlock) void k_round_verdict(const uint8_t *__restrict__ status,
                                                          const uint8_t *__restrict__ vb8,
                                                          const uint32_t *__restrict__ tb_start,
                                                          const uint32_t *__restrict__ tb_end,
                                                          uint32_t n_txn, uint8_t *__restrict__ verdict) {
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < n_txn; t += gridDim.x * blockDim.x)
        verdict[t] = status[t] == ST_UNDEC ? txn_verdict(vb8, tb_start[t], tb_end[t]) : 0;
}

// ---- partitioned: apply the combined verdicts
__global__ __launch_bounds__(kBlock) void k_round_apply(uint8_t *__restrict__ status,
                                                        const uint8_t *__restrict__ verdict,
                                                        uint32_t n_txn, Counters *ctr) {
    uint32_t und = 0;
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < n_txn; t += gridDim.x * blockDim.x) {
        if (status[t] != ST_UNDEC) continue;
        const uint8_t v = verdict[t];
        if (v & V_ABORT) status[t] = ST_ABORT;
        else if (v & V_WAIT) und++;
        else status[t] = ST_COMMIT;
    }
    block_count(und, ctr);
}

__global__ void k_round0_init(uint32_t n, Counters *ctr) { ctr->nlive[0] = n; }

// ------------------------------------------------------------- launchers
static uint32_t txn_grid(uint32_t n_txn) {
    uint32_t g = (n_txn + kBlock - 1) / kBlock;
    return g < 1 ? 1 : (g > 1024 ? 1024 : g);
}

void rounds_epoch_init(hipStream_t s, const RoundBufs &b, uint32_t n_acc) {
    (void)hipMemsetAsync(b.vb8, 0, n_acc ? n_acc : 1, s);
    k_round0_init<<<1, 1, 0, s>>>(n_acc, b.ctr);
}

void round_pass(hipStream_t s, const RoundBufs &b, uint32_t round, int nowait, uint32_t ub_in,
                uint32_t tag, uint32_t ticket, bool settle, RoundPub *pub) {
    const uint32_t nb = ub_in ? (uint32_t)((ub_in + kRTile - 1) / kRTile) : 1;
    const uint64_t *in = round == 0 ? b.el0 : b.rel[(round - 1) & 1];
    uint64_t *out = b.rel[round & 1];
    const uint32_t *n_in = &b.ctr->nlive[round & 1];
    uint32_t *n_out = &b.ctr->nlive[(round + 1) & 1];
    uint32_t *tc = &b.tile_ctr[ticket % kTileCtrs];
    uint32_t *und = settle ? &b.ctr->nund[(round + 1) & 1] : &b.ctr->undecided;
    const uint32_t *und_in = settle && round > 0 ? &b.ctr->nund[round & 1] : nullptr;
    if (round == 0)
        k_round_pass<true><<<nb, kBlock, 0, s>>>(in, n_in, out, n_out, b.status, b.vb8, nowait, b.desc,
                                                  tc, tag, und, nullptr, round, nullptr, b.ctr);
    else
        k_round_pass<false><<<nb, kBlock, 0, s>>>(in, n_in, out, n_out, b.status, b.vb8, nowait,
                                                   b.desc, tc, tag, und, und_in, round, pub, b.ctr);
}

void round_settle(hipStream_t s, const RoundBufs &b, uint32_t round, uint32_t n_txn, uint32_t ub) {
    const uint32_t n = round == 0 ? n_txn : (ub < n_txn ? ub : n_txn);
    const uint32_t nb = n ? (n + kSettleChunk - 1) / kSettleChunk : 1;
    uint32_t *n_out = &b.ctr->nund[(round + 1) & 1];
    if (round == 0)
        k_round_settle<true><<<nb, kBlock, 0, s>>>(b.status, b.vb8, b.tb_start, b.tb_end, nullptr,
                                                   nullptr, n_txn, b.ulist[1], n_out);
    else
        k_round_settle<false><<<nb, kBlock, 0, s>>>(b.status, b.vb8, b.tb_start, b.tb_end,
                                                    b.ulist[round & 1], &b.ctr->nund[round & 1], n_txn,
                                                    b.ulist[(round + 1) & 1], n_out);
}

void round_verdict(hipStream_t s, const RoundBufs &b, uint32_t n_txn, uint8_t *verdict) {
    if (!n_txn) return;
    k_round_verdict<<<txn_grid(n_txn), kBlock, 0, s>>>(b.status, b.vb8, b.tb_start, b.tb_end, n_txn,
                                                      verdict);
}

void round_apply(hipStream_t s, const RoundBufs &b, uint32_t n_txn, const uint8_t *verdict) {
    if (!n_txn) return;
    k_round_apply<<<txn_grid(n_txn), kBlock, 0, s>>>(b.status, verdict, n_txn, b.ctr);
}

}  // namespace dvcc
