// dvcc_common.h -- device helpers shared by the gfx950 kernels: wave64
// primitives, the row-queue element encoding and the single-pass
// (decoupled look-back) segmented scan used by the Calvin grant pass and the
// decision rounds.
#pragma once
#include "dvcc_internal.h"

namespace dvcc {

// ------------------------------------------------------------ wave helpers
// number of set bits of `mask` below this lane
__device__ __forceinline__ uint32_t mask_rank(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// lanes of the wave holding the same 8-bit digit (restricted to `valid`)
__device__ __forceinline__ uint64_t match_digit(uint32_t d, uint64_t valid) {
    uint64_t peers = valid;
#pragma unroll
    for (int b = 0; b < kRadixBits; b++) {
        const uint32_t bit = (d >> b) & 1u;
        const uint64_t m = __ballot(bit);
        peers &= bit ? m : ~m;
    }
    return peers;
}

// exclusive scan of one u32 per thread over a 256-thread block
__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t v, uint32_t *lds4, uint32_t *total) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, 64);
        if (lane >= (uint32_t)off) x += y;
    }
    if (lane == 63) lds4[wave] = x;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < 4; w++) {
        const uint32_t t = lds4[w];
        if (w < (int)wave) pre += t;
        tot += t;
    }
    __syncthreads();
    if (total) *total = tot;
    return pre + x - v;
}

// exclusive scan of c[0, n) in place by one 256-thread block, each thread a
// contiguous chunk; returns the total.  Chunks of up to kChunkRegs entries
// are loaded into registers all at once (a load-add loop waits out one round
// trip per entry); longer ones take the loop.
constexpr uint32_t kChunkRegs = 12;
__device__ __forceinline__ uint32_t block_chunk_scan256(uint32_t *c, uint32_t n, uint32_t *lds4) {
    const uint32_t per = (n + 255) / 256;
    const uint32_t lo = threadIdx.x * per, hi = lo + per < n ? lo + per : n;
    uint32_t tot = 0;
    if (per <= kChunkRegs) {
        uint32_t v[kChunkRegs], sum = 0;
#pragma unroll
        for (uint32_t k = 0; k < kChunkRegs; k++) v[k] = lo + k < hi ? c[lo + k] : 0u;
#pragma unroll
        for (uint32_t k = 0; k < kChunkRegs; k++) sum += v[k];
        uint32_t pre = block_excl_scan256(sum, lds4, &tot);
#pragma unroll
        for (uint32_t k = 0; k < kChunkRegs; k++) {
            if (lo + k < hi) c[lo + k] = pre;
            pre += v[k];
        }
        return tot;
    }
    uint32_t sum = 0;
    for (uint32_t i = lo; i < hi; i++) sum += c[i];
    uint32_t pre = block_excl_scan256(sum, lds4, &tot);
    for (uint32_t i = lo; i < hi; i++) {
        const uint32_t x = c[i];
        c[i] = pre;
        pre += x;
    }
    return tot;
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

__device__ __forceinline__ void set_err(Counters *ctr, uint32_t bit) { atomicOr(&ctr->err, bit); }

// commit bytes (1 = committed) of txns [0, n) from their status bytes, 16 per
// thread per step over the whole grid; returns this thread's committed count
__device__ __forceinline__ uint32_t commit_bytes_grid(const uint8_t *__restrict__ status, uint32_t n,
                                                      uint8_t *__restrict__ out) {
    uint32_t cnt = 0;
    for (uint32_t i0 = (blockIdx.x * blockDim.x + threadIdx.x) * 16u; i0 < n; i0 += gridDim.x * blockDim.x * 16u) {
        if (i0 + 16 <= n && ((uintptr_t)out & 15u) == 0) {
            const uint4 s4 = *reinterpret_cast<const uint4 *>(status + i0);
            uint32_t w[4] = {s4.x, s4.y, s4.z, s4.w};
#pragma unroll
            for (int q = 0; q < 4; q++) {
                // byte == ST_COMMIT (1) -> 1, else 0 (statuses are 0, 1 or 2)
                const uint32_t c = w[q] & ~(w[q] >> 1) & 0x01010101u;
                cnt += __popc(c);
                w[q] = c;
            }
            if (out) *reinterpret_cast<uint4 *>(out + i0) = uint4{w[0], w[1], w[2], w[3]};
        } else {  // (this thread's 16 txns only: a ragged end or an unaligned `out`)
            const uint32_t i1 = n - i0 < 16u ? n : i0 + 16u;
            for (uint32_t i = i0; i < i1; i++) {
                const uint32_t c = status[i] == ST_COMMIT ? 1u : 0u;
                if (out) out[i] = (uint8_t)c;
                cnt += c;
            }
        }
    }
    return cnt;
}

__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x, uint32_t lane) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, 64);
        if (lane >= (uint32_t)off) x += y;
    }
    return x;
}

// ------------------------------------------- segmented scan aggregates
// (f: a row-queue head occurs in the span, v: 5-bit OR value since the last
// head, c: 31-bit count).  OpPlain counts over the whole array (compaction
// offsets); OpSeg restarts the count at every head (grant-group numbers).
struct Agg {
    uint32_t f, v, c;
};
struct OpPlain {
    __device__ static Agg comb(Agg a, Agg b) {
        return Agg{a.f | b.f, b.f ? b.v : (a.v | b.v), a.c + b.c};
    }
};
struct OpSeg {
    __device__ static Agg comb(Agg a, Agg b) {
        return Agg{a.f | b.f, b.f ? b.v : (a.v | b.v), b.f ? b.c : a.c + b.c};
    }
};

template <class Op>
__device__ __forceinline__ Agg wave_incl(Agg p, uint32_t lane) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        Agg o;
        o.f = __shfl_up(p.f, off, 64);
        o.v = __shfl_up(p.v, off, 64);
        o.c = __shfl_up(p.c, off, 64);
        if (lane >= (uint32_t)off) p = Op::comb(o, p);
    }
    return p;
}

template <class Op>
__device__ __forceinline__ Agg wave_excl_from_incl(Agg inc, uint32_t lane) {
    Agg ex;
    ex.f = __shfl_up(inc.f, 1, 64);
    ex.v = __shfl_up(inc.v, 1, 64);
    ex.c = __shfl_up(inc.c, 1, 64);
    if (lane == 0) ex = Agg{0u, 0u, 0u};
    return ex;
}

// ---- decoupled look-back ---------------------------------------------------
// Tiles take tickets in dispatch order (atomicAdd), publish their aggregate as
// ONE 8-byte descriptor with an agent-scope atomic store -- the data is the
// flag (MI355X_MICROARCH.md "Valid forms", R2) -- and wave 0 of each tile folds
// its predecessors' descriptors right-to-left until it meets an inclusive
// prefix.  A tile waits only on tiles with smaller tickets, which are already
// running, so a pass always drains; every spin is bounded (ERRB_SPIN).
// descriptor: [63:39] tag [38:37] state (1 aggregate, 2 inclusive) [36] f
//             [35:31] v [30:0] c
constexpr uint64_t D_AGG = 1ull, D_INC = 2ull;
constexpr uint32_t kSpinLimit = 1u << 22;
constexpr uint32_t kTagBits = 25;

__device__ __forceinline__ uint64_t desc_pack(uint32_t tag, uint64_t state, Agg a) {
    return ((uint64_t)tag << 39) | (state << 37) | ((uint64_t)(a.f & 1u) << 36) |
           ((uint64_t)(a.v & 31u) << 31) | (uint64_t)(a.c & 0x7FFFFFFFu);
}
__device__ __forceinline__ uint32_t desc_tag(uint64_t d) { return (uint32_t)(d >> 39); }
__device__ __forceinline__ uint32_t desc_state(uint64_t d) { return (uint32_t)(d >> 37) & 3u; }
__device__ __forceinline__ Agg desc_agg(uint64_t d) {
    return Agg{(uint32_t)(d >> 36) & 1u, (uint32_t)(d >> 31) & 31u, (uint32_t)d & 0x7FFFFFFFu};
}

// called by ALL lanes of wave 0 of the tile; returns the tile's exclusive prefix
// and publishes its inclusive one.  HEAD: only the OR value in front of the
// tile -- the walk stops at the nearest tile holding a queue head (usually the
// one before), nothing inclusive is published, and only .v of the result is
// the prefix's; a second, full call follows.
template <class Op, bool HEAD = false>
__device__ Agg look_back(uint64_t *desc, uint32_t tile, uint32_t tag, Agg agg, uint32_t lane,
                         Counters *ctr) {
    Agg pre{0u, 0u, 0u};
    if (tile == 0) {
        if (lane == 0)
            __hip_atomic_store(&desc[0], desc_pack(tag, D_INC, agg), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        return pre;
    }
    if (lane == 0)
        __hip_atomic_store(&desc[tile], desc_pack(tag, D_AGG, agg), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    int64_t j = (int64_t)tile - 1;
    uint32_t spins = 0;
    for (;;) {
        const int64_t t = j - (int64_t)lane;
        uint64_t d = 0;
        bool ready = true;
        if (t >= 0) {
            d = __hip_atomic_load(&desc[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ready = desc_tag(d) == tag && desc_state(d) != 0;
        }
        // only the descriptors up to the nearest inclusive one are needed
        // (t < 0 acts as one); later ones may still be unpublished
        const uint64_t incmask =
            __ballot(ready && (t < 0 || desc_state(d) == D_INC || (HEAD && desc_agg(d).f)));
        const uint32_t stop = incmask ? (uint32_t)__builtin_ctzll(incmask) : 64u;
        const uint64_t need = stop >= 63 ? ~0ull : ((2ull << stop) - 1);
        if (__ballot(!ready) & need) {
            if (++spins > kSpinLimit) {
                if (lane == 0) {
                    set_err(ctr, ERRB_SPIN);
                    atomicMax(&ctr->spin_site, 1u);
                }
                break;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        for (uint32_t k = 0; k < 64 && k <= stop; k++) {
            const uint32_t lo = __shfl((uint32_t)d, (int)k, 64);
            const uint32_t hi = __shfl((uint32_t)(d >> 32), (int)k, 64);
            if (j - (int64_t)k < 0) break;
            pre = Op::comb(desc_agg(((uint64_t)hi << 32) | lo), pre);
        }
        if (stop < 64) break;
        j -= 64;
    }
    if (HEAD) return pre;
    if (lane == 0)
        __hip_atomic_store(&desc[tile], desc_pack(tag, D_INC, Op::comb(pre, agg)), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    return pre;
}

// ---- tiles of 64-bit row-queue elements staged through LDS ----------------
// kRIPT consecutive elements per thread; the LDS image pads one slot per
// kRIPT so each lane's ds_read_b64 run is bank-conflict free.
constexpr int kRIPT = 16;
constexpr int kRTile = kBlock * kRIPT;  // 4096 elements per workgroup
__device__ __forceinline__ uint32_t rpad(uint32_t j) { return j + j / kRIPT; }

// coalesced load of elements [base, base + tile_n) into s (padded) and the
// element after the tile into *s_next (`past_end` past the end)
__device__ __forceinline__ void load_tile64(const uint64_t *__restrict__ src, uint32_t base,
                                            uint32_t tile_n, uint32_t n, uint64_t *s,
                                            uint64_t *s_next, uint64_t past_end = EL_HEAD) {
    const uint32_t tid = threadIdx.x;
#pragma unroll
    for (int q = 0; q < kRIPT / 2; q++) {
        const uint32_t j = (q * kBlock + tid) * 2;
        if (j + 1 < tile_n) {
            const ulonglong2 x = *reinterpret_cast<const ulonglong2 *>(src + base + j);
            s[rpad(j)] = x.x;
            s[rpad(j + 1)] = x.y;
        } else if (j < tile_n) {
            s[rpad(j)] = src[base + j];
        }
    }
    if (tid == 0) *s_next = base + tile_n < n ? src[base + tile_n] : past_end;
}

// ------------------------------------------------------------------ probe
// One index probe against table descriptor t.  Callers hand t over from
// where it is uniform or cheap to index: the kernel arguments when the epoch
// names no tables (YCSB: every access probes table 0, scalar registers), an
// LDS copy of the descriptors otherwise -- indexing the kernel-argument array
// with a per-lane table id compiles to a select chain over every descriptor
// field, which cost a config-D probe 64 of its 172 us.
// miss (optional): a missing key ORs true there instead of setting the error
// bit here, so the caller can record it later (the probe keeps the tag
// gather's latency off its path until the access's row is needed)
__device__ __forceinline__ bool probe_row(const TableDesc &t, bool tb_ok, uint64_t key, uint64_t &row,
                                          Counters *ctr, bool *miss = nullptr) {
    if (!tb_ok) {
        set_err(ctr, ERRB_TABLE);
        return false;
    }
    if (t.rep_part != kNoRep) {  // replicated epoch: the key is the row; own keys checked here
        if (t.dense && t.htag == t.rep_part) {
            // every partition a dense map of nbuckets rows (epoch groups
            // require it): the key is there iff its bucket key / P is in range
            // -- one compare, as direct_holds would find for the own keys
            const bool found = key < t.nbuckets * t.part_cnt;
            if (!found) set_err(ctr, ERRB_KEY);
            row = key;
            return found;
        }
        uint64_t lo = 0;
        const uint64_t q = divmod_magic(key, t.part_cnt, t.m_part, lo);
        bool found = q < t.nbuckets;
        if (found && lo == t.rep_part) found = direct_holds(t, q, (uint32_t)lo, key);
        if (!found) set_err(ctr, ERRB_KEY);
        row = key;
        return found;
    }
    if (t.dense && t.part_cnt == 1 && t.htag == 0) {
        // a dense one-partition map (every key 0 .. nbuckets - 1 in bucket =
        // row = key, both hashes): the key check is one compare
        const bool found = key < t.nbuckets;
        if (!found) {
            if (miss) *miss = true;
            else set_err(ctr, ERRB_KEY);
        }
        row = key + t.row_base;
        return found;
    }
    uint32_t tag;
    const uint64_t bk = key_split(t, key, tag);  // (IndexHash::hash, index_hash.h:86-92)
    bool found = false;
    if (t.pkey != nullptr) {                  // direct map, local row = bucket (key tags)
        if (direct_holds(t, bk, tag, key)) { row = bk; found = true; }
    } else if (t.bstart == nullptr) {         // direct map: one {key, row} per bucket
        const IxEntry e = t.ix[bk];
        if (e.key == key) { row = e.row; found = true; }
    } else {                                  // chained bucket (read_item 217-231)
        for (uint32_t j = t.bstart[bk], end = t.bstart[bk + 1]; j < end; j++) {
            const IxEntry e = t.ix[j];
            if (e.key == key) { row = e.row; found = true; break; }
        }
    }
    if (!found) {
        if (miss) *miss = true;
        else set_err(ctr, ERRB_KEY);
    }
    row += t.row_base;
    return found;
}

// the row of a KillKeys epoch's key (k_kill / k_kill_emit with keys): DENSE
// (KillKeys::dense_lim) one compare -- a missing key rejects the epoch --
// else the full probe
template <bool DENSE>
__device__ __forceinline__ bool kk_row(const KillKeys &kk, uint64_t key, uint64_t &row, Counters *ctr) {
    if constexpr (DENSE) {
        row = key + kk.dense_base;
        if (key < kk.dense_lim) return true;
        set_err(ctr, ERRB_KEY);
        return false;
    } else {
        return probe_row(kk.tabs.t[0], kk.tabs.n > 0, key, row, ctr);
    }
}

}  // namespace dvcc
