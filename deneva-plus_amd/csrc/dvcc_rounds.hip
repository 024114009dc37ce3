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
//   blocker committed           -> the access (so its txn) aborts
//   blocker still undecided     -> wait
//   no non-aborted blocker      -> the access is OK, permanently
// A txn commits once all its accesses are OK.  The lowest undecided txn always
// decides, so rounds terminate; zipf 0.9 epochs of 1M txns take ~20.
//
// Work per round shrinks: the downsweep compacts away accesses of aborted txns
// and accesses alone in their row queue, and each access pushes its verdict to
// its txn at most once (an atomic decrement of the txn's count of accesses not
// yet OK, or a plain store of the abort flag).  Cross-workgroup dependencies
// go through kernel boundaries only.
#include "dvcc_internal.h"

namespace dvcc {

namespace {

// scan value bits (OR): 1 committed / 2 undecided (any access), 4 committed /
// 8 undecided (WR accesses), 16 = the access is kept for the next round
constexpr uint32_t B_CA = 1u, B_UA = 2u, B_CW = 4u, B_UW = 8u, B_KEEP = 16u;

struct Seg {
    uint32_t f;  // a segment head occurs in the span
    uint32_t v;  // OR of the values since the last head
};
__device__ __forceinline__ Seg seg_or(Seg a, Seg b) { return Seg{a.f | b.f, b.f ? b.v : (a.v | b.v)}; }

__device__ __forceinline__ Seg wave_incl(Seg p, uint32_t lane) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        Seg o;
        o.f = __shfl_up(p.f, off, 64);
        o.v = __shfl_up(p.v, off, 64);
        if (lane >= (uint32_t)off) p = seg_or(o, p);
    }
    return p;
}

__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x, uint32_t lane) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, 64);
        if (lane >= (uint32_t)off) x += y;
    }
    return x;
}

// this thread's kIPT consecutive elements plus the element after them
__device__ __forceinline__ int load_chunk(const uint32_t *__restrict__ el, uint32_t n, uint32_t first,
                                          uint32_t (&e)[kIPT], uint32_t &next) {
    int cnt;
    if (first + kIPT <= n) {
        const uint4 *p = reinterpret_cast<const uint4 *>(el + first);
#pragma unroll
        for (int q = 0; q < kIPT / 4; q++) {
            const uint4 x = p[q];
            e[4 * q] = x.x; e[4 * q + 1] = x.y; e[4 * q + 2] = x.z; e[4 * q + 3] = x.w;
        }
        cnt = kIPT;
    } else {
        cnt = 0;
#pragma unroll
        for (int j = 0; j < kIPT; j++) {
            const bool ok = first + j < n;
            e[j] = ok ? el[first + j] : EL_HEAD;
            cnt += ok;
        }
    }
    next = (first + kIPT < n) ? el[first + kIPT] : EL_HEAD;
    return cnt;
}

// per-element scan value from the txn's status; a row queue of one access and
// accesses of aborted txns are not kept
__device__ __forceinline__ uint32_t elem_value(uint32_t e, uint32_t next_head, uint8_t s, int nowait) {
    const bool single = (e & EL_HEAD) && next_head;
    const uint32_t wr = e & EL_WR;
    if (s == ST_COMMIT) return (nowait ? B_CA : 0u) | (wr ? B_CW : 0u) | (single ? 0u : B_KEEP);
    if (s == ST_UNDEC) return (nowait ? B_UA : 0u) | (wr ? B_UW : 0u) | (single ? 0u : B_KEEP);
    return 0u;
}

struct Chunk {
    uint32_t e[kIPT];
    uint32_t v[kIPT];
    int cnt;
    Seg agg;
    uint32_t kept;
    uint32_t umask;  // bit j: item j's txn is undecided
};

template <bool FIRST>
__device__ __forceinline__ void eval_chunk(const uint32_t *__restrict__ el, uint32_t n, uint32_t first,
                                           const uint8_t *__restrict__ status, int nowait, Chunk &c) {
    uint32_t next;
    c.cnt = first < n ? load_chunk(el, n, first, c.e, next) : 0;
    c.agg = Seg{0u, 0u};
    c.kept = 0;
    c.umask = 0;
#pragma unroll
    for (int j = 0; j < kIPT; j++) {
        c.v[j] = 0;
        if (j < c.cnt) {
            uint32_t nh;  // is the next access the head of another row queue?
            if (j + 1 < c.cnt) nh = c.e[j + 1] & EL_HEAD;
            else if (c.cnt < kIPT) nh = 1u;
            else nh = next & EL_HEAD;
            const uint8_t s = FIRST ? (uint8_t)ST_UNDEC : status[c.e[j] >> 4];
            c.umask |= (s == ST_UNDEC ? 1u : 0u) << j;
            c.v[j] = elem_value(c.e[j], nh, s, nowait);
            if (c.e[j] & EL_HEAD) c.agg = Seg{1u, c.v[j]};
            else c.agg.v |= c.v[j];
            c.kept += (c.v[j] & B_KEEP) ? 1u : 0u;
        }
    }
}

}  // namespace

// ---- one decision round in ONE pass: decoupled look-back segmented scan.
// Tiles take tickets in launch order (atomicAdd), publish their aggregate as
// one 8-byte descriptor (agent-scope atomic store: the data is the flag,
// MI355X_MICROARCH.md "Valid forms", R2), and wave 0 of each tile folds its
// predecessors' descriptors right-to-left until it meets an inclusive prefix.
// A tile waits only on tiles with smaller tickets, which are already running,
// so the pass always drains; every spin is bounded (ERRB_SPIN).
//
// descriptor: [63:39] tag (round id) [38:37] state (1 aggregate, 2 inclusive)
//             [36] head seen [35:31] OR value [30:0] kept count
namespace {
constexpr uint64_t D_AGG = 1ull, D_INC = 2ull;
__device__ __forceinline__ uint64_t desc_pack(uint32_t tag, uint64_t state, Seg s, uint32_t cnt) {
    return ((uint64_t)tag << 39) | (state << 37) | ((uint64_t)(s.f & 1u) << 36) |
           ((uint64_t)(s.v & 31u) << 31) | (uint64_t)(cnt & 0x7FFFFFFFu);
}
__device__ __forceinline__ uint32_t desc_tag(uint64_t d) { return (uint32_t)(d >> 39); }
__device__ __forceinline__ uint32_t desc_state(uint64_t d) { return (uint32_t)(d >> 37) & 3u; }
__device__ __forceinline__ Seg desc_seg(uint64_t d) {
    return Seg{(uint32_t)(d >> 36) & 1u, (uint32_t)(d >> 31) & 31u};
}
__device__ __forceinline__ uint32_t desc_cnt(uint64_t d) { return (uint32_t)d & 0x7FFFFFFFu; }
constexpr uint32_t kSpinLimit = 1u << 22;
}  // namespace

template <bool FIRST>
__global__ __launch_bounds__(kBlock) void k_round_pass(
    const uint32_t *__restrict__ el_in, const uint32_t *__restrict__ n_in,
    const uint8_t *__restrict__ status, int nowait, uint32_t *__restrict__ el_out,
    uint32_t *__restrict__ n_out, uint32_t *__restrict__ need, uint8_t *__restrict__ abortf,
    uint64_t *desc, uint32_t *tile_ctr, uint32_t tag, Counters *ctr) {
    __shared__ uint32_t s_tile;
    __shared__ Seg wt[4];
    __shared__ uint32_t wc[4];
    __shared__ Seg s_pre;
    __shared__ uint32_t s_pos, s_tot;
    const uint32_t n = *n_in;
    const uint32_t ntiles = (n + kTile - 1) / kTile;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) s_tile = atomicAdd(tile_ctr, 1u);
    __syncthreads();
    const uint32_t tile = s_tile;
    if (tile >= ntiles) {
        if (ntiles == 0 && tile == 0 && tid == 0) { *n_out = 0; ctr->undecided = 0; }
        return;
    }
    Chunk c;
    eval_chunk<FIRST>(el_in, n, tile * kTile + tid * kIPT, status, nowait, c);
    const Seg inc = wave_incl(c.agg, lane);
    const uint32_t ks = wave_incl_sum(c.kept, lane);
    if (lane == 63) { wt[wave] = inc; wc[wave] = ks; }
    __syncthreads();
    if (wave == 0) {
        Seg agg = wt[0];
        uint32_t cnt = wc[0];
        for (int w = 1; w < 4; w++) { agg = seg_or(agg, wt[w]); cnt += wc[w]; }
        Seg pre{0u, 0u};
        uint32_t pcnt = 0;
        if (tile == 0) {
            if (lane == 0)
                __hip_atomic_store(&desc[0], desc_pack(tag, D_INC, agg, cnt), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        } else {
            if (lane == 0)
                __hip_atomic_store(&desc[tile], desc_pack(tag, D_AGG, agg, cnt), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            // look-back: lane k reads tile (j - k); fold nearest-first
            int64_t j = (int64_t)tile - 1;
            Seg acc{0u, 0u};  // covers (window start, tile)
            uint32_t accc = 0;
            bool done = false;
            uint32_t spins = 0;
            while (!done) {
                const int64_t t = j - (int64_t)lane;
                uint64_t d = 0;
                bool ready = true;
                if (t >= 0) {
                    d = __hip_atomic_load(&desc[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    ready = desc_tag(d) == tag && desc_state(d) != 0;
                }
                if (!__all(ready)) {
                    if (++spins > kSpinLimit) {
                        if (lane == 0) atomicOr(&ctr->err, ERRB_SPIN);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                // lanes with t < 0 act as an inclusive identity
                const uint64_t incmask = __ballot(t < 0 || desc_state(d) == D_INC);
                const uint32_t stop = incmask ? (uint32_t)__builtin_ctzll(incmask) : 64u;
                // fold lanes 0..stop (nearest first): acc = d_k o acc
                for (uint32_t k = 0; k < 64 && k <= stop; k++) {
                    const uint32_t lo = __shfl((uint32_t)d, (int)k, 64);
                    const uint32_t hi = __shfl((uint32_t)(d >> 32), (int)k, 64);
                    const int64_t tk = j - (int64_t)k;
                    if (tk < 0) break;
                    const uint64_t dk = ((uint64_t)hi << 32) | lo;
                    acc = seg_or(desc_seg(dk), acc);
                    accc += desc_cnt(dk);
                }
                if (stop < 64) done = true;
                else j -= 64;
            }
            pre = acc;
            pcnt = accc;
            if (lane == 0)
                __hip_atomic_store(&desc[tile], desc_pack(tag, D_INC, seg_or(pre, agg), pcnt + cnt),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) {
            s_pre = pre;
            s_pos = pcnt;
            s_tot = pcnt + cnt;
            if (tile == 0) ctr->undecided = 0;  // re-counted by this round's settle
        }
    }
    __syncthreads();
    Seg ex;
    ex.f = __shfl_up(inc.f, 1, 64);
    ex.v = __shfl_up(inc.v, 1, 64);
    if (lane == 0) ex = Seg{0u, 0u};
    Seg pre = s_pre;
    uint32_t pos = s_pos + ks - c.kept;
    for (uint32_t w = 0; w < wave; w++) {
        pre = seg_or(pre, wt[w]);
        pos += wc[w];
    }
    uint32_t run = seg_or(pre, ex).v;
#pragma unroll
    for (int jj = 0; jj < kIPT; jj++) {
        if (jj < c.cnt) {
            uint32_t e = c.e[jj];
            const uint32_t v = c.v[jj];
            const uint32_t excl = (e & EL_HEAD) ? 0u : run;
            const uint32_t txn = e >> 4;
            if (((c.umask >> jj) & 1u) && !(e & EL_DONE)) {
                // NO_WAIT/WAIT_DIE: a WR conflicts with any earlier access, a RD
                // with earlier WRs; OCC: any access with earlier committed writes
                const uint32_t sel = (nowait && (e & EL_WR)) ? (excl & (B_CA | B_UA))
                                                             : ((excl >> 2) & (B_CA | B_UA));
                if (sel & B_CA) {
                    abortf[txn] = 1;                   // Abort (row_lock.cpp:86-90 / occ.cpp:219)
                } else if (!(sel & B_UA)) {
                    atomicSub(&need[txn], 1u);         // granted / validated: permanently OK
                    e |= EL_DONE;
                }
            }
            if (v & B_KEEP)
                el_out[pos++] = (txn << 4) | (e & (EL_DONE | EL_WR)) | ((excl & B_KEEP) ? 0u : EL_HEAD);
            run = (e & EL_HEAD) ? v : (run | v);
        }
    }
    if (tile == ntiles - 1 && tid == 0) *n_out = s_tot;
}

// ---- K4: single-GPU settle -- status from the pushed verdicts, count undecided
__global__ __launch_bounds__(kBlock) void k_round_settle(uint32_t *__restrict__ status4,
                                                         const uint4 *__restrict__ need4,
                                                         const uint32_t *__restrict__ abort4, uint32_t nw,
                                                         Counters *ctr) {
    __shared__ uint32_t part[4];
    uint32_t und = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nw; i += gridDim.x * blockDim.x) {
        const uint32_t s = status4[i];
        if ((s & 0xFFu) && (s & 0xFF00u) && (s & 0xFF0000u) && (s & 0xFF000000u)) continue;
        const uint4 nd = need4[i];
        const uint32_t ab = abort4[i];
        const uint32_t need[4] = {nd.x, nd.y, nd.z, nd.w};
        uint32_t ns = 0;
#pragma unroll
        for (int b = 0; b < 4; b++) {
            uint32_t sb = (s >> (8 * b)) & 0xFFu;
            if (sb == ST_UNDEC) {
                if ((ab >> (8 * b)) & 0xFFu) sb = ST_ABORT;
                else if (need[b] == 0) sb = ST_COMMIT;
                else und++;
            }
            ns |= sb << (8 * b);
        }
        if (ns != s) status4[i] = ns;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) und += __shfl_down(und, off, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = und;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t t = part[0] + part[1] + part[2] + part[3];
        if (t) atomicAdd(&ctr->undecided, t);
    }
}

// ---- K4a (partitioned): this partition's verdict byte per txn
//      (bit1 abort, bit0 wait; combined across partitions by MAX)
__global__ __launch_bounds__(kBlock) void k_round_verdict(const uint32_t *__restrict__ status4,
                                                          const uint4 *__restrict__ need4,
                                                          const uint32_t *__restrict__ abort4,
                                                          uint32_t nw, uint32_t *__restrict__ verdict4) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nw; i += gridDim.x * blockDim.x) {
        const uint32_t s = status4[i];
        const uint4 nd = need4[i];
        const uint32_t ab = abort4[i];
        const uint32_t need[4] = {nd.x, nd.y, nd.z, nd.w};
        uint32_t v = 0;
#pragma unroll
        for (int b = 0; b < 4; b++) {
            if (((s >> (8 * b)) & 0xFFu) != ST_UNDEC) continue;
            const uint32_t vb = ((ab >> (8 * b)) & 0xFFu) ? V_ABORT : (need[b] ? V_WAIT : 0u);
            v |= vb << (8 * b);
        }
        verdict4[i] = v;
    }
}

// ---- K4b (partitioned): apply the combined verdicts
__global__ __launch_bounds__(kBlock) void k_round_apply(uint32_t *__restrict__ status4,
                                                        const uint32_t *__restrict__ verdict4,
                                                        uint32_t nw, Counters *ctr) {
    __shared__ uint32_t part[4];
    uint32_t und = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nw; i += gridDim.x * blockDim.x) {
        const uint32_t s = status4[i];
        const uint32_t v = verdict4[i];
        uint32_t ns = 0;
#pragma unroll
        for (int b = 0; b < 4; b++) {
            uint32_t sb = (s >> (8 * b)) & 0xFFu;
            const uint32_t vb = (v >> (8 * b)) & 0xFFu;
            if (sb == ST_UNDEC) {
                if (vb & V_ABORT) sb = ST_ABORT;
                else if (vb & V_WAIT) und++;
                else sb = ST_COMMIT;
            }
            ns |= sb << (8 * b);
        }
        if (ns != s) status4[i] = ns;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) und += __shfl_down(und, off, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = und;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t t = part[0] + part[1] + part[2] + part[3];
        if (t) atomicAdd(&ctr->undecided, t);
    }
}

__global__ void k_round0_init(uint32_t n, Counters *ctr) { ctr->nlive[0] = n; }

// ------------------------------------------------------------- launchers
static uint32_t grid_for_txn_words(uint32_t nw) {
    uint32_t g = (nw + kBlock - 1) / kBlock;
    return g < 1 ? 1 : (g > 64 ? 64 : g);
}

// per epoch: need[] is filled by the probe (one atomic per txn run), so only
// the flags, the tile tickets and the round-0 live count are reset here
void rounds_epoch_init(hipStream_t s, uint32_t n_acc, uint32_t n_txn_pad, uint32_t *need,
                       uint8_t *abortf, uint32_t *tile_ctr, Counters *ctr) {
    (void)need;
    (void)hipMemsetAsync(abortf, 0, n_txn_pad ? n_txn_pad : 4, s);
    (void)hipMemsetAsync(tile_ctr, 0, kTileCtrs * sizeof(uint32_t), s);
    k_round0_init<<<1, 1, 0, s>>>(n_acc, ctr);
}

void round_pass(hipStream_t s, bool first, int nowait, const uint32_t *el_in, uint32_t *el_out,
                uint32_t ub_in, const uint32_t *n_in, uint32_t *n_out, const uint8_t *status,
                uint32_t *need, uint8_t *abortf, uint64_t *desc, uint32_t *tile_ctr, uint32_t tag,
                Counters *ctr) {
    const uint32_t nb = ub_in ? nblocks_for(ub_in) : 1;
    if (first)
        k_round_pass<true><<<nb, kBlock, 0, s>>>(el_in, n_in, status, nowait, el_out, n_out, need,
                                                  abortf, desc, tile_ctr, tag, ctr);
    else
        k_round_pass<false><<<nb, kBlock, 0, s>>>(el_in, n_in, status, nowait, el_out, n_out, need,
                                                   abortf, desc, tile_ctr, tag, ctr);
}

void round_settle(hipStream_t s, uint8_t *status, const uint32_t *need, const uint8_t *abortf,
                  uint32_t n_txn_pad, Counters *ctr) {
    const uint32_t nw = n_txn_pad / 4;
    if (!nw) return;
    k_round_settle<<<grid_for_txn_words(nw), kBlock, 0, s>>>(
        reinterpret_cast<uint32_t *>(status), reinterpret_cast<const uint4 *>(need),
        reinterpret_cast<const uint32_t *>(abortf), nw, ctr);
}

void round_verdict(hipStream_t s, const uint8_t *status, const uint32_t *need, const uint8_t *abortf,
                   uint32_t n_txn_pad, uint8_t *verdict) {
    const uint32_t nw = n_txn_pad / 4;
    if (!nw) return;
    k_round_verdict<<<grid_for_txn_words(nw), kBlock, 0, s>>>(
        reinterpret_cast<const uint32_t *>(status), reinterpret_cast<const uint4 *>(need),
        reinterpret_cast<const uint32_t *>(abortf), nw, reinterpret_cast<uint32_t *>(verdict));
}

void round_apply(hipStream_t s, uint8_t *status, const uint8_t *verdict, uint32_t n_txn_pad,
                 Counters *ctr) {
    const uint32_t nw = n_txn_pad / 4;
    if (!nw) return;
    k_round_apply<<<grid_for_txn_words(nw), kBlock, 0, s>>>(
        reinterpret_cast<uint32_t *>(status), reinterpret_cast<const uint32_t *>(verdict), nw, ctr);
}

}  // namespace dvcc
