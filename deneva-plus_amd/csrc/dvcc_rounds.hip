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
            const uint8_t s = status[c.e[j] >> 4];
            c.umask |= (s == ST_UNDEC ? 1u : 0u) << j;
            c.v[j] = elem_value(c.e[j], nh, s, nowait);
            if (c.e[j] & EL_HEAD) c.agg = Seg{1u, c.v[j]};
            else c.agg.v |= c.v[j];
            c.kept += (c.v[j] & B_KEEP) ? 1u : 0u;
        }
    }
}

}  // namespace

// ---- K1: block aggregates (segmented OR + kept count)
__global__ __launch_bounds__(kBlock) void k_round_reduce(const uint32_t *__restrict__ el_in,
                                                         const uint32_t *__restrict__ n_in,
                                                         const uint8_t *__restrict__ status, int nowait,
                                                         uint32_t *__restrict__ agg_f,
                                                         uint32_t *__restrict__ agg_v,
                                                         uint32_t *__restrict__ agg_c) {
    __shared__ Seg wt[4];
    __shared__ uint32_t wc[4];
    const uint32_t n = *n_in;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if ((uint64_t)blockIdx.x * kTile >= n) {
        if (tid == 0) { agg_f[blockIdx.x] = 0; agg_v[blockIdx.x] = 0; agg_c[blockIdx.x] = 0; }
        return;
    }
    Chunk c;
    eval_chunk(el_in, n, blockIdx.x * kTile + tid * kIPT, status, nowait, c);
    const Seg inc = wave_incl(c.agg, lane);
    const uint32_t ks = wave_incl_sum(c.kept, lane);
    if (lane == 63) { wt[wave] = inc; wc[wave] = ks; }
    __syncthreads();
    if (tid == 0) {
        Seg t = wt[0];
        for (int w = 1; w < 4; w++) t = seg_or(t, wt[w]);
        agg_f[blockIdx.x] = t.f;
        agg_v[blockIdx.x] = t.v;
        agg_c[blockIdx.x] = wc[0] + wc[1] + wc[2] + wc[3];
    }
}

// ---- K2: scan of block aggregates -> carry-in value and output offset per block
__global__ __launch_bounds__(1024) void k_round_blocks(const uint32_t *__restrict__ agg_f,
                                                       const uint32_t *__restrict__ agg_v,
                                                       const uint32_t *__restrict__ agg_c, uint32_t nb,
                                                       uint32_t *__restrict__ carry,
                                                       uint32_t *__restrict__ off, uint32_t *n_out,
                                                       Counters *ctr) {
    __shared__ Seg wt[16];
    __shared__ uint32_t wc[16];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t per = (nb + 1023) / 1024;
    const uint32_t lo = tid * per;
    const uint32_t hi = lo + per < nb ? lo + per : nb;
    Seg a{0u, 0u};
    uint32_t cs = 0;
    for (uint32_t i = lo; i < hi; i++) {
        a = seg_or(a, Seg{agg_f[i], agg_v[i]});
        cs += agg_c[i];
    }
    const Seg inc = wave_incl(a, lane);
    const uint32_t ics = wave_incl_sum(cs, lane);
    if (lane == 63) { wt[wave] = inc; wc[wave] = ics; }
    Seg ex;
    ex.f = __shfl_up(inc.f, 1, 64);
    ex.v = __shfl_up(inc.v, 1, 64);
    if (lane == 0) ex = Seg{0u, 0u};
    uint32_t exs = ics - cs;
    __syncthreads();
    Seg pre{0u, 0u};
    uint32_t pres = 0, tot = 0;
    for (uint32_t w = 0; w < 16; w++) {
        if (w < wave) { pre = seg_or(pre, wt[w]); pres += wc[w]; }
        tot += wc[w];
    }
    Seg run = seg_or(pre, ex);
    uint32_t pos = pres + exs;
    for (uint32_t i = lo; i < hi; i++) {
        carry[i] = run.v;
        off[i] = pos;
        run = seg_or(run, Seg{agg_f[i], agg_v[i]});
        pos += agg_c[i];
    }
    if (tid == 0) {
        *n_out = tot;
        ctr->undecided = 0;  // re-counted by the settle kernel of this round
    }
}

// ---- K3: downsweep -- verdict push (once per access) and compaction
__global__ __launch_bounds__(kBlock) void k_round_down(
    const uint32_t *__restrict__ el_in, const uint32_t *__restrict__ n_in,
    const uint8_t *__restrict__ status, int nowait, const uint32_t *__restrict__ carry,
    const uint32_t *__restrict__ off, uint32_t *__restrict__ el_out, uint32_t *__restrict__ need,
    uint8_t *__restrict__ abortf) {
    __shared__ Seg wt[4];
    __shared__ uint32_t wc[4];
    const uint32_t n = *n_in;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if ((uint64_t)blockIdx.x * kTile >= n) return;
    Chunk c;
    eval_chunk(el_in, n, blockIdx.x * kTile + tid * kIPT, status, nowait, c);
    const Seg inc = wave_incl(c.agg, lane);
    const uint32_t ks = wave_incl_sum(c.kept, lane);
    if (lane == 63) { wt[wave] = inc; wc[wave] = ks; }
    Seg ex;
    ex.f = __shfl_up(inc.f, 1, 64);
    ex.v = __shfl_up(inc.v, 1, 64);
    if (lane == 0) ex = Seg{0u, 0u};
    __syncthreads();
    Seg pre{0u, carry[blockIdx.x]};
    uint32_t pos = off[blockIdx.x] + ks - c.kept;
    for (uint32_t w = 0; w < wave; w++) {
        pre = seg_or(pre, wt[w]);
        pos += wc[w];
    }
    uint32_t run = seg_or(pre, ex).v;
#pragma unroll
    for (int j = 0; j < kIPT; j++) {
        if (j < c.cnt) {
            uint32_t e = c.e[j];
            const uint32_t v = c.v[j];
            const uint32_t excl = (e & EL_HEAD) ? 0u : run;
            const uint32_t txn = e >> 4;
            if (((c.umask >> j) & 1u) && !(e & EL_DONE)) {
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
            if (v & B_KEEP) {
                el_out[pos++] = (txn << 4) | (e & (EL_DONE | EL_WR)) | ((excl & B_KEEP) ? 0u : EL_HEAD);
            }
            run = (e & EL_HEAD) ? v : (run | v);
        }
    }
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

// ---- per-epoch init: need[t] = this partition's accesses of txn t
//      (input order: acc_txn is non-decreasing), live count of round 0
__global__ __launch_bounds__(kBlock) void k_need_init(const uint32_t *__restrict__ acc_txn, uint32_t n,
                                                      uint32_t *__restrict__ need, Counters *ctr) {
    if (blockIdx.x == 0 && threadIdx.x == 0) ctr->nlive[0] = n;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t t = acc_txn[i];
        if (i + 1 < n && acc_txn[i + 1] == t) continue;  // not the txn's last access
        uint32_t s = i;
        while (s > 0 && acc_txn[s - 1] == t) s--;
        need[t] = i + 1 - s;
    }
}

// ------------------------------------------------------------- launchers
static uint32_t grid_for_txn_words(uint32_t nw) {
    uint32_t g = (nw + kBlock - 1) / kBlock;
    return g < 1 ? 1 : (g > 512 ? 512 : g);
}

void rounds_epoch_init(hipStream_t s, const uint32_t *acc_txn, uint32_t n_acc, uint32_t n_txn_pad,
                       uint32_t *need, uint8_t *abortf, Counters *ctr) {
    (void)hipMemsetAsync(need, 0, (size_t)(n_txn_pad ? n_txn_pad : 4) * 4, s);
    (void)hipMemsetAsync(abortf, 0, n_txn_pad ? n_txn_pad : 4, s);
    uint32_t g = (n_acc + kBlock - 1) / kBlock;
    g = g < 1 ? 1 : (g > 4096 ? 4096 : g);
    k_need_init<<<g, kBlock, 0, s>>>(acc_txn, n_acc, need, ctr);
}

void round_scan(hipStream_t s, int nowait, const uint32_t *el_in, uint32_t *el_out, uint32_t ub_in,
                const uint32_t *n_in, uint32_t *n_out, const uint8_t *status, uint32_t *need,
                uint8_t *abortf, uint32_t *agg_f, uint32_t *agg_v, uint32_t *agg_c, uint32_t *carry,
                uint32_t *off, Counters *ctr) {
    const uint32_t nb = ub_in ? nblocks_for(ub_in) : 1;
    k_round_reduce<<<nb, kBlock, 0, s>>>(el_in, n_in, status, nowait, agg_f, agg_v, agg_c);
    k_round_blocks<<<1, 1024, 0, s>>>(agg_f, agg_v, agg_c, nb, carry, off, n_out, ctr);
    k_round_down<<<nb, kBlock, 0, s>>>(el_in, n_in, status, nowait, carry, off, el_out, need, abortf);
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
