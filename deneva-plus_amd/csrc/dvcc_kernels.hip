// dvcc_kernels.hip -- gfx950 (CDNA4) kernels of the batched CC engine.
//
// Epoch pipeline (DESIGN.md "Kernels"):
//   k_probe         IndexHash::index_read (storage/index_hash.cpp:137-153) for every access,
//                   emitting one packed u64 per access: row << 32 | txn << 1 | is_wr
//   radix sort      stable LSD sort of those pairs by row (8-bit digits, wave64 ballot
//                   multisplit ranks, LDS-staged coalesced scatter) -> per-row FIFO queues
//                   in sequence order, i.e. the waiter/owner lists of Row_lock
//                   (concurrency_control/row_lock.h:20-59) for the whole epoch at once
//   k_seg_prepare   row-segment heads, same-txn repeats, Calvin grant-group boundaries
//   segmented scans Calvin grant groups (row_lock.cpp:78-81,152-170,318-358) or one
//                   decision round of NO_WAIT/WAIT_DIE lock_get (row_lock.cpp:69,86-90)
//                   / OCC central_validate (occ.cpp:185-199, test_valid 319-327)
//   k_round_apply   per-txn vote combine (TxnManager::received_response, txn.cpp:544-554)
//   k_exec          run_ycsb_1 (benchmarks/ycsb_txn.cpp:227-254) for committed txns
//
// Every tiled kernel uses 256-thread workgroups (4 wave64s) and 4096-element
// tiles; every cross-workgroup dependency goes through a kernel boundary (no
// in-launch hand-offs), so no result depends on dispatch order or XCD placement.
#include "dvcc_internal.h"

namespace dvcc {

// ------------------------------------------------------------ wave helpers
__device__ __forceinline__ uint32_t lane_id() {
    return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}
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

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

// exclusive scan of one u32 per thread over a 256-thread block
__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t v, uint32_t *lds4,
                                                        uint32_t *total) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        uint32_t y = __shfl_up(x, off, 64);
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

__device__ __forceinline__ void set_err(Counters *ctr, uint32_t bit) { atomicOr(&ctr->err, bit); }

// ------------------------------------------------------------------ probe
__device__ __forceinline__ uint64_t bucket_of(const TableDesc &t, uint64_t key) {
    return t.hash_kind == DV_HASH_YCSB ? (key / t.part_cnt) % t.nbuckets : key % t.nbuckets;
}

template <bool VALS, bool NEED>
__global__ __launch_bounds__(kBlock) void k_probe(Tables tabs, const uint64_t *__restrict__ keys,
                                                  const uint8_t *__restrict__ types,
                                                  const uint32_t *__restrict__ acc_txn,
                                                  const uint8_t *__restrict__ tables, uint64_t n,
                                                  uint32_t n_txn, uint64_t *__restrict__ pairs,
                                                  uint32_t *__restrict__ vals,
                                                  uint32_t *__restrict__ need, Counters *ctr) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint32_t lane = threadIdx.x & 63;
    // block-uniform trip count so every lane takes part in the wave ballots
    for (uint64_t b0 = (uint64_t)blockIdx.x * blockDim.x; b0 < n; b0 += stride) {
        const uint64_t i = b0 + threadIdx.x;
        const bool valid = i < n;
        uint32_t txn = valid ? acc_txn[i] : 0xFFFFFFFFu;
        if (valid) {
            const uint64_t key = keys[i];
            const uint32_t tb = tables ? tables[i] : 0u;
            const uint32_t wr = types[i] == DV_WR ? 1u : 0u;
            uint64_t row = 0;
            if (tb >= tabs.n) {
                set_err(ctr, ERRB_TABLE);
            } else {
                const TableDesc &t = tabs.t[tb];
                const uint64_t bk = bucket_of(t, key);
                bool found = false;
                if (t.bstart == nullptr) {                // YCSB: one key per bucket
                    const IxEntry e = t.ix[bk];
                    if (e.key == key) { row = e.row; found = true; }
                } else {                                  // chained bucket (read_item 217-231)
                    for (uint32_t j = t.bstart[bk], end = t.bstart[bk + 1]; j < end; j++) {
                        const IxEntry e = t.ix[j];
                        if (e.key == key) { row = e.row; found = true; break; }
                    }
                }
                if (!found) set_err(ctr, ERRB_KEY);
                row += t.row_base;
            }
            uint32_t t_ok = txn;
            if (txn >= n_txn || (i > 0 && acc_txn[i - 1] > txn)) {
                set_err(ctr, ERRB_TXN);
                t_ok = 0;
            }
            pairs[i] = (row << 32) | ((uint64_t)t_ok << 1) | wr;
            if (VALS) vals[i] = (uint32_t)i;
        }
        if (NEED) {
            // need[t] = this partition's accesses of txn t: one atomic per run of
            // equal txns inside the wave (acc_txn is non-decreasing)
            const uint32_t tprev = __shfl_up(txn, 1, 64);
            const bool start = valid && (lane == 0 || tprev != txn);
            const uint64_t smask = __ballot(start);
            const uint32_t nvalid = (uint32_t)__popcll(__ballot(valid));
            if (start && txn < n_txn) {
                const uint64_t above = lane == 63 ? 0ull : ((smask >> (lane + 1)) << (lane + 1));
                const uint32_t next = above ? (uint32_t)__builtin_ctzll(above) : nvalid;
                atomicAdd(&need[txn], next - lane);
            }
        }
    }
}

void launch_probe(hipStream_t s, const Tables &tabs, const uint64_t *keys, const uint8_t *types,
                  const uint32_t *acc_txn, const uint8_t *tables, uint64_t n_acc, uint32_t n_txn,
                  uint64_t *pairs, uint32_t *vals, uint32_t *need, Counters *ctr) {
    if (n_acc == 0) return;
    uint64_t blocks = (n_acc + kBlock - 1) / kBlock;
    if (blocks > 8192) blocks = 8192;
    const uint32_t g = (uint32_t)blocks;
    if (vals)
        k_probe<true, false><<<g, kBlock, 0, s>>>(tabs, keys, types, acc_txn, tables, n_acc, n_txn,
                                                  pairs, vals, need, ctr);
    else if (need)
        k_probe<false, true><<<g, kBlock, 0, s>>>(tabs, keys, types, acc_txn, tables, n_acc, n_txn,
                                                  pairs, vals, need, ctr);
    else
        k_probe<false, false><<<g, kBlock, 0, s>>>(tabs, keys, types, acc_txn, tables, n_acc, n_txn,
                                                   pairs, vals, need, ctr);
}

// ------------------------------------------------------------- radix sort
// Each wave owns a contiguous 1024-element sub-tile and walks it in 16 steps of
// 64 consecutive elements, so (step, lane) order == input order: the ballot
// ranks below are stable.

__global__ __launch_bounds__(kBlock) void k_radix_hist(const uint64_t *__restrict__ in, uint64_t n,
                                                       int shift, uint32_t *__restrict__ counts,
                                                       uint32_t nblocks) {
    __shared__ uint32_t wc[4][kRadix];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (uint32_t d = tid; d < 4 * kRadix; d += kBlock) (&wc[0][0])[d] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * kTile + wave * (64 * kIPT);
    uint64_t k[kIPT];
#pragma unroll
    for (int j = 0; j < kIPT; j++) {
        const uint64_t idx = base + j * 64 + lane;
        k[j] = idx < n ? in[idx] : 0;
    }
#pragma unroll
    for (int j = 0; j < kIPT; j++) {
        const uint64_t idx = base + j * 64 + lane;
        const bool valid = idx < n;
        const uint32_t d = (uint32_t)(k[j] >> shift) & (kRadix - 1);
        const uint64_t vmask = __ballot(valid);
        const uint64_t peers = match_digit(d, vmask);
        if (valid && lane == (uint32_t)__builtin_ctzll(peers)) wc[wave][d] += (uint32_t)__popcll(peers);
    }
    __syncthreads();
    for (uint32_t d = tid; d < kRadix; d += kBlock)
        counts[(uint64_t)d * nblocks + blockIdx.x] = wc[0][d] + wc[1][d] + wc[2][d] + wc[3][d];
}

// exclusive scan of counts[d][0..nblocks) in place, one workgroup per digit
__global__ __launch_bounds__(kBlock) void k_radix_scan(uint32_t *__restrict__ counts, uint32_t nblocks,
                                                       uint32_t *__restrict__ digit_tot) {
    __shared__ uint32_t lds4[4];
    uint32_t *c = counts + (uint64_t)blockIdx.x * nblocks;
    const uint32_t per = (nblocks + kBlock - 1) / kBlock;
    const uint32_t lo = threadIdx.x * per;
    uint32_t hi = lo + per;
    if (hi > nblocks) hi = nblocks;
    uint32_t sum = 0;
    for (uint32_t i = lo; i < hi; i++) sum += c[i];
    uint32_t tot;
    uint32_t pre = block_excl_scan256(sum, lds4, &tot);
    for (uint32_t i = lo; i < hi; i++) {
        const uint32_t v = c[i];
        c[i] = pre;
        pre += v;
    }
    if (threadIdx.x == 0) digit_tot[blockIdx.x] = tot;
}

template <bool VALS>
__global__ __launch_bounds__(kBlock) void k_radix_scatter(
    const uint64_t *__restrict__ in, uint64_t *__restrict__ out, const uint32_t *__restrict__ vin,
    uint32_t *__restrict__ vout, uint64_t n, int shift, const uint32_t *__restrict__ counts,
    const uint32_t *__restrict__ digit_tot, uint32_t nblocks) {
    __shared__ __attribute__((aligned(16))) uint64_t skeys[kTile];
    __shared__ uint32_t svals[VALS ? kTile : 1];
    __shared__ uint32_t wc[4][kRadix];
    __shared__ uint32_t dstart[kRadix];
    __shared__ uint64_t gbase[kRadix];
    __shared__ uint32_t lds4[4];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t tile0 = (uint64_t)blockIdx.x * kTile;

    // global base of each digit for this tile: sum of smaller digits + this
    // block's exclusive prefix within the digit
    {
        const uint32_t d = tid;  // kBlock == kRadix
        const uint32_t dex = block_excl_scan256(digit_tot[d], lds4, nullptr);
        gbase[d] = (uint64_t)dex + counts[(uint64_t)d * nblocks + blockIdx.x];
        for (int w = 0; w < 4; w++) wc[w][d] = 0;
    }
    __syncthreads();

    const uint64_t base = tile0 + wave * (64 * kIPT);
    uint64_t k[kIPT];
    uint32_t v[VALS ? kIPT : 1];
    uint32_t r[kIPT];
#pragma unroll
    for (int j = 0; j < kIPT; j++) {
        const uint64_t idx = base + j * 64 + lane;
        k[j] = idx < n ? in[idx] : 0;
        if (VALS) v[j] = idx < n ? vin[idx] : 0;
    }
#pragma unroll
    for (int j = 0; j < kIPT; j++) {
        const uint64_t idx = base + j * 64 + lane;
        const bool valid = idx < n;
        const uint32_t d = (uint32_t)(k[j] >> shift) & (kRadix - 1);
        const uint64_t vmask = __ballot(valid);
        const uint64_t peers = match_digit(d, vmask);
        const uint32_t before = wc[wave][d];
        r[j] = before + mask_rank(peers);
        if (valid && lane == (uint32_t)__builtin_ctzll(peers)) wc[wave][d] = before + (uint32_t)__popcll(peers);
    }
    __syncthreads();
    {
        const uint32_t d = tid;
        const uint32_t c0 = wc[0][d], c1 = wc[1][d], c2 = wc[2][d], c3 = wc[3][d];
        wc[0][d] = 0;
        wc[1][d] = c0;
        wc[2][d] = c0 + c1;
        wc[3][d] = c0 + c1 + c2;
        const uint32_t ds = block_excl_scan256(c0 + c1 + c2 + c3, lds4, nullptr);
        dstart[d] = ds;
        gbase[d] -= ds;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kIPT; j++) {
        const uint64_t idx = base + j * 64 + lane;
        if (idx < n) {
            const uint32_t d = (uint32_t)(k[j] >> shift) & (kRadix - 1);
            const uint32_t pos = dstart[d] + wc[wave][d] + r[j];
            skeys[pos] = k[j];
            if (VALS) svals[pos] = v[j];
        }
    }
    __syncthreads();
    const uint32_t tile_n = (uint32_t)((n - tile0) < (uint64_t)kTile ? (n - tile0) : kTile);
    for (uint32_t p = tid; p < tile_n; p += kBlock) {
        const uint64_t key = skeys[p];
        const uint32_t d = (uint32_t)(key >> shift) & (kRadix - 1);
        const uint64_t dst = gbase[d] + p;
        out[dst] = key;
        if (VALS) vout[dst] = svals[p];
    }
}

int radix_sort_rows(hipStream_t s, uint64_t *pairs[2], uint32_t *vals[2], uint64_t n, int key_bits,
                    uint32_t *counts, uint32_t *digit_tot, hipEvent_t *scatter_ev) {
    if (n == 0) return 0;
    const uint32_t nb = nblocks_for(n);
    int cur = 0, pass = 0;
    for (int bit = 0; bit < key_bits; bit += kRadixBits, pass++) {
        const int shift = 32 + bit;
        k_radix_hist<<<nb, kBlock, 0, s>>>(pairs[cur], n, shift, counts, nb);
        k_radix_scan<<<kRadix, kBlock, 0, s>>>(counts, nb, digit_tot);
        if (scatter_ev) (void)hipEventRecord(scatter_ev[2 * pass], s);
        if (vals)
            k_radix_scatter<true><<<nb, kBlock, 0, s>>>(pairs[cur], pairs[cur ^ 1], vals[cur],
                                                        vals[cur ^ 1], n, shift, counts, digit_tot, nb);
        else
            k_radix_scatter<false><<<nb, kBlock, 0, s>>>(pairs[cur], pairs[cur ^ 1], nullptr,
                                                         nullptr, n, shift, counts, digit_tot, nb);
        if (scatter_ev) (void)hipEventRecord(scatter_ev[2 * pass + 1], s);
        cur ^= 1;
    }
    return cur;
}

// ------------------------------------------------------- segment prepare
__global__ __launch_bounds__(kBlock) void k_seg_prepare(const uint64_t *__restrict__ pairs, uint64_t n,
                                                        int calvin, uint32_t *__restrict__ el,
                                                        Counters *ctr) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t p = pairs[i];
        const uint32_t row = (uint32_t)(p >> 32), txn = (uint32_t)(p >> 1) & 0x7FFFFFFFu;
        const uint32_t wr = (uint32_t)p & 1u;
        uint32_t head = 1, dup = 0, bnd = 1;
        if (i > 0) {
            const uint64_t q = pairs[i - 1];
            if ((uint32_t)(q >> 32) == row) {
                head = 0;
                if (((uint32_t)(q >> 1) & 0x7FFFFFFFu) == txn) dup = 1;
                // previous queue entry's lock type: a repeat access keeps the lock
                // type of its txn's first access to the row (TxnManager::get_lock,
                // system/txn.cpp:778-788)
                uint64_t e = i - 1;
                while (e > 0) {
                    const uint64_t qq = pairs[e - 1];
                    if ((uint32_t)(qq >> 32) != row ||
                        ((uint32_t)(qq >> 1) & 0x7FFFFFFFu) != ((uint32_t)(pairs[e] >> 1) & 0x7FFFFFFFu))
                        break;
                    e--;
                }
                const uint32_t prev_entry_wr = (uint32_t)pairs[e] & 1u;
                bnd = dup ? 0u : ((wr | prev_entry_wr) ? 1u : 0u);
            }
        }
        if (dup && !calvin) set_err(ctr, ERRB_DUP);
        el[i] = (txn << 4) | ((calvin && bnd) ? EL_BND : 0u) | (dup ? EL_DUP : 0u) | (head ? EL_HEAD : 0u) | wr;
    }
}

void launch_seg_prepare(hipStream_t s, const uint64_t *pairs, uint64_t n, int calvin, uint32_t *el,
                        Counters *ctr) {
    if (n == 0) return;
    uint64_t blocks = (n + kBlock - 1) / kBlock;
    if (blocks > 8192) blocks = 8192;
    k_seg_prepare<<<(uint32_t)blocks, kBlock, 0, s>>>(pairs, n, calvin, el, ctr);
}

// ----------------------------------------------------- segmented scans
// A scan element is (head, value).  The segmented operator
//   (f1,v1) o (f2,v2) = (f1|f2, f2 ? v2 : comb(v1,v2))
// is associative; the exclusive value at a head is the identity.
struct SegPair {
    uint32_t f;
    uint32_t v;
};

// Calvin: low 31 bits count grant-group boundaries, bit 31 = a WR access seen
struct OpCalvin {
    static constexpr uint32_t kId = 0;
    __device__ static uint32_t comb(uint32_t a, uint32_t b) {
        return ((a & 0x7FFFFFFFu) + (b & 0x7FFFFFFFu)) | ((a | b) & 0x80000000u);
    }
};

template <class Op>
__device__ __forceinline__ SegPair seg_comb(SegPair a, SegPair b) {
    return SegPair{a.f | b.f, b.f ? b.v : Op::comb(a.v, b.v)};
}

template <class Op>
__device__ __forceinline__ SegPair wave_incl_scan(SegPair p, uint32_t lane) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        SegPair o;
        o.f = __shfl_up(p.f, off, 64);
        o.v = __shfl_up(p.v, off, 64);
        if (lane >= (uint32_t)off) p = seg_comb<Op>(o, p);
    }
    return p;
}

// load this thread's kIPT consecutive elements of a tile (blocked arrangement)
__device__ __forceinline__ int load_el(const uint32_t *__restrict__ el, uint64_t n, uint64_t first,
                                       uint32_t (&e)[kIPT]) {
    if (first + kIPT <= n) {
        const uint4 *p = reinterpret_cast<const uint4 *>(el + first);
#pragma unroll
        for (int q = 0; q < kIPT / 4; q++) {
            const uint4 x = p[q];
            e[4 * q] = x.x; e[4 * q + 1] = x.y; e[4 * q + 2] = x.z; e[4 * q + 3] = x.w;
        }
        return kIPT;
    }
    int cnt = 0;
#pragma unroll
    for (int j = 0; j < kIPT; j++) {
        const bool ok = first + j < n;
        e[j] = ok ? el[first + j] : EL_HEAD;
        cnt += ok;
    }
    return cnt;
}

struct ValCalvin {
    __device__ uint32_t operator()(uint32_t e) const {
        return ((e & EL_BND) ? 1u : 0u) | ((e & EL_WR) ? 0x80000000u : 0u);
    }
};

template <class Op, class Val>
__global__ __launch_bounds__(kBlock) void k_segscan_reduce(const uint32_t *__restrict__ el, uint64_t n,
                                                           Val val, uint32_t *__restrict__ agg_f,
                                                           uint32_t *__restrict__ agg_v) {
    __shared__ SegPair wt[4];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t first = (uint64_t)blockIdx.x * kTile + (uint64_t)tid * kIPT;
    uint32_t e[kIPT];
    const int cnt = first < n ? load_el(el, n, first, e) : 0;
    SegPair a{0u, Op::kId};
#pragma unroll
    for (int j = 0; j < kIPT; j++) {
        if (j < cnt) {
            const uint32_t v = val(e[j]);
            if (e[j] & EL_HEAD) { a.f = 1; a.v = v; }
            else a.v = Op::comb(a.v, v);
        }
    }
    SegPair inc = wave_incl_scan<Op>(a, lane);
    if (lane == 63) wt[wave] = inc;
    __syncthreads();
    if (tid == 0) {
        SegPair t = wt[0];
        for (int w = 1; w < 4; w++) t = seg_comb<Op>(t, wt[w]);
        agg_f[blockIdx.x] = t.f;
        agg_v[blockIdx.x] = t.v;
    }
}

// exclusive segmented scan of the block aggregates (one workgroup of 1024)
template <class Op>
__global__ __launch_bounds__(1024) void k_segscan_blocks(const uint32_t *__restrict__ agg_f,
                                                         const uint32_t *__restrict__ agg_v,
                                                         uint32_t nb, uint32_t *__restrict__ carry) {
    __shared__ SegPair wt[16];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t per = (nb + 1023) / 1024;
    const uint32_t lo = tid * per;
    uint32_t hi = lo + per;
    if (hi > nb) hi = nb;
    SegPair a{0u, Op::kId};
    for (uint32_t i = lo; i < hi; i++) a = seg_comb<Op>(a, SegPair{agg_f[i], agg_v[i]});
    SegPair inc = wave_incl_scan<Op>(a, lane);
    if (lane == 63) wt[wave] = inc;
    SegPair ex;
    ex.f = __shfl_up(inc.f, 1, 64);
    ex.v = __shfl_up(inc.v, 1, 64);
    if (lane == 0) ex = SegPair{0u, Op::kId};
    __syncthreads();
    SegPair pre{0u, Op::kId};
    for (uint32_t w = 0; w < wave; w++) pre = seg_comb<Op>(pre, wt[w]);
    SegPair run = seg_comb<Op>(pre, ex);
    for (uint32_t i = lo; i < hi; i++) {
        carry[i] = run.v;
        run = seg_comb<Op>(run, SegPair{agg_f[i], agg_v[i]});
    }
}

// downsweep: per element exclusive value -> apply
struct ApplyCalvin {
    const uint32_t *vals;
    uint32_t *grant;
    uint8_t *ew;
    __device__ void operator()(uint64_t i, uint32_t e, uint32_t excl, uint32_t v) const {
        const uint32_t inc = OpCalvin::comb(excl, v);
        if (grant) grant[vals[i]] = (inc & 0x7FFFFFFFu) - 1u;
        ew[i] = (uint8_t)(((e & EL_HEAD) ? 0u : (excl >> 31)) & 1u);
    }
};

template <class Op, class Val, class Apply>
__global__ __launch_bounds__(kBlock) void k_segscan_down(const uint32_t *__restrict__ el, uint64_t n,
                                                         Val val, const uint32_t *__restrict__ agg_f,
                                                         const uint32_t *__restrict__ carry,
                                                         Apply apply) {
    __shared__ SegPair wt[4];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t first = (uint64_t)blockIdx.x * kTile + (uint64_t)tid * kIPT;
    uint32_t e[kIPT], v[kIPT];
    const int cnt = first < n ? load_el(el, n, first, e) : 0;
    SegPair a{0u, Op::kId};
#pragma unroll
    for (int j = 0; j < kIPT; j++) {
        v[j] = 0;
        if (j < cnt) {
            v[j] = val(e[j]);
            if (e[j] & EL_HEAD) { a.f = 1; a.v = v[j]; }
            else a.v = Op::comb(a.v, v[j]);
        }
    }
    SegPair inc = wave_incl_scan<Op>(a, lane);
    if (lane == 63) wt[wave] = inc;
    SegPair ex;
    ex.f = __shfl_up(inc.f, 1, 64);
    ex.v = __shfl_up(inc.v, 1, 64);
    if (lane == 0) ex = SegPair{0u, Op::kId};
    __syncthreads();
    SegPair pre{0u, carry[blockIdx.x]};
    for (uint32_t w = 0; w < wave; w++) pre = seg_comb<Op>(pre, wt[w]);
    uint32_t run = seg_comb<Op>(pre, ex).v;
#pragma unroll
    for (int j = 0; j < kIPT; j++) {
        if (j < cnt) {
            const uint32_t excl = (e[j] & EL_HEAD) ? Op::kId : run;
            apply(first + j, e[j], excl, v[j]);
            run = (e[j] & EL_HEAD) ? v[j] : Op::comb(run, v[j]);
        }
    }
}

template <class Op, class Val, class Apply>
static void segscan(hipStream_t s, const uint32_t *el, uint64_t n, Val val, Apply apply,
                    uint32_t *agg_f, uint32_t *agg_v, uint32_t *carry) {
    if (n == 0) return;
    const uint32_t nb = nblocks_for(n);
    k_segscan_reduce<Op, Val><<<nb, kBlock, 0, s>>>(el, n, val, agg_f, agg_v);
    k_segscan_blocks<Op><<<1, 1024, 0, s>>>(agg_f, agg_v, nb, carry);
    k_segscan_down<Op, Val, Apply><<<nb, kBlock, 0, s>>>(el, n, val, agg_f, carry, apply);
}

void calvin_grant(hipStream_t s, const uint32_t *el, const uint32_t *vals, uint64_t n,
                  uint32_t *grant_out, uint8_t *ew, uint32_t *agg_f, uint32_t *agg_v,
                  uint32_t *carry) {
    segscan<OpCalvin>(s, el, n, ValCalvin{}, ApplyCalvin{vals, grant_out, ew}, agg_f, agg_v, carry);
}

__global__ void k_status_init(uint8_t *status, uint32_t n_txn, uint32_t n_pad, uint8_t value) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n_pad) status[i] = i < n_txn ? value : (uint8_t)ST_ABORT;
}

void launch_status_init(hipStream_t s, uint8_t *status, uint32_t n_txn, uint32_t n_txn_pad4,
                        uint8_t value) {
    if (!n_txn_pad4) return;
    k_status_init<<<(n_txn_pad4 + kBlock - 1) / kBlock, kBlock, 0, s>>>(status, n_txn, n_txn_pad4,
                                                                        value);
}

// ---------------------------------------------------------------- execute
// run_ycsb_1 (ycsb_txn.cpp:227-254) for committed txns: a RD loads the 8-byte
// F0 prefix, a WR stores 0.  Reads see the epoch's initial image unless an
// earlier WR of another txn precedes them in the row queue (Calvin only; under
// NO_WAIT/OCC a committed reader never follows a committed writer).
__global__ __launch_bounds__(kBlock) void k_exec_reads(const uint64_t *__restrict__ pairs,
                                                       const uint32_t *__restrict__ el,
                                                       const uint8_t *__restrict__ ew, uint64_t n,
                                                       const uint8_t *__restrict__ status,
                                                       const uint64_t *__restrict__ f0,
                                                       const uint64_t *__restrict__ pkey,
                                                       Counters *ctr) {
    __shared__ unsigned long long part[4];
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    unsigned long long dig = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t e = el[i];
        if (e & EL_WR) continue;
        const uint32_t txn = e >> 4;
        if (status[txn] != ST_COMMIT) continue;
        const uint64_t row = pairs[i] >> 32;
        const uint64_t val = (ew && ew[i]) ? 0ull : f0[row];
        dig += mix64(val ^ mix64(((uint64_t)txn << 32) ^ pkey[row]));
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) dig += __shfl_down(dig, off, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = dig;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long t = part[0] + part[1] + part[2] + part[3];
        if (t) atomicAdd(&ctr->read_digest, t);
    }
}

__global__ __launch_bounds__(kBlock) void k_exec_writes(const uint64_t *__restrict__ pairs,
                                                        const uint32_t *__restrict__ el, uint64_t n,
                                                        const uint8_t *__restrict__ status,
                                                        uint64_t *__restrict__ f0, Counters *ctr) {
    __shared__ uint32_t part[4];
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t cnt = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t e = el[i];
        if (!(e & EL_WR)) continue;
        if (status[e >> 4] != ST_COMMIT) continue;
        f0[pairs[i] >> 32] = 0;  // *(uint64_t*)&data[0] = 0 (ycsb_txn.cpp:239-242)
        cnt++;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) cnt += __shfl_down(cnt, off, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t t = part[0] + part[1] + part[2] + part[3];
        if (t) atomicAdd(&ctr->write_cnt, (unsigned long long)t);
    }
}

void launch_exec(hipStream_t s, int calvin, const uint64_t *pairs, const uint32_t *el,
                 const uint8_t *ew, uint64_t n, const uint8_t *status, uint64_t *f0,
                 const uint64_t *pkey, Counters *ctr) {
    if (n == 0) return;
    uint64_t blocks = (n + kBlock - 1) / kBlock;
    if (blocks > 4096) blocks = 4096;
    k_exec_reads<<<(uint32_t)blocks, kBlock, 0, s>>>(pairs, el, calvin ? ew : nullptr, n, status, f0,
                                                     pkey, ctr);
    k_exec_writes<<<(uint32_t)blocks, kBlock, 0, s>>>(pairs, el, n, status, f0, ctr);
}

__global__ __launch_bounds__(kBlock) void k_commit_out(const uint8_t *__restrict__ status, uint32_t n,
                                                       uint8_t *__restrict__ out, Counters *ctr) {
    __shared__ uint32_t part[4];
    const uint32_t stride = gridDim.x * blockDim.x;
    uint32_t cnt = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t c = status[i] == ST_COMMIT ? 1u : 0u;
        if (out) out[i] = (uint8_t)c;
        cnt += c;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) cnt += __shfl_down(cnt, off, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t t = part[0] + part[1] + part[2] + part[3];
        if (t) atomicAdd(&ctr->committed, t);
    }
}

void launch_commit_out(hipStream_t s, const uint8_t *status, uint32_t n_txn, uint8_t *d_commit,
                       Counters *ctr) {
    if (!n_txn) return;
    uint32_t blocks = (n_txn + kBlock - 1) / kBlock;
    if (blocks > 2048) blocks = 2048;
    k_commit_out<<<blocks, kBlock, 0, s>>>(status, n_txn, d_commit, ctr);
}

// ------------------------------------------------------------- loaders
// YCSBWorkload::init_table_slice (ycsb_wl.cpp:144-203) for one partition:
// local row r holds key r*P + part; F0 = "hello\0" + key bytes 6..7 (H3);
// YCSB bucket (key/P) % rows == r, so the index is a direct map.
__global__ void k_ycsb_load(uint64_t rows, uint32_t part_cnt, uint32_t part_id, uint64_t *f0,
                            uint64_t *pkey, IxEntry *ix) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += stride) {
        const uint64_t key = r * part_cnt + part_id;
        f0[r] = 0x00006F6C6C6568ull | (key & 0xFFFF000000000000ull);
        pkey[r] = key;
        ix[r] = IxEntry{key, r};
    }
}

void launch_ycsb_load(hipStream_t s, uint64_t rows, uint32_t part_cnt, uint32_t part_id,
                      uint64_t *f0, uint64_t *pkey, IxEntry *ix) {
    k_ycsb_load<<<2048, kBlock, 0, s>>>(rows, part_cnt, part_id, f0, pkey, ix);
}

__global__ void k_gather_rows(Tables tabs, uint32_t table, const uint64_t *keys, uint64_t n,
                              const uint64_t *f0, uint64_t *out, Counters *ctr) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const TableDesc &t = tabs.t[table];
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t key = keys[i];
        const uint64_t b = bucket_of(t, key);
        bool found = false;
        uint64_t row = 0;
        if (t.bstart == nullptr) {
            const IxEntry e = t.ix[b];
            if (e.key == key) { row = e.row; found = true; }
        } else {
            for (uint32_t j = t.bstart[b], end = t.bstart[b + 1]; j < end; j++) {
                const IxEntry e = t.ix[j];
                if (e.key == key) { row = e.row; found = true; break; }
            }
        }
        if (!found) { set_err(ctr, ERRB_KEY); out[i] = 0; continue; }
        out[i] = f0[t.row_base + row];
    }
}

void launch_gather_rows(hipStream_t s, const Tables &tabs, uint32_t table, const uint64_t *keys,
                        uint64_t n, const uint64_t *f0, uint64_t *out, Counters *ctr) {
    if (!n) return;
    k_gather_rows<<<1024, kBlock, 0, s>>>(tabs, table, keys, n, f0, out, ctr);
}

__global__ void k_split_access(const dv_access *acc, uint64_t n, uint64_t *keys, uint8_t *types,
                               uint32_t *acc_txn, uint8_t *tables) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const dv_access a = acc[i];
        keys[i] = a.key;
        types[i] = a.type;
        acc_txn[i] = a.txn_seq;
        tables[i] = a.table;
    }
}

void launch_split_access(hipStream_t s, const dv_access *acc, uint64_t n, uint64_t *keys,
                         uint8_t *types, uint32_t *acc_txn, uint8_t *tables) {
    if (!n) return;
    k_split_access<<<2048, kBlock, 0, s>>>(acc, n, keys, types, acc_txn, tables);
}

}  // namespace dvcc
