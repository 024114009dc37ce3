// dvcc_carry.hip -- abort carry-over into the next epoch.
//
// The reference retries an aborted txn: WorkerThread::abort (worker_thread.cpp:
// 160-172) hands its id to AbortQueue::enqueue, which holds it for a penalty
// and re-enqueues it as RTXN with its query unchanged (abort_queue.cpp:26-82).
// Here the penalty is one epoch: after an epoch is decided, the accesses of
// its aborted txns are compacted on the device, in sequence order and
// renumbered from 0, to open the next epoch ahead of the new txns -- they are
// older, so they keep their priority (WAIT_DIE keeps a restarted txn's
// timestamp).  Three launches: per-block counts, one scan of the block
// counts, then every carried txn copies its accesses.
#include "dvcc_common.h"

namespace dvcc {

constexpr uint32_t kCarryTpb = kBlock;  // txns per block: one per thread

__device__ __forceinline__ bool carried(const uint8_t *status, uint32_t t) {
    return status[t] != ST_COMMIT;  // aborted (nothing is undecided after the rounds)
}

// per block: aborted txns and their accesses
__global__ __launch_bounds__(kBlock) void k_carry_count(const uint8_t *__restrict__ status,
                                                        const uint32_t *__restrict__ tb_start,
                                                        const uint32_t *__restrict__ tb_end,
                                                        uint32_t n_txn, uint32_t *__restrict__ bt,
                                                        uint32_t *__restrict__ ba) {
    __shared__ uint32_t lds4[4];
    const uint32_t t = blockIdx.x * kCarryTpb + threadIdx.x;
    const bool cr = t < n_txn && carried(status, t);
    const uint32_t nt = cr ? 1u : 0u, na = cr ? tb_end[t] - tb_start[t] : 0u;
    uint32_t tt = 0, ta = 0;
    (void)block_excl_scan256(nt, lds4, &tt);
    (void)block_excl_scan256(na, lds4, &ta);
    if (threadIdx.x == 0) {
        bt[blockIdx.x] = tt;
        ba[blockIdx.x] = ta;
    }
}

// one block: exclusive scans of the block counts, in place
__global__ __launch_bounds__(kBlock) void k_carry_scan(uint32_t *__restrict__ bt, uint32_t *__restrict__ ba,
                                                       uint32_t nb) {
    __shared__ uint32_t lds4[4];
    const uint32_t per = (nb + kBlock - 1) / kBlock;
    const uint32_t lo = threadIdx.x * per, hi = lo + per < nb ? lo + per : nb;
    constexpr uint32_t kR = 16;  // (nb <= 4,096 blocks, 1M txns: a thread's chunk in registers)
    if (per <= kR) {  // every load in flight at once (the loop waited out one round trip per entry: 10 us)
        uint32_t vt[kR], va[kR], st = 0, sa = 0;
#pragma unroll
        for (uint32_t k = 0; k < kR; k++) {
            const bool in = k < per && lo + k < nb;
            vt[k] = in ? bt[lo + k] : 0u;
            va[k] = in ? ba[lo + k] : 0u;
        }
#pragma unroll
        for (uint32_t k = 0; k < kR; k++) {
            st += vt[k];
            sa += va[k];
        }
        uint32_t pt = block_excl_scan256(st, lds4, nullptr);
        uint32_t pa = block_excl_scan256(sa, lds4, nullptr);
#pragma unroll
        for (uint32_t k = 0; k < kR; k++) {
            if (k < per && lo + k < nb) {
                bt[lo + k] = pt;
                ba[lo + k] = pa;
            }
            pt += vt[k];
            pa += va[k];
        }
        return;
    }
    uint32_t st = 0, sa = 0;
    for (uint32_t i = lo; i < hi; i++) {
        st += bt[i];
        sa += ba[i];
    }
    uint32_t pt = block_excl_scan256(st, lds4, nullptr);
    uint32_t pa = block_excl_scan256(sa, lds4, nullptr);
    for (uint32_t i = lo; i < hi; i++) {
        const uint32_t vt = bt[i], va = ba[i];
        bt[i] = pt;
        ba[i] = pa;
        pt += vt;
        pa += va;
    }
}

// every carried txn with a new id below max_txn is copied; the last one
// reports the carried epoch's size (tot[0] txns, tot[1] accesses).  A wave
// holds 64 consecutive txns, whose carried accesses are contiguous in the
// output: its lanes copy them together (a prefix sum of the lengths picks
// each access's txn), so reads and writes are coalesced.
__global__ __launch_bounds__(kBlock) void k_carry_copy(
    const uint8_t *__restrict__ status, const uint32_t *__restrict__ tb_start,
    const uint32_t *__restrict__ tb_end, uint32_t n_txn, const uint32_t *__restrict__ bt,
    const uint32_t *__restrict__ ba, uint32_t max_txn, const uint64_t *__restrict__ keys,
    const uint8_t *__restrict__ types, const uint8_t *__restrict__ tables, uint64_t *__restrict__ okeys,
    uint8_t *__restrict__ otypes, uint32_t *__restrict__ otxn, uint8_t *__restrict__ otables,
    uint32_t *__restrict__ tot, const uint32_t *__restrict__ skip, const uint32_t *__restrict__ recs,
    uint32_t *__restrict__ orecs, uint32_t *__restrict__ otb) {
    __shared__ uint32_t lds4[4];
    if (skip && *skip) return;  // (a refill behind a halted epoch: k_refill_plan)
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t t = blockIdx.x * kCarryTpb + threadIdx.x;
    const bool cr = t < n_txn && carried(status, t);
    const uint32_t a0 = cr ? tb_start[t] : 0u;
    uint32_t len = cr ? tb_end[t] - a0 : 0u;
    const uint32_t id = bt[blockIdx.x] + block_excl_scan256(cr ? 1u : 0u, lds4, nullptr);
    const uint32_t pos = ba[blockIdx.x] + block_excl_scan256(len, lds4, nullptr);
    const uint32_t total_txn = tot[2];  // carried txns before the cap (k_carry_total)
    const uint32_t last = total_txn < max_txn ? total_txn : max_txn;
    if (cr && id < max_txn && id + 1 == last) {
        tot[0] = last;
        tot[1] = pos + len;
    }
    if (!cr || id >= max_txn) len = 0;  // (ids grow with t: the cap cuts a suffix)
    else if (otb) otb[id] = pos;        // (tb form: the carried txn's boundary, dv_epoch_dev::txn_begin)
#ifndef DVCC_CARRY_COPY_WAVE
    // The block's txns hold one contiguous run of source accesses: the block
    // streams it (coalesced loads and stores), each access going to its txn's
    // destination plus its offset in the txn.  An access's txn: the last one
    // starting at or before it, by a binary search over the block's starts in
    // LDS -- made monotone by a suffix minimum, since an empty txn's range
    // (never written by the probe) may hold anything.  (The wave form below
    // spread each wave's carried accesses over its lanes by a shuffle search:
    // at a ~97 % carry rate that search, not the bytes, set its time.)
    {
        constexpr uint32_t kNone = 0xFFFFFFFFu;
        __shared__ uint32_t s_a0[kCarryTpb], s_id[kCarryTpb], s_sh[kCarryTpb], s_w[2][kCarryTpb / 64];
        const uint32_t tid = threadIdx.x, wave = tid >> 6;
        const uint32_t a0s = t < n_txn ? tb_start[t] : 0u;
        const uint32_t src_len = t < n_txn ? tb_end[t] - a0s : 0u;
        uint32_t v = src_len ? a0s : kNone;  // suffix min of the non-empty txns' starts
        uint32_t e = src_len ? a0s + src_len : 0u;  // and the block's end of accesses (max)
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t o = __shfl_down(v, off, 64), oe = __shfl_down(e, off, 64);
            if (lane + (uint32_t)off < 64u) {
                v = o < v ? o : v;
                e = oe > e ? oe : e;
            }
        }
        if (lane == 0) {
            s_w[0][wave] = v;  // (lane 0: the wave's whole suffix)
            s_w[1][wave] = e;
        }
        __syncthreads();
        uint32_t hi = 0;
        for (uint32_t w = 0; w < kCarryTpb / 64; w++) {
            if (w > wave) v = s_w[0][w] < v ? s_w[0][w] : v;
            hi = s_w[1][w] > hi ? s_w[1][w] : hi;
        }
        s_a0[tid] = v;
        s_id[tid] = len ? id : kNone;
        s_sh[tid] = pos - a0;  // (mod 2^32: destination = source + shift)
        __syncthreads();
        const uint32_t lo = s_a0[0];
        for (uint32_t i = lo + tid; lo != kNone && i < hi; i += kCarryTpb) {
            uint32_t k = 0;
#pragma unroll
            for (uint32_t w = kCarryTpb / 2; w > 0; w >>= 1)
                if (s_a0[k + w] <= i) k += w;
            const uint32_t sid = s_id[k];
            if (sid == kNone) continue;
            const uint32_t o = i + s_sh[k];
            if (orecs) orecs[o] = recs[i];  // tb form: the 4-byte records (key | write << 31)
            if (!okeys) continue;
            okeys[o] = keys[i];
            otypes[o] = types[i];
            otxn[o] = sid;
            if (tables) otables[o] = tables[i];
        }
        return;
    }
#endif
    uint32_t incl = len;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t o = __shfl_up(incl, off, 64);
        if (lane >= (uint32_t)off) incl += o;
    }
    const uint32_t pre = incl - len, wtot = __shfl(incl, 63, 64);
    // the wave's first carried access goes where its first carried txn's does
    const uint64_t first = __ballot(len != 0);
    if (!first) return;
    const uint32_t wpos = __shfl(pos, (int)__builtin_ctzll(first), 64);
    for (uint32_t g0 = 0; g0 < wtot; g0 += 64) {  // wave-uniform trips: shuffles read every lane
        const uint32_t g = g0 + lane;
        uint32_t src = 0;
#pragma unroll
        for (uint32_t w = 32; w > 0; w >>= 1) {
            const uint32_t cand = src + w;
            const uint32_t pv = __shfl(pre, (int)(cand & 63u), 64);
            if (cand < 64 && pv <= g) src = cand;
        }
        const uint32_t sa0 = __shfl(a0, (int)src, 64), spre = __shfl(pre, (int)src, 64);
        const uint32_t sid = __shfl(id, (int)src, 64);
        if (g >= wtot) continue;
        const uint32_t in = sa0 + (g - spre), o = wpos + g;
        if (orecs) orecs[o] = recs[in];  // tb form: the 4-byte records (key | write << 31)
        if (!okeys) continue;
        okeys[o] = keys[in];
        otypes[o] = types[in];
        otxn[o] = sid;
        if (tables) otables[o] = tables[in];
    }
}

// tot[2] = carried txns before the cap: the last block's exclusive prefix plus
// its own count; tot[0..1] cleared for k_carry_copy
__global__ void k_carry_total(const uint8_t *__restrict__ status, uint32_t n_txn, const uint32_t *bt,
                              uint32_t nb, uint32_t *tot) {
    uint32_t c = 0;
    for (uint32_t t = (nb - 1) * kCarryTpb + threadIdx.x; t < n_txn; t += blockDim.x)
        c += carried(status, t) ? 1u : 0u;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
    if (threadIdx.x == 0) {
        tot[0] = 0;
        tot[1] = 0;
        tot[2] = bt[nb - 1] + c;
    }
}

// ---- the closed loop on the device (dv_epoch_refill): the next epoch is the
// carried txns (as above, capped at n_out), then fresh txns taken in order
// from a pool, starting at a device-side cursor that wraps around the pool.
// Nothing is read back: the epoch's access count stays on the device
// (dv_epoch_dev::n_acc_dev).  An epoch whose rounds halted has no final
// statuses yet: then every refill kernel is a no-op (the host redoes both).
// tot: [0] carried txns, [1] their accesses, [2] aborted before the cap,
// [3] the cursor's value, [4] skip (halted), [5] fresh txns (kRefillTot)
__device__ __forceinline__ bool refill_skip(const Counters *ctr) {
    return ctr && (ctr->halt || ctr->a_halt || input_err(ctr));  // (no ctr: the loop's first epoch)
}

__global__ void k_refill_plan(const uint8_t *__restrict__ status, uint32_t n_txn, const uint32_t *bt, uint32_t nb,
                              uint32_t *tot, uint32_t n_out, uint32_t *cursor, uint32_t pool_n,
                              const Counters *ctr) {
    uint32_t c = 0;
    for (uint32_t t = (nb ? nb - 1 : 0) * kCarryTpb + threadIdx.x; nb && t < n_txn; t += blockDim.x)
        c += carried(status, t) ? 1u : 0u;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
    if (threadIdx.x != 0) return;
    const uint32_t skip = refill_skip(ctr) ? 1u : 0u;
    const uint32_t total = nb ? bt[nb - 1] + c : 0u;
    const uint32_t C = total < n_out ? total : n_out;
    const uint32_t cur = *cursor, F = n_out - C;
    tot[0] = 0;
    tot[1] = 0;
    tot[2] = skip ? 0u : total;  // (skip: k_carry_copy copies nothing)
    tot[3] = cur;
    tot[4] = skip;
    tot[5] = F;
    if (!skip) *cursor = (uint32_t)(((uint64_t)cur + F) % pool_n);
}

// the fresh txns [cur, cur + F) of the pool (wrapping), renumbered after the
// C carried ones, their accesses after the carried accesses; the epoch's
// access count into *n_acc_dev
__global__ __launch_bounds__(kBlock) void k_refill_fresh(const uint64_t *__restrict__ keys,
                                                         const uint8_t *__restrict__ types,
                                                         const uint8_t *__restrict__ tables,
                                                         const uint32_t *__restrict__ txn,
                                                         const uint32_t *__restrict__ tb, uint32_t pool_n,
                                                         const uint32_t *__restrict__ tot, uint32_t n_out,
                                                         uint64_t *__restrict__ okeys, uint8_t *__restrict__ otypes,
                                                         uint32_t *__restrict__ otxn, uint8_t *__restrict__ otables,
                                                         uint32_t *__restrict__ n_acc_dev,
                                                         const uint32_t *__restrict__ precs,
                                                         uint32_t *__restrict__ orecs, uint32_t *__restrict__ otb) {
    if (tot[4]) return;
    const uint32_t C = tot[2] < n_out ? tot[2] : n_out, A = tot[1], cur = tot[3], F = tot[5];
    const uint32_t e1 = cur + F < pool_n ? cur + F : pool_n;     // [cur, e1) then [0, F - (e1 - cur))
    const uint32_t n2 = F - (e1 - cur);
    const uint32_t b1 = tb[cur], fa1 = tb[e1] - b1, fa2 = tb[n2] - tb[0];
    if (blockIdx.x == 0 && threadIdx.x == 0) *n_acc_dev = A + fa1 + fa2;
    if (orecs) {  // tb form: the fresh txns' boundaries (and the epoch's end), then their records
        for (uint32_t f = blockIdx.x * kBlock + threadIdx.x; f <= F; f += gridDim.x * kBlock) {
            const uint32_t n1 = e1 - cur;
            otb[C + f] = A + (f <= n1 ? tb[cur + f] - b1 : fa1 + (tb[f - n1] - tb[0]));
        }
        for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < fa1 + fa2; i += gridDim.x * kBlock)
            orecs[A + i] = precs[i < fa1 ? b1 + i : tb[0] + (i - fa1)];
    }
    if (!okeys) return;
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < fa1 + fa2; i += gridDim.x * kBlock) {
        const bool first = i < fa1;
        const uint32_t src = first ? b1 + i : tb[0] + (i - fa1);
        const uint32_t t = first ? txn[src] - cur : txn[src] + (pool_n - cur);
        okeys[A + i] = keys[src];
        otypes[A + i] = types[src];
        otxn[A + i] = C + t;
        if (otables) otables[A + i] = tables ? tables[src] : 0;
    }
}

void launch_refill(hipStream_t s, const uint8_t *status, const uint32_t *tb_start, const uint32_t *tb_end,
                   uint32_t n_txn, const uint64_t *keys, const uint8_t *types, const uint8_t *tables,
                   const uint64_t *pkeys, const uint8_t *ptypes, const uint8_t *ptables, const uint32_t *ptxn,
                   const uint32_t *ptb, uint32_t pool_n, uint32_t *cursor, uint32_t n_out, uint64_t fresh_bound,
                   uint64_t *okeys, uint8_t *otypes, uint32_t *otxn, uint8_t *otables, uint32_t *n_acc_dev,
                   uint32_t *bt, uint32_t *ba, uint32_t *tot, const Counters *ctr, const uint32_t *recs,
                   const uint32_t *precs, uint32_t *orecs, uint32_t *otb) {
    const uint32_t nb = carry_blocks(n_txn);
    if (nb) {
        DV_LAUNCH(k_carry_count, nb, kBlock, 0, s, status, tb_start, tb_end, n_txn, bt, ba);
        DV_LAUNCH(k_carry_scan, 1, kBlock, 0, s, bt, ba, nb);
    }
    DV_LAUNCH(k_refill_plan, 1, 64, 0, s, status, n_txn, bt, nb, tot, n_out, cursor, pool_n, ctr);
    if (nb)
        DV_LAUNCH(k_carry_copy, nb, kBlock, 0, s, status, tb_start, tb_end, n_txn, bt, ba, n_out, keys, types, tables,
                  okeys, otypes, otxn, otables, tot, (const uint32_t *)(tot + 4), recs, orecs, otb);
    const uint64_t g = (fresh_bound + kBlock - 1) / kBlock;
    DV_LAUNCH(k_refill_fresh, (uint32_t)(g < 1 ? 1 : (g > 4096 ? 4096 : g)), kBlock, 0, s, pkeys, ptypes, ptables,
              ptxn, ptb, pool_n, tot, n_out, okeys, otypes, otxn, otables, n_acc_dev, precs, orecs, otb);
}

// a client batch's per-txn access ranges from its acc_txn (non-decreasing;
// ids at or past n_txn were rejected by the run that decided it): zeroed
// first (a txn without accesses keeps an empty range), then each run's ends
__global__ void k_txn_ranges_zero(uint32_t *__restrict__ tbs, uint32_t *__restrict__ tbe, uint32_t n_txn) {
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < n_txn; t += gridDim.x * blockDim.x)
        tbs[t] = tbe[t] = 0;
}
__global__ void k_txn_ranges(const uint32_t *__restrict__ acc_txn, uint64_t n, uint32_t n_txn,
                             uint32_t *__restrict__ tbs, uint32_t *__restrict__ tbe) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t t = acc_txn[i];
        if (t >= n_txn) continue;
        if (i == 0 || acc_txn[i - 1] != t) tbs[t] = (uint32_t)i;
        if (i + 1 == n || acc_txn[i + 1] != t) tbe[t] = (uint32_t)(i + 1);
    }
}

void launch_txn_ranges(hipStream_t s, const uint32_t *acc_txn, uint64_t n, uint32_t n_txn, uint32_t *tbs,
                       uint32_t *tbe) {
    if (!n_txn) return;
    const uint32_t gt = (n_txn + kBlock - 1) / kBlock;
    DV_LAUNCH(k_txn_ranges_zero, gt < 2048 ? gt : 2048, kBlock, 0, s, tbs, tbe, n_txn);
    if (!n) return;
    const uint64_t ga = (n + kBlock - 1) / kBlock;
    DV_LAUNCH(k_txn_ranges, (uint32_t)(ga < 4096 ? ga : 4096), kBlock, 0, s, acc_txn, n, n_txn, tbs, tbe);
}

uint32_t carry_blocks(uint32_t n_txn) { return n_txn ? (n_txn + kCarryTpb - 1) / kCarryTpb : 0; }

void launch_carry(hipStream_t s, const uint8_t *status, const uint32_t *tb_start, const uint32_t *tb_end,
                  uint32_t n_txn, uint32_t max_txn, const uint64_t *keys, const uint8_t *types,
                  const uint8_t *tables, uint64_t *okeys, uint8_t *otypes, uint32_t *otxn,
                  uint8_t *otables, uint32_t *bt, uint32_t *ba, uint32_t *tot) {
    const uint32_t nb = carry_blocks(n_txn);
    if (!nb) {
        (void)hipMemsetAsync(tot, 0, 3 * sizeof(uint32_t), s);
        return;
    }
    DV_LAUNCH(k_carry_count, nb, kBlock, 0, s, status, tb_start, tb_end, n_txn, bt, ba);
    DV_LAUNCH(k_carry_scan, 1, kBlock, 0, s, bt, ba, nb);
    DV_LAUNCH(k_carry_total, 1, 64, 0, s, status, n_txn, bt, nb, tot);
    DV_LAUNCH(k_carry_copy, nb, kBlock, 0, s, status, tb_start, tb_end, n_txn, bt, ba, max_txn, keys, types, tables,
                                       okeys, otypes, otxn, otables, tot, (const uint32_t *)nullptr,
                                       (const uint32_t *)nullptr, (uint32_t *)nullptr, (uint32_t *)nullptr);
}

}  // namespace dvcc
