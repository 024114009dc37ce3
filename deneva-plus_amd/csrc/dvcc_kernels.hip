// dvcc_kernels.hip -- gfx950 (CDNA4) kernels of the batched CC engine.
//
// Epoch pipeline (DESIGN.md "Kernels"):
//   k_probe         IndexHash::index_read (storage/index_hash.cpp:137-153) for every access,
//                   emitting one packed u64 per access: row << 32 | txn << 8 | pos << 1 | wr
//   radix sort      stable LSD sort of those keys by row (8-bit digits, wave64 ballot
//                   multisplit ranks, LDS-staged coalesced scatter) -> per-row FIFO queues
//                   in sequence order, i.e. the waiter/owner lists of Row_lock
//                   (concurrency_control/row_lock.h:20-59) for the whole epoch at once
//   k_seg_prepare   queue heads, same-txn repeats, Calvin grant-group boundaries
//   k_calvin_pass   Calvin grant groups (row_lock.cpp:78-81,152-170,318-358), single pass
//   rounds          NO_WAIT / WAIT_DIE / OCC decisions (dvcc_rounds.hip)
//   k_exec_*        run_ycsb_1 (benchmarks/ycsb_txn.cpp:227-254) for committed txns
//
// Cross-workgroup dependencies go through kernel boundaries, except the
// decoupled look-back of the single-pass scans (dvcc_common.h), whose
// protocol is independent of dispatch order and XCD placement.
#include <hip/hip_ext.h>

#include "dvcc_common.h"
#include "dvcc_tpcc.h"

#ifndef DVCC_PROBE_HIST_WAVES
#define DVCC_PROBE_HIST_WAVES 6
#endif

namespace dvcc {

// ------------------------------------------------------------------ probe

// Input order: a txn's accesses are contiguous.  Each thread takes kPV
// consecutive accesses (vector loads, kPV independent index probes in
// flight).  Besides the sort key it records each txn's access range
// [tb_start, tb_end) and every access's position in it: the start of the run
// of equal txns is a max-scan of run-start indices over the wave; a run that
// began in an earlier wave is walked back in memory (at most one per wave).
// Repeated rows inside a txn are detected later, in row order (seg_prepare).
constexpr int kPV = 4;  // (8 measured slower: fewer waves per SIMD)
// RSV (TPC-C): CUST_LAST accesses name a customer by last name, resolved
// here against the name index and rsv_cols (tpcc_last_name_key)
template <bool HIST, bool RSV>
__device__ __forceinline__ void probe_body(const Tables &tabs, const uint64_t *__restrict__ keys,
                                           const uint32_t *__restrict__ keys32,
                                                  const uint8_t *__restrict__ types,
                                                  const uint32_t *__restrict__ acc_txn,
                                                  const uint8_t *__restrict__ tables, uint64_t n,
                                                  uint32_t n_txn, uint32_t slog,
                                                  uint64_t *__restrict__ pairs,
                                                  uint32_t *__restrict__ tb_start,
                                                  uint32_t *__restrict__ tb_end,
                                                  uint8_t *__restrict__ tlen,
                                                  uint32_t *__restrict__ acc_row, Counters *ctr,
                                                  uint32_t *__restrict__ counts, uint32_t ntiles,
                                                  uint32_t pair_limit, const uint64_t *__restrict__ ts,
                                                  const uint32_t *__restrict__ n_dev,
                                                  const uint64_t *__restrict__ rsv_cols) {
    if (n_dev && (uint64_t)*n_dev < n) n = *n_dev;  // (the real count of a device-built epoch)
    if (blockIdx.x == 0 && threadIdx.x == 0) ctr->n_acc = (uint32_t)n;
    // The first radix pass's histogram (digit = row bits [0, 8)) is counted
    // here, per 4096-access sort tile, so the sort skips that k_radix_hist
    // launch and its 8-byte-per-access re-read of the pairs.
    __shared__ uint32_t wc[4][kRadix];
    __shared__ TableDesc s_td[kMaxTables];  // per-lane table ids index this copy
    // RSV: a chunk's last-name keys, resolved in place (unused otherwise)
    __shared__ uint64_t s_rk[RSV ? kBlock * kPV : 1];
    __shared__ uint32_t s_rn;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (tables) {
        if (threadIdx.x < kMaxTables) s_td[threadIdx.x] = tabs.t[threadIdx.x];
        __syncthreads();
    }
    const uint64_t per_block = (uint64_t)kBlock * kPV;
    static_assert(kTile % (kBlock * kPV) == 0, "probe chunks tile the sort tiles");
    // work unit of a block: a whole sort tile when counting, else one chunk
    // (small epochs keep one chunk per block so the launch fills the GPU)
    const uint64_t unit = HIST ? (uint64_t)kTile : per_block;
    const uint64_t nunits = (n + unit - 1) / unit;
    // one 1024-access chunk starting at b0 (block-uniform, so every lane
    // takes part in the wave scans)
    auto chunk = [&](const uint64_t b0) {
        const uint64_t wave0 = b0 + (threadIdx.x & ~63u) * kPV;   // first access of this wave
        const uint64_t i0 = b0 + (uint64_t)threadIdx.x * kPV;       // first access of this thread
        uint32_t txn[kPV], wr[kPV], tb[kPV];
        uint64_t key[kPV], row[kPV];
        if (i0 + kPV <= n) {
#pragma unroll
            for (int q = 0; q < kPV; q += 4) {
                const uint4 t4 = *reinterpret_cast<const uint4 *>(acc_txn + i0 + q);
                txn[q] = t4.x; txn[q + 1] = t4.y; txn[q + 2] = t4.z; txn[q + 3] = t4.w;
                if (keys32) {  // replicated epochs: 32-bit row ids (dvcc_comm.hip)
                    const uint4 k4 = *reinterpret_cast<const uint4 *>(keys32 + i0 + q);
                    key[q] = k4.x; key[q + 1] = k4.y; key[q + 2] = k4.z; key[q + 3] = k4.w;
                } else {
                    const ulonglong2 k0 = *reinterpret_cast<const ulonglong2 *>(keys + i0 + q);
                    const ulonglong2 k1 = *reinterpret_cast<const ulonglong2 *>(keys + i0 + q + 2);
                    key[q] = k0.x; key[q + 1] = k0.y; key[q + 2] = k1.x; key[q + 3] = k1.y;
                }
                const uint32_t tt = tables ? *reinterpret_cast<const uint32_t *>(tables + i0 + q) : 0u;
                if (types) {
                    const uint32_t ty = *reinterpret_cast<const uint32_t *>(types + i0 + q);
#pragma unroll
                    for (int j = 0; j < 4; j++) wr[q + j] = ((ty >> (8 * j)) & 0xFFu) == DV_WR ? 1u : 0u;
                } else {  // epoch groups: row id | wr << 31 (keys32 only)
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        wr[q + j] = (uint32_t)(key[q + j] >> 31);
                        key[q + j] &= 0x7FFFFFFFull;
                    }
                }
#pragma unroll
                for (int j = 0; j < 4; j++) tb[q + j] = (tt >> (8 * j)) & 0xFFu;
            }
        } else {
#pragma unroll
            for (int j = 0; j < kPV; j++) {
                const bool ok = i0 + j < n;
                txn[j] = ok ? acc_txn[i0 + j] : 0xFFFFFFFFu;
                key[j] = ok ? (keys32 ? (uint64_t)keys32[i0 + j] : keys[i0 + j]) : 0ull;
                wr[j] = ok && (types ? types[i0 + j] == DV_WR : (key[j] >> 31) != 0) ? 1u : 0u;
                if (!types) key[j] &= 0x7FFFFFFFull;
                tb[j] = ok && tables ? tables[i0 + j] : 0u;
            }
        }
        bool miss = false, ts_bad = false;
        // the chunk's last names first: listed in LDS and resolved one per
        // thread (a name lookup is a chain of dependent loads; taken by the
        // thread that holds the access, four per thread, the probe ran 32 us
        // per TPC-C launch against 12 + 13 for the probe and a resolve launch)
        if (RSV && tables) {
            uint32_t slot[kPV];
            if (threadIdx.x == 0) s_rn = 0;
            __syncthreads();
#pragma unroll
            for (int j = 0; j < kPV; j++) {
                slot[j] = ~0u;
                if (i0 + j < n && tb[j] == DV_TPCC_CUST_LAST && tb[j] < tabs.n) {  // (else: the missing table reported)
                    slot[j] = atomicAdd(&s_rn, 1u);
                    s_rk[slot[j]] = key[j];
                }
            }
            __syncthreads();
            for (uint32_t u = threadIdx.x; u < s_rn; u += kBlock)
                s_rk[u] = tpcc_last_name_key(s_td[DV_TPCC_CUST_LAST], rsv_cols, s_rk[u]);
            __syncthreads();
#pragma unroll
            for (int j = 0; j < kPV; j++)
                if (slot[j] != ~0u) {
                    key[j] = s_rk[slot[j]];
                    tb[j] = DV_TPCC_CUSTOMER;
                }
        }
#pragma unroll
        for (int j = 0; j < kPV; j++) {
            row[j] = 0;
            if (i0 + j < n) {
                if (tables)
                    probe_row(s_td[tb[j] < kMaxTables ? tb[j] : 0], tb[j] < tabs.n, key[j], row[j], ctr, &miss);
                else
                    probe_row(tabs.t[0], tabs.n > 0, key[j], row[j], ctr, &miss);
            }
        }
        // run starts and their max-scan (32-bit: an epoch holds < kMaxAcc accesses)
        uint32_t prev = __shfl_up(txn[kPV - 1], 1, 64);
        if (lane == 0) prev = wave0 > 0 && wave0 - 1 < n ? acc_txn[wave0 - 1] : 0xFFFFFFFEu;
        uint32_t st[kPV];
        uint32_t mx = 0;
        bool bad = false;
#pragma unroll
        for (int j = 0; j < kPV; j++) {
            const uint32_t pt = j == 0 ? prev : txn[j - 1];
            const bool valid = i0 + j < n;
            const bool start = valid && (i0 + j == 0 || pt != txn[j]);
            if (valid && (txn[j] >= n_txn || (i0 + j > 0 && pt > txn[j] && pt != 0xFFFFFFFEu))) bad = true;
            mx = start ? (uint32_t)(i0 + j + 1) : mx;  // +1: 0 means "no start yet"
            st[j] = mx;
        }
        uint32_t inc = mx;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t o = __shfl_up(inc, off, 64);
            if (lane >= (uint32_t)off && o > inc) inc = o;
        }
        uint32_t ex = __shfl_up(inc, 1, 64);
        if (lane == 0) ex = 0;
        // the wave's first run may have begun before the wave: its start, found
        // 64 earlier accesses per step by the whole wave (one load, a ballot)
        uint32_t carry = 0;
        if (wave0 > 0 && wave0 < n) {  // (wave-uniform)
            const uint32_t t0 = __shfl(txn[0], 0, 64);
            for (uint64_t base = wave0;; base -= 64) {
                const bool same = base > lane && acc_txn[base - 1 - lane] == t0;
                const uint64_t m = __ballot(!same);
                if (m) {
                    const uint32_t f = (uint32_t)__ffsll((unsigned long long)m) - 1;  // accesses [base - f, base) continue the run
                    carry = base - f == wave0 ? 0u : (uint32_t)(base - f + 1);
                    break;
                }
            }
        }
        if (ex == 0) ex = carry;
        const uint32_t nxt_lane = __shfl_down(txn[0], 1, 64);
        const uint64_t in_last = i0 + kPV;
        uint32_t nxt_last = lane == 63 ? (in_last < n ? acc_txn[in_last] : 0xFFFFFFFFu) : nxt_lane;
        if (i0 + kPV > n) nxt_last = 0xFFFFFFFFu;
        if (bad) set_err(ctr, ERRB_TXN);
        if (miss) set_err(ctr, ERRB_KEY);
        uint64_t out[kPV];
#pragma unroll
        for (int j = 0; j < kPV; j++) {
            const uint64_t i = i0 + j;
            out[j] = 0;
            if (i >= n) continue;
            const uint32_t start = (st[j] ? st[j] : ex) - 1u;
            const uint32_t pos = (uint32_t)i - start;
            // a txn longer than the epoch's declared bound (1 << slog verdict
            // bytes per txn): an input error; positions and lengths are clamped
            // so every later index stays inside its txn's slot (the epoch is
            // rejected before anything executes, input_err)
            const bool big = (pos >> slog) != 0;
            if (big) set_err(ctr, ERRB_BIG);
            const uint32_t t = txn[j] < n_txn ? txn[j] : 0u;
            out[j] = pair_pack(row[j], t, big ? 0u : pos, wr[j]);
            if (txn[j] < n_txn) {
                if (pos == 0) {
                    tb_start[t] = (uint32_t)i;
                    // WAIT_DIE: owners must be older than every later txn
                    if (ts && t > 0 && ts[t] <= ts[t - 1]) ts_bad = true;
                }
                const uint32_t nt = j + 1 < kPV ? txn[j + 1] : nxt_last;
                if (i + 1 == n || nt != txn[j]) {
                    tb_end[t] = (uint32_t)(i + 1);
                    if (tlen) tlen[t] = (uint8_t)(big ? (1u << slog) : pos + 1);
                }
            }
        }
        if (ts_bad) set_err(ctr, ERRB_TS);
        if (acc_row) {
            uint32_t ar[kPV];
#pragma unroll
            for (int j = 0; j < kPV; j++) ar[j] = (uint32_t)row[j] | (wr[j] ? AR_WR : 0u);
            if (i0 + kPV <= n) {
                *reinterpret_cast<uint4 *>(acc_row + i0) = uint4{ar[0], ar[1], ar[2], ar[3]};
            } else {
                for (int j = 0; j < kPV; j++)
                    if (i0 + j < n) acc_row[i0 + j] = ar[j];
            }
        }
        if (pair_limit >= n_txn) {
            if (i0 + kPV <= n) {
                *reinterpret_cast<ulonglong2 *>(pairs + i0) = ulonglong2{out[0], out[1]};
                *reinterpret_cast<ulonglong2 *>(pairs + i0 + 2) = ulonglong2{out[2], out[3]};
            } else {
                for (int j = 0; j < kPV; j++)
                    if (i0 + j < n) pairs[i0 + j] = out[j];
            }
        } else {
            // prefix-kill epochs: sort keys only for the prefix txns (the first
            // accesses of the epoch); their count is the index after the last
            // one, stored by the one thread that holds it (txns ascend) -- a
            // counter atomic per wave serialised ~1,300 waves on one word
            if (i0 + kPV <= n && txn[kPV - 1] < pair_limit) {
                *reinterpret_cast<ulonglong2 *>(pairs + i0) = ulonglong2{out[0], out[1]};
                *reinterpret_cast<ulonglong2 *>(pairs + i0 + 2) = ulonglong2{out[2], out[3]};
            } else {
#pragma unroll
                for (int j = 0; j < kPV; j++)
                    if (i0 + j < n && txn[j] < pair_limit) pairs[i0 + j] = out[j];
            }
#pragma unroll
            for (int j = 0; j < kPV; j++) {
                const uint32_t nt = j + 1 < kPV ? txn[j + 1] : nxt_last;
                if (i0 + j < n && txn[j] < pair_limit && (nt >= pair_limit || i0 + j + 1 == n))
                    ctr->a_acc = (uint32_t)(i0 + j + 1);
            }
        }
        // digit-0 counts of the emitted pairs (as k_radix_hist: a step whose
        // keys share one digit adds once)
        if (HIST) {
#pragma unroll
        for (int j = 0; j < kPV; j++) {
            const bool valid = i0 + j < n;
            const uint32_t d = (uint32_t)row[j] & (kRadix - 1);
            const uint32_t d0 = __builtin_amdgcn_readfirstlane(d);
            const uint64_t vmask = __ballot(valid);
            if (__ballot(valid && d == d0) == vmask) {
                if (lane == 0) wc[wave][d0] += (uint32_t)__popcll(vmask);
            } else if (valid) {
                atomicAdd(&wc[wave][d], 1u);
            }
        }
        }
    };
    if (!HIST) {
        for (uint64_t b0 = (uint64_t)blockIdx.x * per_block; b0 < n; b0 += (uint64_t)gridDim.x * per_block)
            chunk(b0);
        return;
    }
    for (uint64_t tile = blockIdx.x; tile < nunits; tile += gridDim.x) {
        for (uint32_t d = threadIdx.x; d < 4 * kRadix; d += kBlock) (&wc[0][0])[d] = 0;
        __syncthreads();
        for (uint64_t b0 = tile * unit; b0 < n && b0 < (tile + 1) * unit; b0 += per_block) chunk(b0);
        __syncthreads();
        for (uint32_t d = threadIdx.x; d < kRadix; d += kBlock)
            counts[(uint64_t)d * ntiles + tile] = wc[0][d] + wc[1][d] + wc[2][d] + wc[3][d];
        __syncthreads();
    }
}

// the fused-histogram variant needs more registers: capped at 6 waves per SIMD
template <bool RSV>
__global__ __launch_bounds__(kBlock) void k_probe(Tables tabs, const uint64_t *__restrict__ keys,
                                                  const uint32_t *__restrict__ keys32,
                                                  const uint8_t *__restrict__ types,
                                                  const uint32_t *__restrict__ acc_txn,
                                                  const uint8_t *__restrict__ tables, uint64_t n, uint32_t n_txn,
                                                  uint32_t slog, uint64_t *__restrict__ pairs,
                                                  uint32_t *__restrict__ tb_start, uint32_t *__restrict__ tb_end,
                                                  uint8_t *__restrict__ tlen, uint32_t *__restrict__ acc_row,
                                                  Counters *ctr, uint32_t pair_limit, const uint64_t *__restrict__ ts,
                                                  const uint32_t *__restrict__ n_dev,
                                                  const uint64_t *__restrict__ rsv_cols) {
    probe_body<false, RSV>(tabs, keys, keys32, types, acc_txn, tables, n, n_txn, slog, pairs, tb_start, tb_end, tlen,
                           acc_row, ctr, nullptr, 0, pair_limit, ts, n_dev, rsv_cols);
}
template <bool RSV>
__global__ __launch_bounds__(kBlock, DVCC_PROBE_HIST_WAVES) void k_probe_hist(
    Tables tabs, const uint64_t *__restrict__ keys, const uint32_t *__restrict__ keys32,
    const uint8_t *__restrict__ types,
    const uint32_t *__restrict__ acc_txn, const uint8_t *__restrict__ tables, uint64_t n, uint32_t n_txn,
    uint32_t slog, uint64_t *__restrict__ pairs, uint32_t *__restrict__ tb_start, uint32_t *__restrict__ tb_end,
    uint8_t *__restrict__ tlen, uint32_t *__restrict__ acc_row, Counters *ctr, uint32_t *__restrict__ counts,
    uint32_t ntiles, const uint64_t *__restrict__ ts, const uint64_t *__restrict__ rsv_cols) {
    probe_body<true, RSV>(tabs, keys, keys32, types, acc_txn, tables, n, n_txn, slog, pairs, tb_start, tb_end, tlen,
                          acc_row, ctr, counts, ntiles, n_txn, ts, nullptr, rsv_cols);
}

void launch_probe(hipStream_t s, const Tables &tabs, const uint64_t *keys, const uint8_t *types,
                  const uint32_t *acc_txn, const uint8_t *tables, uint64_t n_acc, uint32_t n_txn,
                  uint32_t slog, uint64_t *pairs, uint32_t *tb_start, uint32_t *tb_end,
                  uint8_t *tlen, uint32_t *acc_row, Counters *ctr, uint32_t *counts, uint32_t pair_limit,
                  hipEvent_t ev0, hipEvent_t ev1, const uint32_t *keys32, const uint64_t *ts,
                  const uint32_t *n_dev, const uint64_t *rsv_cols) {
    if (n_acc == 0) return;
    const uint32_t ntiles = nblocks_for(n_acc);
    if (pair_limit < n_txn || n_dev) counts = nullptr;  // the prefix's keys only / a device count: no first histogram
    const uint64_t units = counts ? ntiles : (n_acc + (uint64_t)kBlock * kPV - 1) / ((uint64_t)kBlock * kPV);
    const uint32_t blocks = units > 4096 ? 4096u : (uint32_t)units;
    // (ev0 / ev1: the launch's own dispatch timestamps, no extra packets)
    const uint32_t lim = pair_limit < n_txn ? pair_limit : n_txn;
    if (counts && rsv_cols)
        DV_LAUNCH_EV(k_probe_hist<true>, blocks, kBlock, 0, s, ev0, ev1, tabs, keys, keys32, types,
                              acc_txn, tables, n_acc, n_txn, slog, pairs, tb_start, tb_end, tlen, acc_row, ctr,
                              counts, ntiles, ts, rsv_cols);
    else if (counts)
        DV_LAUNCH_EV(k_probe_hist<false>, blocks, kBlock, 0, s, ev0, ev1, tabs, keys, keys32, types,
                              acc_txn, tables, n_acc, n_txn, slog, pairs, tb_start, tb_end, tlen, acc_row, ctr,
                              counts, ntiles, ts, nullptr);
    else if (rsv_cols)
        DV_LAUNCH_EV(k_probe<true>, blocks, kBlock, 0, s, ev0, ev1, tabs, keys, keys32, types, acc_txn,
                              tables, n_acc, n_txn, slog, pairs, tb_start, tb_end, tlen, acc_row, ctr, lim, ts, n_dev,
                              rsv_cols);
    else
        DV_LAUNCH_EV(k_probe<false>, blocks, kBlock, 0, s, ev0, ev1, tabs, keys, keys32, types, acc_txn,
                              tables, n_acc, n_txn, slog, pairs, tb_start, tb_end, tlen, acc_row, ctr, lim, ts, n_dev,
                              nullptr);
}

// The probe of a prefix-kill epoch whose txn boundaries come with it
// (dv_epoch_dev::txn_begin): nothing per access is derived here any more --
// each txn's range is [txn_begin[t], txn_begin[t + 1]) for every later kernel
// -- so this launch touches only what the prefix's decision needs: a thread
// per prefix txn (t < K) probes its accesses (IndexHash::index_read,
// index_hash.cpp:137-153) into acc_row and the prefix's sort keys, and every
// txn's boundaries are checked (ascending from 0 to n_acc: else ERRB_TXN; a
// txn longer than 1 << slog: ERRB_BIG; WAIT_DIE timestamps rising: else
// ERRB_TS).  The accesses after the prefix are probed by the kill pass
// (k_kill with keys), which reads their keys once anyway.  Config D: 4.4 MB of
// boundaries + the prefix's 3.3 MB instead of 190 MB.
__global__ __launch_bounds__(kBlock) void k_probe_tb(Tables tabs, const uint64_t *__restrict__ keys,
                                                     const uint8_t *__restrict__ types,
                                                     const uint32_t *__restrict__ recs,
                                                     const uint32_t *__restrict__ txn_begin, uint64_t n_acc,
                                                     uint32_t n_txn, uint32_t K, uint32_t slog,
                                                     uint64_t *__restrict__ pairs, uint8_t *__restrict__ tlen,
                                                     uint32_t *__restrict__ acc_row, Counters *ctr,
                                                     const uint64_t *__restrict__ ts,
                                                     const uint32_t *__restrict__ n_acc_dev) {
    // (a device-side count: n_acc is its bound -- the closed loop's epochs)
    if (n_acc_dev && (uint64_t)*n_acc_dev < n_acc) n_acc = *n_acc_dev;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        ctr->n_acc = (uint32_t)n_acc;
        const uint64_t ak = txn_begin[K];
        ctr->a_acc = (uint32_t)(ak < n_acc ? ak : n_acc);  // (a bad boundary is ERRB_TXN below)
        if (txn_begin[0] != 0u || txn_begin[n_txn] != n_acc) set_err(ctr, ERRB_TXN);
    }
    bool bad = false, big_seen = false, ts_bad = false;
    for (uint32_t t = blockIdx.x * kBlock + threadIdx.x; t < n_txn; t += gridDim.x * kBlock) {
        const uint32_t a0 = txn_begin[t], a1 = txn_begin[t + 1];
        if (a1 < a0 || a1 > n_acc) {
            bad = true;
            continue;
        }
        const uint32_t len = a1 - a0;
        const bool big = len > (1u << slog);
        big_seen |= big;
        if (ts && t > 0 && ts[t] <= ts[t - 1]) ts_bad = true;
        if (t >= K) continue;
        tlen[t] = (uint8_t)(big ? (1u << slog) : len);
        constexpr uint32_t kU = 8;  // (a chunk's key and type loads in flight together)
        for (uint32_t j0 = 0; j0 < len; j0 += kU) {
            uint64_t key[kU];
            uint32_t wrs[kU];
            const KillKeys kk{tabs, keys, types, recs, 0, 0};
#pragma unroll
            for (uint32_t j = 0; j < kU; j++) {
                wrs[j] = 0;
                key[j] = j0 + j < len ? kk_key(kk, a0 + j0 + j, wrs[j]) : 0ull;
            }
#pragma unroll
            for (uint32_t j = 0; j < kU; j++) {
                if (j0 + j >= len) break;
                uint64_t row = 0;
                probe_row(tabs.t[0], tabs.n > 0, key[j], row, ctr);
                const uint32_t wr = wrs[j];
                const uint32_t pos = j0 + j;
                acc_row[a0 + pos] = (uint32_t)row | (wr ? AR_WR : 0u);
                pairs[a0 + pos] = pair_pack(row, t, (pos >> slog) ? 0u : pos, wr);
            }
        }
    }
    if (bad) set_err(ctr, ERRB_TXN);
    if (big_seen) set_err(ctr, ERRB_BIG);
    if (ts_bad) set_err(ctr, ERRB_TS);
}

void launch_probe_tb(hipStream_t s, const Tables &tabs, const uint64_t *keys, const uint8_t *types,
                     const uint32_t *recs, const uint32_t *txn_begin, uint64_t n_acc, uint32_t n_txn, uint32_t K,
                     uint32_t slog, uint64_t *pairs, uint8_t *tlen, uint32_t *acc_row, Counters *ctr,
                     const uint64_t *ts, hipEvent_t ev0, hipEvent_t ev1, const uint32_t *n_acc_dev) {
#ifndef DVCC_PROBE_TB_GRID
#define DVCC_PROBE_TB_GRID 4096  // (2048: 9.5-9.6 us, 4096: 9.2-9.3, 1024: 11.1 -- profiles/r05_ai)
#endif
    uint32_t g = (n_txn + kBlock - 1) / kBlock;
    g = g < 1 ? 1 : (g > DVCC_PROBE_TB_GRID ? DVCC_PROBE_TB_GRID : g);
    DV_LAUNCH_EV(k_probe_tb, g, kBlock, 0, s, ev0, ev1, tabs, keys, types, recs, txn_begin, n_acc, n_txn, K, slog,
                 pairs, tlen, acc_row, ctr, ts, n_acc_dev);
}

// ------------------------------------------------------------- radix sort
// Each wave owns a contiguous 1024-element sub-tile and walks it in 16 steps of
// 64 consecutive elements, so (step, lane) order == input order: the ballot
// ranks below are stable.

// n_dev (optional): the key count lives on the device (a sub-epoch's size, known
// only to the kernels before it); n and the grid are then upper bounds and the
// tiles past the real count leave at once.
__device__ __forceinline__ uint64_t sort_n(uint64_t n, const uint32_t *n_dev) {
    return n_dev && (uint64_t)*n_dev < n ? (uint64_t)*n_dev : n;
}

// the radix digit of a sort key: bits [shift, shift + W) -- or, for the one
// pass of a bucket sort (hmul != 0), the top W bits of the row's hash
// h = row * hmul mod 2^hbits (a bijection on hbits-bit rows: rows sharing a
// bucket differ in h's low hbits - W bits, which k_bucket_sort sorts by).
// Low row bits would bucket TPC-C's NURand ids -- whose low bits lean to
// ones -- a tenth of them into one bucket.
__device__ __forceinline__ uint32_t row_hash(uint64_t key, uint32_t hmul, int hbits) {
    return ((uint32_t)(key >> 32) * hmul) & ((1u << hbits) - 1u);
}
template <int W>
__device__ __forceinline__ uint32_t key_digit(uint64_t key, int shift, uint32_t hmul, int hbits) {
    return hmul ? row_hash(key, hmul, hbits) >> (hbits - W) : (uint32_t)(key >> shift) & ((1u << W) - 1u);
}

__global__ __launch_bounds__(kBlock) void k_radix_hist(const uint64_t *__restrict__ in, uint64_t n,
                                                       int shift, uint32_t *__restrict__ counts,
                                                       uint32_t nblocks, const uint32_t *__restrict__ n_dev,
                                                       uint32_t hmul, int hbits) {
    __shared__ uint32_t wc[4][kRadix];
    n = sort_n(n, n_dev);
    if ((uint64_t)blockIdx.x * kTile >= n) return;
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
    // counts only: one LDS atomic per key into the wave's own histogram (the
    // ballot multisplit that ranks keys in the scatter costs 8 ballots each)
    // (a step whose keys all share one digit -- hot rows, high digits of
    // small row ids -- adds once instead of 64 times to one LDS word)
#pragma unroll
    for (int j = 0; j < kIPT; j++) {
        const uint64_t idx = base + j * 64 + lane;
        const bool valid = idx < n;
        const uint32_t d = key_digit<kRadixBits>(k[j], shift, hmul, hbits);
        const uint32_t d0 = __builtin_amdgcn_readfirstlane(d);
        const uint64_t vmask = __ballot(valid);
        if (__ballot(valid && d == d0) == vmask) {
            if (lane == 0) wc[wave][d0] += (uint32_t)__popcll(vmask);
        } else if (valid) {
            atomicAdd(&wc[wave][d], 1u);
        }
    }
    __syncthreads();
    for (uint32_t d = tid; d < kRadix; d += kBlock)
        counts[(uint64_t)d * nblocks + blockIdx.x] = wc[0][d] + wc[1][d] + wc[2][d] + wc[3][d];
}

// exclusive scan of counts[d][0..nblocks) in place, one workgroup per digit.
// (Folding it into the histogram launch -- the last-arriving tile scanning
// every digit over write-through counts -- measured 47 us per pass against
// 5.5 + 4.2: one workgroup's dependent cross-XCD loads cost more than the
// kernel boundary they save.)
__global__ __launch_bounds__(kBlock) void k_radix_scan(uint32_t *__restrict__ counts, uint32_t nblocks,
                                                       uint32_t *__restrict__ digit_tot,
                                                       const uint32_t *__restrict__ n_dev) {
    __shared__ uint32_t lds4[4];
    uint32_t *c = counts + (uint64_t)blockIdx.x * nblocks;  // (row stride: the upper bound)
    if (n_dev && nblocks_for(*n_dev) < nblocks) nblocks = nblocks_for(*n_dev);
    const uint32_t tot = block_chunk_scan256(c, nblocks, lds4);
    if (threadIdx.x == 0) digit_tot[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kBlock) void k_radix_scatter(
    const uint64_t *__restrict__ in, uint64_t *__restrict__ out, uint64_t n, int shift, const uint32_t *__restrict__ counts,
    const uint32_t *__restrict__ digit_tot, uint32_t nblocks, const uint32_t *__restrict__ n_dev,
    uint32_t hmul, int hbits) {
    __shared__ __attribute__((aligned(16))) uint64_t skeys[kTile];
    n = sort_n(n, n_dev);
    if ((uint64_t)blockIdx.x * kTile >= n) return;
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
    uint32_t r[kIPT];
#pragma unroll
    for (int j = 0; j < kIPT; j++) {
        const uint64_t idx = base + j * 64 + lane;
        k[j] = idx < n ? in[idx] : 0;
    }
#pragma unroll
    for (int j = 0; j < kIPT; j++) {
        const uint64_t idx = base + j * 64 + lane;
        const bool valid = idx < n;
        const uint32_t d = key_digit<kRadixBits>(k[j], shift, hmul, hbits);
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
            const uint32_t d = key_digit<kRadixBits>(k[j], shift, hmul, hbits);
            const uint32_t pos = dstart[d] + wc[wave][d] + r[j];
            skeys[pos] = k[j];
        }
    }
    __syncthreads();
    const uint32_t tile_n = (uint32_t)((n - tile0) < (uint64_t)kTile ? (n - tile0) : kTile);
    for (uint32_t p = tid; p < tile_n; p += kBlock) {
        const uint64_t key = skeys[p];
        const uint32_t d = key_digit<kRadixBits>(key, shift, hmul, hbits);
        const uint64_t dst = gbase[d] + p;
        out[dst] = key;
    }
}

// ---- 9- and 10-bit digits: one pass fewer where that is all it takes
// (27-bit global rows of an 8-partition epoch group: 3 passes of 9 instead of
// 4 of 8; 17-20-bit rows: 2 of 9-10 instead of 3).  Wider digits were
// measured slower per pass than they save (rejected).  Same
// structure: per-tile histograms, one scan block per digit (k_radix_scan), a
// stable scatter ranking keys by wave ballots (W per step).
template <int W>
__global__ __launch_bounds__(kBlock) void k_radix_hist_w(const uint64_t *__restrict__ in, uint64_t n, int shift,
                                                         uint32_t *__restrict__ counts, uint32_t nblocks,
                                                         const uint32_t *__restrict__ n_dev, uint32_t hmul,
                                                         int hbits) {
    constexpr uint32_t R = 1u << W;
    __shared__ uint32_t wc[4][R];
    n = sort_n(n, n_dev);
    if ((uint64_t)blockIdx.x * kTile >= n) return;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (uint32_t d = tid; d < 4 * R; d += kBlock) (&wc[0][0])[d] = 0;
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
        const uint32_t d = key_digit<W>(k[j], shift, hmul, hbits);
        const uint32_t d0 = __builtin_amdgcn_readfirstlane(d);
        const uint64_t vmask = __ballot(valid);
        if (__ballot(valid && d == d0) == vmask) {
            if (lane == 0) wc[wave][d0] += (uint32_t)__popcll(vmask);
        } else if (valid) {
            atomicAdd(&wc[wave][d], 1u);
        }
    }
    __syncthreads();
    for (uint32_t d = tid; d < R; d += kBlock)
        counts[(uint64_t)d * nblocks + blockIdx.x] = wc[0][d] + wc[1][d] + wc[2][d] + wc[3][d];
}

template <int W>
__global__ __launch_bounds__(kBlock) void k_radix_scatter_w(const uint64_t *__restrict__ in, uint64_t *__restrict__ out,
                                                            uint64_t n, int shift, const uint32_t *__restrict__ counts,
                                                            const uint32_t *__restrict__ digit_tot, uint32_t nblocks,
                                                            const uint32_t *__restrict__ n_dev, uint32_t hmul,
                                                            int hbits) {
    constexpr uint32_t R = 1u << W, PER = R / kBlock;  // digits per thread in the digit scans
    __shared__ __attribute__((aligned(16))) uint64_t skeys[kTile];
    __shared__ uint32_t wc[4][R];
    __shared__ uint32_t dstart[R];
    __shared__ uint32_t gbase[R];  // (an epoch holds < 2^32 accesses)
    __shared__ uint32_t lds4[4];
    n = sort_n(n, n_dev);
    if ((uint64_t)blockIdx.x * kTile >= n) return;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t tile0 = (uint64_t)blockIdx.x * kTile;
    {
        // global base of each digit for this tile: the smaller digits' totals
        // + this tile's exclusive prefix within the digit
        uint32_t t[PER], sum = 0;
#pragma unroll
        for (uint32_t q = 0; q < PER; q++) {
            t[q] = digit_tot[tid * PER + q];
            sum += t[q];
        }
        uint32_t pre = block_excl_scan256(sum, lds4, nullptr);
#pragma unroll
        for (uint32_t q = 0; q < PER; q++) {
            const uint32_t d = tid * PER + q;
            gbase[d] = pre + counts[(uint64_t)d * nblocks + blockIdx.x];
            pre += t[q];
            wc[0][d] = wc[1][d] = wc[2][d] = wc[3][d] = 0;
        }
    }
    __syncthreads();
    const uint64_t base = tile0 + wave * (64 * kIPT);
    uint64_t k[kIPT];
    uint32_t r[kIPT];
#pragma unroll
    for (int j = 0; j < kIPT; j++) {
        const uint64_t idx = base + j * 64 + lane;
        k[j] = idx < n ? in[idx] : 0;
    }
#pragma unroll
    for (int j = 0; j < kIPT; j++) {
        const uint64_t idx = base + j * 64 + lane;
        const bool valid = idx < n;
        const uint32_t d = key_digit<W>(k[j], shift, hmul, hbits);
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < W; b++) {
            const uint32_t bit = (d >> b) & 1u;
            const uint64_t m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
        const uint32_t before = wc[wave][d];
        r[j] = before + mask_rank(peers);
        if (valid && lane == (uint32_t)__builtin_ctzll(peers)) wc[wave][d] = before + (uint32_t)__popcll(peers);
    }
    __syncthreads();
    {
        uint32_t tot[PER], sum = 0;
#pragma unroll
        for (uint32_t q = 0; q < PER; q++) {
            const uint32_t d = tid * PER + q;
            const uint32_t c0 = wc[0][d], c1 = wc[1][d], c2 = wc[2][d], c3 = wc[3][d];
            wc[0][d] = 0;
            wc[1][d] = c0;
            wc[2][d] = c0 + c1;
            wc[3][d] = c0 + c1 + c2;
            tot[q] = c0 + c1 + c2 + c3;
            sum += tot[q];
        }
        uint32_t ds = block_excl_scan256(sum, lds4, nullptr);
#pragma unroll
        for (uint32_t q = 0; q < PER; q++) {
            const uint32_t d = tid * PER + q;
            dstart[d] = ds;
            gbase[d] -= ds;
            ds += tot[q];
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kIPT; j++) {
        const uint64_t idx = base + j * 64 + lane;
        if (idx < n) {
            const uint32_t d = key_digit<W>(k[j], shift, hmul, hbits);
            skeys[dstart[d] + wc[wave][d] + r[j]] = k[j];
        }
    }
    __syncthreads();
    const uint32_t tile_n = (uint32_t)((n - tile0) < (uint64_t)kTile ? (n - tile0) : kTile);
    for (uint32_t p = tid; p < tile_n; p += kBlock) {
        const uint64_t key = skeys[p];
        const uint32_t d = key_digit<W>(key, shift, hmul, hbits);
        out[(uint64_t)gbase[d] + p] = key;
    }
}

template <int W>
void wide_pass(hipStream_t s, const uint64_t *in, uint64_t *out, uint64_t n, int shift, uint32_t *counts,
               uint32_t *digit_tot, uint32_t nb, const uint32_t *n_dev, hipEvent_t e0, hipEvent_t e1,
               uint32_t hmul = 0, int hbits = 0) {
    DV_LAUNCH((k_radix_hist_w<W>), nb, kBlock, 0, s, in, n, shift, counts, nb, n_dev, hmul, hbits);
    DV_LAUNCH(k_radix_scan, 1u << W, kBlock, 0, s, counts, nb, digit_tot, n_dev);
    DV_LAUNCH_EV((k_radix_scatter_w<W>), nb, kBlock, 0, s, e0, e1, in, out, n, shift,
                          (const uint32_t *)counts, (const uint32_t *)digit_tot, nb, n_dev, hmul, hbits);
}

// ---- bucket sort (small sorts, dvcc_internal.h bucket_sort_applies) --------
// After one stable pass on the top digit of the row's hash (key_digit) every
// bucket holds its keys in sequence order; a workgroup per bucket then sorts
// them stably by the hash's remaining bits, which tell its rows apart.  The keys stay where they are: the workgroup
// sorts 32-bit tags (remaining row bits << 14 | the key's index in the
// bucket) in LDS with 8-bit digits, wave-ballot ranks as in k_radix_scatter,
// and finally gathers the keys (L2-resident: the bucket was just read) into
// place.  A bucket larger than its LDS (a hot row read by many survivors)
// is sorted the same way from global memory, in 16K-key chunks, with the
// bucket's region of the input buffer as the ping-pong scratch.
constexpr int kBucketThreads = 1024;
constexpr int kBucketWaves = kBucketThreads / 64;
constexpr int kBucketIdxBits = 32 - kBucketHiMax;
constexpr uint32_t kBucketCap = 1u << kBucketIdxBits;       // keys a workgroup sorts in LDS
constexpr int kBucketSteps = (int)kBucketCap / kBucketThreads;  // 64-key steps per wave, at most
// two tag arrays + per-wave digit counts: one workgroup per CU on gfx950
static_assert((2 * kBucketCap + (kBucketWaves + 2) * kRadix + kBucketWaves) * sizeof(uint32_t) <= 160u * 1024u,
              "k_bucket_sort's LDS exceeds gfx950's 160 KiB per workgroup");

// stable rank of this lane's digit among the wave's keys so far (wcw: the
// wave's running digit counts, updated)
__device__ __forceinline__ uint32_t bucket_rank(uint32_t d, bool valid, uint32_t *wcw, uint32_t lane) {
    const uint64_t peers = match_digit(d, __ballot(valid));
    const uint32_t before = wcw[d];
    if (valid && lane == (uint32_t)__builtin_ctzll(peers)) wcw[d] = before + (uint32_t)__popcll(peers);
    return before + mask_rank(peers);
}

// wc[w][d] (keys of digit d in wave w's part of the chunk) -> the position of
// that part's first key: run[d] (the digit's next free slot; advanced by the
// digit's chunk total) or, with run == nullptr, the chunk's own digit-major
// offsets.  Called by every thread.
__device__ __forceinline__ void bucket_bases(uint32_t (*wc)[kRadix], uint32_t *tot, uint32_t *run) {
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    uint32_t sum = 0;
    if (tid < (uint32_t)kRadix) {
#pragma unroll
        for (int w = 0; w < kBucketWaves; w++) {
            const uint32_t c = wc[w][tid];
            wc[w][tid] = sum;
            sum += c;
        }
        if (!run) tot[tid] = sum;
    }
    __syncthreads();
    if (!run && tid < 64) {  // exclusive scan of the 256 digit totals, 4 per lane
        uint32_t v[4], s4 = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            v[q] = tot[4 * lane + q];
            s4 += v[q];
        }
        uint32_t pre = wave_incl_sum(s4, lane) - s4;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            tot[4 * lane + q] = pre;
            pre += v[q];
        }
    }
    if (!run) __syncthreads();
    if (tid < (uint32_t)kRadix) {
        const uint32_t b = run ? run[tid] : tot[tid];
        if (run) run[tid] = b + sum;
#pragma unroll
        for (int w = 0; w < kBucketWaves; w++) wc[w][tid] += b;
    }
    __syncthreads();
}

#ifdef DVCC_BUCKET_STAMPS
// measurement builds only (tools/exp_variant.sh ... -DDVCC_BUCKET_STAMPS): per
// bucket, summed over launches -- [0] launches, [1] wall-clock ticks (100 MHz)
// from the workgroup's start to its end, [2] keys, [3] the most ticks of one
// launch; g_bucket_launch: [0] launches, [1] sum of the launch's slowest
// bucket's ticks, [2] that bucket's keys, [3] the last-workgroup ticket
__device__ unsigned long long g_bucket_stamps[1024 * 4];
__device__ unsigned long long g_bucket_launch[4];
__device__ unsigned long long g_bucket_lmax;
struct BucketStamp {
    uint64_t t0;
    __device__ BucketStamp() : t0(wall_clock64()) {}
    __device__ void done(uint32_t b, uint32_t m) {
        __syncthreads();
        if (threadIdx.x != 0) return;
        const unsigned long long dt = wall_clock64() - t0;
        unsigned long long *w = g_bucket_stamps + (size_t)b * 4;
        atomicAdd(w + 0, 1ull);
        atomicAdd(w + 1, dt);
        atomicAdd(w + 2, (unsigned long long)m);
        atomicMax(w + 3, dt);
        atomicMax(&g_bucket_lmax, (dt << 20) | m);
        __threadfence();
        if (atomicAdd(&g_bucket_launch[3], 1ull) == (unsigned long long)gridDim.x - 1) {
            __threadfence();
            const unsigned long long mx = atomicExch(&g_bucket_lmax, 0ull);
            atomicAdd(&g_bucket_launch[0], 1ull);
            atomicAdd(&g_bucket_launch[1], mx >> 20);
            atomicAdd(&g_bucket_launch[2], mx & 0xFFFFFull);
            g_bucket_launch[3] = 0;
        }
    }
};
extern "C" int dv_debug_bucket_stamps(uint64_t *out, uint64_t *launch) {
    if (!out || !launch) return DV_ERR_ARG;
    if (hipDeviceSynchronize() != hipSuccess) return DV_ERR_HIP;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bucket_stamps), 1024 * 4 * 8) != hipSuccess) return DV_ERR_HIP;
    if (hipMemcpyFromSymbol(launch, HIP_SYMBOL(g_bucket_launch), 4 * 8) != hipSuccess) return DV_ERR_HIP;
    static const unsigned long long zero[1024 * 4] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_bucket_stamps), zero, sizeof(zero)) != hipSuccess) return DV_ERR_HIP;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_bucket_launch), zero, 4 * 8) != hipSuccess) return DV_ERR_HIP;
    return DV_OK;
}
#endif

__global__ __launch_bounds__(kBucketThreads) void k_bucket_sort(uint64_t *__restrict__ in, uint64_t *__restrict__ out,
                                                                const uint32_t *__restrict__ digit_tot,
                                                                uint32_t hmul, int hbits, int hi_bits) {
#ifdef DVCC_BUCKET_STAMPS
    BucketStamp stamp_;
    struct StampAtExit {
        BucketStamp &s;
        uint32_t b, m;
        __device__ ~StampAtExit() { s.done(b, m); }
    } stamp_exit_{stamp_, blockIdx.x, 0u};
#endif
    __shared__ uint32_t tg[2][kBucketCap];
    __shared__ uint32_t wc[kBucketWaves][kRadix];
    __shared__ uint32_t tot[kRadix], run[kRadix];
    __shared__ uint32_t s_part[kBucketWaves];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, b = blockIdx.x;
    {  // the bucket's offset: the sizes of the buckets before it (gridDim.x <= kBucketThreads)
        uint32_t v = tid < b ? digit_tot[tid] : 0u;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        if (lane == 0) s_part[wave] = v;
    }
    __syncthreads();
    uint32_t base = 0;
#pragma unroll
    for (int w = 0; w < kBucketWaves; w++) base += s_part[w];
    const uint32_t m = digit_tot[b];
#ifdef DVCC_BUCKET_STAMPS
    stamp_exit_.m = m;
#endif
    if (m <= 1) {  // nothing to order (one key: copied into place)
        if (m == 1 && tid == 0) out[base] = in[base];
        return;
    }
    const int passes = (hi_bits + kRadixBits - 1) / kRadixBits;
    const uint32_t hmask = (1u << hi_bits) - 1u;
    if (m <= kBucketCap) {
        {  // every key's load in flight at once (a loop would wait on each)
            uint64_t kv[kBucketSteps];
#pragma unroll
            for (int s = 0; s < kBucketSteps; s++) {
                const uint32_t i = s * kBucketThreads + tid;
                kv[s] = i < m ? in[base + i] : 0ull;
            }
#pragma unroll
            for (int s = 0; s < kBucketSteps; s++) {
                const uint32_t i = s * kBucketThreads + tid;
                if (i < m) tg[0][i] = ((row_hash(kv[s], hmul, hbits) & hmask) << kBucketIdxBits) | i;
            }
        }
        __syncthreads();
        const uint32_t steps = (m + kBucketThreads - 1) / kBucketThreads;
        int cur = 0;
        for (int p = 0; p < passes; p++) {
            const int sh = kBucketIdxBits + kRadixBits * p;
            for (uint32_t d = lane; d < (uint32_t)kRadix; d += 64) wc[wave][d] = 0;
            uint32_t t[kBucketSteps], r[kBucketSteps];
#pragma unroll
            for (int s = 0; s < kBucketSteps; s++) {
                if ((uint32_t)s < steps) {
                    const uint32_t e = (wave * steps + s) * 64 + lane;
                    const bool valid = e < m;
                    t[s] = valid ? tg[cur][e] : 0u;
                    r[s] = bucket_rank((t[s] >> sh) & (kRadix - 1), valid, wc[wave], lane);
                }
            }
            __syncthreads();
            bucket_bases(wc, tot, nullptr);
#pragma unroll
            for (int s = 0; s < kBucketSteps; s++) {
                if ((uint32_t)s < steps) {
                    const uint32_t e = (wave * steps + s) * 64 + lane;
                    if (e < m) tg[cur ^ 1][wc[wave][(t[s] >> sh) & (kRadix - 1)] + r[s]] = t[s];
                }
            }
            __syncthreads();
            cur ^= 1;
        }
        uint64_t kv[kBucketSteps];
#pragma unroll
        for (int s = 0; s < kBucketSteps; s++) {
            const uint32_t i = s * kBucketThreads + tid;
            kv[s] = i < m ? in[base + (tg[cur][i] & (kBucketCap - 1))] : 0ull;
        }
#pragma unroll
        for (int s = 0; s < kBucketSteps; s++) {
            const uint32_t i = s * kBucketThreads + tid;
            if (i < m) out[base + i] = kv[s];
        }
        return;
    }
    // a bucket larger than the LDS: the same passes over global memory, the
    // bucket's region of `in` as scratch
    uint64_t *A = in + base, *B = out + base;
    for (int p = 0; p < passes; p++) {
        const uint64_t *src = (p & 1) ? B : A;
        uint64_t *dst = (p & 1) ? A : B;
        const int sh = kRadixBits * p;
        if (tid < (uint32_t)kRadix) tot[tid] = 0;
        __syncthreads();
        for (uint32_t i0 = 0; i0 < m; i0 += kBucketThreads) {
            const uint32_t i = i0 + tid;
            const bool valid = i < m;
            const uint32_t d = valid ? ((row_hash(src[i], hmul, hbits) & hmask) >> sh) & (kRadix - 1) : 0u;
            const uint32_t d0 = __builtin_amdgcn_readfirstlane(d);
            const uint64_t vm = __ballot(valid);
            if (__ballot(valid && d == d0) == vm) {  // a hot row: one add for the wave
                if (lane == 0 && vm) atomicAdd(&tot[d0], (uint32_t)__popcll(vm));
            } else if (valid) {
                atomicAdd(&tot[d], 1u);
            }
        }
        __syncthreads();
        if (tid < 64) {
            uint32_t v[4], s4 = 0;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                v[q] = tot[4 * lane + q];
                s4 += v[q];
            }
            uint32_t pre = wave_incl_sum(s4, lane) - s4;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                run[4 * lane + q] = pre;
                pre += v[q];
            }
        }
        __syncthreads();
        for (uint32_t c0 = 0; c0 < m; c0 += kBucketCap) {
            const uint32_t mc = m - c0 < kBucketCap ? m - c0 : kBucketCap;
            const uint32_t steps = (mc + kBucketThreads - 1) / kBucketThreads;
            for (uint32_t d = lane; d < (uint32_t)kRadix; d += 64) wc[wave][d] = 0;
            uint64_t k[kBucketSteps];
            uint32_t r[kBucketSteps];
#pragma unroll
            for (int s = 0; s < kBucketSteps; s++) {
                if ((uint32_t)s < steps) {
                    const uint32_t e = (wave * steps + s) * 64 + lane;
                    const bool valid = e < mc;
                    k[s] = valid ? src[c0 + e] : 0ull;
                    r[s] = bucket_rank(((row_hash(k[s], hmul, hbits) & hmask) >> sh) & (kRadix - 1), valid,
                                       wc[wave], lane);
                }
            }
            __syncthreads();
            bucket_bases(wc, tot, run);
#pragma unroll
            for (int s = 0; s < kBucketSteps; s++) {
                if ((uint32_t)s < steps) {
                    const uint32_t e = (wave * steps + s) * 64 + lane;
                    if (e < mc) dst[wc[wave][((row_hash(k[s], hmul, hbits) & hmask) >> sh) & (kRadix - 1)] + r[s]] = k[s];
                }
            }
            __syncthreads();
        }
    }
    if (!(passes & 1)) {  // the result is in the scratch region
        for (uint32_t i = tid; i < m; i += kBucketThreads) B[i] = A[i];
    }
}

int radix_sort_rows(hipStream_t s, uint64_t *pairs[2], uint64_t n, int key_bits, uint32_t *counts,
                    uint32_t *digit_tot, hipEvent_t *scatter_ev, bool hist0_done, const uint32_t *n_dev,
                    bool lsd_only) {
    if (n == 0) return 0;
    const uint32_t nb = nblocks_for(n);
    int cur = 0, pass = 0;
    if (!lsd_only && bucket_sort_applies(n, key_bits, hist0_done, n_dev != nullptr)) {
        const int lo = kBucketLoBits(key_bits);
        const uint32_t hmul = kRowHashMul;
        hipEvent_t e0 = scatter_ev ? scatter_ev[0] : nullptr, e1 = scatter_ev ? scatter_ev[1] : nullptr;
        if (lo == 9)
            wide_pass<9>(s, pairs[0], pairs[1], n, 32, counts, digit_tot, nb, n_dev, e0, e1, hmul, key_bits);
        else if (lo == 10)
            wide_pass<10>(s, pairs[0], pairs[1], n, 32, counts, digit_tot, nb, n_dev, e0, e1, hmul, key_bits);
        else {
            DV_LAUNCH(k_radix_hist, nb, kBlock, 0, s, pairs[0], n, 32, counts, nb, n_dev, hmul, key_bits);
            DV_LAUNCH(k_radix_scan, kRadix, kBlock, 0, s, counts, nb, digit_tot, n_dev);
            DV_LAUNCH_EV(k_radix_scatter, nb, kBlock, 0, s, e0, e1, (const uint64_t *)pairs[0], pairs[1], n, 32,
                         (const uint32_t *)counts, (const uint32_t *)digit_tot, nb, n_dev, hmul, key_bits);
        }
        DV_LAUNCH_EV(k_bucket_sort, 1u << lo, kBucketThreads, 0, s, scatter_ev ? scatter_ev[2] : nullptr,
                     scatter_ev ? scatter_ev[3] : nullptr, pairs[1], pairs[0], (const uint32_t *)digit_tot,
                     hmul, key_bits, key_bits - lo);
        return 0;
    }
    const int wbits = radix_digit_bits(key_bits, hist0_done);
    if (wbits > kRadixBits) {
        for (int bit = 0; bit < key_bits; bit += wbits, pass++) {
            hipEvent_t e0 = scatter_ev ? scatter_ev[2 * pass] : nullptr, e1 = scatter_ev ? scatter_ev[2 * pass + 1] : nullptr;
            if (wbits == 9)
                wide_pass<9>(s, pairs[cur], pairs[cur ^ 1], n, 32 + bit, counts, digit_tot, nb, n_dev, e0, e1);
            else
                wide_pass<10>(s, pairs[cur], pairs[cur ^ 1], n, 32 + bit, counts, digit_tot, nb, n_dev, e0, e1);
            cur ^= 1;
        }
        return cur;
    }
    for (int bit = 0; bit < key_bits; bit += kRadixBits, pass++) {
        const int shift = 32 + bit;
        if (pass > 0 || !hist0_done)
            DV_LAUNCH(k_radix_hist, nb, kBlock, 0, s, pairs[cur], n, shift, counts, nb, n_dev, 0u, 0);
        DV_LAUNCH(k_radix_scan, kRadix, kBlock, 0, s, counts, nb, digit_tot, n_dev);
        // timing: events recorded by the dispatch itself (no extra packets)
        DV_LAUNCH_EV(k_radix_scatter, nb, kBlock, 0, s, scatter_ev ? scatter_ev[2 * pass] : nullptr,
                     scatter_ev ? scatter_ev[2 * pass + 1] : nullptr, (const uint64_t *)pairs[cur], pairs[cur ^ 1], n,
                     shift, (const uint32_t *)counts, (const uint32_t *)digit_tot, nb, n_dev, 0u, 0);
        cur ^= 1;
    }
    return cur;
}

// ------------------------------------------------------- queue elements
// Row-queue element of sorted position i: queue heads, repeats of one txn on
// one row (an error for 2PL/OCC; Calvin merges them into one lock request),
// Calvin grant-group boundaries, and the access id tb_start[txn] + pos.
// kPV consecutive keys per thread, vector loads and stores.
__device__ __forceinline__ uint32_t prev_entry_wr(const uint64_t *__restrict__ pairs, uint64_t e) {
    // lock type of the queue entry ending at e: a repeat access keeps the type
    // of its txn's first access to the row (TxnManager::get_lock, txn.cpp:778-788)
    const uint64_t pe = pairs[e];
    while (e > 0) {
        const uint64_t qq = pairs[e - 1];
        if (pair_row(qq) != pair_row(pe) || pair_txn(qq) != pair_txn(pe)) break;
        e--;
    }
    return (uint32_t)pairs[e] & 1u;
}

__global__ __launch_bounds__(kBlock) void k_seg_prepare(const uint64_t *__restrict__ pairs, uint64_t n,
                                                        int calvin,
                                                        const uint32_t *__restrict__ tb_start,
                                                        uint64_t *__restrict__ el, Counters *ctr) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t per_block = (uint64_t)kBlock * kPV;
    const uint64_t stride = (uint64_t)gridDim.x * per_block;
    for (uint64_t b0 = (uint64_t)blockIdx.x * per_block; b0 < n; b0 += stride) {
        const uint64_t i0 = b0 + (uint64_t)threadIdx.x * kPV;
        uint64_t p[kPV];
        if (i0 + kPV <= n) {
            const ulonglong2 a0 = *reinterpret_cast<const ulonglong2 *>(pairs + i0);
            const ulonglong2 a1 = *reinterpret_cast<const ulonglong2 *>(pairs + i0 + 2);
            p[0] = a0.x; p[1] = a0.y; p[2] = a1.x; p[3] = a1.y;
        } else {
#pragma unroll
            for (int j = 0; j < kPV; j++) p[j] = i0 + j < n ? pairs[i0 + j] : ~0ull;
        }
        uint64_t q = __shfl_up(p[kPV - 1], 1, 64);
        if (lane == 0) q = i0 > 0 && i0 - 1 < n ? pairs[i0 - 1] : ~0ull;
        uint32_t acc[kPV];
#pragma unroll
        for (int j = 0; j < kPV; j++) acc[j] = i0 + j < n ? tb_start[pair_txn(p[j])] + pair_pos(p[j]) : 0u;
        uint64_t out[kPV];
        bool dup_err = false;
#pragma unroll
        for (int j = 0; j < kPV; j++) {
            const uint64_t i = i0 + j;
            const uint64_t pj = p[j];
            const uint64_t pq = j == 0 ? q : p[j - 1];
            const uint32_t wr = (uint32_t)pj & 1u;
            uint32_t head = 1, dup = 0, bnd = 1;
            if (i > 0 && pair_row(pq) == pair_row(pj)) {
                head = 0;
                dup = pair_txn(pq) == pair_txn(pj);
                if (calvin) {
                    uint32_t pwr = (uint32_t)pq & 1u;
                    if (i >= 2 && pair_txn(pairs[i - 2]) == pair_txn(pq) && pair_row(pairs[i - 2]) == pair_row(pq))
                        pwr = prev_entry_wr(pairs, i - 1);  // the previous entry is itself a repeat run
                    bnd = dup ? 0u : ((wr | pwr) ? 1u : 0u);
                }
            }
            dup_err |= dup && i < n;
            out[j] = el_pack(pair_txn(pj), acc[j],
                             ((calvin && bnd) ? EL_BND : 0u) | (dup ? EL_DUP : 0u) | (head ? EL_HEAD : 0u) | wr);
        }
        if (dup_err) {
            if (calvin) ctr->calvin_dups = 1u;  // k_calvin_dup_fix has work
            else set_err(ctr, ERRB_DUP);
        }
        if (i0 + kPV <= n) {
            *reinterpret_cast<ulonglong2 *>(el + i0) = ulonglong2{out[0], out[1]};
            *reinterpret_cast<ulonglong2 *>(el + i0 + 2) = ulonglong2{out[2], out[3]};
        } else {
            for (int j = 0; j < kPV; j++)
                if (i0 + j < n) el[i0 + j] = out[j];
        }
    }
}

void launch_seg_prepare(hipStream_t s, const uint64_t *pairs, uint64_t n, int calvin,
                        const uint32_t *tb_start, uint64_t *el, Counters *ctr) {
    if (n == 0) return;
    uint64_t blocks = (n + (uint64_t)kBlock * kPV - 1) / ((uint64_t)kBlock * kPV);
    if (blocks > 4096) blocks = 4096;
    DV_LAUNCH(k_seg_prepare, (uint32_t)blocks, kBlock, 0, s, pairs, n, calvin, tb_start, el, ctr);
}

// ------------------------------------------------------- Calvin grants
// Per row queue (sequence order), a request is granted together with the
// requests in front of it when they are all shared: grant groups are maximal
// runs of SH requests, each EX alone (CALVIN lock_get queues behind any
// waiter, row_lock.cpp:78-81, 152-170; lock_release promotes compatible FIFO
// waiters, 318-358).  grant group = (boundaries so far in the queue) - 1, one
// OpSeg scan; ew = a WR of an earlier txn precedes the access in its queue
// (its read sees that write under the serial order).
__global__ __launch_bounds__(kBlock) void k_calvin_pass(const uint64_t *__restrict__ el, uint32_t n,
                                                        uint32_t *__restrict__ grant,
                                                        uint8_t *__restrict__ ew, uint64_t *desc,
                                                        uint32_t *tile_ctr, uint32_t tag,
                                                        Counters *ctr) {
    __shared__ uint64_t s_el[kRTile + kRTile / kRIPT];
    __shared__ uint64_t s_next;
    __shared__ uint32_t s_tile;
    __shared__ Agg wt[4];
    __shared__ Agg s_pre;
    const uint32_t ntiles = (n + kRTile - 1) / kRTile;
    if (blockIdx.x >= ntiles) return;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) s_tile = atomicAdd(tile_ctr, 1u);
    __syncthreads();
    const uint32_t tile = s_tile;
    const uint32_t base = tile * kRTile;
    const uint32_t tile_n = n - base < (uint32_t)kRTile ? n - base : (uint32_t)kRTile;
    load_tile64(el, base, tile_n, n, s_el, &s_next);
    __syncthreads();
    const uint32_t first = tid * kRIPT;
    const int cnt = first >= tile_n ? 0 : (tile_n - first < (uint32_t)kRIPT ? (int)(tile_n - first) : kRIPT);
    uint64_t e[kRIPT];
    Agg a{0u, 0u, 0u};
#pragma unroll
    for (int j = 0; j < kRIPT; j++) {
        e[j] = j < cnt ? s_el[rpad(first + j)] : (uint64_t)EL_HEAD;
        if (j < cnt) {
            const Agg x{(uint32_t)((e[j] & EL_HEAD) != 0), (uint32_t)(e[j] & EL_WR),
                        (uint32_t)((e[j] & EL_BND) != 0)};
            a = OpSeg::comb(a, x);
        }
    }
    const Agg inc = wave_incl<OpSeg>(a, lane);
    if (lane == 63) wt[wave] = inc;
    __syncthreads();
    if (wave == 0) {
        Agg bagg = wt[0];
        for (int w = 1; w < 4; w++) bagg = OpSeg::comb(bagg, wt[w]);
        const Agg pre = look_back<OpSeg>(desc, tile, tag, bagg, lane, ctr);
        if (lane == 0) s_pre = pre;
    }
    __syncthreads();
    Agg run = s_pre;
    for (uint32_t w = 0; w < wave; w++) run = OpSeg::comb(run, wt[w]);
    run = OpSeg::comb(run, wave_excl_from_incl<OpSeg>(inc, lane));
#pragma unroll
    for (int j = 0; j < kRIPT; j++) {
        if (j < cnt) {
            const bool head = (e[j] & EL_HEAD) != 0;
            const uint32_t bnd = (e[j] & EL_BND) ? 1u : 0u;
            const uint32_t incl = (head ? 0u : run.c) + bnd;
            if (grant) grant[el_acc(e[j])] = incl - 1u;
            ew[base + first + j] = (uint8_t)(head ? 0u : (run.v & 1u));
            run = OpSeg::comb(run, Agg{head ? 1u : 0u, (uint32_t)(e[j] & EL_WR), bnd});
        }
    }
}

// A txn that touches a row several times reads it before any of its own
// writes (run_calvin_txn: the reads, then the writes, ycsb_txn.cpp:327-353),
// so a repeat access's "earlier WR" flag is its group's first access's:
// own writes in front of it do not count.  Only launched work when
// k_seg_prepare saw a repeat.
__global__ __launch_bounds__(kBlock) void k_calvin_dup_fix(const uint64_t *__restrict__ el, uint64_t n,
                                                           uint8_t *__restrict__ ew, const Counters *ctr) {
    if (!ctr->calvin_dups) return;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock) {
        if (!(el[i] & EL_DUP)) continue;
        uint64_t j = i;
        while (j > 0 && (el[j] & EL_DUP)) j--;
        ew[i] = ew[j];
    }
}

void calvin_grant(hipStream_t s, const uint64_t *el, uint64_t n, uint32_t *grant_out, uint8_t *ew,
                  uint64_t *desc, uint32_t *tile_ctr, uint32_t tag, Counters *ctr) {
    if (n == 0) return;
    const uint32_t nb = (uint32_t)((n + kRTile - 1) / kRTile);
    DV_LAUNCH(k_calvin_pass, nb, kBlock, 0, s, el, (uint32_t)n, grant_out, ew, desc, tile_ctr, tag, ctr);
    const uint64_t fb = (n + kBlock - 1) / kBlock;
    DV_LAUNCH(k_calvin_dup_fix, (uint32_t)(fb > 1024 ? 1024 : fb), kBlock, 0, s, el, n, ew, ctr);
}

// ---------------------------------------------------------------- status
// Per-epoch state in one launch (instead of a fill per buffer): the counters
// block and tile tickets (block 0), every txn's status byte (padding txns
// aborted), and its access range / count (txns without accesses here keep an
// empty range).
__global__ __launch_bounds__(kBlock) void k_epoch_clear(uint8_t *__restrict__ status, uint32_t n_txn,
                                                        uint32_t n_pad, uint8_t value,
                                                        uint32_t *__restrict__ tb_start,
                                                        uint32_t *__restrict__ tb_end,
                                                        uint8_t *__restrict__ tlen,
                                                        uint32_t *__restrict__ tile_ctr,
                                                        const uint32_t *__restrict__ err_seed, Counters *ctr,
                                                        uint4 *__restrict__ zero, uint64_t zero_n, int gate,
                                                        Counters *hctr, unsigned long long *hseq,
                                                        unsigned long long seq, uint64_t *__restrict__ zero8,
                                                        uint64_t *__restrict__ desc, uint32_t n_desc) {
    if (blockIdx.x == 0) {
        // pipelined epochs: the previous epoch's counters into their host
        // mirror first (what k_ctr_out would have done as one more launch)
        if (hctr) {
            const uint32_t *src = reinterpret_cast<const uint32_t *>(ctr);
            uint32_t *dst = reinterpret_cast<uint32_t *>(hctr);
            for (uint32_t i = threadIdx.x; i < sizeof(Counters) / 4; i += kBlock) dst[i] = src[i];
            __threadfence_system();
            __syncthreads();
            if (threadIdx.x == 0) __hip_atomic_store(hseq, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        // gate (pipelined epochs, dv_epoch_run_device_batch): the previous
        // epoch is still unread by the host; if it halted or failed, this one
        // starts halted, so nothing of it reaches the tables or the commit bytes
        __shared__ uint32_t s_gate;
        if (threadIdx.x == 0) s_gate = gate && (ctr->halt | ctr->a_halt | ctr->err | ctr->peer_err) ? 1u : 0u;
        __syncthreads();
        uint32_t *w = reinterpret_cast<uint32_t *>(ctr);
        for (uint32_t i = threadIdx.x; i < sizeof(Counters) / 4; i += kBlock) w[i] = 0;
        for (uint32_t i = threadIdx.x; i < kTileCtrs; i += kBlock) tile_ctr[i] = 0;
        // an epoch replayed from a graph reuses its look-back tags: no
        // descriptor of an earlier epoch may carry one of them
        for (uint32_t i = threadIdx.x; i < n_desc; i += kBlock) desc[i] = 0;
        __syncthreads();
        // errors found before the epoch began (the host-record check)
        if (threadIdx.x == 0 && err_seed) ctr->err = *err_seed;
        if (threadIdx.x == 0 && s_gate) ctr->halt = 1u;
    }
    const uint32_t stride = gridDim.x * kBlock;
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n_pad; i += stride) {
        status[i] = i < n_txn ? value : (uint8_t)ST_ABORT;
        if (tb_start) {  // (null: the epoch's ranges come with it, dv_epoch_dev::txn_begin)
            tb_start[i] = 0;
            tb_end[i] = 0;
        }
        if (tlen) tlen[i] = 0;
        if (zero8 && i < n_txn) zero8[i] = 0;
    }
    for (uint64_t i = blockIdx.x * kBlock + threadIdx.x; i < zero_n; i += stride) zero[i] = uint4{0, 0, 0, 0};
}

// the counters into their host-mapped mirror, then the sequence word the
// host spins on (sync_counters): no blit and no stream synchronisation
// between an epoch's last kernel and the host reading its outcome
__global__ __launch_bounds__(kBlock) void k_ctr_out(const Counters *__restrict__ ctr, Counters *hctr,
                                                    unsigned long long *hseq, unsigned long long seq) {
    const uint32_t *src = reinterpret_cast<const uint32_t *>(ctr);
    uint32_t *dst = reinterpret_cast<uint32_t *>(hctr);
    for (uint32_t i = threadIdx.x; i < sizeof(Counters) / 4; i += kBlock) dst[i] = src[i];
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(hseq, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

void launch_ctr_out(hipStream_t s, const Counters *ctr, Counters *hctr, unsigned long long *hseq,
                    unsigned long long seq) {
    DV_LAUNCH(k_ctr_out, 1, kBlock, 0, s, ctr, hctr, hseq, seq);
}

// Decision lanes' execution order (run_lanes), kept on the device in words
// that stay the same from epoch to epoch, so an epoch's execution can be part
// of its replayed graph: each lane holds its next turn in the chain of
// executions (*turn), the lanes share one word *done = (turns executed << 1)
// | gate, the gate set when the last one halted or failed.  An execution
// waits until *done reaches its turn and starts halted when the gate is set
// (nothing of it executes; the host runs both again, in order); after it,
// its lane posts turn + 1 with its own gate and advances its turn by the
// lane count.  The host sets the words while the lanes are idle (run_lanes,
// at the start of every run of pipelined epochs).  Kernel boundaries on
// either side order the rows: the execution's writes are released before the
// post, the next execution starts after the wait.  (An event recorded on one
// lane's stream and waited for on the next cost the host 13-15 us per graph
// launch behind it instead of 3-4.)
__global__ void k_lane_post(uint32_t *turn, uint32_t *done, uint32_t n_lanes, const Counters *__restrict__ ctr) {
    if (threadIdx.x != 0) return;
    const uint32_t t = *turn;
    const uint32_t gate = (ctr->halt | ctr->a_halt | ctr->err | ctr->peer_err) ? 1u : 0u;
    // done only moves forward: a successor whose wait timed out has posted a
    // later turn already (halted, gate set), and a late post must not take it back
    const uint32_t want = ((t + 1u) << 1) | gate;
    uint32_t old = __hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while ((int32_t)((old >> 1) - (t + 1u)) < 0 &&
           !__hip_atomic_compare_exchange_strong(done, &old, want, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)) {
    }
    *turn = t + n_lanes;
}

// the wait is bounded: a predecessor that has not posted after kLaneWaitTicks
// (1 s of the 100-MHz clock) halts this epoch too, so the grid always drains
constexpr uint64_t kLaneWaitTicks = 100000000ull;
__global__ void k_lane_wait(const uint32_t *turn, const uint32_t *done, Counters *ctr) {
    if (threadIdx.x != 0) return;
    const uint32_t t = *turn & 0x7FFFFFFFu;
    const uint64_t t0 = wall_clock64();
    uint32_t v;
    // (past this turn already: a later epoch timed out and posted, gate set)
    while ((int32_t)(((v = __hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 1) - t) < 0) {
        if (wall_clock64() - t0 > kLaneWaitTicks) {
            ctr->halt = 1u;
            return;
        }
        __builtin_amdgcn_s_sleep(2);
    }
    if (v & 1u) ctr->halt = 1u;
}

void launch_lane_post(hipStream_t s, uint32_t *turn, uint32_t *done, uint32_t n_lanes, const Counters *ctr) {
    DV_LAUNCH(k_lane_post, 1, 64, 0, s, turn, done, n_lanes, ctr);
}

void launch_lane_wait(hipStream_t s, const uint32_t *turn, const uint32_t *done, Counters *ctr) {
    DV_LAUNCH(k_lane_wait, 1, 64, 0, s, turn, done, ctr);
}

void launch_epoch_clear(hipStream_t s, uint8_t *status, uint32_t n_txn, uint32_t n_txn_pad4, uint8_t value,
                        uint32_t *tb_start, uint32_t *tb_end, uint8_t *tlen, uint32_t *tile_ctr,
                        const uint32_t *err_seed, Counters *ctr, uint32_t *zero, uint64_t zero_words, bool gate,
                        Counters *hctr, unsigned long long *hseq, unsigned long long seq, uint64_t *txn_zero8,
                        uint64_t *desc, uint32_t n_desc) {
#ifndef DVCC_CLEAR_GRID
#define DVCC_CLEAR_GRID 2048
#endif
    uint32_t g = (n_txn_pad4 + kBlock - 1) / kBlock;
    g = g < 1 ? 1 : (g > DVCC_CLEAR_GRID ? DVCC_CLEAR_GRID : g);
    // zero: a 16-byte aligned area of zero_words 32-bit words (a multiple of 4)
    DV_LAUNCH(k_epoch_clear, g, kBlock, 0, s, status, n_txn, n_txn_pad4, value, tb_start, tb_end, tlen, tile_ctr,
                                       err_seed, ctr, reinterpret_cast<uint4 *>(zero), zero ? zero_words / 4 : 0,
                                       gate ? 1 : 0, hctr, hseq, seq, txn_zero8, desc, n_desc);
}

// ---------------------------------------------------------------- execute
// run_ycsb_1 (ycsb_txn.cpp:227-254) for committed txns: a RD loads the 8-byte
// F0 prefix, a WR stores 0.  Reads see the epoch's initial image unless an
// earlier WR of another txn precedes them in the row queue (Calvin only; under
// NO_WAIT/OCC a committed reader never follows a committed writer).  Reads
// run before writes (two launches) so every read sees the pre-epoch image.
template <bool WRITES>
__global__ __launch_bounds__(kBlock) void k_exec(const uint64_t *__restrict__ pairs,
                                                 const uint64_t *__restrict__ el,
                                                 const uint8_t *__restrict__ ew, uint64_t n,
                                                 const uint8_t *__restrict__ status,
                                                 uint64_t *__restrict__ f0,
                                                 const uint64_t *__restrict__ pkey, Counters *ctr, RowMap rm) {
    __shared__ unsigned long long part[4];
    if (input_err(ctr)) return;  // a rejected epoch changes no row
    const uint64_t per_block = (uint64_t)kBlock * kPV;
    const uint64_t stride = (uint64_t)gridDim.x * per_block;
    unsigned long long acc = 0;
    for (uint64_t i0 = (uint64_t)blockIdx.x * per_block + (uint64_t)threadIdx.x * kPV; i0 < n;
         i0 += stride) {
        uint64_t e[kPV];
        if (i0 + kPV <= n) {
            const ulonglong2 a0 = *reinterpret_cast<const ulonglong2 *>(el + i0);
            const ulonglong2 a1 = *reinterpret_cast<const ulonglong2 *>(el + i0 + 2);
            e[0] = a0.x; e[1] = a0.y; e[2] = a1.x; e[3] = a1.y;
        } else {
#pragma unroll
            for (int j = 0; j < kPV; j++) e[j] = i0 + j < n ? el[i0 + j] : (WRITES ? 0ull : EL_WR);
        }
        uint8_t st[kPV];
#pragma unroll
        for (int j = 0; j < kPV; j++) {
            const bool mine = i0 + j < n && (((e[j] & EL_WR) != 0) == WRITES);
            st[j] = mine ? status[el_txn(e[j])] : (uint8_t)ST_ABORT;
        }
#pragma unroll
        for (int j = 0; j < kPV; j++) {
            if (st[j] != ST_COMMIT) continue;
            uint64_t row = pair_row(pairs[i0 + j]);
            if (!own_row(rm, row)) continue;  // (replicated epochs: another partition's row)
            if (WRITES) {
                f0[row] = 0;  // *(uint64_t*)&data[0] = 0 (ycsb_txn.cpp:239-242)
                acc++;
            } else {
                const uint64_t val = (ew && ew[i0 + j]) ? 0ull : f0[row];
                acc += mix64(val ^ mix64(((uint64_t)el_txn(e[j]) << 32) ^ pkey[row]));
            }
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long t = part[0] + part[1] + part[2] + part[3];
        if (t) atomicAdd(WRITES ? &my_slot(ctr).write_cnt : &my_slot(ctr).read_digest, t);
    }
}

void launch_exec(hipStream_t s, const uint64_t *pairs, const uint64_t *el, const uint8_t *ew,
                 uint64_t n, const uint8_t *status, uint64_t *f0, const uint64_t *pkey,
                 Counters *ctr, RowMap rm) {
    if (n == 0) return;
    uint64_t blocks = (n + (uint64_t)kBlock * kPV - 1) / ((uint64_t)kBlock * kPV);
    if (blocks > 2048) blocks = 2048;
    DV_LAUNCH((k_exec<false>), (uint32_t)blocks, kBlock, 0, s, pairs, el, ew, n, status, f0, pkey, ctr, rm);
    DV_LAUNCH((k_exec<true>), (uint32_t)blocks, kBlock, 0, s, pairs, el, ew, n, status, f0, pkey, ctr, rm);
}

// NO_WAIT / WAIT_DIE / OCC: run_ycsb_1 for the committed txns only (acc_row
// from the probe).  A committed reader never sees a committed writer's value
// here (2PL: the two conflict, so one launch does both; OCC: reads happen in
// the access phase, occ.cpp:116-294, so the reads run in a launch before the
// writes).  Each wave takes 64 consecutive txns and spreads the accesses of
// its committed ones over its lanes (a prefix sum of their lengths): at a
// ~2 % commit rate a thread per txn left most lanes idle behind a few serial
// access loops, and at high commit rates this keeps every lane busy.
// COMMIT (the launch that reads, the first): also the commit bytes and the
// committed count, what k_commit_out does -- for a rejected epoch too, whose
// rows stay untouched.
enum : int { EX_READS = 1, EX_WRITES = 2, EX_COMMIT = 4 };
template <int MODE>
__global__ __launch_bounds__(kBlock) void k_exec_txn(const uint32_t *__restrict__ tb_start,
                                                     const uint32_t *__restrict__ tb_end,
                                                     const uint32_t *__restrict__ acc_row,
                                                     uint32_t n_txn,
                                                     const uint8_t *__restrict__ status,
                                                     uint64_t *__restrict__ f0,
                                                     const uint64_t *__restrict__ pkey,
                                                     Counters *ctr, RowMap rm, uint8_t *__restrict__ commit_out,
                                                     int pk_dense, uint64_t pk_base) {
    __shared__ unsigned long long part[3][4];
    if (ctr->halt) return;  // rounds not finished (dv_epoch_finish resumes them)
    const bool rows = !input_err(ctr);  // a rejected epoch changes no row
    if (!(MODE & EX_COMMIT) && !rows) return;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    unsigned long long dig = 0, wcnt = 0, ncom = 0;
    const uint32_t step = gridDim.x * (kBlock / 64) * 64;
    for (uint32_t base = (blockIdx.x * (kBlock / 64) + wave) * 64; base < n_txn; base += step) {
        const uint32_t t = base + lane;
        const bool com = t < n_txn && status[t] == ST_COMMIT;
        const uint64_t cm = __ballot(com);
        if (MODE & EX_COMMIT) {
            if (commit_out && t < n_txn) commit_out[t] = com ? 1u : 0u;
            if (lane == 0) ncom += (unsigned long long)__popcll(cm);
        }
        if (cm == 0 || !rows) continue;
        const uint32_t a0 = com ? tb_start[t] : 0u;
        const uint32_t len = com ? tb_end[t] - a0 : 0u;
        uint32_t incl = len;  // inclusive prefix of the lengths over the wave
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t o = __shfl_up(incl, off, 64);
            if (lane >= (uint32_t)off) incl += o;
        }
        const uint32_t pre = incl - len, total = __shfl(incl, 63, 64);
        // wave-uniform trip count: the shuffles below read every lane
        for (uint32_t g0 = 0; g0 < total; g0 += 64) {
            const uint32_t g = g0 + lane;
            // the last lane whose prefix is <= g owns access g (empty lanes
            // share the next lane's prefix and lose to it)
            uint32_t src = 0;
#pragma unroll
            for (uint32_t w = 32; w > 0; w >>= 1) {
                const uint32_t cand = src + w;
                const uint32_t pv = __shfl(pre, (int)(cand & 63u), 64);
                if (cand < 64 && pv <= g) src = cand;
            }
            const uint32_t sa0 = __shfl(a0, (int)src, 64), spre = __shfl(pre, (int)src, 64);
            if (g >= total) continue;
            const uint32_t tt = base + src;
            const uint32_t ar = acc_row[sa0 + (g - spre)];
            uint64_t row = ar & ~AR_WR;
            if (!own_row(rm, row)) continue;  // (replicated epochs: another partition's row)
            if ((MODE & EX_READS) && !(ar & AR_WR))
                dig += mix64(f0[row] ^ mix64(((uint64_t)tt << 32) ^ (pk_dense ? row - pk_base : pkey[row])));
            if ((MODE & EX_WRITES) && (ar & AR_WR)) {
                f0[row] = 0;  // *(uint64_t*)&data[0] = 0 (ycsb_txn.cpp:239-242)
                wcnt++;
            }
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        dig += __shfl_down(dig, off, 64);
        wcnt += __shfl_down(wcnt, off, 64);
    }
    if (lane == 0) {
        part[0][wave] = dig;
        part[1][wave] = wcnt;
        part[2][wave] = ncom;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long d = part[0][0] + part[0][1] + part[0][2] + part[0][3];
        const unsigned long long w = part[1][0] + part[1][1] + part[1][2] + part[1][3];
        const unsigned long long n = part[2][0] + part[2][1] + part[2][2] + part[2][3];
        if (d) atomicAdd(&my_slot(ctr).read_digest, d);
        if (w) atomicAdd(&my_slot(ctr).write_cnt, w);
        if ((MODE & EX_COMMIT) && n) atomicAdd(&my_slot(ctr).committed, (uint32_t)n);
    }
}

void launch_exec_txn(hipStream_t s, const uint32_t *tb_start, const uint32_t *tb_end,
                     const uint32_t *acc_row, uint32_t n_txn, const uint8_t *status, uint64_t *f0,
                     const uint64_t *pkey, bool fused, Counters *ctr, RowMap rm, uint8_t *d_commit,
                     bool pk_dense, uint64_t pk_base) {
    const int pkd = pk_dense && rm.P == 0 ? 1 : 0;  // (replicated epochs read the column)
    if (n_txn == 0) return;
    uint32_t blocks = (n_txn + kBlock - 1) / kBlock;
    if (blocks > 4096) blocks = 4096;
    if (fused) {
        DV_LAUNCH((k_exec_txn<EX_READS | EX_WRITES | EX_COMMIT>), blocks, kBlock, 0, s, tb_start, tb_end, acc_row, n_txn,
                                                                              status, f0, pkey, ctr, rm, d_commit, pkd, pk_base);
    } else {
        DV_LAUNCH((k_exec_txn<EX_READS | EX_COMMIT>), blocks, kBlock, 0, s, tb_start, tb_end, acc_row, n_txn, status, f0,
                                                                   pkey, ctr, rm, d_commit, pkd, pk_base);
        DV_LAUNCH((k_exec_txn<EX_WRITES>), blocks, kBlock, 0, s, tb_start, tb_end, acc_row, n_txn, status, f0,
                                                        pkey, ctr, rm, nullptr, pkd, pk_base);
    }
}

__global__ __launch_bounds__(kBlock) void k_commit_out(const uint8_t *__restrict__ status, uint32_t n,
                                                       uint8_t *__restrict__ out, Counters *ctr) {
    __shared__ uint32_t part[4];
    if (ctr->halt) return;  // the rounds resume first (dv_epoch_finish)
    uint32_t cnt = commit_bytes_grid(status, n, out);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) cnt += __shfl_down(cnt, off, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t t = part[0] + part[1] + part[2] + part[3];
        if (t) atomicAdd(&my_slot(ctr).committed, t);
    }
}

void launch_commit_out(hipStream_t s, const uint8_t *status, uint32_t n_txn, uint8_t *d_commit,
                       Counters *ctr) {
    if (!n_txn) return;
    uint32_t blocks = (n_txn + kBlock * 16 - 1) / (kBlock * 16);
    if (blocks > 1024) blocks = 1024;
    DV_LAUNCH(k_commit_out, blocks, kBlock, 0, s, status, n_txn, d_commit, ctr);
}

// ------------------------------------------------------------- loaders
// YCSBWorkload::init_table_slice (ycsb_wl.cpp:144-203) for one partition:
// local row r holds key r*P + part; F0 = "hello\0" + key bytes 6..7 (H3);
// YCSB bucket (key/P) % rows == r, so the index is a direct map with local
// row == bucket: an implicit-row map over the pkey column (TableDesc::pkey).
__global__ void k_ycsb_load(uint64_t rows, uint32_t part_cnt, uint32_t part_id, uint64_t *f0,
                            uint64_t *pkey, uint8_t *ktag) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rows; r += stride) {
        const uint64_t key = r * part_cnt + part_id;
        f0[r] = 0x00006F6C6C6568ull | (key & 0xFFFF000000000000ull);
        pkey[r] = key;
        ktag[r] = key_tag(DV_HASH_YCSB, rows, part_cnt, key);
    }
}

void launch_ycsb_load(hipStream_t s, uint64_t rows, uint32_t part_cnt, uint32_t part_id,
                      uint64_t *f0, uint64_t *pkey, uint8_t *ktag) {
    DV_LAUNCH(k_ycsb_load, 2048, kBlock, 0, s, rows, part_cnt, part_id, f0, pkey, ktag);
}

__global__ void k_home_bits(const uint8_t *__restrict__ ktag, uint64_t n, uint32_t htag, uint32_t *__restrict__ bits) {
    const uint64_t nw = (n + 31) / 32;
    for (uint64_t w = blockIdx.x * (uint64_t)kBlock + threadIdx.x; w < nw; w += (uint64_t)gridDim.x * kBlock) {
        uint32_t v = 0;
        for (uint32_t j = 0; j < 32 && w * 32 + j < n; j++) v |= (ktag[w * 32 + j] == htag ? 1u : 0u) << j;
        bits[w] = v;
    }
}
void launch_home_bits(hipStream_t s, const uint8_t *ktag, uint64_t n, uint32_t htag, uint32_t *bits) {
    if (n) DV_LAUNCH(k_home_bits, 2048, kBlock, 0, s, ktag, n, htag, bits);
}

__global__ void k_gather_rows(Tables tabs, uint32_t table, const uint64_t *keys, uint64_t n,
                              const uint64_t *f0, uint32_t cstride, uint64_t *out, Counters *ctr) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint64_t row = 0;
        out[i] = probe_row(tabs.t[table < kMaxTables ? table : 0], table < tabs.n, keys[i], row, ctr)
                     ? f0[row * cstride]
                     : 0ull;
    }
}

void launch_gather_rows(hipStream_t s, const Tables &tabs, uint32_t table, const uint64_t *keys,
                        uint64_t n, const uint64_t *f0, uint32_t cstride, uint64_t *out, Counters *ctr) {
    if (!n) return;
    DV_LAUNCH(k_gather_rows, 1024, kBlock, 0, s, tabs, table, keys, n, f0, cstride, out, ctr);
}

// host records -> the epoch's arrays; with txn_begin (CSR), every record's
// txn_seq must own its index (ERRB_TXN otherwise)
__global__ void k_split_access(const dv_access *acc, uint64_t n, const uint32_t *tb, uint32_t n_txn,
                               uint64_t *keys, uint8_t *types, uint32_t *acc_txn, uint8_t *tables,
                               uint32_t *err) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    bool bad = false;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const dv_access a = acc[i];
        keys[i] = a.key;
        types[i] = a.type;
        acc_txn[i] = a.txn_seq;
        tables[i] = a.table;
        if (tb) bad |= a.txn_seq >= n_txn || i < tb[a.txn_seq] || i >= tb[a.txn_seq + 1];
    }
    if (bad) atomicOr(err, ERRB_TXN);
}

// 4-byte host records (dv_epoch_stage_host_rows): row | write << 31, txn ids
// from the CSR txn_begin.  A wave owns 64 consecutive txns, whose accesses
// are one contiguous range: its lanes walk that range together (coalesced)
// and find each access's txn among the 64 starts by a binary search over the
// lanes' registers.
__global__ __launch_bounds__(kBlock) void k_split_rows(const uint32_t *__restrict__ rw, const uint32_t *__restrict__ tb,
                                                       uint32_t n_txn, uint64_t *__restrict__ keys,
                                                       uint8_t *__restrict__ types, uint32_t *__restrict__ acc_txn,
                                                       uint8_t *__restrict__ tables) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t waves = gridDim.x * (kBlock / 64);
    for (uint32_t t0 = (blockIdx.x * kBlock + threadIdx.x) / 64 * 64; t0 < n_txn; t0 += waves * 64) {
        const uint32_t t = t0 + lane;
        const uint32_t start = tb[t < n_txn ? t : n_txn];           // (n_txn: the end)
        const uint32_t lo = __shfl(start, 0, 64);
        const uint32_t hi = tb[t0 + 64 < n_txn ? t0 + 64 : n_txn];
        const uint32_t trips = (hi - lo + 63) / 64;  // (wave-uniform: the shuffles read every lane)
        for (uint32_t k = 0; k < trips; k++) {
            const uint32_t a = lo + k * 64 + lane;
            // the last of the 64 txns starting at or before a (lanes past
            // n_txn hold the end, never <= a; empty txns share a start with
            // the next one, which wins)
            uint32_t src = 0;
#pragma unroll
            for (uint32_t w = 32; w > 0; w >>= 1) {
                const uint32_t cand = src + w;
                if (__shfl(start, (int)cand, 64) <= a) src = cand;
            }
            if (a >= hi) continue;
            const uint32_t v = rw[a];
            keys[a] = v & 0x7FFFFFFFu;
            types[a] = (uint8_t)(v >> 31);  // DV_WR = 1, DV_RD = 0
            acc_txn[a] = t0 + src;
            tables[a] = 0;
        }
    }
}

void launch_split_rows(hipStream_t s, const uint32_t *rw, uint64_t n, const uint32_t *tb, uint32_t n_txn,
                       uint64_t *keys, uint8_t *types, uint32_t *acc_txn, uint8_t *tables) {
    if (!n || !n_txn) return;
    const uint32_t waves = (n_txn + 63) / 64, per = kBlock / 64;
    const uint32_t g = (waves + per - 1) / per;
    DV_LAUNCH(k_split_rows, g < 4096 ? g : 4096, kBlock, 0, s, rw, tb, n_txn, keys, types, acc_txn, tables);
}

void launch_split_access(hipStream_t s, const dv_access *acc, uint64_t n, const uint32_t *tb, uint32_t n_txn,
                         uint64_t *keys, uint8_t *types, uint32_t *acc_txn, uint8_t *tables, uint32_t *err) {
    if (!n) return;
    DV_LAUNCH(k_split_access, 2048, kBlock, 0, s, acc, n, tb, n_txn, keys, types, acc_txn, tables, err);
}

}  // namespace dvcc
