// dvcc_tpcc.hip -- TPC-C on the epoch path (config E), gfx950.
//
// Two pieces around the generic probe -> sort -> decide pipeline:
//
// last names       Payment's customer-by-last-name lookup (run_payment_4,
//                  tpcc_txn.cpp:600-626): index_read on i_customer_last
//                  returns the item list of the key, newest insert first
//                  (BucketHeader::insert_item prepends, index_hash.cpp:
//                  197-200), and the txn takes element floor(n/2) (`mid`
//                  advances on every second element).  The chained index keeps
//                  equal keys grouped newest first (dv_load_table), so the
//                  lookup counts the key's entries and takes the middle one;
//                  its payload (col 0) is the customer's primary key.  The
//                  probe does this in place (tpcc_last_name_key, dvcc_tpcc.h)
//                  and probes CUSTOMER/custKey: no launch or scratch copy of
//                  the epoch of its own.
//
// execution        run_payment_1/3/5 and new_order_5/9 (tpcc_txn.cpp:530-933)
//                  for committed txns, over the row-sorted pairs so that every
//                  row's accesses are visited in sequence order (CALVIN: all
//                  txns commit and a row's updates apply serially in that
//                  order; NO_WAIT / WAIT_DIE / OCC: a written row has at most
//                  one committed accessor that writes it).
//   - Additive updates (W_YTD, D_YTD, C_BALANCE, C_YTD_PAYMENT, C_PAYMENT_CNT,
//     S_YTD, S_ORDER_CNT) are integer-valued: every partial sum is an integer
//     below 2^53, so device-scope atomic adds give the serial result exactly
//     in any order.  C_PAYMENT_CNT is loaded as the integer 1 and read as a
//     double (a denormal): denormal + 1.0 rounds to 1.0 either way.
//   - D_NEXT_O_ID: o_id of a NewOrder = D_NEXT_O_ID + 1 + (committed NewOrders
//     before it in the district's queue).  NO_WAIT / WAIT_DIE / OCC commit at
//     most one writer of a district row (NewOrder and Payment both write it),
//     so the update pass sets o_id = ++D_NEXT_O_ID itself.  CALVIN commits
//     them all: the apply pass snapshots D_NEXT_O_ID at each district queue's
//     head, then one single-pass segmented count (decoupled look-back,
//     dvcc_common.h) numbers the committed NewOrders of every queue and the
//     queue's last element stores the grown word.
//   - The three state columns of a row are one 24-byte group (row-major): a
//     row's updates touch one or two 128-B lines instead of three.
//   - S_QUANTITY is piecewise (s > q + 10 ? s - q : s - q + 91): the queue
//     head walks its stock row's queue in order (stock queues are short: the
//     NURand(8191) item choice spreads over max_items x warehouses rows).
#include "dvcc_internal.h"
#include "dvcc_common.h"
#include "dvcc_tpcc.h"

namespace dvcc {

namespace {

constexpr uint64_t kOpMask = (1ull << 56) - 1;



// pass 1: additive updates, stock queues, D_NEXT_O_ID snapshots at the
// district queue heads.
// Each wave takes 64 consecutive sorted accesses; the additive contributions
// of a row's run inside the wave are summed by a segmented shuffle reduction
// (rows are contiguous in sort order) and the run's first lane issues one
// atomic per column: a hot row (CALVIN: every Payment of a warehouse) takes
// one same-address atomic per wave instead of one per access.
__global__ __launch_bounds__(kBlock) void k_tpcc_apply(const uint64_t *__restrict__ pairs, uint64_t n,
                                                       const uint8_t *__restrict__ status,
                                                       const uint32_t *__restrict__ tb_start,
                                                       const uint64_t *__restrict__ args, uint64_t *cols,
                                                       int oid_direct, uint64_t *__restrict__ oid,
                                                       uint64_t *__restrict__ dsnap, uint64_t dist_base,
                                                       uint64_t dist_rows, Counters *ctr, uint32_t n_txn,
                                                       uint8_t *__restrict__ commit_out) {
    if (ctr->halt) return;  // rounds not finished
    const uint32_t lane = threadIdx.x & 63;
    {  // the commit bytes and the committed count (k_commit_out's work, one launch fewer)
        uint32_t cc = commit_bytes_grid(status, n_txn, commit_out);
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) cc += __shfl_down(cc, off, 64);
        if (lane == 0 && cc) atomicAdd(&my_slot(ctr).committed, cc);
    }
    if (input_err(ctr)) return;  // a rejected epoch changes no row
    unsigned long long wcnt = 0;
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    for (uint64_t base = (uint64_t)blockIdx.x * kBlock + (threadIdx.x & ~63u); base < n; base += stride) {
        const uint64_t i = base + lane;
        const bool valid = i < n;
        const uint64_t p = valid ? pairs[i] : ~0ull;
        const uint32_t row = valid ? pair_row(p) : 0xFFFFFFFFu, txn = pair_txn(p);
        const bool com = valid && status[txn] == ST_COMMIT;
        const uint64_t w = valid ? args[tb_start[txn] + pair_pos(p)] : 0ull;
        const uint32_t op = (uint32_t)(w >> 56);
        const uint64_t v = w & kOpMask;
        const uint32_t prow = __shfl_up(row, 1, 64);
        const bool head = valid && (i == 0 || (lane ? prow : pair_row(pairs[i - 1])) != row);
        const bool dist_row = row >= dist_base && row < dist_base + dist_rows;
        uint64_t *rc = cols + (uint64_t)row * kTpccCols;  // the row's three columns (24 B)
        if (oid_direct) {
            // the district's only committed writer: o_id = ++D_NEXT_O_ID (new_order_5)
            if (com && dist_row && op == DV_TOP_NO_DIST) {
                const uint64_t o = rc[1] + 1;
                rc[1] = o;
                if (oid) oid[txn] = o;
            }
        } else if (head && dist_row) {
            dsnap[row - dist_base] = rc[1];  // D_NEXT_O_ID before the epoch
        }
        if (com && (p & 1)) wcnt++;
        double a0 = 0.0, a1 = 0.0, a2 = 0.0;
        if (com) {
            if (op == DV_TOP_PAY_WH || op == DV_TOP_PAY_DIST) {  // W_YTD / D_YTD += h (run_payment_1/3)
                a0 = (double)v;
            } else if (op == DV_TOP_PAY_CUST) {  // run_payment_5
                a0 = -(double)v;
                a1 = (double)v;
                a2 = 1.0;
            }
        }
        // suffix sums over the row's run inside the wave (integer-valued: exact)
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const double o0 = __shfl_down(a0, off, 64), o1 = __shfl_down(a1, off, 64),
                         o2 = __shfl_down(a2, off, 64);
            const uint32_t orow = __shfl_down(row, off, 64);
            if (lane + off < 64 && orow == row) {
                a0 += o0;
                a1 += o1;
                a2 += o2;
            }
        }
        const bool run_first = valid && (lane == 0 || prow != row);
        if (run_first) {
            if (a0 != 0.0) atomicAdd(reinterpret_cast<double *>(rc), a0);
            if (a1 != 0.0) atomicAdd(reinterpret_cast<double *>(rc + 1), a1);
            if (a2 != 0.0) atomicAdd(reinterpret_cast<double *>(rc + 2), a2);
        }
        if (head && op == DV_TOP_NO_STOCK) {  // new_order_9 in queue order
            uint64_t s = rc[0];
            int64_t ytd = (int64_t)rc[1], ocnt = (int64_t)rc[2];
            bool any = false;
            for (uint64_t j = i; j < n; j++) {
                const uint64_t q = pairs[j];
                if (pair_row(q) != row) break;
                const uint32_t t = pair_txn(q);
                if (status[t] != ST_COMMIT) continue;
                const uint64_t qty = args[tb_start[t] + pair_pos(q)] & kOpMask;
                ytd += (int64_t)qty;
                ocnt += 1;
                s = s > qty + 10 ? s - qty : s - qty + 91;
                any = true;
            }
            if (any) {
                rc[0] = s;
                rc[1] = (uint64_t)ytd;
                rc[2] = (uint64_t)ocnt;
            }
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) wcnt += __shfl_down(wcnt, off, 64);
    if (lane == 0 && wcnt) atomicAdd(&my_slot(ctr).write_cnt, wcnt);
}

// pass 2: o_id of every committed NewOrder (new_order_5: o_id = ++D_NEXT_O_ID,
// in sequence order per district) -- an OpSeg count over the row queues (head
// = f, committed NewOrder on a DISTRICT row = c), one launch: tiles of kRTile
// sorted accesses taken by ticket, decoupled look-back across tiles.  o_id =
// snapshot + inclusive count; the queue's last element stores D_NEXT_O_ID =
// snapshot + its inclusive count (one writer per row, no atomics).  An
// operation word naming another table is ignored.
__global__ __launch_bounds__(kBlock) void k_tpcc_oid(const uint64_t *__restrict__ pairs, uint32_t n,
                                                     const uint8_t *__restrict__ status,
                                                     const uint32_t *__restrict__ tb_start,
                                                     const uint64_t *__restrict__ args,
                                                     const uint64_t *__restrict__ dsnap, uint64_t dist_base,
                                                     uint64_t dist_rows, uint64_t *__restrict__ cols,
                                                     uint64_t *__restrict__ oid, uint64_t *desc,
                                                     uint32_t *tile_ctr, uint32_t tag, Counters *ctr) {
    __shared__ uint64_t s_el[kRTile + kRTile / kRIPT];
    __shared__ uint64_t s_next, s_prev;
    __shared__ uint32_t s_tile;
    __shared__ Agg wt[4];
    __shared__ Agg s_pre;
    const uint32_t ntiles = (n + kRTile - 1) / kRTile;
    if (blockIdx.x >= ntiles || input_err(ctr) || ctr->halt) return;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) s_tile = atomicAdd(tile_ctr, 1u);
    __syncthreads();
    const uint32_t tile = s_tile, base = tile * kRTile;
    const uint32_t tile_n = n - base < (uint32_t)kRTile ? n - base : (uint32_t)kRTile;
    load_tile64(pairs, base, tile_n, n, s_el, &s_next, ~0ull);
    if (tid == 0) s_prev = base ? pairs[base - 1] : ~0ull;
    __syncthreads();
    const uint32_t first = tid * kRIPT;
    const int cnt = first >= tile_n ? 0 : (tile_n - first < (uint32_t)kRIPT ? (int)(tile_n - first) : kRIPT);
    uint64_t e[kRIPT];
    uint32_t flags = 0, heads = 0, dmask = 0;
    Agg a{0u, 0u, 0u};
    uint64_t pp = first == 0 ? s_prev : s_el[rpad(first - 1)];
#pragma unroll
    for (int j = 0; j < kRIPT; j++) {
        e[j] = j < cnt ? s_el[rpad(first + j)] : ~0ull;
        const uint32_t row = pair_row(e[j]);
        dmask |= (j < cnt && row >= dist_base && row < dist_base + dist_rows ? 1u : 0u) << j;
    }
    // the district elements' status and first-access words, then their
    // operation words: every load of a step in flight together (one at a time
    // they were three round trips per district element)
    uint8_t sv[kRIPT];
    uint32_t tbv[kRIPT];
#pragma unroll
    for (int j = 0; j < kRIPT; j++) {
        const uint32_t t = (dmask >> j) & 1u ? pair_txn(e[j]) : 0u;
        sv[j] = (dmask >> j) & 1u ? status[t] : (uint8_t)ST_ABORT;
        tbv[j] = (dmask >> j) & 1u ? tb_start[t] : 0u;
    }
    uint64_t av[kRIPT];
#pragma unroll
    for (int j = 0; j < kRIPT; j++) av[j] = sv[j] == ST_COMMIT ? args[tbv[j] + pair_pos(e[j])] : 0ull;
#pragma unroll
    for (int j = 0; j < kRIPT; j++) {
        if (j < cnt) {
            const uint32_t row = pair_row(e[j]);
            const bool head = pair_row(pp) != row;
            const bool f = sv[j] == ST_COMMIT && (uint32_t)(av[j] >> 56) == DV_TOP_NO_DIST;
            flags |= (f ? 1u : 0u) << j;
            heads |= (head ? 1u : 0u) << j;
            a = OpSeg::comb(a, Agg{head ? 1u : 0u, 0u, f ? 1u : 0u});
            pp = e[j];
        }
    }
    const uint64_t nxt = first + kRIPT < tile_n ? s_el[rpad(first + kRIPT)] : s_next;
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
            const uint32_t f = (flags >> j) & 1u;
            run = OpSeg::comb(run, Agg{(heads >> j) & 1u, 0u, f});  // inclusive count since the head
            const uint32_t row = pair_row(e[j]);
            if (row >= dist_base && row < dist_base + dist_rows) {
                const uint64_t snap = dsnap[row - dist_base];
                if (f && oid) oid[pair_txn(e[j])] = snap + run.c;
                const uint64_t q = j + 1 < cnt ? e[j + 1] : (j + 1 < kRIPT ? ~0ull : nxt);
                if (pair_row(q) != row && run.c) cols[(uint64_t)row * kTpccCols + 1] = snap + run.c;  // queue's last
            }
        }
    }
}

uint32_t grid_for(uint64_t n) {
    uint64_t g = (n + kBlock - 1) / kBlock;
    return (uint32_t)(g < 1 ? 1 : (g > 4096 ? 4096 : g));
}

}  // namespace

void launch_tpcc_exec(hipStream_t s, const TpccExec &x) {
    if (x.n == 0) {  // (no access to update: the commit bytes alone)
        launch_commit_out(s, x.status, x.n_txn, x.commit_out, x.ctr);
        return;
    }
    const uint64_t g = std::max<uint64_t>(x.n, (x.n_txn + 15u) / 16u);
    DV_LAUNCH(k_tpcc_apply, grid_for(g), kBlock, 0, s, x.pairs, x.n, x.status, x.tb_start, x.args, x.cols,
              x.oid_direct ? 1 : 0, x.oid, x.dsnap, x.dist_base, x.dist_rows, x.ctr, x.n_txn, x.commit_out);
    if (x.oid_direct) return;
    const uint32_t ntiles = (uint32_t)((x.n + kRTile - 1) / kRTile);
    DV_LAUNCH(k_tpcc_oid, ntiles, kBlock, 0, s, x.pairs, (uint32_t)x.n, x.status, x.tb_start, x.args, x.dsnap,
                                         x.dist_base, x.dist_rows, x.cols, x.oid, x.desc, x.tile_ctr, x.tag, x.ctr);
}

}  // namespace dvcc
