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
//     head and records where the queue starts, then a wave per district
//     (k_tpcc_oid) numbers the queue's committed NewOrders by ballot ranks and
//     stores the grown word.
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
            dsnap[dist_rows + row - dist_base] = i;  // ... and where the row's queue starts (k_tpcc_oid)
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

// CALVIN's o_id numbering: every committed NewOrder of a district, in the
// district row's queue order (sequence order), takes D_NEXT_O_ID + its rank
// among them (new_order_5, tpcc_txn.cpp:774-781), and the row's D_NEXT_O_ID
// grows by their count.  The update pass recorded each district row's
// snapshot and where its queue starts in the sorted pairs (dsnap, dsnap +
// dist_rows); a wave per district walks its queue 64 accesses per step,
// ranking the committed NewOrders by ballot -- no tiles, no look-back (the
// tiled version with a decoupled look-back across every tile of the epoch
// took 25.7 us per launch under four lanes).  A start recorded by an earlier
// epoch is recognised as stale (not the head of that row's queue now) and
// skipped, with the row.  An operation word naming another table is ignored.
__global__ __launch_bounds__(kBlock) void k_tpcc_oid(const uint64_t *__restrict__ pairs, uint32_t n,
                                                     const uint8_t *__restrict__ status,
                                                     const uint32_t *__restrict__ tb_start,
                                                     const uint64_t *__restrict__ args,
                                                     const uint64_t *__restrict__ dsnap, uint64_t dist_base,
                                                     uint64_t dist_rows, uint64_t *__restrict__ cols,
                                                     uint64_t *__restrict__ oid, Counters *ctr) {
    if (input_err(ctr) || ctr->halt) return;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t d = (uint64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    if (d >= dist_rows) return;  // (wave-uniform)
    const uint32_t row = (uint32_t)(dist_base + d);
    const uint64_t i0 = dsnap[dist_rows + d];
    if (i0 >= n || pair_row(pairs[i0]) != row || (i0 > 0 && pair_row(pairs[i0 - 1]) == row)) return;
    const uint64_t snap = dsnap[d];
    uint64_t count = 0;
    for (uint64_t base = i0;; base += 64) {
        const uint64_t i = base + lane;
        const uint64_t p = i < n ? pairs[i] : ~0ull;
        const bool inq = i < n && pair_row(p) == row;
        const uint32_t t = pair_txn(p);
        const bool com = inq && status[t] == ST_COMMIT;
        const bool f = com && (uint32_t)(args[tb_start[t] + pair_pos(p)] >> 56) == DV_TOP_NO_DIST;
        const uint64_t m = __ballot(f);
        if (f && oid) oid[t] = snap + count + (uint64_t)__popcll(m & ((1ull << lane) - 1ull)) + 1u;
        count += (uint64_t)__popcll(m);
        if (__ballot(inq) != ~0ull) break;  // (the queue ends inside this step)
    }
    if (lane == 0 && count) cols[(uint64_t)row * kTpccCols + 1] = snap + count;  // the grown D_NEXT_O_ID
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
    if (!x.dist_rows) return;
    const uint32_t blocks = (uint32_t)((x.dist_rows + kBlock / 64 - 1) / (kBlock / 64));  // (a wave per district)
    DV_LAUNCH(k_tpcc_oid, blocks, kBlock, 0, s, x.pairs, (uint32_t)x.n, x.status, x.tb_start, x.args, x.dsnap,
                                         x.dist_base, x.dist_rows, x.cols, x.oid, x.ctr);
}

}  // namespace dvcc
