// dvcc_tpcc.h -- TPC-C kernels (dvcc_tpcc.hip) used by the epoch runtime.
#pragma once
#include "dvcc_internal.h"

namespace dvcc {


struct TpccExec {
    const uint64_t *pairs;     // row-sorted pairs of the epoch
    uint64_t n;                // accesses
    const uint8_t *status;     // per txn
    const uint32_t *tb_start;  // per txn: first access
    const uint64_t *args;      // per access: op << 56 | operand
    uint64_t *cols;            // state columns, row-major: cols[3 * row + k] (global row id)
    bool oid_direct;           // NO_WAIT / WAIT_DIE / OCC: at most one committed writer per district
                               // row, so o_id = D_NEXT_O_ID + 1 in the update pass (no numbering pass)
    uint64_t *dsnap;           // per district row: D_NEXT_O_ID before the epoch, then where its queue
                               // starts in pairs ([2 * dist_rows], scratch, CALVIN)
    uint64_t dist_base, dist_rows;
    uint64_t *oid;             // per txn (may be null)
    Counters *ctr;
    uint32_t n_txn;            // the commit bytes of every txn (and the committed count) ...
    uint8_t *commit_out;       // ... written by the update pass (may be null: the count only)
};
// updates (+ D_NEXT_O_ID snapshots) and the commit bytes, then -- CALVIN,
// several committed NewOrders per district -- the o_id numbering
constexpr uint32_t kTpccCols = 3;

// A customer-by-last-name access (payment / order-status by last name,
// tpcc_txn.cpp:600-626): the customer it names is the middle one of the
// name's entries in i_customer_last (t: the CUST_LAST table; equal keys are
// contiguous in a chained bucket, the floor(cnt/2)-th is taken) -- its
// custKey, column 0 of that CUST_LAST row -- or key ~0 when the name has no
// customer (the probe then reports DV_ERR_KEY_NOT_FOUND).  The probe resolves
// these in place (k_probe<HIST, true>), so the access is a CUSTOMER access
// from there on.
__device__ inline uint64_t tpcc_last_name_key(const TableDesc &t, const uint64_t *__restrict__ cols, uint64_t key) {
    uint32_t tag;
    const uint64_t bk = key_split(t, key, tag);
    uint64_t row = ~0ull;
    if (t.pkey != nullptr) {
        if (direct_holds(t, bk, tag, key)) row = bk;
    } else if (t.bstart == nullptr) {
        if (t.ix[bk].key == key) row = t.ix[bk].row;
    } else {
        const uint32_t lo = t.bstart[bk], hi = t.bstart[bk + 1];
        uint32_t cnt = 0, first = hi;
        for (uint32_t j0 = lo; j0 < hi; j0 += 4) {  // (four entries' keys in flight per step)
            uint64_t k4[4];
#pragma unroll
            for (uint32_t q = 0; q < 4; q++) k4[q] = j0 + q < hi ? t.ix[j0 + q].key : ~key;
#pragma unroll
            for (uint32_t q = 0; q < 4; q++)
                if (k4[q] == key) {
                    if (first == hi) first = j0 + q;
                    cnt++;
                }
        }
        if (cnt) row = t.ix[first + cnt / 2].row;
    }
    return row == ~0ull ? ~0ull : cols[(t.row_base + row) * kTpccCols];
}
void launch_tpcc_exec(hipStream_t s, const TpccExec &x);

}  // namespace dvcc
