// dvcc_tpcc.h -- TPC-C kernels (dvcc_tpcc.hip) used by the epoch runtime.
#pragma once
#include "dvcc_internal.h"

namespace dvcc {

// customer-by-last-name accesses -> CUSTOMER/custKey; every other access copied
void launch_tpcc_resolve(hipStream_t s, const Tables &tabs, const uint64_t *keys, const uint8_t *tables,
                         uint64_t n, const uint64_t *cols, uint64_t *okeys, uint8_t *otables, Counters *ctr);

struct TpccExec {
    const uint64_t *pairs;     // row-sorted pairs of the epoch
    uint64_t n;                // accesses
    const uint8_t *status;     // per txn
    const uint32_t *tb_start;  // per txn: first access
    const uint64_t *args;      // per access: op << 56 | operand
    uint64_t *cols;            // state columns, row-major: cols[3 * row + k] (global row id)
    bool oid_direct;           // NO_WAIT / WAIT_DIE / OCC: at most one committed writer per district
                               // row, so o_id = D_NEXT_O_ID + 1 in the update pass (no numbering pass)
    uint64_t *dsnap;           // per district row: D_NEXT_O_ID before the epoch (scratch, CALVIN)
    uint64_t dist_base, dist_rows;
    uint64_t *desc;            // look-back descriptors (>= n / kRTile), tagged
    uint32_t tag;
    uint32_t *tile_ctr;        // a zeroed tile ticket
    uint64_t *oid;             // per txn (may be null)
    Counters *ctr;
    uint32_t n_txn;            // the commit bytes of every txn (and the committed count) ...
    uint8_t *commit_out;       // ... written by the update pass (may be null: the count only)
    ExecGate gate;             // decision lanes: read by the first launch, written by the last
};
// updates (+ D_NEXT_O_ID snapshots) and the commit bytes, then -- CALVIN,
// several committed NewOrders per district -- the o_id numbering
constexpr uint32_t kTpccCols = 3;
bool launch_tpcc_exec(hipStream_t s, const TpccExec &x);

}  // namespace dvcc
