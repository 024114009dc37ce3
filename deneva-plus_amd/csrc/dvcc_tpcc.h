// dvcc_tpcc.h -- TPC-C kernels (dvcc_tpcc.hip) used by the epoch runtime.
#pragma once
#include "dvcc_internal.h"

namespace dvcc {

// customer-by-last-name accesses -> CUSTOMER/custKey; every other access copied
void launch_tpcc_resolve(hipStream_t s, const Tables &tabs, const uint64_t *keys, const uint8_t *tables,
                         uint64_t n, const uint64_t *col0, uint64_t *okeys, uint8_t *otables, Counters *ctr);

struct TpccExec {
    const uint64_t *pairs;     // row-sorted pairs of the epoch
    uint64_t n;                // accesses
    const uint8_t *status;     // per txn
    const uint32_t *tb_start;  // per txn: first access
    const uint64_t *args;      // per access: op << 56 | operand
    uint64_t *c0, *c1, *c2;    // state columns (global row id)
    uint64_t *dsnap;           // per district row: D_NEXT_O_ID before the epoch (scratch)
    uint64_t dist_base, dist_rows;
    uint64_t *desc;            // look-back descriptors (>= n / kRTile), tagged
    uint32_t tag;
    uint32_t *tile_ctr;        // a zeroed tile ticket
    uint64_t *oid;             // per txn (may be null)
    Counters *ctr;
};
// two launches: updates + D_NEXT_O_ID snapshots, then the o_id numbering
void launch_tpcc_exec(hipStream_t s, const TpccExec &x);

}  // namespace dvcc
