// dvcc_internal.h -- shared declarations between the epoch runtime and the
// gfx950 kernels.  Not part of the public ABI (see include/dvcc.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dvcc.h"

namespace dvcc {

constexpr int kBlock = 256;           // 4 waves of 64
constexpr int kIPT = 16;              // items per thread in tiled kernels
constexpr int kTile = kBlock * kIPT;  // 4096 elements per workgroup tile
constexpr int kRadixBits = 8;
constexpr int kRadix = 1 << kRadixBits;
constexpr int kMaxTables = 8;

// per-txn decision state (one byte per txn)
enum : uint8_t { ST_UNDEC = 0, ST_COMMIT = 1, ST_ABORT = 2 };
// verdict bits (combined across partitions by element-wise MAX)
enum : uint8_t { V_WAIT = 1, V_ABORT = 2 };

// sorted-element encoding: txn << 4 | bnd << 3 | dup << 2 | head << 1 | wr
//   head: first access of a row segment; dup: repeat access of the same txn to
//   the same row; bnd: Calvin grant-group boundary.
constexpr uint32_t EL_WR = 1u, EL_HEAD = 2u, EL_DUP = 4u, EL_BND = 8u;
// decision-round arrays reuse bit 3: the access is already OK (verdict pushed)
constexpr uint32_t EL_DONE = 8u;
constexpr uint32_t kMaxTxn = 1u << 28;

// device counters block (zeroed per epoch)
struct Counters {
    uint32_t err;         // ERRB_* bits of every failure seen
    uint32_t undecided;   // txns still undecided after the last round
    uint32_t committed;
    uint32_t pad0;
    uint32_t nlive[2];    // live accesses of the current / next decision round
    uint32_t pad1[2];
    unsigned long long write_cnt;
    unsigned long long read_digest;
};

struct IxEntry {
    uint64_t key;
    uint64_t row;
};

struct TableDesc {
    const IxEntry *ix;        // index entries (direct: [nbuckets]; chained: sorted by bucket)
    const uint32_t *bstart;   // chained: [nbuckets+1] bucket starts; nullptr = direct map
    uint64_t nbuckets;
    uint64_t row_base;        // global row id of local row 0
    uint32_t hash_kind;       // DV_HASH_*
    uint32_t part_cnt;
};

struct Tables {
    TableDesc t[kMaxTables];
    uint32_t n;
};

// error bits recorded by kernels
enum : uint32_t { ERRB_KEY = 1, ERRB_DUP = 2, ERRB_TXN = 4, ERRB_TABLE = 8, ERRB_SPIN = 16 };

// ---- launchers (dvcc_kernels.hip) ----
void launch_probe(hipStream_t s, const Tables &tabs, const uint64_t *keys, const uint8_t *types,
                  const uint32_t *acc_txn, const uint8_t *tables, uint64_t n_acc, uint32_t n_txn,
                  uint64_t *pairs, uint32_t *vals, uint32_t *need, Counters *ctr);

// stable LSD radix sort of pairs on bits [32, 32 + key_bits); returns the index
// (0/1) of the buffer holding the result.  counts: >= kRadix * nblocks(n),
// digit_tot: kRadix.  scatter_ev (optional): 2 events per pass for timing.
int radix_sort_rows(hipStream_t s, uint64_t *pairs[2], uint32_t *vals[2], uint64_t n, int key_bits,
                    uint32_t *counts, uint32_t *digit_tot, hipEvent_t *scatter_ev);

void launch_seg_prepare(hipStream_t s, const uint64_t *pairs, uint64_t n, int calvin,
                        uint32_t *el, Counters *ctr);

// segmented scans: block aggregates / carries live in agg_f, agg_v, carry (>= nblocks)
void calvin_grant(hipStream_t s, const uint32_t *el, const uint32_t *vals, uint64_t n,
                  uint32_t *grant_out, uint8_t *ew, uint32_t *agg_f, uint32_t *agg_v,
                  uint32_t *carry);
// decision rounds (dvcc_rounds.hip)
constexpr uint32_t kTileCtrs = 1024;  // per-round tile tickets, reset every kTileCtrs rounds
void rounds_epoch_init(hipStream_t s, uint32_t n_acc, uint32_t n_txn_pad, uint32_t *need,
                       uint8_t *abortf, uint32_t *tile_ctr, Counters *ctr);
void round_pass(hipStream_t s, bool first, int nowait, const uint32_t *el_in, uint32_t *el_out,
                uint32_t ub_in, const uint32_t *n_in, uint32_t *n_out, const uint8_t *status,
                uint32_t *need, uint8_t *abortf, uint64_t *desc, uint32_t *tile_ctr, uint32_t tag,
                Counters *ctr);
void round_settle(hipStream_t s, uint8_t *status, const uint32_t *need, const uint8_t *abortf,
                  uint32_t n_txn_pad, Counters *ctr);
void round_verdict(hipStream_t s, const uint8_t *status, const uint32_t *need, const uint8_t *abortf,
                   uint32_t n_txn_pad, uint8_t *verdict);
void round_apply(hipStream_t s, uint8_t *status, const uint8_t *verdict, uint32_t n_txn_pad,
                 Counters *ctr);
void launch_status_init(hipStream_t s, uint8_t *status, uint32_t n_txn, uint32_t n_txn_pad4,
                        uint8_t value);
void launch_exec(hipStream_t s, int calvin, const uint64_t *pairs, const uint32_t *el,
                 const uint8_t *ew, uint64_t n, const uint8_t *status, uint64_t *f0,
                 const uint64_t *pkey, Counters *ctr);
void launch_commit_out(hipStream_t s, const uint8_t *status, uint32_t n_txn, uint8_t *d_commit,
                       Counters *ctr);
void launch_ycsb_load(hipStream_t s, uint64_t rows, uint32_t part_cnt, uint32_t part_id,
                      uint64_t *f0, uint64_t *pkey, IxEntry *ix);
void launch_gather_rows(hipStream_t s, const Tables &tabs, uint32_t table, const uint64_t *keys,
                        uint64_t n, const uint64_t *f0, uint64_t *out, Counters *ctr);
void launch_split_access(hipStream_t s, const dv_access *acc, uint64_t n, uint64_t *keys,
                         uint8_t *types, uint32_t *acc_txn, uint8_t *tables);

inline uint32_t nblocks_for(uint64_t n) { return (uint32_t)((n + kTile - 1) / kTile); }

}  // namespace dvcc
