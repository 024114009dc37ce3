/*
 * oracle.h -- CPU restatement of Deneva's transaction-scheduling hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (deneva-plus_amd/, include/)
 * may include, link or call this.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py use it, and only as the checker.
 *
 * Parity status: the reference (elrodrigues/deneva-plus) ships no tests, no
 * golden vectors and cannot be compiled here (boost/jemalloc/nanomsg absent,
 * compile attempt denied -- SURVEY.md 8c).  This oracle is therefore pinned by
 * known-answer tests derived by hand from the reference source text
 * (tests/test_oracle_kat.py) and by the literal-vs-indexed cross checks; the
 * reference binary itself is "parity unpinned".
 *
 * Semantics follow SURVEY.md 8.0 (the "E-schedule"): one worker thread, one
 * seeded epoch, sequence order, TS_CAS counters starting at 1.
 */
#ifndef DENEVA_ORACLE_H
#define DENEVA_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* enums restated from system/global.h:236-291 */
enum { OR_RCOK = 0, OR_COMMIT = 1, OR_ABORT = 2, OR_WAIT = 3 };
enum { OR_RD = 0, OR_WR = 1, OR_XP = 2, OR_SCAN = 3 };
enum { OR_LOCK_EX = 0, OR_LOCK_SH = 1, OR_LOCK_NONE = 2 };
/* CC_ALG values restated from config.h (NO_WAIT 1, WAIT_DIE 2, OCC 8, CALVIN 10) */
enum { OR_NO_WAIT = 1, OR_WAIT_DIE = 2, OR_OCC = 8, OR_CALVIN = 10 };

/* ---- myrand (system/helper.cpp:140-147) ---- */
uint64_t or_myrand_next(uint64_t *seed);

/* ---- zipf (benchmarks/ycsb_query.cpp:181-202) ---- */
double or_zeta(uint64_t n, double theta);

typedef struct {
    uint64_t synth_table_size;   /* g_synth_table_size            */
    uint32_t part_cnt;           /* g_part_cnt                    */
    uint32_t req_per_query;      /* g_req_per_query               */
    double   zipf_theta;         /* g_zipf_theta                  */
    double   txn_write_perc;     /* g_txn_write_perc  (read = 1-) */
    double   tup_write_perc;     /* g_tup_write_perc  (read = 1-) */
    uint32_t part_per_txn;       /* g_part_per_txn                */
    uint32_t strict_ppt;         /* g_strict_ppt                  */
    double   mpr;                /* <0: reference zipf (no MPR gate); >=0: gate (SURVEY 8.0 note) */
} or_ycsb_params;

/* Generates n_txn YCSB queries exactly as gen_requests_zipf
 * (ycsb_query.cpp:303-376) from myrand seeded with `seed`.
 * keys/types are n_txn*req_per_query long; txn_begin is n_txn+1 long. */
int or_ycsb_gen(const or_ycsb_params *p, uint64_t seed, uint32_t home_part,
                uint32_t n_txn, uint64_t *keys, uint8_t *types, uint32_t *txn_begin);

/* ---- hash index (storage/index_hash.{h,cpp}) ---- */
typedef struct or_index or_index;
/* ycsb_hash!=0: (key/part_cnt)%nbuckets (index_hash.h:86-89) else key%nbuckets */
or_index *or_index_create(uint64_t nbuckets, uint32_t part_cnt, int ycsb_hash, uint64_t cap);
void      or_index_free(or_index *ix);
int       or_index_insert(or_index *ix, uint64_t key, uint64_t row);    /* index_hash.cpp:69-83, 172-201 */
int       or_index_read(const or_index *ix, uint64_t key, uint64_t *row); /* index_hash.cpp:137-153, 217-231 */

/* run_payment_4's last-name lookup: element floor(n/2) of the key's item list
 * (tpcc_txn.cpp:600-626) */
int       or_index_read_mid(const or_index *ix, uint64_t key, uint64_t *row);

/* ---- YCSB table F0 prefix (ycsb_wl.cpp:144-203, row.cpp:107-115; hazard H3) ---- */
uint64_t or_ycsb_f0_init(uint64_t key);
/* init_table_slice (ycsb_wl.cpp:144-203) for one partition: keys part_id,
 * part_id+part_cnt, ... get rows 0,1,... in key order; index_insert each. */
int or_ycsb_load(or_index *ix, uint64_t *f0, uint64_t rows_per_part, uint32_t part_cnt,
                 uint32_t part_id);
int or_index_insert_many(or_index *ix, const uint64_t *keys, const uint64_t *rows, uint64_t n);

/* ---- conflict_lock (row_lock.cpp:375-382) ---- */
int or_conflict_lock(int l1, int l2);

/* ---- E-schedule epoch ----
 * accesses of txn t are [txn_begin[t], txn_begin[t+1]) in request order;
 * keys are probed through `ix`; f0 is the row store (indexed by row id) and is
 * updated in place with the committed writes.
 * out_commit[t] = 1 commit / 0 abort; out_grant (Calvin only, may be NULL)
 * = grant-group id of every access; read_digest = sum over committed reads of
 * mix64(value ^ mix64(txn<<32 ^ key)).
 * occ_literal: 1 = literal active-set central_validate (O(N^2)), 0 = indexed. */
typedef struct {
    uint64_t committed;
    uint64_t aborted;
    uint64_t read_digest;
    uint64_t write_cnt;       /* committed WR accesses */
} or_epoch_stats;

int or_epoch_run(int cc_alg, const or_index *ix, uint64_t *f0, uint64_t nrows,
                 uint32_t n_txn, const uint32_t *txn_begin, const uint64_t *keys,
                 const uint8_t *types, uint8_t *out_commit, uint32_t *out_grant,
                 int occ_literal, or_epoch_stats *st);

/* decisions only, on pre-resolved row ids (stats: committed / aborted / write_cnt) */
int or_epoch_decide(int cc_alg, const uint64_t *rows, uint64_t nrows, uint32_t n_txn,
                    const uint32_t *txn_begin, const uint8_t *types, uint8_t *out_commit,
                    uint32_t *out_grant, or_epoch_stats *st);

/* ---- TPC-C (tpcc.c) ---- */
typedef struct { int32_t st[31]; int f, r; } or_grand;   /* glibc random_r TYPE_3 state */
void     or_grand_seed(or_grand *g, uint32_t seed);      /* srandom_r */
uint32_t or_grand_next(or_grand *g);                     /* random_r  */

typedef struct {
    uint32_t num_wh, dist_per_wh, cust_per_dist, max_items, max_items_per_txn;
    uint32_t part_cnt, part_per_txn, wh_update;
    double perc_payment, mpr;
} or_tpcc_params;
enum { OR_T_WH = 0, OR_T_DIST = 1, OR_T_CUST = 2, OR_T_ITEM = 3, OR_T_STOCK = 4, OR_T_CLAST = 5 };
typedef struct or_tpcc_db or_tpcc_db;
or_tpcc_db *or_tpcc_load(const or_tpcc_params *p, uint64_t seed, uint32_t part_id);
/* the same with i_customer_last kept per partition of an ix_parts-partition
 * layout (tpcc.c clast_key): the all-warehouse image of PART_CNT = ix_parts */
or_tpcc_db *or_tpcc_load_layout(const or_tpcc_params *p, uint64_t seed, uint32_t part_id, uint32_t ix_parts);
void     or_tpcc_free(or_tpcc_db *db);
uint64_t or_tpcc_rows(const or_tpcc_db *db, uint32_t table);
/* keys and the three state columns of a table (NULL = skip) */
int or_tpcc_table(const or_tpcc_db *db, uint32_t table, uint64_t *keys, uint64_t *c0, uint64_t *c1,
                  uint64_t *c2);
int or_tpcc_gen(const or_tpcc_params *p, uint64_t seed, uint32_t home_part, uint32_t n_txn,
                uint64_t *keys, uint8_t *types, uint8_t *tables, uint64_t *args, uint32_t *txn_begin,
                uint8_t *txn_type, uint8_t *owner);
/* one epoch: decisions (E-schedule) then the committed txns' TPC-C operations
 * in sequence order; out_oid[t] = o_id of a committed NewOrder, else 0 */
int or_tpcc_epoch(or_tpcc_db *db, int cc_alg, uint32_t n_txn, const uint32_t *txn_begin,
                  const uint64_t *keys, const uint8_t *types, const uint8_t *tables,
                  const uint64_t *args, uint8_t *out_commit, uint64_t *out_oid, or_epoch_stats *st);
/* owner[a]: the partition an access runs on (a by-name lookup reads that
 * partition's list); required when the db was loaded with ix_parts > 1 */
int or_tpcc_epoch_owner(or_tpcc_db *db, int cc_alg, uint32_t n_txn, const uint32_t *txn_begin,
                        const uint64_t *keys, const uint8_t *types, const uint8_t *tables,
                        const uint64_t *args, const uint8_t *owner, uint8_t *out_commit, uint64_t *out_oid,
                        or_epoch_stats *st);

uint64_t or_mix64(uint64_t z);
uint64_t or_table_digest(const uint64_t *f0, uint64_t n);

/* ---- Deneva-style multi-threaded NO_WAIT engine (mt_engine.c),
 * a throughput baseline; its aborts depend on the interleaving ---- */
uint64_t or_mt_lock_words(uint64_t nrows);  /* the lock array or_mt_epoch_run takes */
int or_mt_epoch_run(const or_index *ix, uint64_t *f0, uint32_t *lock, uint64_t nrows, uint32_t n_txn,
                    const uint32_t *tb, const uint64_t *keys, const uint8_t *types, int threads,
                    uint64_t *committed, uint64_t *digest);

#ifdef __cplusplus
}
#endif
#endif
