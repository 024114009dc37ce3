/*
 * dvcc.h -- C ABI of the MI355X batched concurrency-control engine.
 *
 * This is the drop-in boundary for Deneva's transaction-scheduling hot path.
 * Plain pointers and sizes only; no exceptions cross it; every call returns
 * DV_OK (0) or a negative DV_ERR_* code.  A context owns one HIP device, one
 * stream and all device memory; it is not thread-safe (one host thread per
 * context / GPU, like one CalvinLockThread per node).
 *
 * Which reference interface each entry point replaces (paths relative to the
 * elrodrigues/deneva-plus tree):
 *
 *   dv_open / dv_close          row_t::init_manager (storage/row.cpp:54-74),
 *                               Row_lock::init (concurrency_control/row_lock.cpp:24-44),
 *                               Row_occ::init (row_occ.cpp:22-31), OptCC::init (occ.cpp:31-38)
 *   dv_create_table /           Workload::init_schema (system/wl.cpp:31-149),
 *   dv_load_table               IndexHash::init/index_insert (storage/index_hash.cpp:22-83),
 *                               table_t::get_new_row (storage/table.cpp:43-54)
 *   dv_load_ycsb_partition      YCSBWorkload::init_table_slice (benchmarks/ycsb_wl.cpp:144-203)
 *   dv_epoch_run /              the per-epoch hot path:
 *   dv_epoch_run_device           IndexHash::index_read (index_hash.cpp:137-153) via
 *                                 TxnManager::index_read (system/txn.cpp:906-932);
 *                                 Row_lock::lock_get / lock_release (row_lock.cpp:52-373)
 *                                 for NO_WAIT, WAIT_DIE and CALVIN;
 *                                 OptCC::validate / finish (occ.cpp:42-60, 116-294) and
 *                                 Row_occ::access/validate/write (row_occ.cpp:33-79) for OCC;
 *                                 Calvin's Sequencer::send_next_batch ->
 *                                 QWorkQueue::sched_dequeue -> acquire_locks handoff
 *                                 (sequencer.cpp:283-326, work_queue.cpp:105-151,
 *                                 ycsb_txn.cpp:49-88);
 *                                 YCSBTxnManager::run_ycsb_1 execution (ycsb_txn.cpp:227-254)
 *   dv_epoch_begin /            the same path split at the points where a multi-node
 *   dv_epoch_round_local /      Deneva exchanges RQRY/RPREPARE/RACK_PREP votes and
 *   dv_epoch_round_apply /      combines them in TxnManager::received_response
 *   dv_epoch_finish             (system/txn.cpp:544-554; worker_thread.cpp:277-451)
 *   dv_read_rows /              row_t::get_value on the F0 prefix (storage/row.cpp:130-180)
 *   dv_read_table
 *   dv_ycsb_gen                 YCSBQueryGenerator::gen_requests_zipf
 *                               (benchmarks/ycsb_query.cpp:29-38, 181-202, 303-376)
 *   dv_tpcc_load                TPCCWorkload::init / init_tab_* (benchmarks/tpcc_wl.cpp:95-420)
 *                               with the secondary index i_customer_last
 *   dv_tpcc_gen                 TPCCQueryGenerator::create_query / gen_payment /
 *                               gen_new_order (benchmarks/tpcc_query.cpp:26-263) and the
 *                               access lists of TPCCTxnManager::acquire_locks /
 *                               run_txn_state (tpcc_txn.cpp:117-244, 500-933)
 *   dv_tpcc_epoch_run_device    the hot path for TPC-C: the customer-by-last-name
 *                               index_read + mid selection (tpcc_txn.cpp:600-626),
 *                               then dv_epoch_run_device's probe/lock/validate, then
 *                               run_payment_1/3/5 and new_order_5/9 (tpcc_txn.cpp:530-933)
 *                               for the committed txns
 *   dv_load_table_cols /        row_t::set_value / get_value on the mutated TPC-C
 *   dv_read_table_col           columns (storage/row.cpp:95-180)
 *   dv_tpcc_gen_queries /       TPCCQueryGenerator::gen_payment / gen_new_order's TPCCQuery
 *   dv_tpcc_expand              (tpcc_query.cpp:150-263), then TPCCTxnManager's access lists
 *   dv_wire_open / _decode /    the server's receive path: Transport::recv_msg ->
 *   dv_wire_decode_batches      Message::create_messages -> *ClientQueryMessage::copy_from_buf
 *                               (transport/transport.cpp:245-300; transport/message.cpp:29-59,
 *                               493-510, 620-655, 889-903) into an epoch's host arrays
 *   dv_wire_respond             CL_RSP / CALVIN_ACK replies (worker_thread.cpp:127-152;
 *                               message.cpp:921-949, 1057-1110) packed as MessageThread does
 *                               (transport/msg_thread.cpp:53-111)
 *
 * Decisions follow SURVEY.md 8.0 ("E-schedule"): commit/abort of every txn and
 * the final table state equal a single worker thread running the same epoch
 * in sequence order with the reference's CC plugin.
 */
#ifndef DVCC_H
#define DVCC_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes (the reference returns enum RC, system/global.h:236) */
#define DV_OK 0
#define DV_ERR_ARG (-1)           /* bad argument / capacity exceeded (also: a txn
                                     longer than the epoch's max_txn_acc, a WAIT_DIE
                                     ts array not rising in sequence order)       */
#define DV_ERR_HIP (-2)           /* HIP runtime error                            */
#define DV_ERR_NOMEM (-3)         /* device allocation failed                     */
#define DV_ERR_KEY_NOT_FOUND (-4) /* index probe missed (M_ASSERT_V, index_hash.cpp:225) */
#define DV_ERR_DUP_ROW (-5)       /* reserved (repeated rows in a txn are supported:
                                     dvcc_rounds.hip, round 0)                    */
#define DV_ERR_NO_TABLE (-6)      /* table id not created / not loaded            */
#define DV_ERR_STATE (-7)         /* call out of order (e.g. round before begin)  */
#define DV_ERR_NO_DEVICE (-8)     /* no usable HIP device                         */
#define DV_ERR_TXN_RANGE (-9)     /* an access names a txn >= n_txn, or txns unordered */

/* CC_ALG values as in config.h */
#define DV_NO_WAIT 1
#define DV_WAIT_DIE 2
#define DV_OCC 8
#define DV_CALVIN 10

/* WORKLOAD values as in config.h */
#define DV_YCSB 1
#define DV_TPCC 2 /* contexts keep three 8-byte state columns per row (col 0 = the F0 column) */

/* access_t (system/global.h:287) */
#define DV_RD 0
#define DV_WR 1
#define DV_SCAN 3

/* index hash (storage/index_hash.h:86-92) */
#define DV_HASH_YCSB 0 /* (key / part_cnt) % nbuckets */
#define DV_HASH_MOD 1  /* key % nbuckets               */

/* dv_config.flags */
#define DV_FLAG_TIMING 1u  /* record HIP-event timings per stage into dv_stats
                              (implies DV_FLAG_KERNEL_TIMING)                */
#define DV_FLAG_KERNEL_TIMING 16u /* only the sort-scatter and round-pass
                              launches' own dispatch timestamps (ms_scatter,
                              ms_pass): no marker packets between kernels   */
#define DV_FLAG_KERNEL_PROFILE 32u /* every launch dispatched with its own
                              start / stop timestamps, summed per kernel for
                              dv_kernel_times (measurement legs only: each
                              timed launch costs a few us of latency)       */
#define DV_FLAG_NO_TAIL 2u /* never finish the decision rounds in the single-
                              workgroup tail kernel (testing) */
#define DV_FLAG_EL64 4u    /* always use 64-bit round elements (testing)     */
#define DV_FLAG_LSD_SORT 64u /* sort every epoch's row queues with the plain
                              LSD radix passes, never the one-pass-plus-
                              bucket form of small sorts (testing, A/B)      */
#define DV_FLAG_NO_ASYNC 8u /* never finish the decision rounds in the
                               asynchronous multi-workgroup kernel (that
                               kernel wants every workgroup of its launch
                               resident at once; when co-running work holds
                               CUs its workgroups yield after an idle time,
                               dv_set_async_limits, and the synchronous
                               rounds finish the epoch -- correct either way,
                               this flag only skips the attempt) */

typedef struct dv_ctx dv_ctx;

typedef struct dv_config {
    int32_t device;    /* HIP device ordinal                                  */
    int32_t cc_alg;    /* DV_NO_WAIT / DV_WAIT_DIE / DV_OCC / DV_CALVIN       */
    int32_t workload;  /* DV_YCSB (DV_TPCC reserved)                         */
    uint32_t part_cnt; /* PART_CNT (config.h:14)                              */
    uint32_t part_id;  /* partition owned by this context                     */
    uint32_t max_txn;  /* capacity: txns per epoch (global sequence space)    */
    uint64_t max_acc;  /* capacity: accesses per epoch handled by this context */
    uint32_t flags;    /* DV_FLAG_*                                           */
    uint32_t reserved;
} dv_config;

/* one request of one txn (ycsb_request, benchmarks/ycsb_query.h:35-50) */
typedef struct dv_access {
    uint64_t key;     /* primary key                                          */
    uint32_t txn_seq; /* position of the txn in the epoch's sequence order    */
    uint8_t type;     /* DV_RD / DV_WR / DV_SCAN                              */
    uint8_t table;    /* table id                                             */
    uint16_t flags;   /* reserved, 0                                          */
} dv_access;

/* a device-resident epoch (structure of arrays, all device pointers).
 * Accesses are grouped by txn in sequence order: acc_txn is non-decreasing and
 * a txn's accesses appear in its request order. */
typedef struct dv_epoch_dev {
    const uint64_t *keys;    /* [n_acc]                                     */
    const uint8_t *types;    /* [n_acc] DV_RD / DV_WR / DV_SCAN             */
    const uint32_t *acc_txn; /* [n_acc] txn sequence number of each access  */
    const uint8_t *tables;   /* [n_acc] table ids, or NULL = all table 0    */
    uint64_t n_acc;
    uint32_t n_txn;          /* txns in the epoch (global sequence space)   */
    uint32_t max_txn_acc;    /* upper bound on one txn's accesses in this
                                epoch (e.g. REQ_PER_QUERY); 0 = unknown
                                (<= 128 is always required)                 */
    const uint64_t *ts;      /* [n_txn] WAIT_DIE timestamps (device), or NULL:
                                TS_CAS in sequence order (manager.cpp:52-57), a
                                retried txn keeping its ts and sequenced first.
                                Given, they must rise strictly in sequence order
                                -- else the reference would make txns wait
                                (row_lock.cpp:119-147) -- checked by the probe:
                                DV_ERR_ARG, nothing executes.  Other algorithms
                                never read it.  The partitioned drivers
                                (dv_epoch_run_part, dv_epoch_group_run) take
                                NULL only (DV_ERR_ARG voted on every rank). */
    const uint32_t *n_acc_dev; /* (device) the real access count when it is
                                known only on the device (dv_epoch_refill):
                                n_acc is then an upper bound.  NULL: n_acc is
                                exact.  Single-GPU YCSB entry points, NO_WAIT /
                                WAIT_DIE / OCC (DV_ERR_ARG otherwise). */
    const uint32_t *txn_begin; /* (device, optional) [n_txn + 1] the same epoch's
                                txn boundaries -- txn t's accesses are
                                [txn_begin[t], txn_begin[t + 1]), from 0 to
                                n_acc -- as dv_epoch_run takes them on the
                                host.  Given (with an exact n_acc, no tables),
                                a single-GPU prefix-kill epoch reads each txn's
                                range from it instead of deriving it from
                                acc_txn, and probes the accesses after the
                                prefix inside the kill pass:
                                acc_txn must still describe the same epoch
                                (other paths read it).  Not ascending, or not
                                ending at n_acc: DV_ERR_TXN_RANGE. */
    const uint32_t *recs32;  /* (device, optional, with txn_begin) [n_acc] the same
                                accesses as 4-byte records, key | write << 31
                                (table-0 reads and writes, keys below 2^31: the
                                records of dv_epoch_stage_host_rows).  Given, a
                                prefix-kill epoch reads them instead of keys and
                                types (4 bytes per access instead of 9); keys
                                and types must still describe the same epoch. */
} dv_epoch_dev;

typedef struct dv_stats {
    uint64_t n_txn;
    uint64_t n_acc;
    uint64_t committed;   /* txn_cnt (system/txn.cpp:578)                        */
    uint64_t aborted;     /* total_txn_abort_cnt (statistics/stats.cpp:447)     */
    uint64_t write_cnt;   /* committed WR accesses executed                     */
    uint64_t read_digest; /* sum over committed reads of mix64(v ^ mix64(txn<<32 ^ row)) */
    uint32_t rounds;      /* decision rounds (0 for CALVIN)                     */
    uint32_t sort_passes;
    /* HIP-event timings (ms) when DV_FLAG_TIMING, else 0 */
    float ms_total;
    float ms_probe;
    float ms_sort;
    float ms_decide;
    float ms_exec;
    float ms_scatter;        /* sum over radix-scatter launches                */
    uint32_t scatter_launches;
    uint32_t pass_launches;  /* decision-round pass launches (k_round_pass)    */
    float ms_pass;           /* sum over those launches                        */
    uint16_t async_launches; /* asynchronous-round launches (accepted or not)  */
    uint16_t async_declined; /* ... that found the live set too large          */
    uint64_t pass_live;      /* live accesses those launches read, summed      */
    uint32_t async_yields;   /* asynchronous launches that yielded: the rounds
                                were finished synchronously (dv_set_async_limits) */
    float ms_probe_kernel;   /* the index-probe launch alone, from its own
                                dispatch timestamps (DV_FLAG_KERNEL_TIMING)    */
    /* prefix-kill epochs (dv_set_prefix): the stages' sizes, 0 otherwise */
    uint32_t prefix_txn;     /* txns decided as the prefix                     */
    uint32_t surv_txn;       /* later txns that survived the prefix's kill     */
    uint64_t prefix_acc;     /* the prefix's accesses (its sort keys)          */
    uint64_t surv_acc;       /* the survivors' accesses (their sort keys)      */
    uint64_t async_live;     /* live accesses entering the asynchronous
                                decision launches that ran, summed            */
} dv_stats;

/* per-kernel launch timing (DV_FLAG_KERNEL_PROFILE via dv_set_timing) */
typedef struct dv_kernel_time {
    char name[48];           /* kernel function name, template arguments dropped */
    uint64_t launches;
    double ms_total;         /* sum of the launches' own dispatch-to-end times   */
} dv_kernel_time;

/* parameters of YCSBQueryGenerator (g_* globals, system/global.cpp:65-195) */
typedef struct dv_ycsb_params {
    uint64_t synth_table_size;
    uint32_t part_cnt;
    uint32_t req_per_query;
    double zipf_theta;
    double txn_write_perc;
    double tup_write_perc;
    uint32_t part_per_txn;
    uint32_t strict_ppt;
    double mpr; /* < 0: reference zipf generator; >= 0: MPR gate */
} dv_ycsb_params;

const char *dv_strerror(int code);
int dv_device_count(int *count);

int dv_open(dv_ctx **ctx, const dv_config *cfg);
void dv_close(dv_ctx *ctx);
void *dv_stream(dv_ctx *ctx);     /* the hipStream_t the context launches on */
void *dv_own_stream(dv_ctx *ctx); /* the stream dv_open created              */
/* launch on `stream` exactly as given (NULL = the HIP default stream), e.g. the
 * caller's framework stream, so the engine, the caller's copies and its RCCL
 * collectives share one ordering; dv_set_stream(ctx, dv_own_stream(ctx))
 * returns to the context's own stream */
int dv_set_stream(dv_ctx *ctx, void *stream);
/* switch timing between epochs: flags' DV_FLAG_TIMING / DV_FLAG_KERNEL_TIMING
 * bits replace the context's (the other flags are kept).  Event timing costs
 * launch latency (a marker packet per stage, dispatch timestamps per launch:
 * ~70 us per 1M-txn epoch), so a caller measures with it on and runs without. */
int dv_set_timing(dv_ctx *ctx, uint32_t flags);
/* the per-kernel sums of the launches timed so far under DV_FLAG_KERNEL_PROFILE
 * (waits for the context's stream); fills at most cap entries and returns the
 * number of kernels (>= 0) or an error; reset != 0 starts the sums again */
int dv_kernel_times(dv_ctx *ctx, dv_kernel_time *out, uint32_t cap, int reset);

/* tables: hot column = the 8-byte F0 prefix every YCSB txn reads/writes
 * (ycsb_txn.cpp:227-254); bytes beyond it are never touched by the path (H3). */
int dv_create_table(dv_ctx *ctx, uint32_t table, uint64_t capacity_rows, uint64_t nbuckets,
                    uint32_t hash_kind);
int dv_load_table(dv_ctx *ctx, uint32_t table, const uint64_t *keys, const uint64_t *f0,
                  uint64_t n);
int dv_load_ycsb_partition(dv_ctx *ctx, uint64_t rows_per_part); /* table 0 */
int dv_read_rows(dv_ctx *ctx, uint32_t table, const uint64_t *keys, uint64_t n, uint64_t *out_f0);
int dv_read_table(dv_ctx *ctx, uint32_t table, uint64_t first_row, uint64_t n, uint64_t *out_f0);

/* whole epoch from host buffers (H2D + run + D2H).  ts (may be NULL): one
 * timestamp per txn; WAIT_DIE requires it to rise strictly in sequence order
 * (DV_ERR_ARG otherwise: the reference would make txns wait, row_lock.cpp:
 * 119-147); the other algorithms' decisions do not depend on it.  A txn that
 * touches one row several times: CALVIN locks it once with the first access's
 * type (txn.cpp:778-788); OCC puts it in the write set if any access writes
 * it; NO_WAIT / WAIT_DIE abort the txn unless every access to the row reads
 * (its own lock conflicts, row_lock.cpp:69, 86-90). */
int dv_epoch_run(dv_ctx *ctx, const dv_access *acc, uint64_t n_acc, const uint32_t *txn_begin,
                 uint32_t n_txn, const uint64_t *ts, uint8_t *out_commit,
                 uint32_t *out_grant_group, dv_stats *st);
/* double-buffered host input: dv_epoch_stage_host
 * checks an epoch's host records as dv_epoch_run does and queues their H2D
 * copy into staging slot 0 or 1 on the context's copy stream, returning at
 * once; dv_epoch_run_staged(slot) then runs that epoch on the context's
 * stream (after its copy) and writes the commit bytes to host memory.
 * Staging epoch k+1 before running epoch k overlaps the copy with the
 * decisions.  acc / txn_begin must stay unchanged until the slot's run
 * returns; pinned host memory makes the copy asynchronous (pageable memory
 * is copied before dv_epoch_stage_host returns).  A slot holds one epoch:
 * running an empty slot is DV_ERR_STATE. */
int dv_epoch_stage_host(dv_ctx *ctx, int slot, const dv_access *acc, uint64_t n_acc,
                        const uint32_t *txn_begin, uint32_t n_txn);
/* the same staging from 4-byte records (a quarter of the PCIe bytes): record
 * i = key | (type == DV_WR) << 31 for a table-0 read or write of a key below
 * 2^31 (YCSB keys: rows < 2^31), txn_begin (required, n_txn + 1 offsets)
 * giving each txn's records in sequence order; dv_epoch_run_staged runs it
 * like any staged epoch. */
int dv_epoch_stage_host_rows(dv_ctx *ctx, int slot, const uint32_t *row_wr, uint64_t n_acc,
                             const uint32_t *txn_begin, uint32_t n_txn);
int dv_epoch_run_staged(dv_ctx *ctx, int slot, const uint64_t *ts, uint8_t *out_commit,
                        uint32_t *out_grant_group, dv_stats *st);
/* whole epoch on a device-resident epoch; outputs are device pointers
 * (d_grant_group only for DV_CALVIN, may be NULL) */
int dv_epoch_run_device(dv_ctx *ctx, const dv_epoch_dev *ep, uint8_t *d_commit,
                        uint32_t *d_grant_group, dv_stats *st);

/* abort carry-over: the reference retries an aborted txn with
 * its query unchanged after a penalty (WorkerThread::abort,
 * worker_thread.cpp:160-172 -> AbortQueue::enqueue/process,
 * abort_queue.cpp:26-82).  After dv_epoch_run_device / dv_epoch_finish of
 * `ep` (single GPU, not CALVIN; the context still holds its decisions),
 * writes the accesses of its aborted txns -- in sequence order, renumbered
 * 0..C-1, C = min(aborted, max_txn) -- into out->keys / types / acc_txn
 * (/ tables when ep->tables is set): device arrays with room for ep->n_acc
 * accesses.  Sets out->n_txn = C, out->n_acc, out->max_txn_acc.  The caller
 * opens the next epoch with them, ahead of its new txns (the penalty is one
 * epoch; they keep their priority, as WAIT_DIE keeps a restarted txn's
 * timestamp). */
int dv_epoch_carry(dv_ctx *ctx, const dv_epoch_dev *ep, uint32_t max_txn, dv_epoch_dev *out);

/* RCCL from the engine: one process per GPU, rank r
 * owns partition r (the context's part_cnt / part_id must equal nranks /
 * rank).  Rank 0 makes the id (128 bytes) and the caller hands it to every
 * rank (ncclGetUniqueId / ncclCommInitRank).  dv_epoch_run_part runs a whole
 * partitioned epoch from this rank's client batch `home` (txn ids 0..n_txn-1,
 * global sequence number rank * txns_per_rank + id): split by owner = key %
 * nranks on the device, one all-to-all of the access records, decision
 * rounds closed by all-reduce(MAX) of the undecided txns' verdict bytes
 * (queued two rounds ahead), execution of this rank's rows.  d_commit: device
 * bytes, one per global txn (nranks * txns_per_rank).  Same decisions as
 * deneva-plus_amd/dvcc/partitioned.py over torch.distributed. */
int dv_comm_unique_id(void *id_out);
int dv_comm_init(dv_ctx *ctx, const void *unique_id, int nranks, int rank);
/* the same partitioned epochs for nranks (<= 16) contexts of ONE process --
 * e.g. several partitions on one GPU: ctxs[q] owns partition q; the
 * collectives become device copies between the contexts' streams and a host
 * barrier, so each context must be driven by its own host thread
 * (dv_epoch_run_part called concurrently).  Same protocol, same decisions. */
int dv_comm_init_local(dv_ctx **ctxs, int nranks);
/* the same partitioned epochs for nranks (<= 16) PROCESSES of one node, one
 * context each -- e.g. several ranks sharing one GPU, which RCCL refuses --
 * for testing the protocols across real process boundaries: each rank exports
 * a device staging buffer through a HIP IPC handle and meets the others at a
 * barrier in the POSIX shared-memory segment `name` ("/..." , the same string
 * on every rank, unused before; rank 0 unlinks it once all have joined).
 * Collectives are host-synchronous here (test transport; RCCL is the
 * product's).  Same protocol, same decisions. */
int dv_comm_init_ipc(dv_ctx *ctx, const char *name, int nranks, int rank);
int dv_epoch_run_part(dv_ctx *ctx, const dv_epoch_dev *home, uint32_t txns_per_rank, uint8_t *d_commit,
                      dv_stats *st);
/* how dv_epoch_run_part runs a YCSB epoch.  The list protocol above moves
 * each access to its owner and closes every decision round with an
 * all-reduce; the replicated protocol all-gathers the epoch's accesses (9 B
 * each: 32-bit row id = key, txn id, type) so every rank holds the whole epoch
 * in the global order -- what Calvin's sequencer hands every node -- decides
 * it alone with the single-GPU path (one all-reduce of the owners' key checks
 * after the probe) and executes only its own rows.  mode 0 (default):
 * replicated when every rank's table 0 is a YCSB implicit-row map with a
 * 31-bit global row space and the whole epoch fits the context (max_acc), else
 * the list protocol; 1: always the list protocol; 2: replicated whenever
 * possible, also on a one-rank communicator.  Same decisions either way.
 * OR DV_COMM_WIDE_BATCHES into mode: epoch groups move every batch as 8 bytes
 * per access even where the compact 4-byte form (global rows below 2^30,
 * dense txn ids) applies -- results are identical. */
#define DV_COMM_WIDE_BATCHES 4
/* OR DV_COMM_POSITION_ORDER into mode (epoch groups, and the replicated and
 * list-protocol epochs of dv_epoch_run_part / dv_tpcc_epoch_run_part;
 * NO_WAIT / WAIT_DIE / OCC -- CALVIN keeps the origin order): the sequencer
 * merges the origins'
 * batches of an epoch txn by txn --
 * origin q's txn j is sequence number j * P + q, as clients of all nodes
 * arriving together -- instead of batch by batch (origin q's txn j at
 * q * txns_per_rank + j, Calvin's lock order, which CALVIN always keeps).
 * Decisions are the E-schedule of that sequence (dvcc.sequence_position);
 * every rank must set the same order (else DV_ERR_ARG on every rank).  Why:
 * the decider's prefix (the first n / 32 txns, prefix-kill epochs) then holds
 * every origin's first txns and kills in every partition; origin-major it
 * holds origin 0's only, and at P = 8 four times as many txns survive it. */
#define DV_COMM_POSITION_ORDER 8
int dv_comm_set_mode(dv_ctx *ctx, int mode);

/* Several epochs back to back (the same results as one dv_epoch_run_device
 * per epoch, in order): epoch k+1 is queued on the device before the host
 * reads epoch k's outcome, so the host's turnaround between epochs hides
 * behind the device work (prefix-kill epochs; others run one at a time).  If
 * epoch k's decision rounds halted (an asynchronous launch yielded), epoch
 * k+1 starts halted too -- nothing of it executes -- and both run again
 * synchronously.  d_commits: n device pointers (or NULL; entries may be NULL);
 * sts: n stats (or NULL).  On an error the epochs before the failing one are
 * complete and nothing of the failing one or later ones has executed. */
int dv_epoch_run_device_batch(dv_ctx *ctx, const dv_epoch_dev *eps, uint32_t n, uint8_t *const *d_commits,
                              dv_stats *sts);

/* Decision lanes.  dv_open_lane: a second context (same dv_config, its own
 * stream and workspace) that runs epochs against `owner`'s tables -- no
 * copy; the owner's tables are loaded first and are frozen (dv_create_table /
 * dv_load_* / dv_tpcc_load return DV_ERR_STATE) while it has lanes open; close
 * the lanes before the owner.  Contexts without a communicator only.
 * The reference's analogue is its pool of worker threads deciding txns of
 * the same tables concurrently (worker_thread.cpp:119-180); here the unit is
 * a whole epoch. */
int dv_open_lane(dv_ctx *owner, dv_ctx **lane);

/* n epochs over n_lanes (1..8) contexts -- an owner and its lanes: epoch k
 * is decided on lanes[k % n_lanes], so one epoch's decision (latency-bound
 * rounds) overlaps the next epochs', while executions run strictly in epoch
 * order (epoch k's waits on epoch k-1's, across the lanes' streams, and is
 * skipped when k-1 halted or failed).  Lane l runs on a stream of its own
 * masked to the CUs i with i % n_lanes == l (ordered after the context's
 * stream at the start of the call, and the context's stream after it at the
 * end).  4 lanes measured best on MI355X (2: 1.4x one context's throughput,
 * 4: 1.75x; 3, 6 and 8 less).  The same results, commit bytes, statistics
 * and error behaviour as dv_epoch_run_device_batch on one context; n_lanes
 * == 1 is exactly that. */
int dv_epoch_run_device_lanes(dv_ctx *const *lanes, uint32_t n_lanes, const dv_epoch_dev *eps, uint32_t n,
                              uint8_t *const *d_commits, dv_stats *sts);

/* The closed loop over decision lanes (lanes as for dv_epoch_run_device_lanes,
 * 2..8; n_lanes == 1 is dv_epoch_run_closed_loop): epoch k is decided on
 * lanes[k % n_lanes] and every lane runs a closed loop of its own -- epoch
 * k + n_lanes is epoch k's aborted txns, in sequence order, then fresh txns
 * from the shared pool -- with executions, and the refills drawing on the
 * shared cursor, in epoch order.  One sequence of epochs in which an aborted
 * txn is retried n_lanes epochs later (the reference's AbortQueue retries
 * after a penalty, abort_queue.cpp:26-82).  bufs: 2 * n_lanes buffers (lane
 * l's pair at 2l, 2l + 1); without resume each lane's first epoch is drawn
 * fresh, lane 0 first.  resume continues the previous call: its n_epochs
 * must have been a multiple of 2 * n_lanes (every lane's next epoch is then
 * in its first buffer). */
int dv_epoch_run_closed_loop_lanes(dv_ctx *const *lanes, uint32_t n_lanes, const dv_epoch_dev *pool,
                                   const uint32_t *pool_begin, uint32_t *cursor, uint32_t n_txn, dv_epoch_dev *bufs,
                                   uint64_t buf_cap, uint32_t n_epochs, int resume, uint8_t *const *d_commits,
                                   dv_stats *sts);

/* Ordered lanes for epoch groups (dv_epoch_group_run / _batch, N > 1): an
 * owner and its lanes (1..8; opened before dv_comm_init, each lane then
 * given its OWN communicator) become one execution order -- each on a
 * stream masked to its share of the CUs, driven from its own host thread;
 * lane l runs groups l, l + n_lanes, ... (in every call: hand the groups
 * round the lanes without gaps), decisions of different groups overlap, and
 * a group's execution on this partition waits until the previous group's
 * has been queued (host) and has finished (device).  A group that fails on
 * one lane (every rank fails it, as without lanes) ends the order there: the
 * groups before it execute, every later one returns DV_ERR_STATE; a turn
 * not taken within 120 s also ends it.  n_lanes == 1: that context back on
 * its own stream, unordered.  The epoch groups' results are those of one
 * context running the groups in order.  With communicators (N > 1) each
 * lane's collectives run on its own stream: two lanes' streams must not feed
 * one hardware queue (two RCCL kernels queued in opposite orders on two GPUs
 * would wait for each other), so the call first checks, for every pair of
 * lane streams, that a kernel queued on one runs while a kernel on the other
 * is still running (a bounded probe, ~50 ms at most) and returns
 * DV_ERR_STATE, unordered, if any pair shares a queue.  The
 * reference's analogue: its worker threads processing several txns' remote
 * requests at once on one node while Calvin's sequencer fixes the order
 * (sequencer.cpp:283-326). */
int dv_lanes_order(dv_ctx *const *lanes, uint32_t n_lanes);

/* The closed loop on the device (the reference's retry path,
 * WorkerThread::abort -> AbortQueue, worker_thread.cpp:160-172,
 * abort_queue.cpp:26-82, with a one-epoch penalty): n_epochs epochs of n_txn
 * txns each, single GPU (YCSB, not CALVIN, no communicator).  Epoch k + 1 is
 * epoch k's aborted txns, in sequence order and renumbered from 0 (they keep
 * their priority), then fresh txns taken in order from `pool` starting at
 * *cursor (a device word, advanced and wrapping around pool->n_txn) -- built
 * on the device behind epoch k's execution, its access count left on the
 * device (dv_epoch_dev::n_acc_dev), nothing read back between epochs, epoch
 * k + 1 queued before the host reads epoch k's outcome.
 *   pool: device arrays (keys, types, acc_txn = pool txn ids, tables may be
 *     NULL), n_txn >= n_txn of an epoch, max_txn_acc > 0 (required: it bounds
 *     an epoch's accesses, n_txn * max_txn_acc <= buf_cap and <= the
 *     context's max_acc); pool_begin: device, pool->n_txn + 1 access offsets.
 *   bufs[2]: the epochs' device buffers (keys / types / acc_txn, tables when
 *     the pool has them: buf_cap accesses each; n_acc_dev: a device word);
 *     epoch k lives in bufs[k & 1].
 *   resume 0: epoch 0 is all fresh; 1: epoch 0 is already in bufs[0] (the
 *     epoch a previous call left: on return the next epoch -- the last one's
 *     aborts, then fresh txns -- is in bufs[n_epochs & 1]; swap the buffers
 *     to continue).
 * d_commits / sts: NULL or n_epochs entries (commit bytes of epoch k's txns,
 * its stats; st->n_acc is the real count).  A halted epoch is decided again
 * synchronously before its successor is rebuilt, so the epochs are exactly
 * those of a host loop of dv_epoch_run_device + dv_epoch_carry + the fresh
 * txns (tests/test_closed_loop.py). */
int dv_epoch_run_closed_loop(dv_ctx *ctx, const dv_epoch_dev *pool, const uint32_t *pool_begin, uint32_t *cursor,
                             uint32_t n_txn, dv_epoch_dev *bufs, uint64_t buf_cap, uint32_t n_epochs, int resume,
                             uint8_t *const *d_commits, dv_stats *sts);

/* Epoch groups -- epoch-parallel scheduling for YCSB: a
 * group is P = nranks consecutive epochs of the sequencer, and homes[e]
 * (n_homes == P) is this rank's client batch of epoch e (txn ids local,
 * global sequence number in epoch e: rank * txns_per_rank + id).  Rank e
 * receives every rank's batch of epoch e (all-to-allv, 9 B per access, in
 * origin order = Calvin's sequence), decides epoch e alone with the
 * single-GPU path, and forwards the committed accesses to the partitions
 * owning their rows; every rank then executes epochs 0..P-1 on its own rows,
 * in epoch order.  An epoch's decisions depend only on its own accesses, so
 * the results equal running the P epochs one after the other (dv_epoch_run_part
 * or one GPU): same commit bytes, same final rows.  d_commit (device, P *
 * txns_per_rank bytes, may be NULL): the commit bytes of this rank's txns,
 * epoch e at e * txns_per_rank.  st: committed / aborted / n_txn over the whole
 * group, read_digest / write_cnt of this partition's rows, rounds and
 * timings and n_acc of the epoch this rank decided.
 * Requires every rank's table 0 loaded by dv_load_ycsb_partition (a dense
 * map, so a key's range check is its owner's key check); DV_ERR_ARG on every
 * rank otherwise.  Errors (a key out of range in any epoch, ...) are voted:
 * every rank returns the same code and no row changes.  Batches move as 4 B
 * per access (row id, txn-start and write bits; the decider numbers the txns
 * again) when P x rows < 2^30, else as 8 B (row id, txn id); the compact form
 * needs every txn id below a batch's n_txn to have an access -- a batch with
 * an empty txn fails the group with DV_ERR_ARG on every rank
 * (DV_COMM_WIDE_BATCHES lifts that).  Position-major order
 * (DV_COMM_POSITION_ORDER, dv_comm_set_mode): the decider interleaves the
 * landed batches txn by txn before deciding, the commit bytes come back in
 * origin order as above; a malformed wide batch (txn ids not rising, or past
 * txns_per_rank) fails the group with DV_ERR_ARG on every rank. */
/* Precondition (open loop): the P epochs of a group are decided side by
 * side, so no epoch of a group may depend on the outcome of an earlier epoch
 * of the same group -- in particular a txn aborted in epoch e of group g can
 * be retried at the earliest in group g + 1 (a penalty of up to 2P - 1
 * epochs instead of one; dv_epoch_group_carry builds that retry batch).
 * A caller retrying aborts epoch by epoch needs dv_epoch_run_part. */
int dv_epoch_group_run(dv_ctx *ctx, const dv_epoch_dev *homes, uint32_t n_homes, uint32_t txns_per_rank,
                       uint8_t *d_commit, dv_stats *st);
/* Retries across epoch groups (the reference's AbortQueue, abort_queue.cpp:
 * 26-82, with a penalty of one group = P epochs): after dv_epoch_group_run
 * (or one group of dv_epoch_group_run_batch) returned d_commit for `homes`,
 * writes into outs[e] the accesses of this rank's txns of homes[e] whose
 * commit byte is 0 -- in sequence order, renumbered 0..C-1, C = min(aborted,
 * max_txn) -- into outs[e].keys / types / acc_txn (/ tables when
 * homes[e].tables is set: device arrays with room for homes[e].n_acc
 * accesses), and sets outs[e].n_txn / n_acc / max_txn_acc.  The caller opens
 * rank r's batch of epoch e of group g + 1 with them, ahead of its new txns:
 * a txn aborted in epoch e of group g is retried in epoch e of group g + 1
 * (same epoch slot, so the retries of group g enter group g + 1 in their
 * order), P epochs later instead of one -- the price of deciding a group's
 * epochs side by side (the open-loop precondition above).  Purely local: no
 * collective; one host wait for the counts. */
int dv_epoch_group_carry(dv_ctx *ctx, const dv_epoch_dev *homes, uint32_t n_homes, uint32_t txns_per_rank,
                         const uint8_t *d_commit, uint32_t max_txn, dv_epoch_dev *outs);
/* n_groups consecutive groups, exactly as n_groups dv_epoch_group_run calls
 * (homes: n_groups * n_homes batches, group g's at g * n_homes; d_commits:
 * NULL or one device pointer, each may be NULL, per group; st: NULL or
 * n_groups stats), with one host wait between two groups instead of two:
 * a group's execution digest is read together with the next group's vote.
 * The first failing group's code is returned on every rank and no later
 * group runs; the stats of the groups before it are then unspecified. */
int dv_epoch_group_run_batch(dv_ctx *ctx, const dv_epoch_dev *homes, uint32_t n_groups, uint32_t n_homes,
                             uint32_t txns_per_rank, uint8_t *const *d_commits, dv_stats *st);

/* staged form for partitioned (multi-GPU) epochs.  Every partition holds the
 * same txn statuses after each round, hence the same list of undecided txns
 * (ascending).  dv_epoch_round_local writes this partition's verdict byte for
 * every list entry, in list order, into d_verdict (a device byte array of
 * n_txn entries, rounded up to a multiple of 4; bit1 = abort, bit0 = wait);
 * combine the first U bytes across partitions with an element-wise MAX (U =
 * the list length; any bound on it works, bytes past U are ignored) and hand
 * the result to dv_epoch_round_apply.  Round 0's list is every txn; the list
 * of round r + 1 has the length dv_epoch_round_wait(r) reports.
 * dv_epoch_round_apply with undecided == NULL only enqueues the apply, so
 * rounds can be queued ahead of their outcome (rounds past the fixpoint are
 * no-ops); dv_epoch_round_wait(r) waits for round r's apply and reports the
 * undecided count after it (or after a later round, if that one is already
 * done -- never larger). */
int dv_epoch_begin(dv_ctx *ctx, const dv_epoch_dev *ep, uint32_t *d_grant_group);
int dv_epoch_round_local(dv_ctx *ctx, uint8_t *d_verdict);
int dv_epoch_round_apply(dv_ctx *ctx, const uint8_t *d_verdict, uint32_t *undecided);
int dv_epoch_round_wait(dv_ctx *ctx, uint32_t round, uint32_t *undecided);
int dv_epoch_finish(dv_ctx *ctx, uint8_t *d_commit, dv_stats *st);

/* partitioned epochs, between dv_epoch_begin and the first round: enqueue a
 * copy of this partition's input-error bits (probe: missing key, bad txn
 * order, ...) into the device word d_word; combine the words of all
 * partitions with MAX and hand the result to dv_epoch_errors_combined.  Every
 * partition then treats the epoch as rejected -- rounds are no-ops, each
 * round's outcome reports the error, nothing executes -- so all ranks leave
 * the round loop at the same collective with the same verdict. */
int dv_epoch_errors_local(dv_ctx *ctx, uint32_t *d_word);
int dv_epoch_errors_combined(dv_ctx *ctx, const uint32_t *d_word);

/* asynchronous decision rounds: a workgroup yields after max_iters iterations
 * or idle_us microseconds without a decision (0 = defaults: 2^18, 200 us);
 * the rounds are then finished synchronously (same decisions).  Between
 * epochs; lower values are a testing knob. */
int dv_set_async_limits(dv_ctx *ctx, uint32_t max_iters, uint32_t idle_us);

/* NO_WAIT / WAIT_DIE / OCC epochs of YCSB from 131,072 txns up (single
 * partition) are decided prefix first: the first prefix_txns txns on their
 * own, then every later txn that conflicts with one of their commits aborts at
 * once, and only the survivors go through the rounds (same decisions;
 * dvcc_prefix.hip).  prefix_txns: 0 = automatic (n_txn / 32, clamped to
 * [4096, 65536]), 0xFFFFFFFF = off (every epoch takes the full path), else
 * that many txns for any epoch longer than it.  Between epochs. */
int dv_set_prefix(dv_ctx *ctx, uint32_t prefix_txns);

/* diagnostics: per decision round of the last finished epoch, the live
 * accesses entering the round and the undecided txns before it; returns the
 * number of rounds logged (at most cap, and at most 64) */
int dv_round_log(dv_ctx *ctx, uint32_t *live, uint32_t *undecided, uint32_t cap);

/* host-side epoch builder */
int dv_ycsb_gen(const dv_ycsb_params *p, uint64_t seed, uint32_t home_part, uint32_t n_txn,
                uint64_t *keys, uint8_t *types, uint32_t *txn_begin);

/* ---------------------------------------------------------------- TPC-C (config E)
 * Table ids of this engine (the reference's TPCCTable enum, config.h:200-208,
 * also numbers the insert-only tables; the engine keeps the five tables txns
 * lock plus the i_customer_last secondary index). */
#define DV_TPCC_WAREHOUSE 0
#define DV_TPCC_DISTRICT 1
#define DV_TPCC_CUSTOMER 2
#define DV_TPCC_ITEM 3
#define DV_TPCC_STOCK 4
#define DV_TPCC_CUST_LAST 5 /* key custNPKey (tpcc_helper.cpp:35-43); col 0 = custKey of the row */

/* mutated columns (8-byte words, H4: 4-byte integer parameters zero-extended)
 *   WAREHOUSE  col0 W_YTD (double)          col1 W_TAX (double)
 *   DISTRICT   col0 D_YTD (double)          col1 D_NEXT_O_ID (int64)   col2 D_TAX (double)
 *   CUSTOMER   col0 C_BALANCE (double)      col1 C_YTD_PAYMENT (double)
 *              col2 C_PAYMENT_CNT (loaded as the integer 1, read and written as a double:
 *                   run_payment_5, tpcc_txn.cpp:640-647)
 *   ITEM       col0 I_PRICE (int64)
 *   STOCK      col0 S_QUANTITY (uint64)     col1 S_YTD (int64)         col2 S_ORDER_CNT (int64) */

/* per-access operation word of a TPC-C epoch: op << 56 | operand */
#define DV_TOP_NONE 0      /* a read whose value no output depends on                  */
#define DV_TOP_PAY_WH 1    /* W_YTD += h_amount                 (run_payment_1)        */
#define DV_TOP_PAY_DIST 2  /* D_YTD += h_amount                 (run_payment_3)        */
#define DV_TOP_PAY_CUST 3  /* C_BALANCE -= h, C_YTD_PAYMENT += h, C_PAYMENT_CNT += 1
                              (run_payment_5)                                          */
#define DV_TOP_NO_DIST 4   /* o_id = ++D_NEXT_O_ID              (new_order_5)          */
#define DV_TOP_NO_STOCK 5  /* S_QUANTITY piecewise, S_YTD += q, S_ORDER_CNT += 1
                              (new_order_9); operand = ol_quantity                     */

typedef struct dv_tpcc_params {
    uint32_t num_wh;            /* NUM_WH                                    */
    uint32_t dist_per_wh;       /* DIST_PER_WH (10)                          */
    uint32_t cust_per_dist;     /* g_cust_per_dist (>= 1000, tpcc_wl.cpp)    */
    uint32_t max_items;         /* g_max_items                               */
    uint32_t max_items_per_txn; /* MAX_ITEMS_PER_TXN (15)                    */
    uint32_t part_cnt;          /* PART_CNT; wh_to_part(w) = (w-1) % part_cnt */
    uint32_t part_per_txn;      /* g_part_per_txn                            */
    uint32_t wh_update;         /* WH_UPDATE: Payment writes the warehouse   */
    double perc_payment;        /* PERC_PAYMENT                              */
    double mpr;                 /* g_mpr                                     */
} dv_tpcc_params;

/* rows of each table held by partition part_id (order of dv_tpcc_load) */
int dv_tpcc_table_rows(const dv_tpcc_params *p, uint32_t part_id, uint32_t table, uint64_t *rows);
/* seeded sequential loader for the context's partition (hazard H7: the
 * reference loads with 8 threads sharing glibc rand()); creates and loads the
 * six tables.  The context must be opened with workload DV_TPCC. */
int dv_tpcc_load(dv_ctx *ctx, const dv_tpcc_params *p, uint64_t seed);
/* host side of the same loader: keys and columns of one table (NULL = skip) */
int dv_tpcc_table(const dv_tpcc_params *p, uint64_t seed, uint32_t part_id, uint32_t table,
                  uint64_t *keys, uint64_t *col0, uint64_t *col1, uint64_t *col2);
/* epoch builder: n_txn queries from a glibc-rand stream seeded with `seed`;
 * accesses in run_txn_state order.  Capacity: n_txn * (3 + 2 * max_items_per_txn).
 * txn_type (optional): 1 Payment, 2 NewOrder.  owner (optional): the partition
 * that runs each access (wh_to_part of its warehouse; ITEM reads go with the
 * supply warehouse, as acquire_locks does, tpcc_txn.cpp:210-240). */
int dv_tpcc_gen(const dv_tpcc_params *p, uint64_t seed, uint32_t home_part, uint32_t n_txn,
                uint64_t *keys, uint8_t *types, uint8_t *tables, uint64_t *args,
                uint32_t *txn_begin, uint8_t *txn_type, uint8_t *owner);

/* multi-column tables (DV_TPCC contexts) */
int dv_load_table_cols(dv_ctx *ctx, uint32_t table, const uint64_t *keys, const uint64_t *col0,
                       const uint64_t *col1, const uint64_t *col2, uint64_t n);
int dv_read_table_col(dv_ctx *ctx, uint32_t table, uint32_t col, uint64_t first_row, uint64_t n,
                      uint64_t *out);
/* one TPC-C epoch on the device: ep->tables required; d_args[n_acc] operation
 * words; d_oid[n_txn] (may be NULL) receives o_id of every committed NewOrder
 * whose district is local (0 otherwise) */
int dv_tpcc_epoch_run_device(dv_ctx *ctx, const dv_epoch_dev *ep, const uint64_t *d_args,
                             uint8_t *d_commit, uint64_t *d_oid, dv_stats *st);
/* n TPC-C epochs back to back, pipelined like dv_epoch_run_device_batch
 * (replaces TPCCTxnManager's per-txn loop, tpcc_txn.cpp:117-244, for a
 * stream of epochs): epoch k+1 is queued before epoch k is read back, its
 * clear gated on epoch k (a halted epoch and the one behind it run again
 * synchronously), and its clear writes epoch k's read-back.  d_args[k],
 * d_commits[k] / d_oids[k] (either array, or an entry, may be NULL) as for
 * dv_tpcc_epoch_run_device; sts (may be NULL): n stats.  Stops at the first
 * failing epoch; the ones before it are applied. */
int dv_tpcc_epoch_run_device_batch(dv_ctx *ctx, const dv_epoch_dev *eps, const uint64_t *const *d_args,
                                   uint32_t n, uint8_t *const *d_commits, uint64_t *const *d_oids,
                                   dv_stats *sts);

/* TPC-C epochs over decision lanes (dv_open_lane on a DV_TPCC context), as
 * dv_epoch_run_device_lanes: epoch k decided on lanes[k % n_lanes], executions
 * -- the table updates and each NewOrder's o_id -- in epoch order.  The same
 * results as dv_tpcc_epoch_run_device_batch; n_lanes == 1 is exactly that. */
int dv_tpcc_epoch_run_device_lanes(dv_ctx *const *lanes, uint32_t n_lanes, const dv_epoch_dev *eps,
                                   const uint64_t *const *d_args, uint32_t n, uint8_t *const *d_commits,
                                   uint64_t *const *d_oids, dv_stats *sts);
/* the same from host buffers (H2D + run + D2H; records as dv_epoch_run);
 * out_oid (may be NULL): n_txn words */
int dv_tpcc_epoch_run(dv_ctx *ctx, const dv_access *acc, uint64_t n_acc, const uint32_t *txn_begin,
                      uint32_t n_txn, const uint64_t *args, uint8_t *out_commit, uint64_t *out_oid,
                      dv_stats *st);
/* staged form for partitioned epochs: dv_epoch_begin of a TPC-C epoch (this
 * partition's accesses); then the rounds, and dv_epoch_finish executes the
 * committed txns' operations on this partition's rows.  d_args / d_oid must
 * stay valid until dv_epoch_finish. */
int dv_tpcc_epoch_begin(dv_ctx *ctx, const dv_epoch_dev *ep, const uint64_t *d_args, uint64_t *d_oid);
/* config E from the engine: dv_epoch_run_part for TPC-C
 * contexts after dv_comm_init / dv_comm_init_local.  `home` is this rank's
 * client batch (tables required), d_args its operation words and d_owner
 * the partition of every access (dv_tpcc_gen's owner: the warehouse's
 * partition, ITEM reads with their supply warehouse); records travel to
 * their owner with table and operation word (the RQRY fragments of
 * tpcc_txn.cpp:183-244), each partition resolves last names, decides and
 * executes its rows, and d_oid[nranks * txns_per_rank] ends equal on every
 * rank: the o_id of each committed NewOrder, all-reduced (MAX) from the
 * partition of its district -- Calvin's RFWD forward of o_id
 * (tpcc_txn.cpp:1040, txn.cpp:960-972, transport/message.cpp:982-1025).  An owner byte >= nranks is
 * DV_ERR_ARG on every rank. */
int dv_tpcc_epoch_run_part(dv_ctx *ctx, const dv_epoch_dev *home, const uint64_t *d_args,
                           const uint8_t *d_owner, uint32_t txns_per_rank, uint8_t *d_commit,
                           uint64_t *d_oid, dv_stats *st);

/* ---------------------------------------------------------------- TPC-C queries
 * A client query as TPCCQuery and TPCCClientQueryMessage hold it
 * (benchmarks/tpcc_query.h; transport/message.h:280-312): what runcl sends.
 * dv_tpcc_gen is dv_tpcc_gen_queries followed by dv_tpcc_expand. */
#define DV_TPCC_MAX_OL 62   /* longest NewOrder accepted (MAX_ITEMS_PER_TXN bound here) */
#define DV_TPCC_MAX_PARTS 64
typedef struct dv_tpcc_item {  /* Item_no (benchmarks/tpcc_query.h:30-38) */
    uint64_t ol_i_id, ol_supply_w_id, ol_quantity;
} dv_tpcc_item;
typedef struct dv_tpcc_query {
    uint64_t txn_type;                 /* TPCCTxnType (config.h:209): 1 PAYMENT, 2 NEW_ORDER */
    uint64_t w_id, d_id, c_id;         /* both; c_id: NewOrder, Payment by id          */
    uint64_t d_w_id, c_w_id, c_d_id;   /* Payment                                       */
    char c_last[16];                   /* LASTNAME_LEN, NUL-terminated: Payment by name */
    uint64_t h_amount;                 /* Payment                                       */
    uint8_t by_last_name, rbk, remote, pad_[5];
    uint64_t ol_cnt, o_entry_d;        /* NewOrder                                      */
    uint32_t n_parts, pad2_;           /* BaseQuery::partitions, ascending (std::set)   */
    uint64_t parts[DV_TPCC_MAX_PARTS];
    dv_tpcc_item items[DV_TPCC_MAX_OL];  /* NewOrder: ol_cnt of them                    */
} dv_tpcc_query;

/* the queries of dv_tpcc_gen (same seed, same draws: gen_payment /
 * gen_new_order, tpcc_query.cpp:150-263); fields the reference leaves unset
 * for a txn type are 0 */
int dv_tpcc_gen_queries(const dv_tpcc_params *p, uint64_t seed, uint32_t home_part, uint32_t n_txn,
                        dv_tpcc_query *q);
/* the accesses of n queries in run_txn_state order (tpcc_txn.cpp:500-933),
 * arrays as dv_tpcc_gen's, at most acc_cap accesses (DV_ERR_ARG beyond; a
 * query naming a warehouse, district, customer or item outside p, or an
 * unknown txn type, is DV_ERR_ARG too) */
int dv_tpcc_expand(const dv_tpcc_params *p, const dv_tpcc_query *q, uint32_t n_txn, uint64_t acc_cap,
                   uint64_t *keys, uint8_t *types, uint8_t *tables, uint64_t *args, uint32_t *txn_begin,
                   uint8_t *txn_type, uint8_t *owner);

/* ---------------------------------------------------------------- Deneva wire format
 * Ingress of Deneva's own client stream (transport row): the
 * message batches runcl's MessageThread sends (transport/msg_thread.cpp:
 * 53-111) -- one mbuf of at most MSG_SIZE_MAX bytes, a 12-byte header
 * {u32 dest, u32 src, u32 count} (msg_thread.h:24-62), then `count`
 * messages back to back, each copy_to_buf's fields packed with no padding
 * between them (COPY_BUF, system/helper.h:163-165; x86-64 sizes: RemReqType
 * and access_t 4 bytes, size_t 8, bool 1):
 *   Message header (message.cpp:196-270): rtype u32, txn_id u64, [CALVIN:
 *     batch_id u64], mq_time u64, 7 latency doubles
 *   ClientQueryMessage (856-916): client_startts u64, size_t n, n x u64 partition
 *   YCSBClientQueryMessage (451-526): size_t n, n x ycsb_request (24 bytes:
 *     acctype u32, 4 pad, key u64, value char, 7 pad; ycsb_query.h:35-50)
 *   TPCCClientQueryMessage (544-687): txn_type, w_id, d_id, c_id, d_w_id,
 *     c_w_id, c_d_id (u64), c_last[16], h_amount u64, by_last_name bool,
 *     size_t n, n x Item_no (3 x u64), rbk bool, remote bool, ol_cnt u64,
 *     o_entry_d u64
 *   DoneMessage RDONE (954-977): the header alone (CALVIN: ends a sequencer's batch)
 * The decoder fills a host epoch (dv_epoch_dev's host arrays) straight from
 * the bytes -- Message::create_messages + copy_from_buf + the txn managers'
 * access lists, without a Message object per txn; the epoch then runs as any
 * other (dv_epoch_run / DeviceEpoch).  Replies go back the same way:
 * dv_wire_respond packs the epoch's outcome as CL_RSP batches to the
 * clients (worker_thread.cpp:152; ClientResponseMessage, message.cpp:
 * 921-949), or, under CALVIN, CALVIN_ACK batches to the sequencers
 * (worker_thread.cpp:127-136; AckMessage, message.cpp:1057-1110). */
#define DV_WIRE_MSG_MAX 4096    /* MSG_SIZE_MAX (config.h:94): one mbuf          */
#define DV_WIRE_HDR 12          /* {dest, src, count}                            */
#define DV_WIRE_CL_QRY 3        /* RemReqType (system/global.h:237-262)          */
#define DV_WIRE_RDONE 19
#define DV_WIRE_CL_RSP 20
#define DV_WIRE_CALVIN_ACK 24
#define DV_WIRE_MORE 1          /* dv_wire_decode: the epoch takes no more of this batch */

typedef struct dv_wire_cfg {
    int32_t workload;            /* DV_YCSB / DV_TPCC                                      */
    uint32_t calvin;             /* CC_ALG == CALVIN: the header carries batch_id          */
    uint32_t node_id;            /* g_node_id: every batch's dest                          */
    uint32_t node_cnt;           /* g_node_cnt (servers)                                   */
    uint32_t part_cnt;           /* g_part_cnt: every partition named below it             */
    uint32_t max_req;            /* YCSB: longest request list accepted (<= 128)           */
    uint64_t synth_table_size;   /* YCSB: every key below it (copy_from_buf's assert)      */
    const dv_tpcc_params *tpcc;  /* TPC-C: the knobs the access lists follow               */
} dv_wire_cfg;

typedef struct dv_wire_epoch {
    /* the caller's host buffers and their capacity */
    uint32_t max_txn, pad_;
    uint64_t max_acc;
    uint64_t *keys;              /* [max_acc]                                              */
    uint8_t *types;              /* [max_acc] DV_RD / DV_WR                                */
    uint32_t *txn_begin;         /* [max_txn + 1]                                          */
    uint8_t *tables;             /* [max_acc] TPC-C (NULL for YCSB)                        */
    uint64_t *args;              /* [max_acc] TPC-C operation words                        */
    uint8_t *txn_type;           /* [max_txn] TPC-C, optional                              */
    uint8_t *owner;              /* [max_acc] optional: the partition that runs the access */
    uint64_t *txn_id;            /* [max_txn] optional: the server's txn id (CALVIN: the sequencer's) */
    uint64_t *client_startts;    /* [max_txn] optional: echoed in CL_RSP                   */
    uint32_t *return_node;       /* [max_txn] optional: the batch's src (client / sequencer) */
    /* kept by the decoder */
    uint32_t n_txn, rdone;       /* txns so far; CALVIN: RDONEs taken for batch_id        */
    uint64_t n_acc;
    uint64_t batch_id;           /* CALVIN: the batch its messages name (UINT64_MAX: none yet) */
    uint64_t next_txn;           /* not CALVIN: txn k gets id node_id + node_cnt * k (one worker,
                                    WorkerThread::get_next_txn_id, worker_thread.cpp:453-458);
                                    kept across dv_wire_epoch_reset */
} dv_wire_epoch;

typedef struct dv_wire_cursor {
    const uint8_t *buf;
    uint64_t len;
    uint64_t off;                /* the next message                                       */
    uint32_t left;               /* messages not decoded yet                               */
    uint32_t src;                /* the batch's return node                                */
} dv_wire_cursor;

/* an empty epoch (n_txn = n_acc = 0, txn_begin[0] = 0, batch_id none) */
int dv_wire_epoch_reset(dv_wire_epoch *ep);
/* checks a received batch whole and positions a cursor at its first
 * message: the header (dest == node_id, src != node_id, count >= 1, len
 * within MSG_SIZE_MAX; create_messages' asserts, message.cpp:39-41) and
 * every message -- exactly `count` of them filling exactly `len` bytes, each
 * a CL_QRY (or, under CALVIN, RDONE) with its batch id under CALVIN, keys
 * below synth_table_size, RD / WR requests, at most max_req of them,
 * partitions below part_cnt, TPC-C fields inside the tables (as
 * dv_tpcc_expand checks them).  A malformed batch is DV_ERR_ARG and nothing
 * of it is decoded. */
int dv_wire_open(const dv_wire_cfg *cfg, const uint8_t *batch, uint64_t len, dv_wire_cursor *cur);
/* decodes the cursor's messages into the epoch, in order.  DV_OK: the batch
 * is consumed.  DV_WIRE_MORE: the next message does not fit the epoch's
 * capacity, or (CALVIN) names a later batch -- run the epoch, reset it and
 * call again with the same cursor.  CALVIN: a message naming an earlier
 * batch than the epoch's is DV_ERR_ARG (the cursor stays at it).
 * CALVIN: epoch = one sequencer's batch; RDONE of the epoch's batch_id
 * counts in ep->rdone (the batch is complete at 1 per sequencer); the lock
 * order of several sequencers' batches is origin-major, so decode each
 * sequencer's stream into its own epoch and concatenate them in node order
 * (the Python mirror's dvcc.sequence, QWorkQueue::sched_dequeue,
 * work_queue.cpp:105-151). */
int dv_wire_decode(const dv_wire_cfg *cfg, dv_wire_cursor *cur, dv_wire_epoch *ep);
/* a receive queue's batches at once: batch b is buf[off[b] .. off[b + 1]);
 * decoding starts with what the cursor still holds (cur->buf NULL or
 * cur->left 0: nothing) and goes on from batch *next_batch, which advances
 * past every batch opened.  DV_OK: all consumed.  DV_WIRE_MORE: the epoch
 * is full (or a CALVIN batch ends) -- run it, reset it, call again with the
 * same cursor and *next_batch.  A refused batch (dv_wire_open) returns its
 * error with *next_batch at it. */
int dv_wire_decode_batches(const dv_wire_cfg *cfg, const uint8_t *buf, const uint64_t *off, uint32_t n_batches,
                           dv_wire_cursor *cur, uint32_t *next_batch, dv_wire_epoch *ep);
/* the epoch's replies: not CALVIN, one CL_RSP per committed txn (commit[t]
 * != 0) to its return node; CALVIN, one CALVIN_ACK (rc RCOK) per txn to its
 * sequencer.  Packed into mbufs like MessageThread (a destination's
 * messages in txn order, a batch sent when the next message does not fit),
 * destinations ascending; batch b is out[batch_off[b] .. batch_off[b + 1]).
 * Latency fields are 0 (statistics only).  DV_ERR_ARG if out (cap bytes) or
 * batch_off (max_batches + 1 entries) is too small, or the epoch holds no
 * txn_id / return_node (and, not CALVIN, client_startts) arrays. */
int dv_wire_respond(const dv_wire_cfg *cfg, const dv_wire_epoch *ep, const uint8_t *commit, uint8_t *out,
                    uint64_t cap, uint64_t *batch_off, uint32_t max_batches, uint32_t *n_batches);

#ifdef __cplusplus
}
#endif
#endif
