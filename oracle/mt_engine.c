/*
 * mt_engine.c -- a Deneva-style multi-threaded CPU engine, the second CPU
 * baseline of SURVEY.md 8(d)(ii).
 *
 * TEST / BASELINE INFRASTRUCTURE ONLY (see oracle.h): bench.py's cpu_baseline
 * leg times it; nothing in the product links it.  It is a restatement of how
 * the reference runs NO_WAIT on one node, not the reference binary:
 *   - THREAD_CNT workers take txns in sequence order from a shared counter
 *     (the work queue, system/work_queue.cpp: work_queue.cpp:154-233), in
 *     chunks of MT_CHUNK txns, the counter alone on its cache line;
 *   - per access: IndexHash::index_read (index_hash.cpp:137-153, here
 *     or_index_read), then Row_lock::lock_get with NO_WAIT semantics
 *     (row_lock.cpp:52-90: a conflicting request aborts at once) on a per-row
 *     lock word instead of a mutex-protected owner list -- the MT_HOT lowest
 *     rows (zipf's hottest: a row's id is its rank) one word per 64-B line,
 *     as each reference row_t holds its own latch, the rest packed;
 *   - all locks held: run_ycsb_1 (ycsb_txn.cpp:227-254) -- a RD folds the F0
 *     prefix into the read digest, a WR stores 0 -- then release
 *     (row_lock.cpp:241-257); an abort releases what it holds
 *     (TxnManager::cleanup, txn.cpp:700-776) and is not retried.
 * Which txns abort depends on the interleaving (txns in flight = THREAD_CNT),
 * so its decisions are not the E-schedule's; it is a throughput baseline.
 */
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdlib.h>

#include "oracle.h"

#define MT_WR_BIT 0x80000000u
#define MT_HOT 65536u  /* rows with a lock word of their own line */
#define MT_LINE 16u    /* uint32 words per 64-B line */
#define MT_CHUNK 16u   /* txns taken from the work counter at once */

typedef struct {
    const or_index *ix;
    uint64_t *f0;
    _Atomic uint32_t *lock;  /* per row (mt_lock_ix): writer bit | reader count */
    const uint32_t *tb;
    const uint64_t *keys;
    const uint8_t *types;
    uint64_t nrows;  /* rows the lock array holds (or_mt_lock_words) */
    uint32_t n_txn;
    _Alignas(64) _Atomic uint32_t next;  /* next txn to take: alone on its line */
    _Alignas(64) _Atomic uint64_t committed, digest, writes;
    _Atomic uint32_t err;
} mt_shared;

static inline uint64_t mt_lock_ix(uint64_t r) {
    return r < MT_HOT ? r * MT_LINE : (uint64_t)MT_HOT * MT_LINE + (r - MT_HOT);
}

/* lock words or_mt_epoch_run needs for nrows rows */
uint64_t or_mt_lock_words(uint64_t nrows) {
    return nrows <= MT_HOT ? nrows * MT_LINE : (uint64_t)MT_HOT * MT_LINE + (nrows - MT_HOT);
}

static uint64_t mt_mix(uint64_t z) { /* same mixer as the engine's read digest */
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

static int lock_get(_Atomic uint32_t *w, int wr) {
    if (wr) {  /* EX: only on a free row */
        uint32_t expected = 0;
        return atomic_compare_exchange_strong(w, &expected, MT_WR_BIT);
    }
    uint32_t v = atomic_load_explicit(w, memory_order_relaxed);
    for (;;) {  /* SH: while no writer holds it */
        if (v & MT_WR_BIT) return 0;
        if (atomic_compare_exchange_weak(w, &v, v + 1)) return 1;
    }
}

static void lock_release(_Atomic uint32_t *w, int wr) {
    if (wr) atomic_store_explicit(w, 0, memory_order_release);
    else atomic_fetch_sub_explicit(w, 1, memory_order_release);
}

static void *worker(void *arg) {
    mt_shared *s = (mt_shared *)arg;
    /* (the shared block's read-only fields in registers: no loads from the
     * lines the atomics below write) */
    const or_index *ix = s->ix;
    uint64_t *f0 = s->f0;
    _Atomic uint32_t *lock = s->lock;
    const uint32_t *tb = s->tb;
    const uint64_t *keys = s->keys;
    const uint8_t *types = s->types;
    const uint32_t n_txn = s->n_txn;
    const uint64_t nrows = s->nrows;
    uint64_t rows[128];
    int held_wr[128];
    uint64_t committed = 0, digest = 0, writes = 0;
    uint32_t err = 0;
    for (;;) {
        const uint32_t c0 = atomic_fetch_add_explicit(&s->next, MT_CHUNK, memory_order_relaxed);
        if (c0 >= n_txn) break;
        const uint32_t c1 = n_txn - c0 < MT_CHUNK ? n_txn : c0 + MT_CHUNK;
        for (uint32_t t = c0; t < c1; t++) {
            const uint32_t a0 = tb[t], n = tb[t + 1] - a0;
            if (n > 128) { err |= 1u; continue; }
            uint32_t held = 0;
            int ok = 1;
            for (uint32_t j = 0; j < n && ok; j++) {
                uint64_t r;
                if (or_index_read(ix, keys[a0 + j], &r) != 0 || r >= nrows) { err |= 2u; ok = 0; break; }
                const int wr = types[a0 + j] == OR_WR;
                if (!lock_get(&lock[mt_lock_ix(r)], wr)) { ok = 0; break; }
                rows[held] = r;
                held_wr[held++] = wr;
            }
            if (ok) {
                for (uint32_t j = 0; j < held; j++) {
                    if (held_wr[j]) { f0[rows[j]] = 0; writes++; }
                    else digest += mt_mix(f0[rows[j]] ^ mt_mix(((uint64_t)t << 32) ^ keys[a0 + j]));
                }
                committed++;
            }
            for (uint32_t j = held; j-- > 0;) lock_release(&lock[mt_lock_ix(rows[j])], held_wr[j]);
        }
    }
    if (err) atomic_fetch_or(&s->err, err);
    atomic_fetch_add(&s->committed, committed);
    atomic_fetch_add(&s->digest, digest);
    atomic_fetch_add(&s->writes, writes);
    return NULL;
}

/* one epoch on `threads` workers; lock: or_mt_lock_words(nrows) words, zero
 * on entry and exit.
 * Returns 0, or -1 on a bad argument / missing key. */
int or_mt_epoch_run(const or_index *ix, uint64_t *f0, uint32_t *lock, uint64_t nrows, uint32_t n_txn,
                    const uint32_t *tb, const uint64_t *keys, const uint8_t *types, int threads,
                    uint64_t *committed, uint64_t *digest) {
    if (threads < 1 || threads > 256) return -1;
    mt_shared s;
    s.ix = ix;
    s.f0 = f0;
    s.lock = (_Atomic uint32_t *)lock;
    s.tb = tb;
    s.keys = keys;
    s.types = types;
    s.nrows = nrows;
    s.n_txn = n_txn;
    atomic_init(&s.next, 0);
    atomic_init(&s.committed, 0);
    atomic_init(&s.digest, 0);
    atomic_init(&s.writes, 0);
    atomic_init(&s.err, 0);
    pthread_t th[256];
    for (int i = 1; i < threads; i++)
        if (pthread_create(&th[i], NULL, worker, &s) != 0) return -1;
    worker(&s);
    for (int i = 1; i < threads; i++) pthread_join(th[i], NULL);
    if (committed) *committed = atomic_load(&s.committed);
    if (digest) *digest = atomic_load(&s.digest);
    return atomic_load(&s.err) ? -1 : 0;
}
