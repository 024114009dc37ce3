/*
 * mt_engine.c -- a Deneva-style multi-threaded CPU engine, the second CPU
 * baseline of SURVEY.md 8(d)(ii).
 *
 * TEST / BASELINE INFRASTRUCTURE ONLY (see oracle.h): bench.py's cpu_baseline
 * leg times it; nothing in the product links it.  It is a restatement of how
 * the reference runs NO_WAIT on one node, not the reference binary:
 *   - THREAD_CNT workers take txns in sequence order from a shared counter
 *     (the work queue, system/work_queue.cpp);
 *   - per access: IndexHash::index_read (index_hash.cpp:137-153, here
 *     or_index_read), then Row_lock::lock_get with NO_WAIT semantics
 *     (row_lock.cpp:52-90: a conflicting request aborts at once) on a per-row
 *     lock word instead of a mutex-protected owner list;
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

typedef struct {
    const or_index *ix;
    uint64_t *f0;
    _Atomic uint32_t *lock;  /* per row: writer bit | reader count */
    const uint32_t *tb;
    const uint64_t *keys;
    const uint8_t *types;
    uint32_t n_txn;
    _Atomic uint32_t next;   /* next txn to take */
    _Atomic uint64_t committed, digest, writes;
    _Atomic uint32_t err;
} mt_shared;

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
    uint64_t rows[128];
    int held_wr[128];
    uint64_t committed = 0, digest = 0, writes = 0;
    for (;;) {
        const uint32_t t = atomic_fetch_add_explicit(&s->next, 1, memory_order_relaxed);
        if (t >= s->n_txn) break;
        const uint32_t a0 = s->tb[t], n = s->tb[t + 1] - a0;
        if (n > 128) { atomic_fetch_or(&s->err, 1u); continue; }
        uint32_t held = 0;
        int ok = 1;
        for (uint32_t j = 0; j < n && ok; j++) {
            uint64_t r;
            if (or_index_read(s->ix, s->keys[a0 + j], &r) != 0) { atomic_fetch_or(&s->err, 2u); ok = 0; break; }
            const int wr = s->types[a0 + j] == OR_WR;
            if (!lock_get(&s->lock[r], wr)) { ok = 0; break; }
            rows[held] = r;
            held_wr[held++] = wr;
        }
        if (ok) {
            for (uint32_t j = 0; j < held; j++) {
                if (held_wr[j]) { s->f0[rows[j]] = 0; writes++; }
                else digest += mt_mix(s->f0[rows[j]] ^ mt_mix(((uint64_t)t << 32) ^ s->keys[a0 + j]));
            }
            committed++;
        }
        for (uint32_t j = held; j-- > 0;) lock_release(&s->lock[rows[j]], held_wr[j]);
    }
    atomic_fetch_add(&s->committed, committed);
    atomic_fetch_add(&s->digest, digest);
    atomic_fetch_add(&s->writes, writes);
    return NULL;
}

/* one epoch on `threads` workers; lock: nrows words, zero on entry and exit.
 * Returns 0, or -1 on a bad argument / missing key. */
int or_mt_epoch_run(const or_index *ix, uint64_t *f0, uint32_t *lock, uint64_t nrows, uint32_t n_txn,
                    const uint32_t *tb, const uint64_t *keys, const uint8_t *types, int threads,
                    uint64_t *committed, uint64_t *digest) {
    (void)nrows;
    if (threads < 1 || threads > 256) return -1;
    mt_shared s;
    s.ix = ix;
    s.f0 = f0;
    s.lock = (_Atomic uint32_t *)lock;
    s.tb = tb;
    s.keys = keys;
    s.types = types;
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
