/*
 * tpcc.c -- CPU restatement of TPC-C on Deneva's hot path (config E).
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h): the checker for the product's
 * TPC-C loader (dv_tpcc_table), epoch builder (dv_tpcc_gen) and device path
 * (dv_tpcc_epoch_run_device).  Parity against the reference binary is
 * unpinned; the generator is pinned to glibc's own rand() by a
 * known-answer test (tests/test_tpcc.py), and the rest restates:
 *   keys, Lastname, RAND/URand/NURand, wh_to_part   benchmarks/tpcc_helper.cpp:19-164
 *   loader (values that reach an output)            benchmarks/tpcc_wl.cpp:205-420
 *   create_query, gen_payment, gen_new_order        benchmarks/tpcc_query.cpp:26-263
 *   access lists                                    benchmarks/tpcc_txn.cpp:117-244, 500-933
 *   customer by last name (mid of the item list)    benchmarks/tpcc_txn.cpp:600-626
 *   execution                                       run_payment_1/3/5, new_order_5/9
 * with the determinism rules of DESIGN.md (H4 zero-extension, H5 remote=false /
 * ol_amount=0, H6 district row in Calvin's phase 5, H7 one seeded stream).
 * Decisions are the E-schedule of oracle.c (or_epoch_decide); committed txns
 * then run one at a time in sequence order.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

/* ---------------------------------------------------- glibc random_r TYPE_3 */
void or_grand_seed(or_grand *g, uint32_t seed) { /* __srandom_r */
    int32_t word = (int32_t)(seed ? seed : 1u);
    g->st[0] = word;
    for (int i = 1; i < 31; i++) {
        const int32_t hi = word / 127773, lo = word % 127773;
        word = 16807 * lo - 2836 * hi;
        if (word < 0) word += 2147483647;
        g->st[i] = word;
    }
    g->f = 3;
    g->r = 0;
    for (int i = 0; i < 310; i++) (void)or_grand_next(g);
}

uint32_t or_grand_next(or_grand *g) { /* __random_r */
    uint32_t val = (uint32_t)g->st[g->f] + (uint32_t)g->st[g->r];
    g->st[g->f] = (int32_t)val;
    const uint32_t result = val >> 1;
    if (++g->f >= 31) {
        g->f = 0;
        ++g->r;
    } else if (++g->r >= 31) {
        g->r = 0;
    }
    return result;
}

typedef struct { or_grand g; int cinit[3]; uint64_t C[3]; } trand;
static uint64_t t_rand(trand *t, uint64_t max) { return or_grand_next(&t->g) % max; }  /* RAND */
static uint64_t t_urand(trand *t, uint64_t x, uint64_t y) { return x + t_rand(t, y - x + 1); }
static uint64_t t_nurand(trand *t, uint64_t A, uint64_t x, uint64_t y) {
    int k = A == 255 ? 0 : (A == 1023 ? 1 : 2);
    if (!t->cinit[k]) { t->C[k] = t_urand(t, 0, A); t->cinit[k] = 1; }
    uint64_t a = t_urand(t, 0, A);
    uint64_t b = t_urand(t, x, y);
    return (((a | b) + t->C[k]) % (y - x + 1)) + x;
}
static void t_init(trand *t, uint64_t seed) { memset(t, 0, sizeof(*t)); or_grand_seed(&t->g, (uint32_t)seed); }

static void lastname(uint64_t num, char *name) {
    static const char *n[] = {"BAR", "OUGHT", "ABLE", "PRI", "PRES", "ESE", "ANTI", "CALLY", "ATION", "EING"};
    strcpy(name, n[num / 100]);
    strcat(name, n[(num / 10) % 10]);
    strcat(name, n[num % 10]);
}

static uint64_t k_dist(const or_tpcc_params *p, uint64_t d, uint64_t w) { return w * p->dist_per_wh + d; }
static uint64_t k_cust(const or_tpcc_params *p, uint64_t c, uint64_t d, uint64_t w) {
    return k_dist(p, d, w) * p->cust_per_dist + c;
}
static uint64_t k_stock(const or_tpcc_params *p, uint64_t i, uint64_t w) { return w * p->max_items + i; }
static uint64_t k_custnp(const or_tpcc_params *p, const char *last, uint64_t d, uint64_t w) {
    uint64_t key = 0;
    char offset = 'A';
    for (uint32_t i = 0; i < strlen(last); i++) key = (key << 1) + (uint64_t)(last[i] - offset);
    key = key << 10;
    key += w * p->dist_per_wh + d;
    return key;
}
static uint32_t wh_part(const or_tpcc_params *p, uint64_t w) { return (uint32_t)((w - 1) % p->part_cnt); }
static uint64_t dbl(double v) { uint64_t b; memcpy(&b, &v, 8); return b; }
static double asd(uint64_t b) { double v; memcpy(&v, &b, 8); return v; }

/* ------------------------------------------------------------------ loader */
typedef struct {
    uint64_t n, cap;
    uint64_t *key, *c0, *c1, *c2;
    or_index *ix;
} ttab;

struct or_tpcc_db {
    or_tpcc_params p;
    ttab t[5];
    or_index *clast;   /* i_customer_last: custNPKey -> customer row */
    uint32_t ix_parts; /* partitions of the index layout (or_tpcc_load_layout) */
    uint64_t base[5];  /* global row id of each table's row 0 */
};

static void tab_init(ttab *t, uint64_t cap) {
    t->cap = cap ? cap : 1;
    t->n = 0;
    t->key = (uint64_t *)malloc(t->cap * 8);
    t->c0 = (uint64_t *)calloc(t->cap, 8);
    t->c1 = (uint64_t *)calloc(t->cap, 8);
    t->c2 = (uint64_t *)calloc(t->cap, 8);
    t->ix = or_index_create(t->cap, 1, 0, t->cap);
}
static uint64_t tab_put(ttab *t, uint64_t key, uint64_t a, uint64_t b, uint64_t c) {
    uint64_t r = t->n++;
    t->key[r] = key; t->c0[r] = a; t->c1[r] = b; t->c2[r] = c;
    or_index_insert(t->ix, key, r);  /* index_insert (index_hash.cpp:69-83) */
    return r;
}

/* i_customer_last lists are per partition (IndexHash::index_read reads the
 * buckets of its part_id, index_hash.cpp:137-153; tpcc_wl.cpp:421-422 inserts
 * with wh_to_part(wid)), and custNPKey's w * DIST_PER_WH + d overflows its 10
 * bits from warehouse 103 on (tpcc_helper.cpp:35-43), so with many warehouses
 * the last-name lists -- and the customer a Payment by name picks -- depend on
 * the partition layout.  ix_parts > 1 keeps one list per (key, partition of
 * ix_parts) in this all-warehouse image, as PART_CNT = ix_parts nodes would;
 * or_tpcc_epoch_owner then reads the list of the access's owner partition. */
static uint64_t clast_key(const or_tpcc_db *db, uint64_t key, uint32_t part) {
    return db->ix_parts > 1 ? key * db->ix_parts + part : key;
}

or_tpcc_db *or_tpcc_load_layout(const or_tpcc_params *p, uint64_t seed, uint32_t part_id, uint32_t ix_parts) {
    if (p->cust_per_dist < 1000 || part_id >= p->part_cnt || ix_parts < 1) return NULL;
    or_tpcc_db *db = (or_tpcc_db *)calloc(1, sizeof(or_tpcc_db));
    db->p = *p;
    db->ix_parts = ix_parts;
    uint64_t wh = 0;
    for (uint64_t w = 1; w <= p->num_wh; w++) wh += wh_part(p, w) == part_id;
    const uint64_t ncust = wh * p->dist_per_wh * p->cust_per_dist;
    tab_init(&db->t[OR_T_WH], wh);
    tab_init(&db->t[OR_T_DIST], wh * p->dist_per_wh);
    tab_init(&db->t[OR_T_CUST], ncust);
    tab_init(&db->t[OR_T_ITEM], p->max_items);
    tab_init(&db->t[OR_T_STOCK], wh * p->max_items);
    db->clast = or_index_create(ncust ? ncust : 1, 1, 0, ncust ? ncust : 1);
    trand R;
    t_init(&R, seed);
    /* init_tab_item (tpcc_wl.cpp:205-224) */
    for (uint64_t i = 1; i <= p->max_items; i++) {
        (void)t_urand(&R, 1, 10000);                  /* I_IM_ID */
        uint64_t price = t_urand(&R, 1, 100);         /* I_PRICE */
        (void)t_rand(&R, 10);                         /* I_DATA "original" */
        tab_put(&db->t[OR_T_ITEM], i, price, 0, 0);
    }
    for (uint64_t w = 1; w <= p->num_wh; w++) {
        int mine = wh_part(p, w) == part_id;
        double w_tax = (double)t_urand(&R, 0, 200) / 1000.0;          /* init_tab_wh */
        if (mine) tab_put(&db->t[OR_T_WH], w, dbl(300000.00), dbl(w_tax), 0);
        for (uint64_t d = 1; d <= p->dist_per_wh; d++) {               /* init_tab_dist */
            double d_tax = (double)t_urand(&R, 0, 200) / 1000.0;
            if (mine) tab_put(&db->t[OR_T_DIST], k_dist(p, d, w), dbl(30000.00), 3001, dbl(d_tax));
        }
        for (uint64_t s = 1; s <= p->max_items; s++) {                 /* init_tab_stock */
            uint64_t q = t_urand(&R, 10, 100);
            if (mine) tab_put(&db->t[OR_T_STOCK], k_stock(p, s, w), q, 0, 0);
        }
        for (uint64_t d = 1; d <= p->dist_per_wh; d++) {               /* init_tab_cust */
            for (uint64_t c = 1; c <= p->cust_per_dist; c++) {
                char last[32];
                if (c <= 1000) lastname(c - 1, last);
                else lastname(t_nurand(&R, 255, 0, 999), last);
                (void)t_rand(&R, 10);                                  /* C_CREDIT */
                (void)t_rand(&R, 5000);                                /* C_DISCOUNT */
                if (!mine) continue;
                uint64_t r = tab_put(&db->t[OR_T_CUST], k_cust(p, c, d, w), dbl(-10.0), dbl(10.0), 1);
                or_index_insert(db->clast, clast_key(db, k_custnp(p, last, d, w), (uint32_t)((w - 1) % ix_parts)), r);
            }
        }
    }
    uint64_t b = 0;
    for (int t = 0; t < 5; t++) { db->base[t] = b; b += db->t[t].n; }
    return db;
}

or_tpcc_db *or_tpcc_load(const or_tpcc_params *p, uint64_t seed, uint32_t part_id) {
    return or_tpcc_load_layout(p, seed, part_id, 1);
}

void or_tpcc_free(or_tpcc_db *db) {
    if (!db) return;
    for (int t = 0; t < 5; t++) {
        free(db->t[t].key); free(db->t[t].c0); free(db->t[t].c1); free(db->t[t].c2);
        or_index_free(db->t[t].ix);
    }
    or_index_free(db->clast);
    free(db);
}

uint64_t or_tpcc_rows(const or_tpcc_db *db, uint32_t table) { return table < 5 ? db->t[table].n : 0; }

int or_tpcc_table(const or_tpcc_db *db, uint32_t table, uint64_t *keys, uint64_t *c0, uint64_t *c1,
                  uint64_t *c2) {
    if (table >= 5) return -1;
    const ttab *t = &db->t[table];
    if (keys) memcpy(keys, t->key, t->n * 8);
    if (c0) memcpy(c0, t->c0, t->n * 8);
    if (c1) memcpy(c1, t->c1, t->n * 8);
    if (c2) memcpy(c2, t->c2, t->n * 8);
    return 0;
}

/* ------------------------------------------------------------------ queries */
enum { OP_NONE = 0, OP_PAY_WH = 1, OP_PAY_DIST = 2, OP_PAY_CUST = 3, OP_NO_DIST = 4, OP_NO_STOCK = 5 };

int or_tpcc_gen(const or_tpcc_params *p, uint64_t seed, uint32_t home_part, uint32_t n_txn,
                uint64_t *keys, uint8_t *types, uint8_t *tables, uint64_t *args, uint32_t *txn_begin,
                uint8_t *txn_type, uint8_t *owner) {
    trand R;
    t_init(&R, seed);
    uint64_t n = 0;
#define ACC(tb, k, ty, op, v, wh) do { if (owner) owner[n] = (uint8_t)wh_part(p, (wh)); keys[n] = (k); types[n] = (ty); tables[n] = (tb); \
                                   args[n] = ((uint64_t)(op) << 56) | (v); n++; } while (0)
    for (uint32_t t = 0; t < n_txn; t++) {
        txn_begin[t] = (uint32_t)n;
        double x = (double)(or_grand_next(&R.g) % 100) / 100.0;
        uint64_t w;
        if (x < p->perc_payment) {                             /* gen_payment */
            if (txn_type) txn_type[t] = 1;
            while (wh_part(p, w = t_urand(&R, 1, p->num_wh)) != home_part) {}
            uint64_t d_id = t_urand(&R, 1, p->dist_per_wh);
            uint64_t h_amount = t_urand(&R, 1, 5000);
            double xr = (double)(or_grand_next(&R.g) % 10000) / 10000;
            int y = (int)t_urand(&R, 1, 100);
            uint64_t c_d_id, c_w_id;
            if (xr > 0.15) {
                c_d_id = d_id;
                c_w_id = w;
            } else {
                c_d_id = t_urand(&R, 1, p->dist_per_wh);
                if (p->num_wh > 1) {
                    while ((c_w_id = t_urand(&R, 1, p->num_wh)) == w) {}
                } else {
                    c_w_id = w;
                }
            }
            ACC(OR_T_WH, w, p->wh_update ? OR_WR : OR_RD, p->wh_update ? OP_PAY_WH : OP_NONE, h_amount, w);
            ACC(OR_T_DIST, k_dist(p, d_id, w), OR_WR, OP_PAY_DIST, h_amount, w);
            if (y <= 60) {
                char last[32];
                lastname(t_nurand(&R, 255, 0, 999), last);
                ACC(OR_T_CLAST, k_custnp(p, last, c_d_id, c_w_id), OR_WR, OP_PAY_CUST, h_amount, c_w_id);
            } else {
                uint64_t c_id = t_nurand(&R, 1023, 1, p->cust_per_dist);
                ACC(OR_T_CUST, k_cust(p, c_id, c_d_id, c_w_id), OR_WR, OP_PAY_CUST, h_amount, c_w_id);
            }
        } else {                                               /* gen_new_order */
            if (txn_type) txn_type[t] = 2;
            while (wh_part(p, w = t_urand(&R, 1, p->num_wh)) != home_part) {}
            uint64_t d_id = t_urand(&R, 1, p->dist_per_wh);
            uint64_t c_id = t_nurand(&R, 1023, 1, p->cust_per_dist);
            uint64_t ol_cnt = t_urand(&R, 5, p->max_items_per_txn);
            uint32_t parts[64];
            uint32_t nparts = 0;
            parts[nparts++] = wh_part(p, w);
            double r_mpr = (double)(or_grand_next(&R.g) % 10000) / 10000;
            uint64_t part_limit = r_mpr < p->mpr ? p->part_per_txn : 1;
            ACC(OR_T_WH, w, OR_RD, OP_NONE, 0, w);
            ACC(OR_T_CUST, k_cust(p, c_id, d_id, w), OR_RD, OP_NONE, 0, w);
            ACC(OR_T_DIST, k_dist(p, d_id, w), OR_WR, OP_NO_DIST, 0, w);
            uint64_t ids[64];
            for (uint64_t k = 0; k < ol_cnt; k++) {
                uint64_t i_id;
                for (;;) {
                    i_id = t_nurand(&R, 8191, 1, p->max_items);
                    int seen = 0;
                    for (uint64_t z = 0; z < k; z++) seen |= ids[z] == i_id;
                    if (!seen) break;
                }
                ids[k] = i_id;
                uint64_t qty = t_urand(&R, 1, 10);
                double r_rem = (double)(or_grand_next(&R.g) % 100000) / 100000;
                uint64_t sw;
                if (r_rem > 0.01 || r_mpr > p->mpr || p->num_wh == 1) {
                    sw = w;
                } else if (nparts < part_limit) {
                    sw = t_urand(&R, 1, p->num_wh);
                    uint32_t pp = wh_part(p, sw);
                    int have = 0;
                    for (uint32_t z = 0; z < nparts; z++) have |= parts[z] == pp;
                    if (!have) parts[nparts++] = pp;
                } else {
                    for (;;) {
                        sw = t_urand(&R, 1, p->num_wh);
                        uint32_t pp = wh_part(p, sw);
                        int have = 0;
                        for (uint32_t z = 0; z < nparts; z++) have |= parts[z] == pp;
                        if (have) break;
                    }
                }
                ACC(OR_T_ITEM, i_id, OR_RD, OP_NONE, 0, sw);
                ACC(OR_T_STOCK, k_stock(p, i_id, sw), OR_WR, OP_NO_STOCK, qty, sw);
            }
        }
    }
#undef ACC
    txn_begin[n_txn] = (uint32_t)n;
    return 0;
}

/* ------------------------------------------------------------------ epoch */
int or_tpcc_epoch_owner(or_tpcc_db *db, int cc_alg, uint32_t n_txn, const uint32_t *tb, const uint64_t *keys,
                        const uint8_t *types, const uint8_t *tables, const uint64_t *args, const uint8_t *owner,
                        uint8_t *out_commit, uint64_t *out_oid, or_epoch_stats *st) {
    if (db->ix_parts > 1 && !owner) return -1;
    uint64_t n_acc = tb[n_txn];
    uint64_t *rows = (uint64_t *)malloc((n_acc + 1) * 8);
    uint8_t *tab = (uint8_t *)malloc(n_acc + 1);
    for (uint64_t a = 0; a < n_acc; a++) {
        uint64_t r;
        int rc;
        uint8_t t = tables[a];
        if (t == OR_T_CLAST) {             /* run_payment_4 by last name */
            rc = or_index_read_mid(db->clast, clast_key(db, keys[a], owner ? owner[a] : 0u), &r);
            t = OR_T_CUST;
        } else if (t < 5) {
            rc = or_index_read(db->t[t].ix, keys[a], &r);
        } else {
            rc = -1;
        }
        if (rc) { free(rows); free(tab); return -1; }
        tab[a] = t;
        rows[a] = db->base[t] + r;
    }
    uint64_t nrows = db->base[4] + db->t[4].n;
    int rc = or_epoch_decide(cc_alg, rows, nrows, n_txn, tb, types, out_commit, NULL, st);
    if (rc) { free(rows); free(tab); return rc; }
    /* committed txns in sequence order */
    for (uint32_t t = 0; t < n_txn; t++) {
        if (out_oid) out_oid[t] = 0;
        if (!out_commit[t]) continue;
        for (uint64_t a = tb[t]; a < tb[t + 1]; a++) {
            ttab *T = &db->t[tab[a]];
            uint64_t r = rows[a] - db->base[tab[a]];
            uint64_t op = args[a] >> 56, v = args[a] & ((1ull << 56) - 1);
            double h = (double)v;
            switch (op) {
            case OP_PAY_WH:   /* run_payment_1: W_YTD = w_ytd + h_amount */
            case OP_PAY_DIST: /* run_payment_3: D_YTD = d_ytd + h_amount */
                T->c0[r] = dbl(asd(T->c0[r]) + h);
                break;
            case OP_PAY_CUST: /* run_payment_5 */
                T->c0[r] = dbl(asd(T->c0[r]) - h);
                T->c1[r] = dbl(asd(T->c1[r]) + h);
                T->c2[r] = dbl(asd(T->c2[r]) + 1);
                break;
            case OP_NO_DIST: { /* new_order_5 */
                int64_t o_id = (int64_t)T->c1[r];
                o_id++;
                T->c1[r] = (uint64_t)o_id;
                if (out_oid) out_oid[t] = (uint64_t)o_id;
                break;
            }
            case OP_NO_STOCK: { /* new_order_9 (TPCC_SMALL false, remote false) */
                uint64_t s_quantity = T->c0[r];
                T->c1[r] = (uint64_t)((int64_t)T->c1[r] + (int64_t)v);
                T->c2[r] = (uint64_t)((int64_t)T->c2[r] + 1);
                uint64_t quantity = s_quantity > v + 10 ? s_quantity - v : s_quantity - v + 91;
                T->c0[r] = quantity;
                break;
            }
            default:
                break;
            }
        }
    }
    free(rows);
    free(tab);
    return 0;
}

int or_tpcc_epoch(or_tpcc_db *db, int cc_alg, uint32_t n_txn, const uint32_t *tb, const uint64_t *keys,
                  const uint8_t *types, const uint8_t *tables, const uint64_t *args, uint8_t *out_commit,
                  uint64_t *out_oid, or_epoch_stats *st) {
    return or_tpcc_epoch_owner(db, cc_alg, n_txn, tb, keys, types, tables, args, NULL, out_commit, out_oid, st);
}
