// tpcc_gen.cpp -- host side of TPC-C (config E): seeded loader and epoch builder.
//
// Follows benchmarks/tpcc_helper.cpp (keys 19-71, Lastname 81-89, RAND/URand/
// NURand 91-128, wh_to_part 161-164), tpcc_wl.cpp (init_tab_item/wh/dist/stock/
// cust, 205-420) and tpcc_query.cpp (create_query 26-32, gen_payment 150-205,
// gen_new_order 207-263), with the access lists of TPCCTxnManager::
// acquire_locks / run_txn_state (tpcc_txn.cpp:117-244, 500-933).
//
// Determinism (hazard H7): the reference loads with 8 threads that share glibc
// rand().  Here one glibc-compatible stream (random_r TYPE_3, the generator
// behind rand()) is seeded per loader / per epoch, and the draws that reach an
// output are taken in a fixed order:
//   items i = 1..max_items: I_IM_ID URand(1,10000), I_PRICE URand(1,100), RAND(10)
//   per warehouse w = 1..num_wh (every partition walks all of them):
//     W_TAX URand(0,200); per district D_TAX URand(0,200);
//     per item S_QUANTITY URand(10,100);
//     per district, per customer c: c_last (c <= 1000: Lastname(c-1), else
//     Lastname(NURand(255,0,999))), C_CREDIT RAND(10), C_DISCOUNT RAND(5000)
// NURand's C constants are drawn lazily from the same stream on first use, as
// the reference's function statics are (one set per stream).  The two operands
// of `URand(0,A) | URand(x,y)` are drawn left to right.  TPCCQuery::remote and
// ol_amount are never assigned in the reference (H5): false and 0 here.
#include <cstdint>
#include <cstring>
#include <set>
#include <string>
#include <vector>

#include "dvcc.h"

namespace {

class GlibcRand {  // glibc random_r, TYPE_3 (x**31 + x**3 + 1), as srand/rand use it
public:
    explicit GlibcRand(uint32_t seed) {
        int32_t r[34];
        r[0] = (int32_t)(seed ? seed : 1u);
        for (int i = 1; i < 31; i++) {
            const int64_t w = (16807LL * r[i - 1]) % 2147483647LL;
            r[i] = (int32_t)(w < 0 ? w + 2147483647LL : w);
        }
        for (int i = 31; i < 34; i++) r[i] = r[i - 31];
        for (int i = 0; i < 34; i++) h_[i] = (uint32_t)r[i];
        n_ = 34;
        for (int i = 0; i < 310; i++) step();
    }
    uint32_t next() { return step() >> 1; }  // rand(): 0 .. RAND_MAX
private:
    uint32_t step() {
        const uint32_t v = h_[(n_ - 31) % 34] + h_[(n_ - 3) % 34];
        h_[n_ % 34] = v;
        n_++;
        return v;
    }
    uint32_t h_[34];
    uint64_t n_;
};

class TpccRand {  // tpcc_helper.cpp:91-128
public:
    explicit TpccRand(uint32_t seed) : g_(seed) {}
    uint64_t RAND(uint64_t max) { return g_.next() % max; }
    uint64_t raw() { return g_.next(); }
    uint64_t URand(uint64_t x, uint64_t y) { return x + RAND(y - x + 1); }
    uint64_t NURand(uint64_t A, uint64_t x, uint64_t y) {
        const int k = A == 255 ? 0 : (A == 1023 ? 1 : 2);
        if (!c_init_[k]) {
            c_[k] = URand(0, A);
            c_init_[k] = true;
        }
        const uint64_t a = URand(0, A);
        const uint64_t b = URand(x, y);
        return (((a | b) + c_[k]) % (y - x + 1)) + x;
    }
private:
    GlibcRand g_;
    bool c_init_[3] = {false, false, false};
    uint64_t c_[3] = {0, 0, 0};
};

std::string last_name(uint64_t num) {  // Lastname (tpcc_helper.cpp:81-89)
    static const char *n[] = {"BAR", "OUGHT", "ABLE", "PRI", "PRES", "ESE", "ANTI", "CALLY", "ATION", "EING"};
    return std::string(n[num / 100]) + n[(num / 10) % 10] + n[num % 10];
}

struct Keys {  // tpcc_helper.cpp:19-47
    uint64_t dpw, cpd, items;
    uint64_t dist(uint64_t d, uint64_t w) const { return w * dpw + d; }
    uint64_t cust(uint64_t c, uint64_t d, uint64_t w) const { return dist(d, w) * cpd + c; }
    uint64_t stock(uint64_t i, uint64_t w) const { return w * items + i; }
    uint64_t cust_np(const std::string &last, uint64_t d, uint64_t w) const {
        uint64_t key = 0;
        for (char ch : last) key = (key << 1) + (uint64_t)(ch - 'A');
        key <<= 10;
        return key + w * dpw + d;  // overflows 10 bits past 102 warehouses (H8), kept verbatim
    }
};

uint64_t dbits(double v) {
    uint64_t b;
    std::memcpy(&b, &v, 8);
    return b;
}

bool valid(const dv_tpcc_params *p) {
    return p && p->num_wh >= 1 && p->dist_per_wh >= 1 && p->cust_per_dist >= 1000 && p->max_items >= 1 &&
           p->max_items_per_txn >= 5 && p->max_items_per_txn <= 62 && p->part_cnt >= 1 &&
           p->part_cnt <= p->num_wh && p->max_items_per_txn <= p->max_items;
}

uint32_t wh_to_part(const dv_tpcc_params *p, uint64_t w) { return (uint32_t)((w - 1) % p->part_cnt); }

struct Out {
    uint64_t *keys, *c0, *c1, *c2;
    uint64_t n = 0;
    void put(uint64_t k, uint64_t a, uint64_t b, uint64_t c) {
        if (keys) keys[n] = k;
        if (c0) c0[n] = a;
        if (c1) c1[n] = b;
        if (c2) c2[n] = c;
        n++;
    }
};

}  // namespace

extern "C" int dv_tpcc_table_rows(const dv_tpcc_params *p, uint32_t part_id, uint32_t table, uint64_t *rows) {
    if (!valid(p) || !rows || part_id >= p->part_cnt) return DV_ERR_ARG;
    uint64_t wh = 0;
    for (uint64_t w = 1; w <= p->num_wh; w++) wh += wh_to_part(p, w) == part_id;
    switch (table) {
    case DV_TPCC_WAREHOUSE: *rows = wh; break;
    case DV_TPCC_DISTRICT: *rows = wh * p->dist_per_wh; break;
    case DV_TPCC_CUSTOMER:
    case DV_TPCC_CUST_LAST: *rows = wh * p->dist_per_wh * p->cust_per_dist; break;
    case DV_TPCC_ITEM: *rows = p->max_items; break;  // replicated (tpcc_wl.cpp:219-241)
    case DV_TPCC_STOCK: *rows = wh * p->max_items; break;
    default: return DV_ERR_NO_TABLE;
    }
    return DV_OK;
}

extern "C" int dv_tpcc_table(const dv_tpcc_params *p, uint64_t seed, uint32_t part_id, uint32_t table,
                             uint64_t *keys, uint64_t *col0, uint64_t *col1, uint64_t *col2) {
    uint64_t nrows;
    int r = dv_tpcc_table_rows(p, part_id, table, &nrows);
    if (r) return r;
    const Keys K{p->dist_per_wh, p->cust_per_dist, p->max_items};
    TpccRand R((uint32_t)seed);
    Out o{keys, col0, col1, col2};
    // init_tab_item (tpcc_wl.cpp:205-224)
    for (uint64_t i = 1; i <= p->max_items; i++) {
        R.URand(1, 10000);
        const uint64_t price = R.URand(1, 100);
        R.RAND(10);
        if (table == DV_TPCC_ITEM) o.put(i, price, 0, 0);
    }
    if (table == DV_TPCC_ITEM) return o.n == nrows ? DV_OK : DV_ERR_STATE;
    for (uint64_t w = 1; w <= p->num_wh; w++) {
        const bool mine = wh_to_part(p, w) == part_id;
        // init_tab_wh (226-258): W_YTD 300000.00, W_TAX URand(0,200)/1000
        const double w_tax = (double)R.URand(0, 200) / 1000.0;
        if (mine && table == DV_TPCC_WAREHOUSE) o.put(w, dbits(300000.0), dbits(w_tax), 0);
        // init_tab_dist (259-288): D_YTD 30000.00, D_NEXT_O_ID 3001
        for (uint64_t d = 1; d <= p->dist_per_wh; d++) {
            const double d_tax = (double)R.URand(0, 200) / 1000.0;
            if (mine && table == DV_TPCC_DISTRICT) o.put(K.dist(d, w), dbits(30000.0), 3001, dbits(d_tax));
        }
        // init_tab_stock (289-330): S_QUANTITY URand(10,100), S_YTD 0, S_ORDER_CNT 0
        for (uint64_t i = 1; i <= p->max_items; i++) {
            const uint64_t q = R.URand(10, 100);
            if (mine && table == DV_TPCC_STOCK) o.put(K.stock(i, w), q, 0, 0);
        }
        // init_tab_cust (331-420): C_BALANCE -10.0, C_YTD_PAYMENT 10.0,
        // C_PAYMENT_CNT set_value(int 1) -> zero-extended 8-byte integer 1 (H4)
        for (uint64_t d = 1; d <= p->dist_per_wh; d++) {
            for (uint64_t c = 1; c <= p->cust_per_dist; c++) {
                const std::string last = c <= 1000 ? last_name(c - 1) : last_name(R.NURand(255, 0, 999));
                R.RAND(10);
                R.RAND(5000);
                if (!mine) continue;
                if (table == DV_TPCC_CUSTOMER)
                    o.put(K.cust(c, d, w), dbits(-10.0), dbits(10.0), 1);
                else if (table == DV_TPCC_CUST_LAST)  // index_insert(i_customer_last, custNPKey, row)
                    o.put(K.cust_np(last, d, w), K.cust(c, d, w), 0, 0);
            }
        }
    }
    return o.n == nrows ? DV_OK : DV_ERR_STATE;
}

// the client queries (gen_payment / gen_new_order, tpcc_query.cpp:150-263),
// every draw in the reference's order; fields the reference leaves unset for
// a txn type stay 0, TPCCQuery::remote is never assigned (H5)
extern "C" int dv_tpcc_gen_queries(const dv_tpcc_params *p, uint64_t seed, uint32_t home_part, uint32_t n_txn,
                                   dv_tpcc_query *q) {
    if (!valid(p) || home_part >= p->part_cnt || (!q && n_txn)) return DV_ERR_ARG;
    TpccRand R((uint32_t)seed);
    auto home_wh = [&]() {  // FIRST_PART_LOCAL (config.h:158)
        uint64_t w;
        while (wh_to_part(p, w = R.URand(1, p->num_wh)) != home_part) {}
        return w;
    };
    for (uint32_t t = 0; t < n_txn; t++) {
        dv_tpcc_query &o = q[t];
        std::memset(&o, 0, sizeof(o));
        std::set<uint64_t> parts;
        const double x = (double)(R.raw() % 100) / 100.0;  // create_query (tpcc_query.cpp:26-32)
        if (x < p->perc_payment) {
            o.txn_type = 1;  // TPCC_PAYMENT
            o.w_id = o.d_w_id = home_wh();
            parts.insert(wh_to_part(p, o.w_id));
            o.d_id = R.URand(1, p->dist_per_wh);
            o.h_amount = R.URand(1, 5000);
            const double xr = (double)(R.raw() % 10000) / 10000;
            const uint64_t y = R.URand(1, 100);
            if (xr > 0.15) {  // home warehouse
                o.c_d_id = o.d_id;
                o.c_w_id = o.w_id;
            } else {          // remote warehouse
                o.c_d_id = R.URand(1, p->dist_per_wh);
                if (p->num_wh > 1) {
                    while ((o.c_w_id = R.URand(1, p->num_wh)) == o.w_id) {}
                    parts.insert(wh_to_part(p, o.c_w_id));
                } else {
                    o.c_w_id = o.w_id;
                }
            }
            if (y <= 60) {
                o.by_last_name = 1;
                const std::string last = last_name(R.NURand(255, 0, 999));
                std::memcpy(o.c_last, last.c_str(), last.size() + 1);
            } else {
                o.c_id = R.NURand(1023, 1, p->cust_per_dist);
            }
        } else {
            o.txn_type = 2;  // TPCC_NEW_ORDER
            o.w_id = home_wh();
            o.d_id = R.URand(1, p->dist_per_wh);
            o.c_id = R.NURand(1023, 1, p->cust_per_dist);
            o.ol_cnt = R.URand(5, p->max_items_per_txn);
            o.o_entry_d = 2013;
            parts.insert(wh_to_part(p, o.w_id));
            const double r_mpr = (double)(R.raw() % 10000) / 10000;
            const uint64_t part_limit = r_mpr < p->mpr ? p->part_per_txn : 1;
            std::set<uint64_t> ids;
            for (uint64_t k = 0; k < o.ol_cnt; k++) {
                dv_tpcc_item &it = o.items[k];
                while (ids.count(it.ol_i_id = R.NURand(8191, 1, p->max_items)) > 0) {}
                ids.insert(it.ol_i_id);
                it.ol_quantity = R.URand(1, 10);
                const double r_rem = (double)(R.raw() % 100000) / 100000;
                if (r_rem > 0.01 || r_mpr > p->mpr || p->num_wh == 1) {
                    it.ol_supply_w_id = o.w_id;
                } else if (parts.size() < part_limit) {
                    it.ol_supply_w_id = R.URand(1, p->num_wh);
                    parts.insert(wh_to_part(p, it.ol_supply_w_id));
                } else {
                    while (parts.count(wh_to_part(p, it.ol_supply_w_id = R.URand(1, p->num_wh))) == 0) {}
                }
            }
        }
        for (uint64_t v : parts) o.parts[o.n_parts++] = v;
    }
    return DV_OK;
}

// TPCCTxnManager's access lists (acquire_locks / run_txn_state,
// tpcc_txn.cpp:117-244, 500-933) of n queries
extern "C" int dv_tpcc_expand(const dv_tpcc_params *p, const dv_tpcc_query *q, uint32_t n_txn, uint64_t acc_cap,
                              uint64_t *keys, uint8_t *types, uint8_t *tables, uint64_t *args, uint32_t *txn_begin,
                              uint8_t *txn_type, uint8_t *owner) {
    if (!valid(p) || (!q && n_txn) || !keys || !types || !tables || !args || !txn_begin) return DV_ERR_ARG;
    const Keys K{p->dist_per_wh, p->cust_per_dist, p->max_items};
    constexpr uint64_t kOperand = (1ull << 56) - 1;
    auto wh_ok = [&](uint64_t w) { return w >= 1 && w <= p->num_wh; };
    auto d_ok = [&](uint64_t d) { return d >= 1 && d <= p->dist_per_wh; };
    uint64_t n = 0;
    // owner: the partition whose node runs the access (acquire_locks tests
    // GET_NODE_ID(wh_to_part(...)) per access; ITEM goes with its supply
    // warehouse's stock access, tpcc_txn.cpp:210-240)
    auto acc = [&](uint8_t table, uint64_t key, uint8_t type, uint64_t op, uint64_t v, uint64_t wh) {
        if (owner) owner[n] = (uint8_t)wh_to_part(p, wh);
        keys[n] = key;
        types[n] = type;
        tables[n] = table;
        args[n] = op << 56 | v;
        n++;
    };
    for (uint32_t t = 0; t < n_txn; t++) {
        const dv_tpcc_query &o = q[t];
        txn_begin[t] = (uint32_t)n;
        if (txn_type) txn_type[t] = (uint8_t)o.txn_type;
        if (o.txn_type == 1) {
            if (!wh_ok(o.w_id) || !d_ok(o.d_id) || !wh_ok(o.c_w_id) || !d_ok(o.c_d_id) || o.h_amount > kOperand)
                return DV_ERR_ARG;
            if (!o.by_last_name && (o.c_id < 1 || o.c_id > p->cust_per_dist)) return DV_ERR_ARG;
            if (o.by_last_name && std::memchr(o.c_last, 0, sizeof(o.c_last)) == nullptr) return DV_ERR_ARG;
            if (n + 3 > acc_cap) return DV_ERR_ARG;
            // run_payment_0..5 (tpcc_txn.cpp:500-660): WH, DIST, CUST
            acc(DV_TPCC_WAREHOUSE, o.w_id, p->wh_update ? DV_WR : DV_RD, p->wh_update ? DV_TOP_PAY_WH : DV_TOP_NONE,
                o.h_amount, o.w_id);
            acc(DV_TPCC_DISTRICT, K.dist(o.d_id, o.w_id), DV_WR, DV_TOP_PAY_DIST, o.h_amount, o.w_id);
            if (o.by_last_name)  // index_read(i_customer_last) + mid (600-626)
                acc(DV_TPCC_CUST_LAST, K.cust_np(std::string(o.c_last), o.c_d_id, o.c_w_id), DV_WR, DV_TOP_PAY_CUST,
                    o.h_amount, o.c_w_id);
            else
                acc(DV_TPCC_CUSTOMER, K.cust(o.c_id, o.c_d_id, o.c_w_id), DV_WR, DV_TOP_PAY_CUST, o.h_amount, o.c_w_id);
        } else if (o.txn_type == 2) {
            if (!wh_ok(o.w_id) || !d_ok(o.d_id) || o.c_id < 1 || o.c_id > p->cust_per_dist || o.ol_cnt < 1 ||
                o.ol_cnt > DV_TPCC_MAX_OL)
                return DV_ERR_ARG;
            for (uint64_t k = 0; k < o.ol_cnt; k++) {
                const dv_tpcc_item &it = o.items[k];
                if (it.ol_i_id < 1 || it.ol_i_id > p->max_items || !wh_ok(it.ol_supply_w_id) ||
                    it.ol_quantity > kOperand)
                    return DV_ERR_ARG;
            }
            if (n + 3 + 2 * o.ol_cnt > acc_cap) return DV_ERR_ARG;
            // new_order_0..5 (tpcc_txn.cpp:663-800): WH RD, CUST RD, DIST WR
            acc(DV_TPCC_WAREHOUSE, o.w_id, DV_RD, DV_TOP_NONE, 0, o.w_id);
            acc(DV_TPCC_CUSTOMER, K.cust(o.c_id, o.d_id, o.w_id), DV_RD, DV_TOP_NONE, 0, o.w_id);
            acc(DV_TPCC_DISTRICT, K.dist(o.d_id, o.w_id), DV_WR, DV_TOP_NO_DIST, 0, o.w_id);
            for (uint64_t k = 0; k < o.ol_cnt; k++) {
                const dv_tpcc_item &it = o.items[k];
                // new_order_6..9 (tpcc_txn.cpp:801-933): ITEM RD, STOCK WR
                acc(DV_TPCC_ITEM, it.ol_i_id, DV_RD, DV_TOP_NONE, 0, it.ol_supply_w_id);
                acc(DV_TPCC_STOCK, K.stock(it.ol_i_id, it.ol_supply_w_id), DV_WR, DV_TOP_NO_STOCK, it.ol_quantity,
                    it.ol_supply_w_id);
            }
        } else {
            return DV_ERR_ARG;
        }
    }
    txn_begin[n_txn] = (uint32_t)n;
    return DV_OK;
}

extern "C" int dv_tpcc_gen(const dv_tpcc_params *p, uint64_t seed, uint32_t home_part, uint32_t n_txn,
                           uint64_t *keys, uint8_t *types, uint8_t *tables, uint64_t *args,
                           uint32_t *txn_begin, uint8_t *txn_type, uint8_t *owner) {
    if (!valid(p) || home_part >= p->part_cnt || !keys || !types || !tables || !args || !txn_begin)
        return DV_ERR_ARG;
    std::vector<dv_tpcc_query> q(n_txn ? n_txn : 1);
    int r = dv_tpcc_gen_queries(p, seed, home_part, n_txn, q.data());
    if (r) return r;
    return dv_tpcc_expand(p, q.data(), n_txn, (uint64_t)n_txn * (3 + 2 * p->max_items_per_txn), keys, types, tables,
                          args, txn_begin, txn_type, owner);
}
