// host_driver_test.cpp -- the C++ host mirror (include/dvcc_host.hpp) driven the
// way a Deneva workload driver would drive it, checked against the CPU oracle.
//
// TEST INFRASTRUCTURE: links oracle/build/liboracle.so as the checker.  Run by
// tests/test_host_cpp.py on the GPU box (needs a visible MI355X).
//   YCSB:  YCSBQueryGenerator queries (dv_ycsb_gen) -> acquire_ycsb per txn -> run;
//          commit RCs and the final F0 column vs or_epoch_run.
//   TPC-C: TPCCQuery objects -> acquire_tpcc per txn -> run_tpcc; RCs, o_ids and
//          every state column vs or_tpcc_epoch on the same access lists.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "dvcc_host.hpp"
#include "oracle.h"

using namespace dvcc_host;

static int failures = 0;
#define CHECK(cond, ...)                                   \
    do {                                                   \
        if (!(cond)) {                                     \
            std::printf("FAIL %s:%d: ", __FILE__, __LINE__); \
            std::printf(__VA_ARGS__);                      \
            std::printf("\n");                             \
            failures++;                                    \
        }                                                  \
    } while (0)

static const char *kNames[] = {"BAR", "OUGHT", "ABLE", "PRI", "PRES", "ESE", "ANTI", "CALLY", "ATION", "EING"};
static std::string last_name(unsigned n) {
    return std::string(kNames[n / 100]) + kNames[(n / 10) % 10] + kNames[n % 10];
}

struct Lcg {  // test-local query source (any valid queries will do)
    uint64_t s;
    uint64_t next(uint64_t lo, uint64_t hi) {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        return lo + (s >> 33) % (hi - lo + 1);
    }
};

static void ycsb_case(int cc) {
    const uint64_t rows = 1 << 14;
    const uint32_t n_txn = 4096, R = 10;
    dv_ycsb_params p{rows, 1, R, 0.9, 1.0, 0.5, 1, 0, -1.0};
    std::vector<uint64_t> keys(n_txn * R);
    std::vector<uint8_t> types(n_txn * R);
    std::vector<uint32_t> tb(n_txn + 1);
    CHECK(dv_ycsb_gen(&p, 77, 0, n_txn, keys.data(), types.data(), tb.data()) == DV_OK, "gen");
    EpochRunner run;
    dv_config cfg{0, cc, DV_YCSB, 1, 0, n_txn, (uint64_t)n_txn * R, 0, 0};
    CHECK(run.open(cfg) == DV_OK, "open");
    CHECK(run.load_ycsb(rows) == DV_OK, "load");
    for (uint32_t t = 0; t < n_txn; t++) {
        std::vector<ycsb_request> q;
        for (uint32_t a = tb[t]; a < tb[t + 1]; a++)
            q.push_back(ycsb_request{types[a] == DV_WR ? WR : RD, keys[a], 0});
        CHECK(run.acquire_ycsb(q) == t, "txn numbering");
    }
    std::vector<RC> rc;
    dv_stats st{};
    CHECK(run.run(rc, &st) == DV_OK, "run cc=%d", cc);
    // oracle
    or_index *ix = or_index_create(rows, 1, 1, rows);
    std::vector<uint64_t> f0(rows);
    or_ycsb_load(ix, f0.data(), rows, 1, 0);
    std::vector<uint8_t> commit(n_txn);
    or_epoch_stats os{};
    CHECK(or_epoch_run(cc, ix, f0.data(), rows, n_txn, tb.data(), keys.data(), types.data(), commit.data(),
                       nullptr, 0, &os) == 0, "oracle");
    uint32_t bad = 0;
    for (uint32_t t = 0; t < n_txn; t++) bad += (rc[t] == RCOK) != (commit[t] == 1);
    CHECK(bad == 0, "cc=%d: %u commit mismatches", cc, bad);
    CHECK(st.committed == os.committed && st.read_digest == os.read_digest, "cc=%d stats", cc);
    std::vector<uint64_t> got(rows);
    CHECK(dv_read_table(run.ctx(), 0, 0, rows, got.data()) == DV_OK, "read");
    CHECK(got == f0, "cc=%d: table mismatch", cc);
    or_index_free(ix);
    std::printf("ycsb cc=%d: %llu/%u committed, parity ok\n", cc, (unsigned long long)st.committed, n_txn);
}

static void tpcc_case(int cc) {
    dv_tpcc_params p{2, 10, 1000, 2000, 15, 1, 2, 1, 0.5, 1.0};
    const uint32_t n_txn = 3000;
    EpochRunner run;
    dv_config cfg{0, cc, DV_TPCC, 1, 0, n_txn, (uint64_t)n_txn * 33, 0, 0};
    CHECK(run.open(cfg) == DV_OK, "open");
    CHECK(run.load_tpcc(p, 5) == DV_OK, "load");
    Lcg g{(uint64_t)cc * 1000 + 1};
    for (uint32_t t = 0; t < n_txn; t++) {
        TPCCQuery q;
        q.w_id = q.d_w_id = g.next(1, p.num_wh);
        q.d_id = g.next(1, p.dist_per_wh);
        if (g.next(0, 1)) {
            q.txn_type = TPCC_PAYMENT;
            q.c_w_id = g.next(1, p.num_wh);
            q.c_d_id = g.next(1, p.dist_per_wh);
            q.h_amount = (double)g.next(1, 5000);
            q.by_last_name = g.next(0, 9) < 6;
            if (q.by_last_name)
                q.c_last = last_name((unsigned)g.next(0, 999));
            else
                q.c_id = g.next(1, p.cust_per_dist);
        } else {
            q.txn_type = TPCC_NEW_ORDER;
            q.c_id = g.next(1, p.cust_per_dist);
            const uint64_t cnt = g.next(5, 15);
            while (q.items.size() < cnt) {
                const uint64_t i = g.next(1, p.max_items);
                bool dup = false;
                for (const Item_no &it : q.items) dup |= it.ol_i_id == i;
                if (!dup) q.items.push_back(Item_no{i, g.next(0, 99) ? q.w_id : g.next(1, p.num_wh), g.next(1, 10)});
            }
        }
        run.acquire_tpcc(q);
        if (t == 0) {  // the access list of acquire_locks for this first query
            const auto &a = run.accesses();
            if (q.txn_type == TPCC_PAYMENT) {
                CHECK(a.size() == 3 && a[0].table == DV_TPCC_WAREHOUSE && a[0].key == q.w_id &&
                          a[1].table == DV_TPCC_DISTRICT && a[1].key == q.w_id * 10 + q.d_id &&
                          a[2].type == DV_WR, "payment access list");
            } else {
                CHECK(a.size() == 3 + 2 * q.items.size() && a[1].table == DV_TPCC_CUSTOMER &&
                          a[1].key == (q.w_id * 10 + q.d_id) * 1000 + q.c_id && a[2].type == DV_WR &&
                          a[4].table == DV_TPCC_STOCK &&
                          a[4].key == q.items[0].ol_supply_w_id * 2000 + q.items[0].ol_i_id,
                      "new-order access list");
            }
        }
    }
    // the same access lists for the oracle
    std::vector<uint64_t> keys, args(run.ops());
    std::vector<uint8_t> types, tables;
    std::vector<uint32_t> tb(n_txn + 1, 0);
    for (const dv_access &a : run.accesses()) {
        keys.push_back(a.key);
        types.push_back(a.type);
        tables.push_back(a.table);
        tb[a.txn_seq + 1]++;
    }
    for (uint32_t t = 0; t < n_txn; t++) tb[t + 1] += tb[t];
    std::vector<RC> rc;
    std::vector<uint64_t> oid;
    dv_stats st{};
    CHECK(run.run_tpcc(rc, oid, &st) == DV_OK, "run_tpcc cc=%d", cc);
    or_tpcc_params op{p.num_wh, p.dist_per_wh, p.cust_per_dist, p.max_items, p.max_items_per_txn,
                      p.part_cnt, p.part_per_txn, p.wh_update, p.perc_payment, p.mpr};
    or_tpcc_db *db = or_tpcc_load(&op, 5, 0);
    std::vector<uint8_t> commit(n_txn);
    std::vector<uint64_t> oref(n_txn);
    or_epoch_stats os{};
    CHECK(or_tpcc_epoch(db, cc, n_txn, tb.data(), keys.data(), types.data(), tables.data(), args.data(),
                        commit.data(), oref.data(), &os) == 0, "oracle");
    uint32_t bad = 0;
    for (uint32_t t = 0; t < n_txn; t++) bad += ((rc[t] == RCOK) != (commit[t] == 1)) + (oid[t] != oref[t]);
    CHECK(bad == 0, "cc=%d: %u commit / o_id mismatches", cc, bad);
    for (uint32_t t = 0; t < 5; t++) {
        const uint64_t n = or_tpcc_rows(db, t);
        std::vector<uint64_t> k(n), c0(n), c1(n), c2(n), got(n);
        or_tpcc_table(db, t, k.data(), c0.data(), c1.data(), c2.data());
        const std::vector<uint64_t> *ref[3] = {&c0, &c1, &c2};
        for (uint32_t col = 0; col < 3; col++) {
            CHECK(dv_read_table_col(run.ctx(), t, col, 0, n, got.data()) == DV_OK, "read col");
            CHECK(got == *ref[col], "cc=%d table %u col %u mismatch", cc, t, col);
        }
    }
    or_tpcc_free(db);
    std::printf("tpcc cc=%d: %llu/%u committed, parity ok\n", cc, (unsigned long long)st.committed, n_txn);
}

int main() {
    int ndev = 0;
    if (dv_device_count(&ndev) != DV_OK || ndev < 1) {
        std::printf("no GPU\n");
        return 2;
    }
    for (int cc : {DV_NO_WAIT, DV_WAIT_DIE, DV_OCC, DV_CALVIN}) ycsb_case(cc);
    for (int cc : {DV_NO_WAIT, DV_WAIT_DIE, DV_OCC, DV_CALVIN}) tpcc_case(cc);
    std::printf(failures ? "FAILURES %d\n" : "ALL PASS\n", failures);
    return failures ? 1 : 0;
}
