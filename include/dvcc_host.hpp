// dvcc_host.hpp -- C++ host mirror of Deneva's CC plugin surface over the C ABI.
//
// What a Deneva workload driver (YCSBTxnManager / TPCCTxnManager) includes to
// hand its epoch to the GPU: the reference's own vocabulary (RC, access_t,
// ycsb_request, TPCCQuery, TxnManager::get_lock / acquire_locks) at epoch
// granularity.  Header-only; links libdvcc.so.  Nothing here decides a txn:
// every decision and every row update happens in the HIP engine.
//
//   RC, access_t                  system/global.h:236, 270-271
//   ycsb_request                  benchmarks/ycsb_query.h:35-50
//   TPCCQuery, Item_no            benchmarks/tpcc_query.h:30-99
//   distKey ... stockKey          benchmarks/tpcc_helper.cpp:19-47
//   EpochRunner::get_lock         TxnManager::get_lock + index_read (system/txn.cpp:778-788, 906-932);
//                                 the lock request is queued, as a Calvin txn waits (RC WAIT)
//                                 until the lock thread grants it (row_lock.cpp:152-170)
//   EpochRunner::acquire_ycsb     YCSBTxnManager::acquire_locks (benchmarks/ycsb_txn.cpp:49-88)
//   EpochRunner::acquire_tpcc     TPCCTxnManager::acquire_locks / run_txn_state access order
//                                 (benchmarks/tpcc_txn.cpp:117-244, 500-933)
//   EpochRunner::run / run_tpcc   one epoch: decisions for the queued txns (RCOK / Abort, as
//                                 TxnManager::validate + commit / abort return them)
#ifndef DVCC_HOST_HPP
#define DVCC_HOST_HPP
#include <cstdint>
#include <string>
#include <vector>

#include "dvcc.h"

namespace dvcc_host {

enum RC { RCOK = 0, Commit, Abort, WAIT, WAIT_REM, ERROR, FINISH, NONE };  // global.h:236
enum access_t { RD = 0, WR = 1, XP = 2, SCAN = 3 };                         // global.h:270-271

struct ycsb_request {  // ycsb_query.h:35-50
    access_t acctype;
    uint64_t key;
    char value;
};

enum TPCCTxnType { TPCC_ALL = 0, TPCC_PAYMENT, TPCC_NEW_ORDER };  // config.h:209-214
struct Item_no {                                                   // tpcc_query.h:30-39
    uint64_t ol_i_id, ol_supply_w_id, ol_quantity;
};
struct TPCCQuery {  // the fields Payment / NewOrder read (tpcc_query.h:66-84)
    TPCCTxnType txn_type = TPCC_PAYMENT;
    uint64_t w_id = 0, d_id = 0, c_id = 0, d_w_id = 0, c_w_id = 0, c_d_id = 0;
    std::string c_last;
    double h_amount = 0;
    bool by_last_name = false;
    std::vector<Item_no> items;
};

// tpcc_helper.cpp:19-47
inline uint64_t distKey(uint64_t d_id, uint64_t d_w_id, uint64_t dpw) { return d_w_id * dpw + d_id; }
inline uint64_t custKey(uint64_t c_id, uint64_t c_d_id, uint64_t c_w_id, uint64_t dpw, uint64_t cpd) {
    return distKey(c_d_id, c_w_id, dpw) * cpd + c_id;
}
inline uint64_t custNPKey(const std::string &c_last, uint64_t c_d_id, uint64_t c_w_id, uint64_t dpw) {
    uint64_t key = 0;
    for (char ch : c_last) key = (key << 1) + (uint64_t)(ch - 'A');
    return (key << 10) + c_w_id * dpw + c_d_id;
}
inline uint64_t stockKey(uint64_t s_i_id, uint64_t s_w_id, uint64_t max_items) { return s_w_id * max_items + s_i_id; }

class EpochRunner {
public:
    EpochRunner() = default;
    EpochRunner(const EpochRunner &) = delete;
    EpochRunner &operator=(const EpochRunner &) = delete;
    ~EpochRunner() { close(); }

    // one context per GPU (row_t::init_manager / Row_lock::init / OptCC::init)
    int open(const dv_config &cfg) {
        close();
        return dv_open(&ctx_, &cfg);
    }
    void close() {
        if (ctx_) dv_close(ctx_);
        ctx_ = nullptr;
    }
    dv_ctx *ctx() const { return ctx_; }

    int load_ycsb(uint64_t rows_per_part) { return dv_load_ycsb_partition(ctx_, rows_per_part); }
    int load_tpcc(const dv_tpcc_params &p, uint64_t seed) {
        tp_ = p;
        return dv_tpcc_load(ctx_, &p, seed);
    }

    // ---- TxnManager side: build the epoch one txn at a time
    uint32_t begin_txn() {
        if (begin_.empty()) begin_.push_back(0);
        return (uint32_t)(begin_.size() - 1);
    }
    // TxnManager::get_lock (txn.cpp:778-788) after index_read: the request is
    // queued; its grant or abort comes with the epoch's decisions
    RC get_lock(uint64_t key, access_t type, uint8_t table = 0, uint64_t op = 0) {
        const uint32_t t = begin_txn();
        acc_.push_back(dv_access{key, t, (uint8_t)(type == WR ? DV_WR : (type == SCAN ? DV_SCAN : DV_RD)),
                                 table, 0});
        args_.push_back(op);
        return WAIT;
    }
    void end_txn() {
        if (begin_.empty()) begin_.push_back(0);
        begin_.push_back((uint32_t)acc_.size());
    }
    uint32_t txn_cnt() const { return begin_.empty() ? 0 : (uint32_t)(begin_.size() - 1); }

    // YCSBTxnManager::acquire_locks (ycsb_txn.cpp:49-88): every request of the query
    uint32_t acquire_ycsb(const std::vector<ycsb_request> &requests) {
        const uint32_t t = begin_txn();
        for (const ycsb_request &r : requests) get_lock(r.key, r.acctype);
        end_txn();
        return t;
    }

    // TPCCTxnManager::acquire_locks / run_txn_state order (tpcc_txn.cpp:117-244, 500-933)
    uint32_t acquire_tpcc(const TPCCQuery &q) {
        const uint64_t dpw = tp_.dist_per_wh, cpd = tp_.cust_per_dist, items = tp_.max_items;
        const uint32_t t = begin_txn();
        if (q.txn_type == TPCC_PAYMENT) {
            const uint64_t h = (uint64_t)q.h_amount;
            get_lock(q.w_id, tp_.wh_update ? WR : RD, DV_TPCC_WAREHOUSE,
                     op(tp_.wh_update ? DV_TOP_PAY_WH : DV_TOP_NONE, h));
            get_lock(distKey(q.d_id, q.d_w_id, dpw), WR, DV_TPCC_DISTRICT, op(DV_TOP_PAY_DIST, h));
            if (q.by_last_name)
                get_lock(custNPKey(q.c_last, q.c_d_id, q.c_w_id, dpw), WR, DV_TPCC_CUST_LAST,
                         op(DV_TOP_PAY_CUST, h));
            else
                get_lock(custKey(q.c_id, q.c_d_id, q.c_w_id, dpw, cpd), WR, DV_TPCC_CUSTOMER,
                         op(DV_TOP_PAY_CUST, h));
        } else {
            get_lock(q.w_id, RD, DV_TPCC_WAREHOUSE);
            get_lock(custKey(q.c_id, q.d_id, q.w_id, dpw, cpd), RD, DV_TPCC_CUSTOMER);
            get_lock(distKey(q.d_id, q.w_id, dpw), WR, DV_TPCC_DISTRICT, op(DV_TOP_NO_DIST, 0));
            for (const Item_no &it : q.items) {
                get_lock(it.ol_i_id, RD, DV_TPCC_ITEM);
                get_lock(stockKey(it.ol_i_id, it.ol_supply_w_id, items), WR, DV_TPCC_STOCK,
                         op(DV_TOP_NO_STOCK, it.ol_quantity));
            }
        }
        end_txn();
        return t;
    }

    // ---- one epoch: rc[t] = RCOK (committed) or Abort
    int run(std::vector<RC> &rc, dv_stats *st) {
        std::vector<uint8_t> commit(txn_cnt() ? txn_cnt() : 1);
        const int r = dv_epoch_run(ctx_, acc_.data(), acc_.size(), begins(), txn_cnt(), nullptr,
                                   commit.data(), nullptr, st);
        return finish(r, commit, rc);
    }
    // o_id[t]: D_NEXT_O_ID after new_order_5 for committed NewOrders, else 0
    int run_tpcc(std::vector<RC> &rc, std::vector<uint64_t> &o_id, dv_stats *st) {
        std::vector<uint8_t> commit(txn_cnt() ? txn_cnt() : 1);
        o_id.assign(txn_cnt() ? txn_cnt() : 1, 0);
        const int r = dv_tpcc_epoch_run(ctx_, acc_.data(), acc_.size(), begins(), txn_cnt(), args_.data(),
                                        commit.data(), o_id.data(), st);
        o_id.resize(txn_cnt());
        return finish(r, commit, rc);
    }

    const std::vector<dv_access> &accesses() const { return acc_; }
    const std::vector<uint64_t> &ops() const { return args_; }

private:
    static uint64_t op(uint64_t code, uint64_t v) { return code << 56 | v; }
    const uint32_t *begins() {
        if (begin_.empty()) begin_.push_back(0);
        return begin_.data();
    }
    int finish(int r, const std::vector<uint8_t> &commit, std::vector<RC> &rc) {
        rc.assign(txn_cnt(), Abort);
        if (r == DV_OK)
            for (uint32_t t = 0; t < txn_cnt(); t++) rc[t] = commit[t] ? RCOK : Abort;
        acc_.clear();
        args_.clear();
        begin_.clear();
        return r;
    }
    dv_ctx *ctx_ = nullptr;
    dv_tpcc_params tp_{};
    std::vector<dv_access> acc_;
    std::vector<uint64_t> args_;
    std::vector<uint32_t> begin_;
};

}  // namespace dvcc_host
#endif
