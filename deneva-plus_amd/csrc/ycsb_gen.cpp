// ycsb_gen.cpp -- host epoch builder: Deneva's YCSB query generator.
//
// Produces the integer keys of an epoch on the host (glibc libm `pow`, as the
// reference does) so the GPU never regenerates doubles (hard
// part 5).  Follows YCSBQueryGenerator (benchmarks/ycsb_query.cpp):
//   init            29-38    (zeta(2,theta); denom = zeta(table_size-1, theta))
//   zeta            181-186  (sum of pow(1.0/i, theta), i = 1..n, in order)
//   zipf            188-202
//   gen_requests_zipf 303-376 (FIRST_PART_LOCAL, strict PPT loop, duplicate-key redo)
// with myrand (system/helper.cpp:140-147) and the read/write percentages of
// system/global.cpp:86-89.  Built with -ffp-contract=off so the doubles match
// the reference's un-contracted expressions bit for bit.
//
// Seeding: the reference seeds with the clock (hazard H2); callers pass
// SEED + 97*partition + epoch.  dv_ycsb_params.mpr >= 0 enables
// the MPR gate modelled on gen_requests_hot (ycsb_query.cpp:212-217): the
// reference's zipf generator ignores g_mpr.
#include <cmath>
#include <cstdint>
#include <mutex>

#include "dvcc.h"

namespace {

class MyRand {  // system/helper.cpp:140-147
public:
    explicit MyRand(uint64_t seed) : seed_(seed) {}
    uint64_t next() {
        seed_ = (seed_ * 1103515247UL + 12345UL) % (1UL << 63);
        return (seed_ / 65537) % 2147483647UL;  // RAND_MAX
    }
private:
    uint64_t seed_;
};

double zeta(uint64_t n, double theta) {
    double sum = 0;
    for (uint64_t i = 1; i <= n; i++) sum += std::pow(1.0 / i, theta);
    return sum;
}

// zeta(the_n) is init-time work (O(n)); cache the last value per process
double zeta_denom(uint64_t n, double theta) {
    static std::mutex mu;
    static uint64_t cn = 0;
    static double ct = -1, cv = 0;
    std::lock_guard<std::mutex> g(mu);
    if (n != cn || theta != ct) {
        cv = zeta(n, theta);
        cn = n;
        ct = theta;
    }
    return cv;
}

struct Zipf {
    MyRand *rnd;
    double zetan, zeta_2_theta;
    uint64_t draw(uint64_t n, double theta) {
        double alpha = 1 / (1 - theta);
        double eta = (1 - std::pow(2.0 / n, 1 - theta)) / (1 - zeta_2_theta / zetan);
        double u = (double)(rnd->next() % 10000000) / 10000000;
        double uz = u * zetan;
        if (uz < 1) return 1;
        if (uz < 1 + std::pow(0.5, theta)) return 2;
        return 1 + (uint64_t)(n * std::pow(eta * u - eta + 1, alpha));
    }
};

struct SmallSet {  // the reference uses std::set; R <= 64 here
    uint64_t v[64];
    uint32_t n = 0;
    bool has(uint64_t x) const {
        for (uint32_t i = 0; i < n; i++)
            if (v[i] == x) return true;
        return false;
    }
    void add(uint64_t x) {
        if (!has(x)) v[n++] = x;
    }
};

}  // namespace

extern "C" int dv_ycsb_gen(const dv_ycsb_params *p, uint64_t seed, uint32_t home_part,
                           uint32_t n_txn, uint64_t *keys, uint8_t *types, uint32_t *txn_begin) {
    if (!p || !keys || !types || !txn_begin || p->part_cnt == 0) return DV_ERR_ARG;
    const uint32_t R = p->req_per_query;
    const uint64_t table_size = p->synth_table_size / p->part_cnt;
    if (R == 0 || R > 64 || table_size < 3 || home_part >= p->part_cnt) return DV_ERR_ARG;
    MyRand rnd(seed);
    Zipf z{&rnd, zeta_denom(table_size - 1, p->zipf_theta), zeta(2, p->zipf_theta)};
    const double txn_read_perc = 1.0 - p->txn_write_perc;
    const double tup_read_perc = 1.0 - p->tup_write_perc;
    const bool gate = p->mpr >= 0;
    for (uint32_t t = 0; t < n_txn; t++) {
        SmallSet all_keys, parts;
        uint32_t part_limit = p->part_per_txn;
        if (gate) {
            double r_mpt = (double)(rnd.next() % 10000) / 10000;
            part_limit = r_mpt < p->mpr ? p->part_per_txn : 1;
        }
        double r_twr = (double)(rnd.next() % 10000) / 10000;
        uint32_t rid = 0;
        txn_begin[t] = t * R;
        for (uint32_t i = 0; i < R; i++) {
            double r = (double)(rnd.next() % 10000) / 10000;
            uint64_t partition_id;
            if (rid == 0 || (gate && part_limit == 1)) {
                partition_id = home_part;
            } else {
                partition_id = rnd.next() % p->part_cnt;
                if (p->strict_ppt && part_limit <= p->part_cnt) {
                    while ((parts.n < part_limit && parts.has(partition_id)) ||
                           (parts.n == part_limit && !parts.has(partition_id)))
                        partition_id = rnd.next() % p->part_cnt;
                } else if (gate) {
                    while (parts.n == part_limit && !parts.has(partition_id))
                        partition_id = rnd.next() % p->part_cnt;
                }
            }
            const uint8_t acctype = (r_twr < txn_read_perc || r < tup_read_perc) ? DV_RD : DV_WR;
            const uint64_t row_id = z.draw(table_size - 1, p->zipf_theta);
            const uint64_t primary_key = row_id * p->part_cnt + partition_id;
            (void)(rnd.next() % (1 << 8));  // req->value
            if (all_keys.has(primary_key)) {  // a row is never accessed twice in a txn
                i--;
                continue;
            }
            all_keys.add(primary_key);
            parts.add(partition_id);
            keys[(uint64_t)t * R + rid] = primary_key;
            types[(uint64_t)t * R + rid] = acctype;
            rid++;
        }
    }
    txn_begin[n_txn] = n_txn * R;
    return DV_OK;
}
