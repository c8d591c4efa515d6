// C++-linkage TPC-H drop-ins (declared in sgxamd/tpch.hpp): the reference's
// tpch_q3/q10/q12/q19 (lib/TPCH-Queries/src/tpch.cpp:36-309) and table loaders
// (App/TpcH/TpcHCommons.cpp:193-741) over the mi355_tpch_* C-ABI.
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "sgxamd/rho.h"
#include "sgxamd/tpch.h"
#include "sgxamd/tpch.hpp"

namespace {

const auto g_log_start = std::chrono::steady_clock::now();

// Logger.cpp:53-76 format, as joins_adapter.cpp
void logger(const char *level, const char *color, const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    const double t = std::chrono::duration<double>(std::chrono::steady_clock::now() - g_log_start).count();
    std::printf("%s[%8.4f][%5s] %s\x1b[0m\n", color, t, level, buf);
}
#define LOG_INFO(...) logger("INFO", "\x1b[32m", __VA_ARGS__)
#define LOG_ERROR(...) logger("ERROR", "\x1b[31m", __VA_ARGS__)

int algo_of(const char *name) {
    if (name && std::strcmp(name, "RHO") == 0) return MI355_ALGO_RHO;
    if (name && std::strcmp(name, "RHT") == 0) return MI355_ALGO_RHT;
    LOG_ERROR("Algorithm not found: %s (this library provides RHO and RHT)", name ? name : "(null)");
    std::exit(EXIT_FAILURE);
}

void check(int rc, const char *what) {
    if (rc != MI355_OK) {
        LOG_ERROR("%s failed (%d): %s", what, rc, mi355_last_error());
        std::exit(EXIT_FAILURE);
    }
}

// time_print.cpp:18-35 (times in microseconds)
void print_query_results(const mi355_tpch_stats &st) {
    auto us = [](double ms) { return (unsigned)(ms * 1000.0); };
    const double total = st.ms_total * 1000.0;
    const double sel = (st.ms_selection[0] + st.ms_selection[1] + st.ms_selection[2]) * 1000.0;
    const double join = (st.ms_join[0] + st.ms_join[1] + st.ms_join[2]) * 1000.0;
    LOG_INFO("QueryTimeTotal (us)         : %u", us(st.ms_total));
    LOG_INFO("QueryTimeSelection (us)     : %u (%.2lf%%)", (unsigned)sel, 100 * sel / total);
    LOG_INFO("QueryTimeSelection 1 (us)   : %u", us(st.ms_selection[0]));
    LOG_INFO("QueryTimeSelection 2 (us)   : %u", us(st.ms_selection[1]));
    LOG_INFO("QueryTimeSelection 3 (us)   : %u", us(st.ms_selection[2]));
    LOG_INFO("QueryTimeJoin (us)          : %u (%.2lf%%)", (unsigned)join, 100 * join / total);
    LOG_INFO("QueryTimeCopy (us)          : %u (%.2lf%%)", us(st.ms_copy), 100 * st.ms_copy * 1000.0 / total);
    LOG_INFO("QueryTimeJoin 1 (us)         : %u", us(st.ms_join[0]));
    LOG_INFO("QueryTimeJoin 2 (us)         : %u", us(st.ms_join[1]));
    LOG_INFO("QueryTimeJoin 3 (us)         : %u", us(st.ms_join[2]));
    LOG_INFO("QueryThroughput (M rec/s)   : %.4lf", (double)st.input_tuples / total);
    LOG_INFO("Host->device staging (us)   : %u", us(st.ms_h2d));
}

void fill(result_t *r, const mi355_tpch_stats &st, uint64_t totalresults, const joinconfig_t *cfg) {
    std::memset(r, 0, sizeof(*r));
    r->totalresults = (int64_t)totalresults;
    r->nthreads = cfg ? cfg->NTHREADS : 1;
    r->throughput = st.ms_total > 0 ? (double)st.input_tuples / (st.ms_total * 1000.0) : 0.0;  // M rec/s
}

std::string data_root() {
    const char *e = std::getenv("SGXAMD_TPCH_DATA");
    return e ? e : "../data";
}

}  // namespace

void tpch_q3(result_t *result, const CustomerTable *c, const OrdersTable *o, const LineItemTable *l,
             const char *algorithm, joinconfig_t *config) {
    LOG_INFO("tpch_q3");
    LOG_INFO("LineItemTable size: %lu, OrdersTable size: %lu, CustomerTable size: %lu",
             (unsigned long)l->numTuples, (unsigned long)o->numTuples, (unsigned long)c->numTuples);
    mi355_tpch_stats st{};
    check(mi355_tpch_q3(c, o, l, algo_of(algorithm), &st), "tpch_q3");
    LOG_INFO("Join customers=%lu with orders=%lu", (unsigned long)st.filtered[0], (unsigned long)st.filtered[1]);
    LOG_INFO("U tuples=%lu", (unsigned long)st.join_matches[0]);
    LOG_INFO("Join U=%lu with lineitems=%lu", (unsigned long)st.join_matches[0], (unsigned long)st.filtered[2]);
    if (config) config->MATERIALIZE = false;  // tpch.cpp:100 leaves it off
    fill(result, st, st.join_matches[1], config);
    print_query_results(st);
}

void tpch_q10(result_t *result, const CustomerTable *c, const OrdersTable *o, const LineItemTable *l,
              const NationTable *n, const char *algorithm, joinconfig_t *config) {
    LOG_INFO("tpch_q10");
    LOG_INFO("CustomerTable: %lu, OrdersTable size: %lu, LineItemTable size: %lu, NationTable: %lu",
             (unsigned long)c->numTuples, (unsigned long)o->numTuples, (unsigned long)l->numTuples,
             (unsigned long)n->numTuples);
    mi355_tpch_stats st{};
    check(mi355_tpch_q10(c, o, l, n, algo_of(algorithm), &st), "tpch_q10");
    LOG_INFO("Join Customer=%lu with Orders=%lu", (unsigned long)c->numTuples, (unsigned long)st.filtered[0]);
    LOG_INFO("Join Nation=%lu with U=%lu", (unsigned long)n->numTuples, (unsigned long)st.join_matches[0]);
    LOG_INFO("Join U=%lu with LineItem=%lu", (unsigned long)st.join_matches[1], (unsigned long)st.filtered[1]);
    LOG_INFO("Join result tuples: %lu", (unsigned long)st.join_matches[2]);
    if (config) config->MATERIALIZE = false;
    fill(result, st, st.join_matches[2], config);
    print_query_results(st);
}

void tpch_q12(result_t *result, const LineItemTable *l, const OrdersTable *o, const char *algorithm,
              joinconfig_t *config) {
    LOG_INFO("tpch_q12");
    LOG_INFO("LineItemTable size: %lu, OrdersTable size: %lu", (unsigned long)l->numTuples,
             (unsigned long)o->numTuples);
    mi355_tpch_stats st{};
    check(mi355_tpch_q12(l, o, algo_of(algorithm), &st), "tpch_q12");
    LOG_INFO("Join lineitem=%lu with order=%lu tuples", (unsigned long)st.filtered[0], (unsigned long)o->numTuples);
    if (config) config->MATERIALIZE = false;
    fill(result, st, st.join_matches[0], config);
    print_query_results(st);
}

void tpch_q19(result_t *result, const LineItemTable *l, const PartTable *p, const char *algorithm,
              joinconfig_t *config) {
    LOG_INFO("tpch_q19");
    LOG_INFO("LineItemTable size: %lu, PartTable size: %lu", (unsigned long)l->numTuples,
             (unsigned long)p->numTuples);
    mi355_tpch_stats st{};
    chunked_table_t *join = nullptr;
    check(mi355_tpch_q19(l, p, algo_of(algorithm), &st, 1, &join), "tpch_q19");
    LOG_INFO("Join Part=%lu with LineItem=%lu", (unsigned long)st.filtered[0], (unsigned long)st.filtered[1]);
    LOG_INFO("Number of Tuples: %lu", (unsigned long)join->num_tuples);
    LOG_INFO("Number of Chunks: %lu", (unsigned long)join->num_chunks);
    LOG_INFO("Total matches = %lu", (unsigned long)st.result);
    if (config) config->MATERIALIZE = true;  // tpch.cpp:281
    fill(result, st, st.join_matches[0], config);
    result->materialized = 1;
    result->result = join;
    result->result_type = 1;
    print_query_results(st);
}

std::string getPath(int scale, const std::string &tbl) {
    char buf[32];
    std::snprintf(buf, sizeof(buf), "/scale%03d/", scale);
    return data_root() + buf + tbl;
}

int load_lineitems_from_binary(LineItemTable *t, uint8_t query, uint8_t scale) {
    return mi355_tpch_load_lineitem(t, data_root().c_str(), query, scale, 0);
}
int load_lineitem_from_csv(LineItemTable *t, uint8_t scale) {
    return mi355_tpch_load_lineitem(t, data_root().c_str(), 0, scale, 1);
}
void free_lineitem(LineItemTable *t) { mi355_tpch_free_lineitem(t); }
int load_orders_from_binary(OrdersTable *t, uint8_t query, uint8_t scale) {
    return mi355_tpch_load_orders(t, data_root().c_str(), query, scale, 0);
}
int load_orders_from_csv(OrdersTable *t, uint8_t scale) {
    return mi355_tpch_load_orders(t, data_root().c_str(), 0, scale, 1);
}
void free_orders(OrdersTable *t) { mi355_tpch_free_orders(t); }
int load_customers_from_binary(CustomerTable *t, uint8_t query, uint8_t scale) {
    return mi355_tpch_load_customer(t, data_root().c_str(), query, scale, 0);
}
int load_customer_from_csv(CustomerTable *t, uint8_t scale) {
    return mi355_tpch_load_customer(t, data_root().c_str(), 0, scale, 1);
}
void free_customer(CustomerTable *t) { mi355_tpch_free_customer(t); }
int load_parts_from_binary(PartTable *t, uint8_t query, uint8_t scale) {
    return mi355_tpch_load_part(t, data_root().c_str(), query, scale, 0);
}
int load_part_from_csv(PartTable *t, uint8_t scale) {
    return mi355_tpch_load_part(t, data_root().c_str(), 0, scale, 1);
}
void free_part(PartTable *t) { mi355_tpch_free_part(t); }
int load_nations_from_binary(NationTable *t, uint8_t query, uint8_t scale) {
    return mi355_tpch_load_nation(t, data_root().c_str(), query, scale, 0);
}
int load_nation_from_csv(NationTable *t, uint8_t scale) {
    return mi355_tpch_load_nation(t, data_root().c_str(), 0, scale, 1);
}
void free_nation(NationTable *t) { mi355_tpch_free_nation(t); }
