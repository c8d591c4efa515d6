// TPC-H tables on the host: binary directory load/store, dbgen '|' text load,
// and the synthetic generator (host side of tpch_gen.hpp).
//
// Binary layout = the reference's csv_convert output read by
// App/TpcH/TpcHCommons.cpp:200-214 (size file + one raw array per column),
// per-query column selection as load_*_from_binary (:234-294, 422-451, 505-537,
// 593-623, 708-725).  Text parsing follows load_*_from_csv (:296-345, 378-420,
// 461-503, 547-591, 676-706) with its string encodings (:141-183, 347-353, 625-665).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cerrno>
#include <cstring>
#include <string>
#include <sys/stat.h>
#include <thread>
#include <vector>

#include "sgxamd/tpch.h"
#include "tpch_gen.hpp"

namespace {

using namespace sgxamd::tpch;

template <typename T>
T *alloc_col(uint64_t n) {
    void *p = nullptr;
    if (posix_memalign(&p, 64, std::max<uint64_t>(n, 1) * sizeof(T))) return nullptr;
    return static_cast<T *>(p);
}

template <typename T>
void free_col(T *&p) {
    std::free(p);
    p = nullptr;
}

std::string table_dir(const char *root, int scale, const char *tbl) {
    char buf[32];
    std::snprintf(buf, sizeof(buf), "scale%03d", scale);
    return std::string(root) + "/" + buf + "/" + tbl;
}

bool read_size(const std::string &dir, uint64_t *n) {
    FILE *f = std::fopen((dir + "/size").c_str(), "r");
    if (!f) return false;
    unsigned long long v = 0;
    const bool ok = std::fscanf(f, "%llu", &v) == 1;
    std::fclose(f);
    *n = v;
    return ok;
}

template <typename T>
bool read_col(const std::string &dir, const char *name, uint64_t n, T **out) {
    *out = alloc_col<T>(n);
    if (!*out) return false;
    FILE *f = std::fopen((dir + "/" + name).c_str(), "rb");
    if (!f) return false;
    const size_t got = std::fread(*out, sizeof(T), n, f);
    std::fclose(f);
    return got == n;
}

template <typename T>
bool write_col(const std::string &dir, const char *name, const T *p, uint64_t n) {
    if (!p) return true;
    FILE *f = std::fopen((dir + "/" + name).c_str(), "wb");
    if (!f) return false;
    const size_t put = std::fwrite(p, sizeof(T), n, f);
    std::fclose(f);
    return put == n;
}

bool make_dir(const std::string &d) { return mkdir(d.c_str(), 0755) == 0 || errno == EEXIST; }

bool write_size(const std::string &dir, uint64_t n) {
    FILE *f = std::fopen((dir + "/size").c_str(), "w");
    if (!f) return false;
    std::fprintf(f, "%llu", (unsigned long long)n);
    std::fclose(f);
    return true;
}

// ---- dbgen text
struct TextTable {
    std::string data;
    std::vector<size_t> line_start;  // one entry per '\n'-terminated line
};

bool read_text(const std::string &path, TextTable *t) {
    FILE *f = std::fopen(path.c_str(), "rb");
    if (!f) return false;
    std::fseek(f, 0, SEEK_END);
    const long sz = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    t->data.resize(sz > 0 ? (size_t)sz : 0);
    const bool ok = std::fread(&t->data[0], 1, t->data.size(), f) == t->data.size();
    std::fclose(f);
    if (!ok) return false;
    size_t s = 0;
    for (size_t i = 0; i < t->data.size(); ++i)
        if (t->data[i] == '\n') {  // the reference counts '\n' (getNumberOfLines)
            t->line_start.push_back(s);
            s = i + 1;
        }
    return true;
}

// field k of the line starting at s (fields end at '|' or end of line)
std::string field(const TextTable &t, size_t s, int k) {
    size_t p = s;
    for (int i = 0; i < k; ++i) {
        while (p < t.data.size() && t.data[p] != '|' && t.data[p] != '\n') ++p;
        if (p < t.data.size() && t.data[p] == '|') ++p;
    }
    size_t e = p;
    while (e < t.data.size() && t.data[e] != '|' && t.data[e] != '\n') ++e;
    return t.data.substr(p, e - p);
}

// days since 1970-01-01 of a proleptic Gregorian date (civil calendar)
int64_t days_from_civil(int64_t y, unsigned m, unsigned d) {
    y -= m <= 2;
    const int64_t era = (y >= 0 ? y : y - 399) / 400;
    const unsigned yoe = (unsigned)(y - era * 400);
    const unsigned doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
    const unsigned doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
    return era * 146097 + (int64_t)doe - 719468;
}

// "YYYY-MM-DD" -> seconds at UTC midnight (parseDateToLong_2: mktime(tm) - timezone)
uint64_t parse_date(const std::string &v) {
    int y = 0, m = 0, d = 0;
    if (std::sscanf(v.c_str(), "%d-%d-%d", &y, &m, &d) != 3) return 0;
    return (uint64_t)(days_from_civil(y, (unsigned)m, (unsigned)d) * (int64_t)kDay);
}

uint8_t enc_shipmode(const std::string &v) {
    return v == "MAIL" ? 1 : v == "SHIP" ? 2 : v == "AIR" ? 3 : v == "AIR REG" ? 4 : 0;
}
uint8_t enc_brand(const std::string &v) {
    return v == "Brand#12" ? 1 : v == "Brand#23" ? 2 : v == "Brand#34" ? 3 : 0;
}
uint8_t enc_container(const std::string &v) {
    static const char *names[12] = {"SM CASE", "SM BOX", "SM PACK", "SM PKG", "MED BAG", "MED BOX",
                                    "MED PKG", "MED PACK", "LG CASE", "LG BOX", "LG PACK", "LG PKG"};
    for (int i = 0; i < 12; ++i)
        if (v == names[i]) return (uint8_t)(i + 1);
    return 0;
}

template <typename F>
void parallel_rows(uint64_t n, F f) {
    const unsigned T = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (n < (1u << 16) || T == 1) {
        f(0, n);
        return;
    }
    std::vector<std::thread> th;
    const uint64_t per = (n + T - 1) / T;
    for (unsigned t = 0; t < T; ++t) {
        const uint64_t a = std::min<uint64_t>(n, t * per), b = std::min<uint64_t>(n, a + per);
        th.emplace_back([=] { f(a, b); });
    }
    for (auto &x : th) x.join();
}

}  // namespace

extern "C" {

void mi355_tpch_free_lineitem(LineItemTable *t) {
    if (!t) return;
    t->numTuples = 0;
    free_col(t->l_orderkey);
    free_col(t->l_shipdate);
    free_col(t->l_commitdate);
    free_col(t->l_receiptdate);
    free_col(t->l_shipmode);
    free_col(t->l_partkey);
    free_col(t->l_quantity);
    free_col(t->l_shipinstruct);
    free_col(t->l_returnflag);
}
void mi355_tpch_free_orders(OrdersTable *t) {
    if (!t) return;
    t->numTuples = 0;
    free_col(t->o_orderkey);
    free_col(t->o_orderdate);
    free_col(t->o_custkey);
}
void mi355_tpch_free_customer(CustomerTable *t) {
    if (!t) return;
    t->numTuples = 0;
    free_col(t->c_custkey);
    free_col(t->c_mktsegment);
    free_col(t->c_nationkey);
}
void mi355_tpch_free_part(PartTable *t) {
    if (!t) return;
    t->numTuples = 0;
    free_col(t->p_partkey);
    free_col(t->p_brand);
    free_col(t->p_size);
    free_col(t->p_container);
}
void mi355_tpch_free_nation(NationTable *t) {
    if (!t) return;
    t->numTuples = 0;
    free_col(t->n_nationkey);
}

int mi355_tpch_load_lineitem(LineItemTable *t, const char *root, int query, int scale, int csv) {
    if (!t || !root) return -1;
    std::memset(t, 0, sizeof(*t));
    if (csv) {
        TextTable tx;
        if (!read_text(table_dir(root, scale, "lineitem.tbl"), &tx)) return -1;
        const uint64_t n = tx.line_start.size();
        t->numTuples = n;
        t->l_orderkey = alloc_col<row_t>(n);
        t->l_shipdate = alloc_col<uint64_t>(n);
        t->l_returnflag = alloc_col<char>(n);
        t->l_commitdate = alloc_col<uint64_t>(n);
        t->l_receiptdate = alloc_col<uint64_t>(n);
        t->l_shipmode = alloc_col<uint8_t>(n);
        t->l_partkey = alloc_col<type_key>(n);
        t->l_quantity = alloc_col<float>(n);
        t->l_shipinstruct = alloc_col<uint8_t>(n);
        if (!t->l_orderkey || !t->l_shipdate || !t->l_returnflag || !t->l_commitdate || !t->l_receiptdate ||
            !t->l_shipmode || !t->l_partkey || !t->l_quantity || !t->l_shipinstruct) {
            mi355_tpch_free_lineitem(t);
            return -1;
        }
        parallel_rows(n, [&](uint64_t a, uint64_t b) {
            for (uint64_t i = a; i < b; ++i) {
                const size_t s = tx.line_start[i];
                t->l_orderkey[i].key = (type_key)std::strtoul(field(tx, s, 0).c_str(), nullptr, 10);
                t->l_orderkey[i].payload = (type_value)i;
                t->l_partkey[i] = (type_key)std::strtoul(field(tx, s, 1).c_str(), nullptr, 10);
                t->l_quantity[i] = std::strtof(field(tx, s, 4).c_str(), nullptr);
                const std::string rf = field(tx, s, 8);
                t->l_returnflag[i] = rf.empty() ? 0 : rf[0];
                t->l_shipdate[i] = parse_date(field(tx, s, 10));
                t->l_commitdate[i] = parse_date(field(tx, s, 11));
                t->l_receiptdate[i] = parse_date(field(tx, s, 12));
                t->l_shipinstruct[i] = field(tx, s, 13) == "DELIVER IN PERSON" ? 1 : 0;
                t->l_shipmode[i] = enc_shipmode(field(tx, s, 14));
            }
        });
        return 0;
    }
    if (query != 0 && query != 3 && query != 10 && query != 12 && query != 19) return 0;
    const std::string dir = table_dir(root, scale, "lineitem.tbl.dir");
    uint64_t n;
    if (!read_size(dir, &n)) return -1;
    t->numTuples = n;
    bool ok = read_col(dir, "l_orderkey.bin", n, &t->l_orderkey);
    const bool all = query == 0;
    if (all || query == 3 || query == 12) ok = ok && read_col(dir, "l_shipdate.bin", n, &t->l_shipdate);
    if (all || query == 10) ok = ok && read_col(dir, "l_returnflag.bin", n, &t->l_returnflag);
    if (all || query == 12) {
        ok = ok && read_col(dir, "l_commitdate.bin", n, &t->l_commitdate);
        ok = ok && read_col(dir, "l_receiptdate.bin", n, &t->l_receiptdate);
    }
    if (all || query == 12 || query == 19) ok = ok && read_col(dir, "l_shipmode.bin", n, &t->l_shipmode);
    if (all || query == 19) {
        ok = ok && read_col(dir, "l_partkey.bin", n, &t->l_partkey);
        ok = ok && read_col(dir, "l_quantity.bin", n, &t->l_quantity);
        ok = ok && read_col(dir, "l_shipinstruct.bin", n, &t->l_shipinstruct);
    }
    if (!ok) mi355_tpch_free_lineitem(t);
    return ok ? 0 : -1;
}

int mi355_tpch_load_orders(OrdersTable *t, const char *root, int query, int scale, int csv) {
    if (!t || !root) return -1;
    std::memset(t, 0, sizeof(*t));
    if (csv) {
        TextTable tx;
        if (!read_text(table_dir(root, scale, "orders.tbl"), &tx)) return -1;
        const uint64_t n = tx.line_start.size();
        t->numTuples = n;
        t->o_orderkey = alloc_col<row_t>(n);
        t->o_orderdate = alloc_col<uint64_t>(n);
        t->o_custkey = alloc_col<type_key>(n);
        if (!t->o_orderkey || !t->o_orderdate || !t->o_custkey) {
            mi355_tpch_free_orders(t);
            return -1;
        }
        parallel_rows(n, [&](uint64_t a, uint64_t b) {
            for (uint64_t i = a; i < b; ++i) {
                const size_t s = tx.line_start[i];
                t->o_orderkey[i].key = (type_key)std::strtoul(field(tx, s, 0).c_str(), nullptr, 10);
                t->o_orderkey[i].payload = (type_value)i;
                t->o_custkey[i] = (type_key)std::strtoul(field(tx, s, 1).c_str(), nullptr, 10);
                t->o_orderdate[i] = parse_date(field(tx, s, 4));
            }
        });
        return 0;
    }
    if (query != 0 && query != 3 && query != 10 && query != 12) return 0;
    const std::string dir = table_dir(root, scale, "orders.tbl.dir");
    uint64_t n;
    if (!read_size(dir, &n)) return -1;
    t->numTuples = n;
    bool ok = read_col(dir, "o_orderkey.bin", n, &t->o_orderkey);
    if (query == 0 || query == 3 || query == 10) {
        ok = ok && read_col(dir, "o_orderdate.bin", n, &t->o_orderdate);
        ok = ok && read_col(dir, "o_custkey.bin", n, &t->o_custkey);
    }
    if (!ok) mi355_tpch_free_orders(t);
    return ok ? 0 : -1;
}

int mi355_tpch_load_customer(CustomerTable *t, const char *root, int query, int scale, int csv) {
    if (!t || !root) return -1;
    std::memset(t, 0, sizeof(*t));
    if (csv) {
        TextTable tx;
        if (!read_text(table_dir(root, scale, "customer.tbl"), &tx)) return -1;
        const uint64_t n = tx.line_start.size();
        t->numTuples = n;
        t->c_custkey = alloc_col<row_t>(n);
        t->c_mktsegment = alloc_col<uint8_t>(n);
        t->c_nationkey = alloc_col<type_key>(n);
        if (!t->c_custkey || !t->c_mktsegment || !t->c_nationkey) {
            mi355_tpch_free_customer(t);
            return -1;
        }
        for (uint64_t i = 0; i < n; ++i) {
            const size_t s = tx.line_start[i];
            t->c_custkey[i].key = (type_key)std::strtoul(field(tx, s, 0).c_str(), nullptr, 10);
            t->c_custkey[i].payload = (type_value)i;
            t->c_mktsegment[i] = field(tx, s, 6) == "BUILDING" ? 1 : 0;
            t->c_nationkey[i] = (type_key)std::strtoul(field(tx, s, 3).c_str(), nullptr, 10);
        }
        return 0;
    }
    if (query != 0 && query != 3 && query != 10) return 0;
    const std::string dir = table_dir(root, scale, "customer.tbl.dir");
    uint64_t n;
    if (!read_size(dir, &n)) return -1;
    t->numTuples = n;
    bool ok = read_col(dir, "c_custkey.bin", n, &t->c_custkey);
    if (query == 0 || query == 3) ok = ok && read_col(dir, "c_mktsegment.bin", n, &t->c_mktsegment);
    if (query == 0 || query == 10) ok = ok && read_col(dir, "c_nationkey.bin", n, &t->c_nationkey);
    if (!ok) mi355_tpch_free_customer(t);
    return ok ? 0 : -1;
}

int mi355_tpch_load_part(PartTable *t, const char *root, int query, int scale, int csv) {
    if (!t || !root) return -1;
    std::memset(t, 0, sizeof(*t));
    if (csv) {
        TextTable tx;
        if (!read_text(table_dir(root, scale, "part.tbl"), &tx)) return -1;
        const uint64_t n = tx.line_start.size();
        t->numTuples = n;
        t->p_partkey = alloc_col<row_t>(n);
        t->p_brand = alloc_col<uint8_t>(n);
        t->p_size = alloc_col<uint32_t>(n);
        t->p_container = alloc_col<uint8_t>(n);
        if (!t->p_partkey || !t->p_brand || !t->p_size || !t->p_container) {
            mi355_tpch_free_part(t);
            return -1;
        }
        for (uint64_t i = 0; i < n; ++i) {
            const size_t s = tx.line_start[i];
            t->p_partkey[i].key = (type_key)std::strtoul(field(tx, s, 0).c_str(), nullptr, 10);
            t->p_partkey[i].payload = (type_value)i;
            t->p_brand[i] = enc_brand(field(tx, s, 3));
            t->p_size[i] = (uint32_t)std::strtoul(field(tx, s, 5).c_str(), nullptr, 10);
            t->p_container[i] = enc_container(field(tx, s, 6));
        }
        return 0;
    }
    if (query != 0 && query != 19) return 0;
    const std::string dir = table_dir(root, scale, "part.tbl.dir");
    uint64_t n;
    if (!read_size(dir, &n)) return -1;
    t->numTuples = n;
    bool ok = read_col(dir, "p_partkey.bin", n, &t->p_partkey);
    ok = ok && read_col(dir, "p_brand.bin", n, &t->p_brand);
    ok = ok && read_col(dir, "p_container.bin", n, &t->p_container);
    ok = ok && read_col(dir, "p_size.bin", n, &t->p_size);
    if (!ok) mi355_tpch_free_part(t);
    return ok ? 0 : -1;
}

int mi355_tpch_load_nation(NationTable *t, const char *root, int query, int scale, int csv) {
    if (!t || !root) return -1;
    std::memset(t, 0, sizeof(*t));
    if (csv) {
        TextTable tx;
        if (!read_text(table_dir(root, scale, "nation.tbl"), &tx)) return -1;
        const uint64_t n = tx.line_start.size();
        t->numTuples = n;
        t->n_nationkey = alloc_col<row_t>(n);
        if (!t->n_nationkey) return -1;
        for (uint64_t i = 0; i < n; ++i) {
            t->n_nationkey[i].key = (type_key)std::strtoul(field(tx, tx.line_start[i], 0).c_str(), nullptr, 10);
            t->n_nationkey[i].payload = (type_value)i;
        }
        return 0;
    }
    if (query != 0 && query != 10) return 0;
    const std::string dir = table_dir(root, scale, "nation.tbl.dir");
    uint64_t n;
    if (!read_size(dir, &n)) return -1;
    t->numTuples = n;
    const bool ok = read_col(dir, "n_nationkey.bin", n, &t->n_nationkey);
    if (!ok) mi355_tpch_free_nation(t);
    return ok ? 0 : -1;
}

int mi355_tpch_store(const char *root, int scale, const LineItemTable *l, const OrdersTable *o,
                     const CustomerTable *c, const PartTable *p, const NationTable *n) {
    if (!root) return -1;
    char buf[32];
    std::snprintf(buf, sizeof(buf), "/scale%03d", scale);
    const std::string base = std::string(root) + buf;
    if (!make_dir(root) || !make_dir(base)) return -1;
    bool ok = true;
    if (l && l->numTuples) {
        const std::string d = base + "/lineitem.tbl.dir";
        const uint64_t k = l->numTuples;
        ok = ok && make_dir(d) && write_size(d, k) && write_col(d, "l_orderkey.bin", l->l_orderkey, k) &&
             write_col(d, "l_shipdate.bin", l->l_shipdate, k) && write_col(d, "l_commitdate.bin", l->l_commitdate, k) &&
             write_col(d, "l_receiptdate.bin", l->l_receiptdate, k) &&
             write_col(d, "l_shipmode.bin", l->l_shipmode, k) && write_col(d, "l_partkey.bin", l->l_partkey, k) &&
             write_col(d, "l_quantity.bin", l->l_quantity, k) &&
             write_col(d, "l_shipinstruct.bin", l->l_shipinstruct, k) &&
             write_col(d, "l_returnflag.bin", l->l_returnflag, k);
    }
    if (o && o->numTuples) {
        const std::string d = base + "/orders.tbl.dir";
        const uint64_t k = o->numTuples;
        ok = ok && make_dir(d) && write_size(d, k) && write_col(d, "o_orderkey.bin", o->o_orderkey, k) &&
             write_col(d, "o_custkey.bin", o->o_custkey, k) && write_col(d, "o_orderdate.bin", o->o_orderdate, k);
    }
    if (c && c->numTuples) {
        const std::string d = base + "/customer.tbl.dir";
        const uint64_t k = c->numTuples;
        ok = ok && make_dir(d) && write_size(d, k) && write_col(d, "c_custkey.bin", c->c_custkey, k) &&
             write_col(d, "c_mktsegment.bin", c->c_mktsegment, k) &&
             write_col(d, "c_nationkey.bin", c->c_nationkey, k);
    }
    if (p && p->numTuples) {
        const std::string d = base + "/part.tbl.dir";
        const uint64_t k = p->numTuples;
        ok = ok && make_dir(d) && write_size(d, k) && write_col(d, "p_partkey.bin", p->p_partkey, k) &&
             write_col(d, "p_brand.bin", p->p_brand, k) && write_col(d, "p_container.bin", p->p_container, k) &&
             write_col(d, "p_size.bin", p->p_size, k);
    }
    if (n && n->numTuples) {
        const std::string d = base + "/nation.tbl.dir";
        ok = ok && make_dir(d) && write_size(d, n->numTuples) &&
             write_col(d, "n_nationkey.bin", n->n_nationkey, n->numTuples);
    }
    return ok ? 0 : -1;
}

int mi355_tpch_sizes(uint32_t sm, uint64_t seed, uint64_t *nl, uint64_t *no, uint64_t *nc, uint64_t *np,
                     uint64_t *nn) {
    const uint64_t n_o = n_orders(sm);
    if (nl) {
        std::vector<uint64_t> part(16, 0);
        const uint64_t per = (n_o + 15) / 16;
        std::vector<std::thread> th;
        for (int t = 0; t < 16; ++t)
            th.emplace_back([&, t] {
                uint64_t s = 0;
                for (uint64_t i = t * per; i < std::min<uint64_t>(n_o, (t + 1) * per); ++i) s += o_lines(seed, i);
                part[t] = s;
            });
        for (auto &x : th) x.join();
        uint64_t s = 0;
        for (uint64_t v : part) s += v;
        *nl = s;
    }
    if (no) *no = n_o;
    if (nc) *nc = n_customer(sm);
    if (np) *np = n_part(sm);
    if (nn) *nn = kNations;
    return 0;
}

int mi355_tpch_generate(uint32_t sm, uint64_t seed, LineItemTable *l, OrdersTable *o, CustomerTable *c,
                        PartTable *p, NationTable *n) {
    if (sm == 0) return -1;
    const uint64_t n_c = n_customer(sm), n_o = n_orders(sm), n_p = n_part(sm);
    if (c) {
        std::memset(c, 0, sizeof(*c));
        c->numTuples = n_c;
        c->c_custkey = alloc_col<row_t>(n_c);
        c->c_mktsegment = alloc_col<uint8_t>(n_c);
        c->c_nationkey = alloc_col<type_key>(n_c);
        if (!c->c_custkey || !c->c_mktsegment || !c->c_nationkey) return -1;
        parallel_rows(n_c, [&](uint64_t a, uint64_t b) {
            for (uint64_t i = a; i < b; ++i) {
                c->c_custkey[i] = row_t{(type_key)(i + 1), (type_value)i};
                c->c_mktsegment[i] = c_mktsegment(seed, i);
                c->c_nationkey[i] = c_nationkey(seed, i);
            }
        });
    }
    if (p) {
        std::memset(p, 0, sizeof(*p));
        p->numTuples = n_p;
        p->p_partkey = alloc_col<row_t>(n_p);
        p->p_brand = alloc_col<uint8_t>(n_p);
        p->p_size = alloc_col<uint32_t>(n_p);
        p->p_container = alloc_col<uint8_t>(n_p);
        if (!p->p_partkey || !p->p_brand || !p->p_size || !p->p_container) return -1;
        parallel_rows(n_p, [&](uint64_t a, uint64_t b) {
            for (uint64_t i = a; i < b; ++i) {
                p->p_partkey[i] = row_t{(type_key)(i + 1), (type_value)i};
                p->p_brand[i] = p_brand(seed, i);
                p->p_size[i] = p_size(seed, i);
                p->p_container[i] = p_container(seed, i);
            }
        });
    }
    if (n) {
        std::memset(n, 0, sizeof(*n));
        n->numTuples = kNations;
        n->n_nationkey = alloc_col<row_t>(kNations);
        if (!n->n_nationkey) return -1;
        for (uint64_t i = 0; i < kNations; ++i) n->n_nationkey[i] = row_t{(type_key)i, (type_value)i};
    }
    if (o) {
        std::memset(o, 0, sizeof(*o));
        o->numTuples = n_o;
        o->o_orderkey = alloc_col<row_t>(n_o);
        o->o_orderdate = alloc_col<uint64_t>(n_o);
        o->o_custkey = alloc_col<type_key>(n_o);
        if (!o->o_orderkey || !o->o_orderdate || !o->o_custkey) return -1;
        parallel_rows(n_o, [&](uint64_t a, uint64_t b) {
            for (uint64_t i = a; i < b; ++i) {
                o->o_orderkey[i] = row_t{o_orderkey(i), (type_value)i};
                o->o_orderdate[i] = (uint64_t)o_orderday(seed, i) * kDay;
                o->o_custkey[i] = o_custkey(seed, i, n_c);
            }
        });
    }
    if (l) {
        std::memset(l, 0, sizeof(*l));
        std::vector<uint64_t> off(n_o + 1, 0);
        for (uint64_t i = 0; i < n_o; ++i) off[i + 1] = off[i] + o_lines(seed, i);
        const uint64_t n_l = off[n_o];
        l->numTuples = n_l;
        l->l_orderkey = alloc_col<row_t>(n_l);
        l->l_shipdate = alloc_col<uint64_t>(n_l);
        l->l_commitdate = alloc_col<uint64_t>(n_l);
        l->l_receiptdate = alloc_col<uint64_t>(n_l);
        l->l_shipmode = alloc_col<uint8_t>(n_l);
        l->l_partkey = alloc_col<type_key>(n_l);
        l->l_quantity = alloc_col<float>(n_l);
        l->l_shipinstruct = alloc_col<uint8_t>(n_l);
        l->l_returnflag = alloc_col<char>(n_l);
        if (!l->l_orderkey || !l->l_shipdate || !l->l_commitdate || !l->l_receiptdate || !l->l_shipmode ||
            !l->l_partkey || !l->l_quantity || !l->l_shipinstruct || !l->l_returnflag)
            return -1;
        parallel_rows(n_o, [&](uint64_t a, uint64_t b) {
            for (uint64_t i = a; i < b; ++i) {
                const uint32_t day = o_orderday(seed, i);
                const uint32_t key = o_orderkey(i);
                for (uint64_t r = off[i]; r < off[i + 1]; ++r) {
                    const Line L = make_line(seed, r, day, n_p);
                    l->l_orderkey[r] = row_t{key, (type_value)r};
                    l->l_shipdate[r] = L.shipdate;
                    l->l_commitdate[r] = L.commitdate;
                    l->l_receiptdate[r] = L.receiptdate;
                    l->l_shipmode[r] = L.shipmode;
                    l->l_partkey[r] = L.partkey;
                    l->l_quantity[r] = L.quantity;
                    l->l_shipinstruct[r] = L.shipinstruct;
                    l->l_returnflag[r] = L.returnflag;
                }
            }
        });
    }
    return 0;
}

}  // extern "C"
