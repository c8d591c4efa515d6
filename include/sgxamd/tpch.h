/*
 * sgxamd/tpch.h — C-ABI of the TPC-H callers of the join/scan hot path
 * (SURVEY.md §8(f) rank 3).
 *
 * The reference runs four TPC-H queries as the end-to-end consumers of RHO:
 *     tpch_q3 / tpch_q10 / tpch_q12 / tpch_q19
 * (Join-Benchmarks/lib/TPCH-Queries/include/tpch.hpp:7-21, implemented in
 *  lib/TPCH-Queries/src/tpch.cpp:36-309): column filters (filters.hpp:113-138 and
 *  the Q*Predicates.hpp predicates), one to three RHO joins with MATERIALIZE
 *  toggled per join, result transforms between them (result_transformers.hpp:46-127)
 *  and, for Q19, a predicate over the join result (Q19Predicates.hpp:57-78).
 * The tables are the column sets of TpcHTypes.hpp:39-87 and are read from the
 * binary table directories of App/TpcH/TpcHCommons.cpp:200-741.
 *
 * Here every step runs on the GPU: filters are order-preserving stream
 * compactions, the joins are the RHO/RHT device pipeline of rho.h with
 * device-resident materialisation, the transforms are gathers.  Column
 * pointers may be host or device memory (host columns are staged to HBM and the
 * copy time is reported apart from the query time).
 *
 * The C++ drop-ins with the reference's exact signatures (tpch_q3(result_t*, ...)
 * and the load_*_from_binary / load_*_from_csv / free_* loaders) are declared
 * in sgxamd/tpch.hpp.
 */
#ifndef SGXAMD_TPCH_H
#define SGXAMD_TPCH_H

#include "sgxamd/data_types.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Column codes (TpcHTypes.hpp:7-43). */
#define TPCH_L_SHIPMODE_MAIL 1
#define TPCH_L_SHIPMODE_SHIP 2
#define TPCH_L_SHIPMODE_AIR 3
#define TPCH_L_SHIPMODE_AIR_REG 4
#define TPCH_L_SHIPINSTRUCT_DELIVER_IN_PERSON 1
#define TPCH_MKT_BUILDING 1
#define TPCH_P_BRAND_12 1
#define TPCH_P_BRAND_23 2
#define TPCH_P_BRAND_34 3
#define TPCH_P_CONTAINER_SM_CASE 1
#define TPCH_P_CONTAINER_SM_BOX 2
#define TPCH_P_CONTAINER_SM_PACK 3
#define TPCH_P_CONTAINER_SM_PKG 4
#define TPCH_P_CONTAINER_MED_BAG 5
#define TPCH_P_CONTAINER_MED_BOX 6
#define TPCH_P_CONTAINER_MED_PKG 7
#define TPCH_P_CONTAINER_MED_PACK 8
#define TPCH_P_CONTAINER_LG_CASE 9
#define TPCH_P_CONTAINER_LG_BOX 10
#define TPCH_P_CONTAINER_LG_PACK 11
#define TPCH_P_CONTAINER_LG_PKG 12
#define TPCH_TIMESTAMP_1995_01_01_SECONDS 788918400ull
#define TPCH_TIMESTAMP_1995_03_15_SECONDS 795225600ull
#define TPCH_TIMESTAMP_1995_03_16_SECONDS 795312000ull
#define TPCH_TIMESTAMP_1993_10_01_SECONDS 749433600ull
#define TPCH_TIMESTAMP_1994_01_01_SECONDS 757382400ull
#define TPCH_L_RETURNFLAG_R 'R'

/* Tables: the reference's column structs, field for field (TpcHTypes.hpp:53-87). */
struct LineItemTable {
    uint64_t numTuples;
    struct row_t *l_orderkey; /* key = orderkey, payload = row id */
    uint64_t *l_shipdate;     /* seconds since the epoch, UTC midnight */
    uint64_t *l_commitdate;
    uint64_t *l_receiptdate;
    uint8_t *l_shipmode;
    type_key *l_partkey;
    float *l_quantity;
    uint8_t *l_shipinstruct;
    char *l_returnflag;
};

struct OrdersTable {
    uint64_t numTuples;
    struct row_t *o_orderkey; /* key = orderkey, payload = row id */
    uint64_t *o_orderdate;
    type_key *o_custkey;
};

struct CustomerTable {
    uint64_t numTuples;
    struct row_t *c_custkey; /* key = custkey, payload = row id */
    uint8_t *c_mktsegment;
    type_key *c_nationkey;
};

struct PartTable {
    uint64_t numTuples;
    struct row_t *p_partkey; /* key = partkey, payload = row id */
    uint8_t *p_brand;
    uint32_t *p_size;
    uint8_t *p_container;
};

struct NationTable {
    uint64_t numTuples;
    struct row_t *n_nationkey; /* key = nationkey, payload = row id */
};

/* What one query did.  Times are HIP-event milliseconds of the query's phases on
 * the device (the reference's TPCHTimers, time_print.hpp:6-15), with H2D
 * staging of host columns reported apart. */
typedef struct mi355_tpch_stats {
    uint64_t result;          /* Q3/Q10/Q12: the last join's count; Q19: the final predicate's count */
    uint64_t join_matches[3]; /* cardinality of join 1..3 (0 if the query has fewer) */
    uint64_t filtered[3];     /* rows surviving selection 1..3 */
    double ms_selection[3];
    double ms_join[3];
    double ms_copy;           /* result transforms between joins */
    double ms_total;          /* first filter .. last step, device time */
    double ms_h2d;            /* staging of host columns (not part of ms_total) */
    uint64_t input_tuples;    /* Σ numTuples of the query's tables (throughput numerator) */
    uint64_t column_bytes;    /* bytes of the columns the query reads */
} mi355_tpch_stats;

/* The four queries (tpch.cpp:36-309).  algorithm = MI355_ALGO_RHO or MI355_ALGO_RHT.
 * Return 0 or a negative MI355_ERR_* code (rho.h). */
int mi355_tpch_q3(const struct CustomerTable *c, const struct OrdersTable *o, const struct LineItemTable *l,
                  int algorithm, mi355_tpch_stats *stats);
int mi355_tpch_q10(const struct CustomerTable *c, const struct OrdersTable *o, const struct LineItemTable *l,
                   const struct NationTable *n, int algorithm, mi355_tpch_stats *stats);
int mi355_tpch_q12(const struct LineItemTable *l, const struct OrdersTable *o, int algorithm,
                   mi355_tpch_stats *stats);
/* Q19 also hands back the materialised join 1 (part ⋈ lineitem) when want_join is
 * non-zero: *join_out receives a host chunked_table_t (free with
 * mi355_free_chunked_table), as the reference's result->result (tpch.cpp:281-296). */
int mi355_tpch_q19(const struct LineItemTable *l, const struct PartTable *p, int algorithm,
                   mi355_tpch_stats *stats, int want_join, struct chunked_table_t **join_out);

/* One selection of a query on its own (parity tests, benchmarks): writes the
 * filtered rows of query q's selection `which` (1-based, in the order of
 * tpch.cpp) to out (host or device, capacity rows) in input order, exactly the
 * rows the reference's scalar filter_table (filters.hpp:118-138) produces.
 * *n_out = rows written; MI355_ERR_CAPACITY if capacity is too small. */
int mi355_tpch_filter(int query, int which, const struct CustomerTable *c, const struct OrdersTable *o,
                      const struct LineItemTable *l, const struct PartTable *p, struct row_t *out,
                      uint64_t capacity, uint64_t *n_out);

/*
 * Tables on disk and synthetic tables (host code, no GPU needed).
 *
 * Binary directories as written by the reference's csv_convert
 * (App/TpcH/CSVConvert.cpp) and read by TpcHCommons.cpp:200-741:
 *     <root>/scale%03d/<table>.tbl.dir/size        row count, decimal text
 *     <root>/scale%03d/<table>.tbl.dir/<column>.bin raw column array
 * load: only the columns `query` needs (the reference's per-query selection;
 * query 0 = every column present).  Returns 0, or -1 if a file is missing/short.
 * CSV: the dbgen '|' files <root>/scale%03d/<table>.tbl (TpcHCommons.cpp:296-591).
 * Every table is allocated with 64-B aligned malloc; free with mi355_tpch_free_*.
 */
int mi355_tpch_load_lineitem(struct LineItemTable *t, const char *root, int query, int scale, int csv);
int mi355_tpch_load_orders(struct OrdersTable *t, const char *root, int query, int scale, int csv);
int mi355_tpch_load_customer(struct CustomerTable *t, const char *root, int query, int scale, int csv);
int mi355_tpch_load_part(struct PartTable *t, const char *root, int query, int scale, int csv);
int mi355_tpch_load_nation(struct NationTable *t, const char *root, int query, int scale, int csv);
/* Write every non-null column of the tables to the binary layout (csv_convert). */
int mi355_tpch_store(const char *root, int scale, const struct LineItemTable *l, const struct OrdersTable *o,
                     const struct CustomerTable *c, const struct PartTable *p, const struct NationTable *n);
void mi355_tpch_free_lineitem(struct LineItemTable *t);
void mi355_tpch_free_orders(struct OrdersTable *t);
void mi355_tpch_free_customer(struct CustomerTable *t);
void mi355_tpch_free_part(struct PartTable *t);
void mi355_tpch_free_nation(struct NationTable *t);

/*
 * Deterministic synthetic TPC-H tables (dbgen is not available offline): the
 * TPC-H spec's cardinalities and value distributions for every column above,
 * from a counter-based hash of (seed, table, column, row) — the same values on
 * the host (these calls) and on the device (mi355_tpch_generate_dev).  Encoded
 * the way the reference's CSV loader encodes dbgen text (so "REG AIR" maps to 0,
 * as TpcHCommons.cpp:142-154 does).  scale_milli = scale factor × 1000
 * (1000 = SF1: 150k customers, 1.5M orders, ~6M lineitems, 200k parts, 25 nations).
 * Host tables are malloc'd (free with mi355_tpch_free_*).
 */
int mi355_tpch_generate(uint32_t scale_milli, uint64_t seed, struct LineItemTable *l, struct OrdersTable *o,
                        struct CustomerTable *c, struct PartTable *p, struct NationTable *n);
/* Row counts of a synthetic scale (lineitem needs the per-order draw: exact). */
int mi355_tpch_sizes(uint32_t scale_milli, uint64_t seed, uint64_t *n_lineitem, uint64_t *n_orders,
                     uint64_t *n_customer, uint64_t *n_part, uint64_t *n_nation);
/* Same tables generated in HBM: every column pointer of the structs must point to
 * device memory of the sizes mi355_tpch_sizes reports (NULL columns are skipped). */
int mi355_tpch_generate_dev(uint32_t scale_milli, uint64_t seed, const struct LineItemTable *l,
                            const struct OrdersTable *o, const struct CustomerTable *c, const struct PartTable *p,
                            const struct NationTable *n, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* SGXAMD_TPCH_H */
