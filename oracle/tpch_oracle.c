/*
 * oracle/tpch_oracle.c — CPU restatement of the reference's TPC-H callers.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Follows
 *   Join-Benchmarks/lib/TPCH-Queries/src/tpch.cpp:36-309           (pipelines)
 *   filters.hpp:118-138 filter_table (the scalar path, no -DSIMD)   (selections)
 *   Q3Predicates.hpp:166-195, Q10Predicates.hpp:26-45,
 *   Q12Predicates.hpp:22-37, Q19Predicates.hpp:27-78               (predicates / copies)
 *   result_transformers.hpp:50-64                                   (triple -> row transforms)
 * with the joins done by this oracle's RHO restatement (rho_oracle.c), MATERIALIZE
 * where tpch.cpp sets it.
 *
 * Divergence kept out on purpose: the reference's -DSIMD filter variants differ
 * from filter_table on the last (n mod 8/64) rows of Q10 (q10_filter_order_simd's
 * tail tests o_orderdate < 1995-03-15, q10_filter_lineitem_simd's tail tests
 * l_returnflag == MKT_BUILDING) — those are bugs of one build flavour; this oracle
 * and the GPU restate the scalar predicates.
 */
#include <stdlib.h>
#include <string.h>

#include "oracle.h"
#include "sgxamd/tpch.h"

static int q3_cust(const struct CustomerTable *c, uint64_t i) { return c->c_mktsegment[i] == TPCH_MKT_BUILDING; }
static int q3_ord(const struct OrdersTable *o, uint64_t i) { return o->o_orderdate[i] < TPCH_TIMESTAMP_1995_03_15_SECONDS; }
static int q3_line(const struct LineItemTable *l, uint64_t i) { return l->l_shipdate[i] >= TPCH_TIMESTAMP_1995_03_16_SECONDS; }
static int q10_ord(const struct OrdersTable *o, uint64_t i) {
    return o->o_orderdate[i] >= TPCH_TIMESTAMP_1993_10_01_SECONDS && o->o_orderdate[i] < TPCH_TIMESTAMP_1994_01_01_SECONDS;
}
static int q10_line(const struct LineItemTable *l, uint64_t i) { return l->l_returnflag[i] == TPCH_L_RETURNFLAG_R; }
static int q12_line(const struct LineItemTable *l, uint64_t i) {
    const uint8_t m = l->l_shipmode[i];
    const uint64_t commit = l->l_commitdate[i], ship = l->l_shipdate[i], receipt = l->l_receiptdate[i];
    return (m == TPCH_L_SHIPMODE_MAIL || m == TPCH_L_SHIPMODE_SHIP) && commit < receipt && ship < commit &&
           receipt >= TPCH_TIMESTAMP_1994_01_01_SECONDS && receipt < TPCH_TIMESTAMP_1995_01_01_SECONDS;
}
static int q19_part(const struct PartTable *p, uint64_t i) {
    const uint8_t b = p->p_brand[i], k = p->p_container[i];
    return (b == TPCH_P_BRAND_12 || b == TPCH_P_BRAND_23 || b == TPCH_P_BRAND_34) &&
           (k == TPCH_P_CONTAINER_SM_CASE || k == TPCH_P_CONTAINER_SM_BOX || k == TPCH_P_CONTAINER_SM_PACK ||
            k == TPCH_P_CONTAINER_SM_PKG || k == TPCH_P_CONTAINER_MED_BAG || k == TPCH_P_CONTAINER_MED_BOX ||
            k == TPCH_P_CONTAINER_MED_PKG || k == TPCH_P_CONTAINER_MED_PACK || k == TPCH_P_CONTAINER_LG_CASE ||
            k == TPCH_P_CONTAINER_LG_BOX || k == TPCH_P_CONTAINER_LG_PACK || k == TPCH_P_CONTAINER_LG_PKG) &&
           (p->p_size[i] >= 1 && p->p_size[i] <= 15);
}
static int q19_line(const struct LineItemTable *l, uint64_t i) {
    return (l->l_quantity[i] >= 1 && l->l_quantity[i] <= (20 + 10)) &&
           (l->l_shipmode[i] == TPCH_L_SHIPMODE_AIR || l->l_shipmode[i] == TPCH_L_SHIPMODE_AIR_REG) &&
           (l->l_shipinstruct[i] == TPCH_L_SHIPINSTRUCT_DELIVER_IN_PERSON);
}
/* Q19Predicates.hpp:57-78 */
static int q19_final(const struct PartTable *p, uint64_t rp, const struct LineItemTable *l, uint64_t rl) {
    const uint8_t b = p->p_brand[rp], k = p->p_container[rp];
    const uint32_t sz = p->p_size[rp];
    const float q = l->l_quantity[rl];
    const int p1 = b == TPCH_P_BRAND_12 &&
                   (k == TPCH_P_CONTAINER_SM_CASE || k == TPCH_P_CONTAINER_SM_BOX || k == TPCH_P_CONTAINER_SM_PACK ||
                    k == TPCH_P_CONTAINER_SM_PKG) &&
                   (sz >= 1 && sz <= 5) && (q >= 1 && q <= (1 + 10));
    const int p2 = b == TPCH_P_BRAND_23 &&
                   (k == TPCH_P_CONTAINER_MED_BAG || k == TPCH_P_CONTAINER_MED_BOX || k == TPCH_P_CONTAINER_MED_PKG ||
                    k == TPCH_P_CONTAINER_MED_PACK) &&
                   (sz >= 1 && sz <= 10) && (q >= 10 && q <= (10 + 10));
    const int p3 = b == TPCH_P_BRAND_34 &&
                   (k == TPCH_P_CONTAINER_LG_CASE || k == TPCH_P_CONTAINER_LG_BOX || k == TPCH_P_CONTAINER_LG_PACK ||
                    k == TPCH_P_CONTAINER_LG_PKG) &&
                   (sz >= 1 && sz <= 15) && (q >= 20 && q <= (20 + 10));
    return p1 || p2 || p3;
}

uint64_t oracle_tpch_filter(int query, int which, const struct CustomerTable *c, const struct OrdersTable *o,
                            const struct LineItemTable *l, const struct PartTable *p, struct row_t *out) {
    uint64_t k = 0;
    switch (query * 10 + which) {
        case 31:
            for (uint64_t i = 0; i < c->numTuples; ++i)
                if (q3_cust(c, i)) out[k++] = c->c_custkey[i];
            break;
        case 32:
            for (uint64_t i = 0; i < o->numTuples; ++i)
                if (q3_ord(o, i)) {
                    out[k].key = o->o_custkey[i];
                    out[k++].payload = o->o_orderkey[i].key;
                }
            break;
        case 33:
            for (uint64_t i = 0; i < l->numTuples; ++i)
                if (q3_line(l, i)) out[k++] = l->l_orderkey[i];
            break;
        case 101:
            for (uint64_t i = 0; i < o->numTuples; ++i)
                if (q10_ord(o, i)) {
                    out[k].key = o->o_custkey[i];
                    out[k++].payload = o->o_orderkey[i].payload;
                }
            break;
        case 102:
            for (uint64_t i = 0; i < l->numTuples; ++i)
                if (q10_line(l, i)) out[k++] = l->l_orderkey[i];
            break;
        case 121:
            for (uint64_t i = 0; i < l->numTuples; ++i)
                if (q12_line(l, i)) out[k++] = l->l_orderkey[i];
            break;
        case 191:
            for (uint64_t i = 0; i < p->numTuples; ++i)
                if (q19_part(p, i)) out[k++] = p->p_partkey[i];
            break;
        case 192:
            for (uint64_t i = 0; i < l->numTuples; ++i)
                if (q19_line(l, i)) {
                    out[k].key = l->l_partkey[i];
                    out[k++].payload = l->l_orderkey[i].payload;
                }
            break;
        default:
            break;
    }
    return k;
}

static uint64_t max_rows(uint64_t a, uint64_t b) { return (a > b ? a : b) + 1; }

/* join with materialisation into a fresh buffer (*out owned by the caller) */
static int64_t join_mat(const struct row_t *R, uint64_t nR, const struct row_t *S, uint64_t nS, int nthreads,
                        int rht, struct output_triple_t **out) {
    int64_t m = rht ? oracle_rht_join(R, nR, S, nS, nthreads, 0, NULL, 0)
                    : oracle_rho_join(R, nR, S, nS, nthreads, 0, NULL);
    *out = (struct output_triple_t *)malloc(((size_t)m + 1) * sizeof(struct output_triple_t));
    if (!*out) return -1;
    return rht ? oracle_rht_join(R, nR, S, nS, nthreads, 0, *out, (uint64_t)m)
               : oracle_rho_join_mat(R, nR, S, nS, nthreads, 0, *out, (uint64_t)m);
}
static int64_t join_count(const struct row_t *R, uint64_t nR, const struct row_t *S, uint64_t nS, int nthreads,
                          int rht) {
    return rht ? oracle_rht_join(R, nR, S, nS, nthreads, 0, NULL, 0) : oracle_rho_join(R, nR, S, nS, nthreads, 0, NULL);
}

/* tpch.cpp:36-115.  info: filtered[0..2], join_matches[0..1]. */
int64_t oracle_tpch_q3(const struct CustomerTable *c, const struct OrdersTable *o, const struct LineItemTable *l,
                       int nthreads, int rht, uint64_t *info) {
    struct row_t *f1 = malloc(max_rows(c->numTuples, 0) * sizeof(struct row_t));
    struct row_t *f2 = malloc(max_rows(o->numTuples, 0) * sizeof(struct row_t));
    struct row_t *f3 = malloc(max_rows(l->numTuples, 0) * sizeof(struct row_t));
    const uint64_t n1 = oracle_tpch_filter(3, 1, c, o, l, NULL, f1);
    const uint64_t n2 = oracle_tpch_filter(3, 2, c, o, l, NULL, f2);
    struct output_triple_t *t = NULL;
    const int64_t m1 = join_mat(f1, n1, f2, n2, nthreads, rht, &t);
    struct row_t *u = malloc(((size_t)m1 + 1) * sizeof(struct row_t));
    for (int64_t i = 0; i < m1; ++i) u[i].key = u[i].payload = t[i].Spayload; /* copy_Sp_Sp */
    const uint64_t n3 = oracle_tpch_filter(3, 3, c, o, l, NULL, f3);
    const int64_t m2 = join_count(u, (uint64_t)m1, f3, n3, nthreads, rht);
    if (info) {
        info[0] = n1, info[1] = n2, info[2] = n3, info[3] = (uint64_t)m1, info[4] = (uint64_t)m2;
    }
    free(f1), free(f2), free(f3), free(t), free(u);
    return m2;
}

/* tpch.cpp:117-216.  info: filtered[0..1], join_matches[0..2]. */
int64_t oracle_tpch_q10(const struct CustomerTable *c, const struct OrdersTable *o, const struct LineItemTable *l,
                        const struct NationTable *n, int nthreads, int rht, uint64_t *info) {
    struct row_t *f1 = malloc(max_rows(o->numTuples, 0) * sizeof(struct row_t));
    const uint64_t n1 = oracle_tpch_filter(10, 1, c, o, l, NULL, f1);
    struct output_triple_t *t1 = NULL, *t2 = NULL;
    const int64_t m1 = join_mat(c->c_custkey, c->numTuples, f1, n1, nthreads, rht, &t1);
    struct row_t *u1 = malloc(((size_t)m1 + 1) * sizeof(struct row_t));
    for (int64_t i = 0; i < m1; ++i) { /* copy_RpToKeySp with c_nationkey */
        u1[i].key = c->c_nationkey[t1[i].Rpayload];
        u1[i].payload = t1[i].Spayload;
    }
    const int64_t m2 = join_mat(n->n_nationkey, n->numTuples, u1, (uint64_t)m1, nthreads, rht, &t2);
    struct row_t *u2 = malloc(((size_t)m2 + 1) * sizeof(struct row_t));
    for (int64_t i = 0; i < m2; ++i) { /* copy_SpToTupleST with o_orderkey */
        u2[i].key = o->o_orderkey[t2[i].Spayload].key;
        u2[i].payload = 0;
    }
    struct row_t *f2 = malloc(max_rows(l->numTuples, 0) * sizeof(struct row_t));
    const uint64_t n2 = oracle_tpch_filter(10, 2, c, o, l, NULL, f2);
    const int64_t m3 = join_count(u2, (uint64_t)m2, f2, n2, nthreads, rht);
    if (info) {
        info[0] = n1, info[1] = n2, info[2] = 0, info[3] = (uint64_t)m1, info[4] = (uint64_t)m2,
        info[5] = (uint64_t)m3;
    }
    free(f1), free(f2), free(t1), free(t2), free(u1), free(u2);
    return m3;
}

/* tpch.cpp:218-252.  info: filtered[0], join_matches[0]. */
int64_t oracle_tpch_q12(const struct LineItemTable *l, const struct OrdersTable *o, int nthreads, int rht,
                        uint64_t *info) {
    struct row_t *f1 = malloc(max_rows(l->numTuples, 0) * sizeof(struct row_t));
    const uint64_t n1 = oracle_tpch_filter(12, 1, NULL, o, l, NULL, f1);
    const int64_t m1 = join_count(o->o_orderkey, o->numTuples, f1, n1, nthreads, rht);
    if (info) info[0] = n1, info[3] = (uint64_t)m1;
    free(f1);
    return m1;
}

/* tpch.cpp:254-309.  Returns the final predicate's count; info: filtered[0..1], join_matches[0]. */
int64_t oracle_tpch_q19(const struct LineItemTable *l, const struct PartTable *p, int nthreads, int rht,
                        uint64_t *info) {
    struct row_t *f1 = malloc(max_rows(p->numTuples, 0) * sizeof(struct row_t));
    struct row_t *f2 = malloc(max_rows(l->numTuples, 0) * sizeof(struct row_t));
    const uint64_t n1 = oracle_tpch_filter(19, 1, NULL, NULL, l, p, f1);
    const uint64_t n2 = oracle_tpch_filter(19, 2, NULL, NULL, l, p, f2);
    struct output_triple_t *t = NULL;
    const int64_t m1 = join_mat(f1, n1, f2, n2, nthreads, rht, &t);
    int64_t matches = 0;
    for (int64_t i = 0; i < m1; ++i) matches += q19_final(p, t[i].Rpayload, l, t[i].Spayload);
    if (info) info[0] = n1, info[1] = n2, info[3] = (uint64_t)m1;
    free(f1), free(f2), free(t);
    return matches;
}
