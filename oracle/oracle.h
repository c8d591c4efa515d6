/*
 * oracle/oracle.h — CPU restatement of the reference's hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (the HIP library under
 * sgxv2-analytical-query-processing-benchmarks_amd/) links or calls this code.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load
 * liboracle.so, and only as the checker / the timed CPU baseline.
 *
 * Pinning (see DESIGN.md "Oracle"): building or running the reference itself
 * was denied in this pipeline, so there is no oracle/_ref.
 * The join restatement is pinned by the analytical known-answer tests derived
 * from the reference's generators (pk ⋈ fk → |S|, fk_sel jump rule, Zipf → |S|)
 * and by an independent sort-merge cardinality counter; the scan restatement
 * by the reference's own Catch2 KATs (testsimdscan.cpp: count = N/256 · width
 * over the i % 256 column).  Join parity is therefore "pinned by KATs", not by
 * reference-produced golden vectors.
 */
#ifndef SGXAMD_ORACLE_H
#define SGXAMD_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#include "sgxamd/data_types.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_rho_timing {
    uint32_t radix_bits;
    uint32_t passes;
    uint64_t join_tasks;
    double s_total;      /* max over threads of total_timer (radix_join.cpp:1108,1353) */
    double s_partition;  /* partitioning_total_timer */
    double s_pass1;
    double s_pass2;
    double s_join;       /* join_total_timer ("Build+Join Overall") */
} oracle_rho_timing;

/* radix_join.cpp:295-317 (L2_CACHE_SIZE 1280 KiB, CACHE_DIVISOR 4). */
uint32_t oracle_calc_num_radix_bits(uint64_t num_r, uint64_t nthreads);
/* radix_join.cpp:319-329 */
uint32_t oracle_calc_num_passes(uint32_t num_radix_bits);

/*
 * RHO = join_init_run(R, S, bucket_chaining_join, cfg) (radix_join.cpp:1369-1643),
 * count-only, with nthreads pthreads.  force_two_passes mirrors -DFORCE_2_PHASES.
 * Returns the match count (the reference's result_t.totalresults).
 */
int64_t oracle_rho_join(const struct row_t *R, uint64_t nR, const struct row_t *S, uint64_t nS,
                        int nthreads, int force_two_passes, oracle_rho_timing *timing);

/* Independent check: sum_k cnt_R(k) * cnt_S(k) by sorting the keys. */
/* The same join with MATERIALIZE = 1 (radix_join.cpp:437-446): every match as
 * {S key, R payload, S payload}, per-thread outputs concatenated in thread order
 * into out (at most cap triples written).  Returns the match count. */
int64_t oracle_rho_join_mat(const struct row_t *R, uint64_t nR, const struct row_t *S, uint64_t nS, int nthreads,
                            int force_two_passes, struct output_triple_t *out, uint64_t cap);

/* RHT (radix_join.cpp:1645-1648): the same partitioning with histogram_join
 * (:463-612); out = NULL counts only, else materialises like oracle_rho_join_mat. */
int64_t oracle_rht_join(const struct row_t *R, uint64_t nR, const struct row_t *S, uint64_t nS, int nthreads,
                        int force_two_passes, struct output_triple_t *out, uint64_t cap);

int64_t oracle_count_join_sort(const struct row_t *R, uint64_t nR, const struct row_t *S, uint64_t nS);

/* Stable single-pass radix partition of `in` by bin = (key >> shift) & (2^bits-1)
 * with the reference's per-thread histogram/offset rule (radix_join.cpp:851-931)
 * for `nthreads` contiguous slices, without padding.  out: n tuples;
 * bin_start: 2^bits + 1 entries. */
void oracle_radix_partition(const struct row_t *in, uint64_t n, int nthreads, uint32_t shift,
                            uint32_t bits, struct row_t *out, uint64_t *bin_start);

/* Scalar scans (SIMD512.cpp:7-32, 210-287; ScalarScan.hpp:8-18) over all n values. */
uint64_t oracle_scan_count_u8(uint8_t lo, uint8_t hi, const uint8_t *in, size_t n);
uint64_t oracle_scan_count_i32(int32_t lo, int32_t hi, const int32_t *in, size_t n);
void oracle_scan_bitvector_u8(uint8_t lo, uint8_t hi, const uint8_t *in, size_t n, uint64_t *out);
void oracle_scan_bitvector_i32(int32_t lo, int32_t hi, const int32_t *in, size_t n, uint64_t *out);
uint64_t oracle_scan_index_u8(uint8_t lo, uint8_t hi, const uint8_t *in, size_t n, uint64_t *out);
uint64_t oracle_scan_index_i32(int32_t lo, int32_t hi, const int32_t *in, size_t n, uint64_t *out);
/* SIMD512::explicit_index_scan (SIMD512.cpp:152-208): row r takes
 * index[8*(r/64 + (r%64)/8) + r%8] (the reference's index_compressed[i + j]). */
uint64_t oracle_scan_explicit_index_u8(uint8_t lo, uint8_t hi, const uint64_t *index, const uint8_t *in, size_t n,
                                       uint64_t *out);
uint64_t oracle_scan_values_u8(uint8_t lo, uint8_t hi, const uint8_t *in, size_t n, uint32_t *out);
uint64_t oracle_scan_values_i32(int32_t lo, int32_t hi, const int32_t *in, size_t n, int32_t *out);
/* Multithreaded count for the CPU baseline (contiguous slices, like scan_wrapper). */
/* SIMD512::sum (SIMD512.cpp:34-88). */
uint64_t oracle_scan_sum_u8(uint8_t lo, uint8_t hi, const uint8_t *in, size_t n);
/* dict_scan_{8,16,32}bit_64bit (SIMD512.cpp:289-629): code range via the dictionary with
 * the reference's casts, then dict[code] of every matching row; returns the matches. */
uint64_t oracle_dict_scan(int64_t lo, int64_t hi, const int64_t *dict, uint64_t dict_size, const void *codes,
                          int code_bytes, size_t n, int64_t *out);
uint64_t oracle_scan_count_i32_mt(int32_t lo, int32_t hi, const int32_t *in, size_t n, int nthreads);

/* CPU scan baseline (cpu_baseline.c): kind 0 count / 1 bitvector / 2 index list over
 * a uint8 (width 1) or int32 (width 4) column, nthreads pinned to cpus[t] (NULL: not
 * pinned), the multithreadedscan.cpp slicing; returns the per-call seconds averaged
 * over the threads (-1 on error) and the total matches. */
double oracle_cpu_scan_bench(int kind, int width, int64_t lo, int64_t hi, const void *in, size_t n, int nthreads,
                             const int *cpus, int reps, uint64_t *matches);

/* TPC-H callers (tpch_oracle.c; tables as in sgxamd/tpch.h).  oracle_tpch_filter:
 * filter_table of selection `which` of `query` into out (rows in input order),
 * returns the row count.  The queries return the reference's result (Q19: the
 * final predicate's count) and fill info[0..2] = rows after selection 1..3,
 * info[3..5] = cardinality of join 1..3. */
struct CustomerTable;
struct OrdersTable;
struct LineItemTable;
struct PartTable;
struct NationTable;
uint64_t oracle_tpch_filter(int query, int which, const struct CustomerTable *c, const struct OrdersTable *o,
                            const struct LineItemTable *l, const struct PartTable *p, struct row_t *out);
int64_t oracle_tpch_q3(const struct CustomerTable *c, const struct OrdersTable *o, const struct LineItemTable *l,
                       int nthreads, int rht, uint64_t *info);
int64_t oracle_tpch_q10(const struct CustomerTable *c, const struct OrdersTable *o, const struct LineItemTable *l,
                        const struct NationTable *n, int nthreads, int rht, uint64_t *info);
int64_t oracle_tpch_q12(const struct LineItemTable *l, const struct OrdersTable *o, int nthreads, int rht,
                        uint64_t *info);
int64_t oracle_tpch_q19(const struct LineItemTable *l, const struct PartTable *p, int nthreads, int rht,
                        uint64_t *info);

#ifdef __cplusplus
}
#endif

#endif /* SGXAMD_ORACLE_H */
