/*
 * oracle/scan_oracle.c — scalar restatement of the reference's predicate scans.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Semantics follow Scan-Micro-Benchmarks/shared_libraries/SimdScan/src/SIMD512.cpp:
 *   count            :7-32     popcount of (v >= lo) & (v <= hi), unsigned bytes
 *   bitvector_scan   :210-222  bit j of word i <-> row 64i+j (_store_mask64)
 *   implicit_index_scan(_self_alloc) :225-287  ascending row indexes (uint64)
 *   scan             :91-150   matching values zero-extended to uint32
 * and the scalar driver mode microbenchmarks/SimdScanMulti/shared/ScalarScan.hpp:8-18.
 * All n values are scanned (the AVX-512 code drops the n % 64 tail; callers
 * that want that pass n rounded down).  i32 variants compare signed.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define PRED(v) ((v) >= lo && (v) <= hi)

uint64_t oracle_scan_count_u8(uint8_t lo, uint8_t hi, const uint8_t *in, size_t n) {
    uint64_t c = 0;
    for (size_t i = 0; i < n; i++) c += PRED(in[i]);
    return c;
}

uint64_t oracle_scan_count_i32(int32_t lo, int32_t hi, const int32_t *in, size_t n) {
    uint64_t c = 0;
    for (size_t i = 0; i < n; i++) c += PRED(in[i]);
    return c;
}

void oracle_scan_bitvector_u8(uint8_t lo, uint8_t hi, const uint8_t *in, size_t n, uint64_t *out) {
    memset(out, 0, ((n + 63) / 64) * sizeof(uint64_t));
    for (size_t i = 0; i < n; i++)
        if (PRED(in[i])) out[i / 64] |= 1ull << (i % 64);
}

void oracle_scan_bitvector_i32(int32_t lo, int32_t hi, const int32_t *in, size_t n, uint64_t *out) {
    memset(out, 0, ((n + 63) / 64) * sizeof(uint64_t));
    for (size_t i = 0; i < n; i++)
        if (PRED(in[i])) out[i / 64] |= 1ull << (i % 64);
}

uint64_t oracle_scan_index_u8(uint8_t lo, uint8_t hi, const uint8_t *in, size_t n, uint64_t *out) {
    uint64_t k = 0;
    for (size_t i = 0; i < n; i++)
        if (PRED(in[i])) out[k++] = i;
    return k;
}

uint64_t oracle_scan_index_i32(int32_t lo, int32_t hi, const int32_t *in, size_t n, uint64_t *out) {
    uint64_t k = 0;
    for (size_t i = 0; i < n; i++)
        if (PRED(in[i])) out[k++] = i;
    return k;
}

uint64_t oracle_scan_values_u8(uint8_t lo, uint8_t hi, const uint8_t *in, size_t n, uint32_t *out) {
    uint64_t k = 0;
    for (size_t i = 0; i < n; i++)
        if (PRED(in[i])) out[k++] = in[i];
    return k;
}

uint64_t oracle_scan_values_i32(int32_t lo, int32_t hi, const int32_t *in, size_t n, int32_t *out) {
    uint64_t k = 0;
    for (size_t i = 0; i < n; i++)
        if (PRED(in[i])) out[k++] = in[i];
    return k;
}

typedef struct {
    int32_t lo, hi;
    const int32_t *in;
    size_t n;
    uint64_t result;
} count_arg;

static void *count_worker(void *p) {
    count_arg *a = (count_arg *)p;
    a->result = oracle_scan_count_i32(a->lo, a->hi, a->in, a->n);
    return NULL;
}

/* Contiguous per-thread slices as in scan_wrapper (multithreadedscan.cpp:227-236). */
uint64_t oracle_scan_count_i32_mt(int32_t lo, int32_t hi, const int32_t *in, size_t n, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    pthread_t *th = (pthread_t *)calloc(nthreads, sizeof(pthread_t));
    count_arg *args = (count_arg *)calloc(nthreads, sizeof(count_arg));
    size_t per = n / nthreads;
    for (int t = 0; t < nthreads; t++) {
        args[t].lo = lo;
        args[t].hi = hi;
        args[t].in = in + t * per;
        args[t].n = (t == nthreads - 1) ? n - t * per : per;
        pthread_create(&th[t], NULL, count_worker, &args[t]);
    }
    uint64_t total = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        total += args[t].result;
    }
    free(th);
    free(args);
    return total;
}

/* SIMD512::sum (SIMD512.cpp:34-88), scalar: sum of the u8 codes in [lo, hi]. */
uint64_t oracle_scan_sum_u8(uint8_t lo, uint8_t hi, const uint8_t *in, size_t n) {
    uint64_t s = 0;
    for (size_t i = 0; i < n; i++)
        if (in[i] >= lo && in[i] <= hi) s += in[i];
    return s;
}

/* dict_scan_{8,16,32}bit_64bit (SIMD512.cpp:289-338, 531-579, 581-629) in the
 * scalar form of dict_scan_8bit_64bit_scalar (:505-529): the predicate's code
 * range comes from two std::find_if passes over the dictionary (:297-302), cast to
 * uint8_t (8-bit codes) or uint16_t (16- and 32-bit codes, :588-589); matching
 * rows are decoded to dict[code] in row order.  code_bytes = 1, 2 or 4.  Scans all
 * n codes (the vector versions' block tails are the caller's business). */
uint64_t oracle_dict_scan(int64_t lo, int64_t hi, const int64_t *dict, uint64_t dict_size, const void *codes,
                          int code_bytes, size_t n, int64_t *out) {
    uint64_t low = 0;
    while (low < dict_size && !(dict[low] >= lo)) low++;
    uint64_t end = low;
    while (end < dict_size && !(dict[end] > hi)) end++;
    const int64_t high = (int64_t)end - 1;
    uint32_t clo, chi;
    if (code_bytes == 1) {
        clo = (uint8_t)low;
        chi = (uint8_t)(high & 0xff);
    } else {
        clo = (uint16_t)low;
        chi = (uint16_t)high;
    }
    uint64_t k = 0;
    for (size_t i = 0; i < n; i++) {
        uint32_t c;
        if (code_bytes == 1) c = ((const uint8_t *)codes)[i];
        else if (code_bytes == 2) c = ((const uint16_t *)codes)[i];
        else c = ((const uint32_t *)codes)[i];
        if (c >= clo && c <= chi) {
            if (out) out[k] = dict[c];
            k++;
        }
    }
    return k;
}

/* SIMD512::explicit_index_scan (SIMD512.cpp:152-208), restated as written: for the
 * 64-row block i and its 8-row sub-block j (rows 64i+8j .. 64i+8j+7), the matching
 * rows' entries are compress-stored from the 8 u64 lanes of index_compressed[i + j]
 * (:174, :198) — the vector index is block + sub-block, not 8·block + sub-block — so
 * row r takes index[8·(r/64 + (r%64)/8) + r%8].  Both of the reference's branches
 * (lo == hi via cmpeq, else cmpge & cmple) select the same rows.  The reference only
 * reads index vectors of sub-blocks with a match; so does this loop.  Scans all n
 * rows (the AVX-512 loop drops the n % 64 tail: callers that want it round down). */
uint64_t oracle_scan_explicit_index_u8(uint8_t lo, uint8_t hi, const uint64_t *index, const uint8_t *in, size_t n,
                                       uint64_t *out) {
    uint64_t k = 0;
    for (size_t r = 0; r < n; r++)
        if (PRED(in[r])) out[k++] = index[8 * (r / 64 + (r % 64) / 8) + r % 8];
    return k;
}
