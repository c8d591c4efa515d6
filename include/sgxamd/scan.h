/*
 * sgxamd/scan.h — C-ABI of the MI355X predicate column scan.
 *
 * Replaces the reference's AVX-512 scan functions in namespace SIMD512
 * (Scan-Micro-Benchmarks/shared_libraries/SimdScan/include/SIMD512.hpp:39-84,
 *  implemented in src/SIMD512.cpp):
 *   count                          SIMD512.cpp:7-32    -> mi355_scan_count_*
 *   bitvector_scan                 SIMD512.cpp:210-222 -> mi355_scan_bitvector_*
 *   implicit_index_scan(_self_alloc) SIMD512.cpp:225-287 -> mi355_scan_index_*
 *   explicit_index_scan            SIMD512.cpp:152-208 -> mi355_scan_explicit_index_u8
 *   scan (value materialisation)   SIMD512.cpp:91-150  -> mi355_scan_values_*
 *   sum                            SIMD512.cpp:34-88   -> mi355_scan_sum_u8
 *   dict_scan_8bit_64bit           SIMD512.cpp:289-338 -> mi355_dict_scan_8bit_64bit
 *   dict_scan_16bit_64bit          SIMD512.cpp:531-579 -> mi355_dict_scan_16bit_64bit
 *   dict_scan_32bit_64bit          SIMD512.cpp:581-629 -> mi355_dict_scan_32bit_64bit
 * Predicate semantics: lo <= v <= hi, inclusive; unsigned compare for u8
 * (_mm512_cmpge_epu8_mask / cmple), signed compare for i32.
 *
 * Unlike the AVX-512 code, which silently ignores the n % 64 tail
 * (loops run to input_size / 64), these entry points scan all n values.  The
 * header-only C++ adapter sgxamd/SIMD512_mi355.hpp restores the reference's
 * tail behaviour for drop-in callers.
 *
 * Pointers may be host or device memory (classified per call).  Blocking.
 */
#ifndef SGXAMD_SCAN_H
#define SGXAMD_SCAN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Number of values v[i] with lo <= v[i] <= hi. */
int mi355_scan_count_u8(uint8_t lo, uint8_t hi, const uint8_t *in, size_t n, uint64_t *count);
int mi355_scan_count_i32(int32_t lo, int32_t hi, const int32_t *in, size_t n, uint64_t *count);

/* One bit per row: bit j of word i <-> row 64*i + j (the _store_mask64 layout,
 * SIMD512.cpp:219).  out holds ceil(n/64) words; bits past n are zero. */
int mi355_scan_bitvector_u8(uint8_t lo, uint8_t hi, const uint8_t *in, size_t n, uint64_t *out_words);
int mi355_scan_bitvector_i32(int32_t lo, int32_t hi, const int32_t *in, size_t n, uint64_t *out_words);

/* Ascending uint64 row indexes (relative to `in`) of all matches.  Writes at
 * most cap indexes; *n_out = number of matches.  Returns MI355_ERR_CAPACITY
 * (with *n_out set) when cap < matches. */
int mi355_scan_index_u8(uint8_t lo, uint8_t hi, const uint8_t *in, size_t n,
                        uint64_t *out, size_t cap, uint64_t *n_out);
int mi355_scan_index_i32(int32_t lo, int32_t hi, const int32_t *in, size_t n,
                         uint64_t *out, size_t cap, uint64_t *n_out);

/* SIMD512::explicit_index_scan (SIMD512.cpp:152-208, SIMD512.hpp:60-65): like the index
 * scan, but each match of row r emits the u64 entry index[8*(r/64 + (r%64)/8) + r%8] of a
 * caller-supplied index array (index_len entries, host or device) — the reference's
 * index_compressed[i + j] for 64-row block i and 8-row sub-block j, restated as written.
 * A caller covering every row allocates 8*((n-1)/64 + 7) + 8 entries; a match whose
 * entry lies past index_len fails with MI355_ERR_INVALID.  cap / n_out / CAPACITY as
 * for mi355_scan_index_u8. */
int mi355_scan_explicit_index_u8(uint8_t lo, uint8_t hi, const uint64_t *index, size_t index_len,
                                 const uint8_t *in, size_t n, uint64_t *out, size_t cap, uint64_t *n_out);

/* Matching values in row order: u8 codes zero-extended to uint32 (SIMD512::scan),
 * i32 values as int32. */
int mi355_scan_values_u8(uint8_t lo, uint8_t hi, const uint8_t *in, size_t n,
                         uint32_t *out, size_t cap, uint64_t *n_out);
int mi355_scan_values_i32(int32_t lo, int32_t hi, const int32_t *in, size_t n,
                          int32_t *out, size_t cap, uint64_t *n_out);

/* Sum of the u8 codes v[i] with lo <= v[i] <= hi (SIMD512::sum). */
int mi355_scan_sum_u8(uint8_t lo, uint8_t hi, const uint8_t *in, size_t n, uint64_t *sum);

/*
 * Dictionary scans: codes index a dictionary of int64 values; the value predicate
 * [lo, hi] is turned into a code range the way the reference does (first index
 * with dict[i] >= lo; first index after it with dict[j] > hi, minus one; cast to
 * the code width, uint16_t for the 32-bit variant as at SIMD512.cpp:588-589, so
 * out-of-dictionary predicates wrap exactly like the reference's), and every
 * matching row's dict[code] is written in row order.  At most cap values are
 * written; *n_out = matches (MI355_ERR_CAPACITY when cap < matches).  dict has
 * 256 / 65536 / dict_size entries (host or device).
 */
int mi355_dict_scan_8bit_64bit(int64_t lo, int64_t hi, const int64_t *dict, const uint8_t *in, size_t n,
                               int64_t *out, size_t cap, uint64_t *n_out);
int mi355_dict_scan_16bit_64bit(int64_t lo, int64_t hi, const int64_t *dict, const uint16_t *in, size_t n,
                                int64_t *out, size_t cap, uint64_t *n_out);
int mi355_dict_scan_32bit_64bit(int64_t lo, int64_t hi, const int64_t *dict, size_t dict_size, const uint32_t *in,
                                size_t n, int64_t *out, size_t cap, uint64_t *n_out);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* SGXAMD_SCAN_H */
