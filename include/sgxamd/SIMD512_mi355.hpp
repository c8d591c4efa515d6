// sgxamd/SIMD512_mi355.hpp — header-only drop-in for the reference's SIMD512:: scans.
//
// Same names, argument order and meaning as
// Scan-Micro-Benchmarks/shared_libraries/SimdScan/include/SIMD512.hpp:39-84, including
// the reference's behaviour of ignoring the input_size % 64 tail (its loops run to
// input_size / 64).  The pointer arguments are untyped here so that callers passing
// `const __m512i *` / `__mmask64 *` compile unchanged without AVX-512 headers.
// Errors abort, as the reference has no error channel.
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "sgxamd/scan.h"

extern "C" const char *mi355_last_error(void);

namespace SIMD512 {

constexpr uint8_t BITS_NEEDED = 8;
using pred_t = uint8_t;

namespace detail {
inline void check(int rc, const char *what) {
    if (rc != 0) {
        std::fprintf(stderr, "SIMD512(mi355)::%s failed (%d): %s\n", what, rc, mi355_last_error());
        std::abort();
    }
}
inline size_t whole(size_t n) { return n & ~size_t(63); }
}  // namespace detail

// SIMD512.cpp:7-32
inline size_t count(pred_t lo, pred_t hi, const void *input_compressed, size_t input_size) {
    uint64_t c = 0;
    detail::check(mi355_scan_count_u8(lo, hi, static_cast<const uint8_t *>(input_compressed),
                                      detail::whole(input_size), &c), "count");
    return c;
}

// SIMD512.cpp:210-222; output_buffer holds input_size / 64 words.
inline void bitvector_scan(pred_t lo, pred_t hi, const void *input_compressed, size_t input_size,
                           void *output_buffer) {
    detail::check(mi355_scan_bitvector_u8(lo, hi, static_cast<const uint8_t *>(input_compressed),
                                          detail::whole(input_size), static_cast<uint64_t *>(output_buffer)),
                  "bitvector_scan");
}

// SIMD512.cpp:225-249; like the reference, output_buffer must have room for every match.
inline void implicit_index_scan(pred_t lo, pred_t hi, const void *input_compressed, size_t input_size,
                                size_t *output_buffer) {
    uint64_t n = 0;
    const size_t m = detail::whole(input_size);
    detail::check(mi355_scan_index_u8(lo, hi, static_cast<const uint8_t *>(input_compressed), m,
                                      reinterpret_cast<uint64_t *>(output_buffer), m, &n),
                  "implicit_index_scan");
}

// SIMD512.cpp:251-287; grows the vector as needed, trims it to the match count when cut.
template <typename Vec>
inline void implicit_index_scan_self_alloc(pred_t lo, pred_t hi, const void *input_compressed, size_t input_size,
                                           Vec &output_buffer, bool cut = false) {
    const size_t m = detail::whole(input_size);
    uint64_t c = 0;
    detail::check(mi355_scan_count_u8(lo, hi, static_cast<const uint8_t *>(input_compressed), m, &c),
                  "implicit_index_scan_self_alloc");
    if (output_buffer.size() < c) output_buffer.resize(c);
    uint64_t n = 0;
    detail::check(mi355_scan_index_u8(lo, hi, static_cast<const uint8_t *>(input_compressed), m,
                                      reinterpret_cast<uint64_t *>(output_buffer.data()), output_buffer.size(), &n),
                  "implicit_index_scan_self_alloc");
    if (cut) output_buffer.resize(n);
}

// SIMD512.cpp:91-150: matching codes zero-extended to uint32; returns the match count.
inline size_t scan(pred_t lo, pred_t hi, const void *input_compressed, size_t input_size, uint32_t *output_buffer) {
    uint64_t n = 0;
    const size_t m = detail::whole(input_size);
    detail::check(mi355_scan_values_u8(lo, hi, static_cast<const uint8_t *>(input_compressed), m, output_buffer, m,
                                       &n),
                  "scan");
    return n;
}

}  // namespace SIMD512
