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

#include "sgxamd/rho.h"
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

// SIMD512.cpp:152-208.  index_compressed is the reference's __m512i array of 8 u64 lanes
// per vector; every 8-row sub-block j of 64-row block i gathers from vector i + j, as the
// reference does (read as written).  The reference reads only vectors of sub-blocks with a
// match and has no bound to check; this adapter passes the largest array any row can
// reach, 8 * (input_size / 64 + 7) u64 — a caller's array must be that long.
inline void explicit_index_scan(pred_t lo, pred_t hi, const void *index_compressed, const void *input_compressed,
                                size_t input_size, size_t *output_buffer) {
    uint64_t n = 0;
    const size_t m = detail::whole(input_size);
    detail::check(mi355_scan_explicit_index_u8(lo, hi, static_cast<const uint64_t *>(index_compressed),
                                               m ? 8 * (m / 64 + 7) : 0, static_cast<const uint8_t *>(input_compressed),
                                               m, reinterpret_cast<uint64_t *>(output_buffer), m, &n),
                  "explicit_index_scan");
}

namespace detail {
// Size the reference's vector ends with (SIMD512.cpp:262-266): before each 64-row block
// it grows once, to (64 + size) * 3, when matches-so-far + 64 exceed the size; the last
// check happens before the last block, with the matches of all blocks before it.
inline size_t self_alloc_size(size_t size, size_t blocks, size_t matches_before_last) {
    if (blocks == 0) return size;
    while (matches_before_last + 64 > size) size = (64 + size) * 3;
    return size;
}
}  // namespace detail

// SIMD512.cpp:251-287, in one pass over the column: the scan runs straight into the
// vector; only if it held fewer slots than matches (MI355_ERR_CAPACITY reports how many)
// is the vector grown and the scan repeated.  The vector then takes the size the
// reference's growth rule gives, or the match count when cut.
template <typename Vec>
inline void implicit_index_scan_self_alloc(pred_t lo, pred_t hi, const void *input_compressed, size_t input_size,
                                           Vec &output_buffer, bool cut = false) {
    const size_t m = detail::whole(input_size);
    const auto *in = static_cast<const uint8_t *>(input_compressed);
    const size_t size0 = output_buffer.size();
    uint64_t n = 0;
    int rc = mi355_scan_index_u8(lo, hi, in, m, reinterpret_cast<uint64_t *>(output_buffer.data()),
                                 output_buffer.size(), &n);
    if (rc == MI355_ERR_CAPACITY) {
        output_buffer.resize(detail::self_alloc_size(output_buffer.size(), m / 64, n));
        rc = mi355_scan_index_u8(lo, hi, in, m, reinterpret_cast<uint64_t *>(output_buffer.data()),
                                 output_buffer.size(), &n);
    }
    detail::check(rc, "implicit_index_scan_self_alloc");
    if (cut) {
        output_buffer.resize(n);
        return;
    }
    // matches before the last 64-row block: the indexes are ascending
    size_t before_last = n;
    const uint64_t last_row0 = m >= 64 ? m - 64 : 0;
    const auto *ix = reinterpret_cast<const uint64_t *>(output_buffer.data());
    while (before_last > 0 && ix[before_last - 1] >= last_row0) --before_last;
    const size_t final_size = detail::self_alloc_size(size0, m / 64, before_last);
    if (final_size != output_buffer.size()) output_buffer.resize(final_size);
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

// SIMD512.cpp:34-88: sum of the matching codes.
inline size_t sum(pred_t lo, pred_t hi, const void *input_compressed, size_t input_size) {
    uint64_t v = 0;
    detail::check(mi355_scan_sum_u8(lo, hi, static_cast<const uint8_t *>(input_compressed), detail::whole(input_size),
                                    &v),
                  "sum");
    return v;
}

namespace detail {
// Dictionary scans: the reference processes input_size / BLOCK whole blocks
// (64 / 32 / 16 codes per 512-bit register) and sizes the output vector itself.
template <typename Vec, typename F>
inline void dict_into(Vec &out, size_t max_matches, F &&call, bool trim) {
    if (out.size() < max_matches) out.resize(max_matches);
    uint64_t n = 0;
    check(call(reinterpret_cast<int64_t *>(out.data()), out.size(), &n), "dict_scan");
    if (trim) out.resize(n);
}
}  // namespace detail

// SIMD512.cpp:289-338
template <typename Vec>
inline void dict_scan_8bit_64bit(int64_t lo, int64_t hi, const int64_t *dict, const void *input_compressed,
                                 size_t input_size, Vec &output_buffer, bool cut = false) {
    const size_t m = input_size / 64 * 64;
    detail::dict_into(output_buffer, m, [&](int64_t *o, size_t cap, uint64_t *n) {
        return mi355_dict_scan_8bit_64bit(lo, hi, dict, static_cast<const uint8_t *>(input_compressed), m, o, cap, n);
    }, cut);
}

// SIMD512.cpp:531-579 (always trims, like the reference)
template <typename Vec>
inline void dict_scan_16bit_64bit(int64_t lo, int64_t hi, const int64_t *dict, const void *input_compressed,
                                  size_t input_size, Vec &output_buffer) {
    const size_t m = input_size / 32 * 32;
    detail::dict_into(output_buffer, m, [&](int64_t *o, size_t cap, uint64_t *n) {
        return mi355_dict_scan_16bit_64bit(lo, hi, dict, static_cast<const uint16_t *>(input_compressed), m, o, cap,
                                           n);
    }, true);
}

// SIMD512.cpp:581-629 (always trims, like the reference)
template <typename Vec>
inline void dict_scan_32bit_64bit(int64_t lo, int64_t hi, const int64_t *dict, size_t dict_size,
                                  const void *input_compressed, size_t input_size, Vec &output_buffer) {
    const size_t m = input_size / 16 * 16;
    detail::dict_into(output_buffer, m, [&](int64_t *o, size_t cap, uint64_t *n) {
        return mi355_dict_scan_32bit_64bit(lo, hi, dict, dict_size, static_cast<const uint32_t *>(input_compressed),
                                           m, o, cap, n);
    }, true);
}

}  // namespace SIMD512
