// Internal interface between the scan kernels (scan_kernels.hip) and scan_host.cpp.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace sgxamd {
namespace scan {

constexpr uint64_t kChunkQuantum = 16384;  // rows; multiple of waves * 64 * V * unroll for u8 and i32
#ifndef SGXAMD_SCAN_WGS
#define SGXAMD_SCAN_WGS 2048
#endif
constexpr uint64_t kChunkTarget = SGXAMD_SCAN_WGS;  // workgroups per scan

template <typename T>
hipError_t launch_predicate(const T *in, uint64_t n, T lo, T hi, uint64_t rows_per_chunk, uint32_t nchunks,
                            uint64_t *bv, uint64_t *chunk_counts, hipStream_t s);

// One-pass index (MODE 0) / value (1) / dictionary (2) / explicit index (3) selection
// with decoupled look-back over chunks (scan_kernels.hip k_select).  ticket: two u32
// (after the launch, bit 0 of ticket[1] = a look-back poll gave up, bit 1 = an explicit
// index entry past aux_len), status: one u64 per chunk (select_chunks(n)); both are
// reset by the launch.  *total = matches.
template <typename T, typename OutT, int MODE>
hipError_t launch_select(const T *in, uint64_t n, T lo, T hi, uint32_t *ticket, uint64_t *status, OutT *out,
                         uint64_t cap, uint64_t *total, hipStream_t s, const int64_t *dict = nullptr,
                         uint64_t aux_len = 0);
uint64_t select_chunks(uint64_t n);

// Per-chunk sums of the u8 codes in [lo, hi] (SIMD512::sum).
hipError_t launch_sum_u8(const uint8_t *in, uint64_t n, uint8_t lo, uint8_t hi, uint64_t rows_per_chunk,
                         uint32_t nchunks, uint64_t *chunk_sums, hipStream_t s);

// range[0] = first i with dict[i] >= lo, range[1] = first j >= range[0] with dict[j] > hi
// (each dict_size when none); both must be preset to dict_size.
hipError_t launch_dict_range(const int64_t *dict, uint64_t n, int64_t lo, int64_t hi, uint64_t *range,
                             hipStream_t s);

hipError_t launch_sum(const uint64_t *v, uint32_t n, uint64_t *out, hipStream_t s);

}  // namespace scan
}  // namespace sgxamd
