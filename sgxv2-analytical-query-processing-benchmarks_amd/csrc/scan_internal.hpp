// Internal interface between the scan kernels (scan_kernels.hip) and scan_host.cpp.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace sgxamd {
namespace scan {

constexpr uint64_t kChunkQuantum = 16384;  // rows; multiple of waves * 64 * V * unroll for u8 and i32
constexpr uint64_t kChunkTarget = 2048;    // workgroups per scan

template <typename T>
hipError_t launch_predicate(const T *in, uint64_t n, T lo, T hi, uint64_t rows_per_chunk, uint32_t nchunks,
                            uint64_t *bv, uint64_t *chunk_counts, hipStream_t s);

hipError_t launch_chunk_scan(const uint64_t *counts, uint32_t nchunks, uint64_t *offsets, uint64_t *total,
                             hipStream_t s);

// MODE 0: row indexes (OutT = uint64_t); MODE 1: values (u8 -> uint32_t, i32 -> int32_t)
template <typename T, typename OutT, int MODE>
hipError_t launch_expand(const uint64_t *bv, const T *in, uint64_t n, uint64_t rows_per_chunk, uint32_t nchunks,
                         const uint64_t *chunk_off, OutT *out, uint64_t cap, hipStream_t s);

hipError_t launch_sum(const uint64_t *v, uint32_t n, uint64_t *out, hipStream_t s);

}  // namespace scan
}  // namespace sgxamd
