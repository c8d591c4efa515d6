// HIP kernels of the MI355X predicate column scan (gfx950, wave64).
//
// Replaces the AVX-512 loops of Scan-Micro-Benchmarks/shared_libraries/SimdScan/src/SIMD512.cpp:
//   count            :7-32    -> k_predicate<T, false>  (chunk counts, then a sum)
//   bitvector_scan   :210-222 -> k_predicate<T, true>   (one 64-bit word per 64 rows)
//   implicit_index_scan(_self_alloc) :225-287 -> k_predicate<T, true> + k_chunk_scan + k_expand<.., kIndex>
//   scan             :91-150  -> same pipeline, k_expand<.., kValue>
// A 512-bit compare of the reference covers 64 uint8 codes; here one wave-wide
// 16-byte-per-lane load covers 1024 uint8 codes or 256 int32 values, and the
// predicate mask of 64 consecutive rows is assembled across 4 (u8) or 16 (i32)
// lanes with xor-shuffles into exactly the reference's __mmask64 word layout.
// Index/value compaction is two-phase without inter-workgroup waiting: the
// bitvector pass also emits one match count per chunk, a one-block scan turns
// those into chunk output offsets, and the expand pass reads only the bitvector
// (n/8 bytes) and writes the outputs coalesced (lane j of a wave writes output j).
#include "common.hpp"
#include "scan_internal.hpp"

namespace sgxamd {
namespace scan {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / kWave;
constexpr int kUnroll = 4;

template <typename T>
__device__ __forceinline__ uint32_t match_mask(const uint4 &q, T lo, T hi, uint32_t valid);

// 16 uint8 codes -> 16-bit mask (unsigned compare, _mm512_cmpge/le_epu8_mask).
template <>
__device__ __forceinline__ uint32_t match_mask<uint8_t>(const uint4 &q, uint8_t lo, uint8_t hi, uint32_t valid) {
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
    uint32_t m = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const uint32_t b = __builtin_amdgcn_ubfe(w[j >> 2], (j & 3) * 8, 8);
        m |= (uint32_t)(b >= lo && b <= hi) << j;
    }
    return m & valid;
}

// 4 int32 values -> 4-bit mask (signed compare).
template <>
__device__ __forceinline__ uint32_t match_mask<int32_t>(const uint4 &q, int32_t lo, int32_t hi, uint32_t valid) {
    const int32_t v0 = (int32_t)q.x, v1 = (int32_t)q.y, v2 = (int32_t)q.z, v3 = (int32_t)q.w;
    uint32_t m = (uint32_t)(v0 >= lo && v0 <= hi) | ((uint32_t)(v1 >= lo && v1 <= hi) << 1) |
                 ((uint32_t)(v2 >= lo && v2 <= hi) << 2) | ((uint32_t)(v3 >= lo && v3 <= hi) << 3);
    return m & valid;
}

// 8 uint16 dictionary codes -> 8-bit mask (unsigned, _mm512_cmpge/le_epu16_mask).
template <>
__device__ __forceinline__ uint32_t match_mask<uint16_t>(const uint4 &q, uint16_t lo, uint16_t hi, uint32_t valid) {
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
    uint32_t m = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint32_t c = __builtin_amdgcn_ubfe(w[j >> 1], (j & 1) * 16, 16);
        m |= (uint32_t)(c >= lo && c <= hi) << j;
    }
    return m & valid;
}

// 4 uint32 dictionary codes -> 4-bit mask (unsigned, _mm512_cmpge/le_epu32_mask).
template <>
__device__ __forceinline__ uint32_t match_mask<uint32_t>(const uint4 &q, uint32_t lo, uint32_t hi, uint32_t valid) {
    uint32_t m = (uint32_t)(q.x >= lo && q.x <= hi) | ((uint32_t)(q.y >= lo && q.y <= hi) << 1) |
                 ((uint32_t)(q.z >= lo && q.z <= hi) << 2) | ((uint32_t)(q.w >= lo && q.w <= hi) << 3);
    return m & valid;
}

// Sum of the matching values of one 16-byte lane load (SIMD512::sum, u8 codes).
template <typename T>
__device__ __forceinline__ uint64_t match_sum(const uint4 &q, uint32_t m) {
    constexpr uint32_t V = 16 / sizeof(T), B = 8 * sizeof(T);
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
    uint64_t acc = 0;
#pragma unroll
    for (uint32_t j = 0; j < V; ++j) {
        const uint32_t v = B == 32 ? w[j] : __builtin_amdgcn_ubfe(w[(j * B) / 32], (j * B) % 32, B);
        acc += (m >> j) & 1u ? (uint64_t)v : 0ull;
    }
    return acc;
}

// Count (WRITE=false) or bitvector + count (WRITE=true) of one chunk per workgroup.
// rows_per_chunk is a multiple of kWaves * 64 * V * kUnroll.
// SUM=true accumulates the matching values instead of counting them (SIMD512::sum).
template <typename T, bool WRITE, bool SUM = false>
__global__ __launch_bounds__(kBlock) void k_predicate(const T *__restrict__ in, uint64_t n, T lo, T hi,
                                                      uint64_t rows_per_chunk, uint64_t *__restrict__ bv,
                                                      uint64_t *__restrict__ chunk_counts) {
    constexpr uint32_t V = 16 / sizeof(T);  // rows per lane per load
    constexpr uint32_t LPW = 64 / V;        // lanes per 64-row word
    constexpr uint32_t FULL = (1u << V) - 1u;
    __shared__ uint64_t red[kWaves];
    const uint32_t lane = __lane_id(), wave = threadIdx.x / kWave;
    const uint64_t r0 = (uint64_t)blockIdx.x * rows_per_chunk;
    const uint64_t r1 = (r0 + rows_per_chunk < n) ? r0 + rows_per_chunk : n;
    const uint64_t nwords = (n + 63) / 64;
    constexpr uint64_t STEP = (uint64_t)kWaves * 64 * V;  // rows per block per load round
    uint64_t count = 0;
    for (uint64_t base = r0 + (uint64_t)wave * 64 * V; base < r1; base += STEP * kUnroll) {
        uint4 q[kUnroll];
        uint32_t valid[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const uint64_t row = base + u * STEP + (uint64_t)lane * V;
            if (row + V <= r1) {
                q[u] = ld_nt(reinterpret_cast<const uint4 *>(in + row));
                valid[u] = FULL;
            } else if (row < r1) {  // ragged tail: element loads packed like a uint4
                uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
                for (uint32_t j = 0; j < V; ++j) {
                    const uint32_t val = (row + j < r1) ? (uint32_t)in[row + j] : 0u;
                    constexpr uint32_t B = 8 * sizeof(T);
                    constexpr uint32_t VM = B == 32 ? 0xFFFFFFFFu : ((1u << B) - 1u);
                    w[(j * B) / 32] |= (val & VM) << ((j * B) % 32);
                }
                q[u] = make_uint4(w[0], w[1], w[2], w[3]);
                valid[u] = (1u << (uint32_t)(r1 - row)) - 1u;
            } else {
                q[u] = make_uint4(0, 0, 0, 0);
                valid[u] = 0;
            }
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const uint32_t m = match_mask<T>(q[u], lo, hi, valid[u]);
            if (SUM) count += match_sum<T>(q[u], m);
            else count += __popc(m);
            if (WRITE) {
                uint64_t x = (uint64_t)m << (V * (lane % LPW));
#pragma unroll
                for (uint32_t off = 1; off < LPW; off <<= 1) x |= __shfl_xor(x, off, kWave);
                const uint64_t word = (base + u * STEP) / 64 + lane / LPW;
                if ((lane % LPW) == 0 && word < nwords && (base + u * STEP) < r1) bv[word] = x;
            }
        }
    }
    count = wave_sum_u64(count);
    if (lane == 0) red[wave] = count;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = 0;
        for (int w = 0; w < kWaves; ++w) t += red[w];
        chunk_counts[blockIdx.x] = t;
    }
}

template <typename T>
hipError_t launch_predicate(const T *in, uint64_t n, T lo, T hi, uint64_t rows_per_chunk, uint32_t nchunks,
                            uint64_t *bv, uint64_t *chunk_counts, hipStream_t s) {
    if (nchunks == 0) return hipSuccess;
    if (bv)
        hipLaunchKernelGGL((k_predicate<T, true>), dim3(nchunks), dim3(kBlock), 0, s, in, n, lo, hi, rows_per_chunk,
                           bv, chunk_counts);
    else
        hipLaunchKernelGGL((k_predicate<T, false>), dim3(nchunks), dim3(kBlock), 0, s, in, n, lo, hi,
                           rows_per_chunk, bv, chunk_counts);
    return hipGetLastError();
}

template hipError_t launch_predicate<uint8_t>(const uint8_t *, uint64_t, uint8_t, uint8_t, uint64_t, uint32_t,
                                              uint64_t *, uint64_t *, hipStream_t);
template hipError_t launch_predicate<uint16_t>(const uint16_t *, uint64_t, uint16_t, uint16_t, uint64_t, uint32_t,
                                               uint64_t *, uint64_t *, hipStream_t);
template hipError_t launch_predicate<uint32_t>(const uint32_t *, uint64_t, uint32_t, uint32_t, uint64_t, uint32_t,
                                               uint64_t *, uint64_t *, hipStream_t);

hipError_t launch_sum_u8(const uint8_t *in, uint64_t n, uint8_t lo, uint8_t hi, uint64_t rows_per_chunk,
                         uint32_t nchunks, uint64_t *chunk_sums, hipStream_t s) {
    if (nchunks == 0) return hipSuccess;
    hipLaunchKernelGGL((k_predicate<uint8_t, false, true>), dim3(nchunks), dim3(kBlock), 0, s, in, n, lo, hi,
                       rows_per_chunk, nullptr, chunk_sums);
    return hipGetLastError();
}
template hipError_t launch_predicate<int32_t>(const int32_t *, uint64_t, int32_t, int32_t, uint64_t, uint32_t,
                                              uint64_t *, uint64_t *, hipStream_t);

// One block: exclusive scan of the chunk counts -> chunk offsets, total in *total.
__global__ __launch_bounds__(1024) void k_chunk_scan(const uint64_t *__restrict__ counts, uint32_t nchunks,
                                                     uint64_t *__restrict__ offsets, uint64_t *__restrict__ total) {
    __shared__ uint64_t scratch[1024 / kWave + 1];
    uint64_t carry = 0;
    for (uint32_t b = 0; b < nchunks; b += 1024) {
        const uint32_t i = b + threadIdx.x;
        const uint64_t v = i < nchunks ? counts[i] : 0;
        uint64_t tot;
        const uint64_t ex = block_excl_scan_u64(v, scratch, &tot);
        if (i < nchunks) offsets[i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) *total = carry;
}

hipError_t launch_chunk_scan(const uint64_t *counts, uint32_t nchunks, uint64_t *offsets, uint64_t *total,
                             hipStream_t s) {
    hipLaunchKernelGGL(k_chunk_scan, dim3(1), dim3(1024), 0, s, counts, nchunks, offsets, total);
    return hipGetLastError();
}

// Position of the r-th set bit (0-based) of x (r < popcount(x)).
__device__ __forceinline__ uint32_t select_bit(uint64_t x, uint32_t r) {
    uint32_t pos = 0;
    uint32_t w = (uint32_t)x;
    uint32_t c = __popc(w);
    if (r >= c) {
        r -= c;
        w = (uint32_t)(x >> 32);
        pos = 32;
    }
#pragma unroll
    for (uint32_t half = 16; half >= 1; half >>= 1) {
        const uint32_t lowmask = (1u << half) - 1u;
        c = __popc(w & lowmask);
        if (r >= c) {
            r -= c;
            w >>= half;
            pos += half;
        }
    }
    return pos;
}

// Expand the bitvector of one chunk into row indexes (MODE 0), values (MODE 1) or
// dictionary-decoded values dict[code] (MODE 2, the dict_scan_* family).
// Waves take 64 words at a time; lane j of a wave writes the wave's j-th, (j+64)-th,
// ... output, locating its set bit by binary search over the wave's inclusive
// word-popcount prefix held in LDS.
template <typename T, typename OutT, int MODE>
__global__ __launch_bounds__(kBlock) void k_expand(const uint64_t *__restrict__ bv, const T *__restrict__ in,
                                                   uint64_t n, uint64_t rows_per_chunk,
                                                   const uint64_t *__restrict__ chunk_off, OutT *__restrict__ out,
                                                   uint64_t cap, const int64_t *__restrict__ dict) {
    __shared__ uint32_t incl_s[kWaves][64];
    __shared__ uint64_t word_s[kWaves][64];
    __shared__ uint32_t wtot_s[kWaves];
    const uint32_t lane = __lane_id(), wave = threadIdx.x / kWave;
    const uint64_t nwords = (n + 63) / 64;
    const uint64_t w0 = (uint64_t)blockIdx.x * (rows_per_chunk / 64);
    uint64_t w1 = w0 + rows_per_chunk / 64;
    if (w1 > nwords) w1 = nwords;
    uint64_t base = chunk_off[blockIdx.x];
    for (uint64_t wb = w0; wb < w1; wb += kWaves * 64) {
        const uint64_t wi = wb + (uint64_t)wave * 64 + lane;
        const uint64_t x = wi < w1 ? ld_nt(bv + wi) : 0ull;
        const uint32_t c = __popcll(x);
        const uint32_t incl = wave_incl_scan_u32(c);
        incl_s[wave][lane] = incl;
        word_s[wave][lane] = x;
        const uint32_t wtot = __shfl(incl, 63, kWave);
        if (lane == 0) wtot_s[wave] = wtot;
        __syncthreads();
        uint64_t woff = base;
        uint64_t all = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) {
            const uint32_t t = wtot_s[w];
            if (w < (int)wave) woff += t;
            all += t;
        }
        for (uint32_t m = lane; m < wtot; m += 64) {
            uint32_t lo = 0, hi = 63;  // smallest l with incl[l] > m
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (incl_s[wave][mid] > m) hi = mid; else lo = mid + 1;
            }
            const uint64_t xw = word_s[wave][lo];
            const uint32_t before = incl_s[wave][lo] - (uint32_t)__popcll(xw);
            const uint32_t bit = select_bit(xw, m - before);
            const uint64_t row = (wb + (uint64_t)wave * 64 + lo) * 64 + bit;
            const uint64_t o = woff + m;
            if (o < cap) {
                if (MODE == 0) out[o] = (OutT)row;
                else if (MODE == 1) out[o] = (OutT)in[row];
                else out[o] = (OutT)dict[in[row]];
            }
        }
        base += all;
        __syncthreads();
    }
}

template <typename T, typename OutT, int MODE>
hipError_t launch_expand(const uint64_t *bv, const T *in, uint64_t n, uint64_t rows_per_chunk, uint32_t nchunks,
                         const uint64_t *chunk_off, OutT *out, uint64_t cap, hipStream_t s, const int64_t *dict) {
    if (nchunks == 0) return hipSuccess;
    hipLaunchKernelGGL((k_expand<T, OutT, MODE>), dim3(nchunks), dim3(kBlock), 0, s, bv, in, n, rows_per_chunk,
                       chunk_off, out, cap, dict);
    return hipGetLastError();
}

template hipError_t launch_expand<uint8_t, uint64_t, 0>(const uint64_t *, const uint8_t *, uint64_t, uint64_t,
                                                        uint32_t, const uint64_t *, uint64_t *, uint64_t,
                                                        hipStream_t, const int64_t *);
template hipError_t launch_expand<int32_t, uint64_t, 0>(const uint64_t *, const int32_t *, uint64_t, uint64_t,
                                                        uint32_t, const uint64_t *, uint64_t *, uint64_t,
                                                        hipStream_t, const int64_t *);
template hipError_t launch_expand<uint8_t, uint32_t, 1>(const uint64_t *, const uint8_t *, uint64_t, uint64_t,
                                                        uint32_t, const uint64_t *, uint32_t *, uint64_t,
                                                        hipStream_t, const int64_t *);
template hipError_t launch_expand<int32_t, int32_t, 1>(const uint64_t *, const int32_t *, uint64_t, uint64_t,
                                                       uint32_t, const uint64_t *, int32_t *, uint64_t,
                                                       hipStream_t, const int64_t *);

template hipError_t launch_expand<uint8_t, int64_t, 2>(const uint64_t *, const uint8_t *, uint64_t, uint64_t,
                                                       uint32_t, const uint64_t *, int64_t *, uint64_t, hipStream_t,
                                                       const int64_t *);
template hipError_t launch_expand<uint16_t, int64_t, 2>(const uint64_t *, const uint16_t *, uint64_t, uint64_t,
                                                        uint32_t, const uint64_t *, int64_t *, uint64_t, hipStream_t,
                                                        const int64_t *);
template hipError_t launch_expand<uint32_t, int64_t, 2>(const uint64_t *, const uint32_t *, uint64_t, uint64_t,
                                                        uint32_t, const uint64_t *, int64_t *, uint64_t, hipStream_t,
                                                        const int64_t *);

// Dictionary code range of a predicate on values (dict_scan_* prologue,
// SIMD512.cpp:297-305): lo_idx = first i with dict[i] >= lo (else dict_size),
// hi_end = first j >= lo_idx with dict[j] > hi (else dict_size).  Two passes of
// atomicMin; range[0] / range[1] must be preset to dict_size.
__global__ __launch_bounds__(kBlock) void k_dict_low(const int64_t *__restrict__ dict, uint64_t n, int64_t lo,
                                                     unsigned long long *__restrict__ range) {
    for (uint64_t i = blockIdx.x * (uint64_t)kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock)
        if (dict[i] >= lo) atomicMin(&range[0], (unsigned long long)i);
}
__global__ __launch_bounds__(kBlock) void k_dict_high(const int64_t *__restrict__ dict, uint64_t n, int64_t hi,
                                                      unsigned long long *__restrict__ range) {
    const uint64_t lo_idx = range[0];
    for (uint64_t i = lo_idx + blockIdx.x * (uint64_t)kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock)
        if (dict[i] > hi) atomicMin(&range[1], (unsigned long long)i);
}

hipError_t launch_dict_range(const int64_t *dict, uint64_t n, int64_t lo, int64_t hi, uint64_t *range,
                             hipStream_t s) {
    uint64_t blocks = (n + kBlock - 1) / kBlock;
    if (blocks > 1024) blocks = 1024;
    if (blocks == 0) blocks = 1;
    auto *r = reinterpret_cast<unsigned long long *>(range);
    hipLaunchKernelGGL(k_dict_low, dim3((uint32_t)blocks), dim3(kBlock), 0, s, dict, n, lo, r);
    hipLaunchKernelGGL(k_dict_high, dim3((uint32_t)blocks), dim3(kBlock), 0, s, dict, n, hi, r);
    return hipGetLastError();
}

// Sum of chunk counts (count-only path).
__global__ __launch_bounds__(kBlock) void k_sum(const uint64_t *__restrict__ v, uint32_t n,
                                                uint64_t *__restrict__ out) {
    __shared__ uint64_t red[kWaves];
    uint64_t acc = 0;
    for (uint32_t i = threadIdx.x; i < n; i += kBlock) acc += v[i];
    acc = wave_sum_u64(acc);
    if (__lane_id() == 0) red[threadIdx.x / kWave] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = 0;
        for (int w = 0; w < kWaves; ++w) t += red[w];
        *out = t;
    }
}

hipError_t launch_sum(const uint64_t *v, uint32_t n, uint64_t *out, hipStream_t s) {
    hipLaunchKernelGGL(k_sum, dim3(1), dim3(kBlock), 0, s, v, n, out);
    return hipGetLastError();
}

}  // namespace scan
}  // namespace sgxamd
