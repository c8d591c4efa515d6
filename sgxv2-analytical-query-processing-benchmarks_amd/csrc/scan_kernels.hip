// HIP kernels of the MI355X predicate column scan (gfx950, wave64).
//
// Replaces the AVX-512 loops of Scan-Micro-Benchmarks/shared_libraries/SimdScan/src/SIMD512.cpp:
//   count            :7-32    -> k_predicate<T, false>  (chunk counts, then a sum)
//   bitvector_scan   :210-222 -> k_predicate<T, true>   (one 64-bit word per 64 rows)
//   implicit_index_scan(_self_alloc) :225-287 -> k_select<.., 0> (one pass, decoupled look-back)
//   scan             :91-150  -> k_select<.., 1>
// A 512-bit compare of the reference covers 64 uint8 codes; here one wave-wide
// 16-byte-per-lane load covers 1024 uint8 codes or 256 int32 values, and the
// predicate mask of 64 consecutive rows is assembled across 4 (u8) or 16 (i32)
// lanes with DPP row operations into exactly the reference's __mmask64 word layout.
// Index/value compaction is one pass (k_select): each chunk's bitvector stays in LDS,
// its output offset comes from a decoupled look-back over the chunks before it, and
// each wave's matches are staged in LDS and written coalesced (lane j of a wave
// writes output j).
#include "common.hpp"
#include "scan_internal.hpp"

namespace sgxamd {
namespace scan {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / kWave;
constexpr int kUnroll = 4;

template <typename T>
__device__ __forceinline__ uint32_t match_mask(const uint4 &q, T lo, T hi, uint32_t valid);

// 16 uint8 codes -> 16-bit mask (unsigned compare, _mm512_cmpge/le_epu8_mask), on packed
// 16-bit halves: pair k holds codes k and k + 8 (one v_perm_b32 from words k/4 and
// k/4 + 2), b + 256 - lo has bit 8 set iff b >= lo and hi + 256 - b iff b <= hi (both
// in [1, 511]), so (b + 256 - lo) & (hi + 256 - b) & 0x100 is the predicate of code k,
// and of code k + 8 at bit 24.  The eight pairs' flags are OR-ed in at bits 8 + k /
// 24 + k (v_lshl_or_b32) and one v_perm_b32 takes bytes 1 and 3: 5 VALU per 2 codes,
// against 3 VALU (two SGPR-writing compares and a select) + 1 SALU per code before.
typedef unsigned short u16x2_t __attribute__((ext_vector_type(2)));
template <>
__device__ __forceinline__ uint32_t match_mask<uint8_t>(const uint4 &q, uint8_t lo, uint8_t hi, uint32_t valid) {
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
    const unsigned short c1 = (unsigned short)(256u - lo), c2 = (unsigned short)(256u + hi);
    const u16x2_t vc1 = {c1, c1}, vc2 = {c2, c2};
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint32_t sel = 0x0c000c00u | ((4u + (k & 3)) << 16) | (uint32_t)(k & 3);
        const u16x2_t p = __builtin_bit_cast(u16x2_t, __builtin_amdgcn_perm(w[2 + (k >> 2)], w[k >> 2], sel));
        const uint32_t t = __builtin_bit_cast(uint32_t, p + vc1);
        const uint32_t u = __builtin_bit_cast(uint32_t, vc2 - p);
        const uint32_t f = __builtin_amdgcn_bitop3_b32(t, u, 0x01000100u, 0x80);  // t & u & mask
        if (k == 0) acc = f;
        else  // one v_lshl_or_b32 (left to itself the compiler shifts, then masks, then ORs)
            asm("v_lshl_or_b32 %0, %1, %2, %3" : "=v"(acc) : "v"(f), "i"(k), "v"(acc));
    }
    return __builtin_amdgcn_perm(0u, acc, 0x0c0c0301u) & valid;
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

// OR of x over each group of LPW consecutive lanes (LPW = 4, 8 or 16; the groups'
// bit fields do not overlap, so OR = sum) with DPP row operations on the VALU (no LDS
// round trips): quad_perm [1,0,3,2] and [2,3,0,1], then inside each 16-lane row
// row_ror:4 + row_ror:8 (LPW 16), or the neighbouring quad of the same 8-lane group
// (row_ror:4 reads lane i-4, row_ror:12 lane i+4; LPW 8).  Every lane of a group
// ends with the group's full word.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, true);
}
template <uint32_t LPW>
__device__ __forceinline__ uint64_t group_or(uint64_t x) {
    static_assert(LPW == 4 || LPW == 8 || LPW == 16, "lanes per 64-row word");
    uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    lo |= dpp_u32<0xB1>(lo);
    hi |= dpp_u32<0xB1>(hi);
    lo |= dpp_u32<0x4E>(lo);
    hi |= dpp_u32<0x4E>(hi);
    if (LPW == 8) {
        const bool upper = (__lane_id() & 4u) != 0;  // quad 1 or 3 of the row: partner is i-4
        const uint32_t plo_a = dpp_u32<0x124>(lo), phi_a = dpp_u32<0x124>(hi);
        const uint32_t plo_b = dpp_u32<0x12C>(lo), phi_b = dpp_u32<0x12C>(hi);
        lo |= upper ? plo_a : plo_b;
        hi |= upper ? phi_a : phi_b;
    }
    if (LPW == 16) {
        lo |= dpp_u32<0x124>(lo);
        hi |= dpp_u32<0x124>(hi);
        lo |= dpp_u32<0x128>(lo);
        hi |= dpp_u32<0x128>(hi);
    }
    return (uint64_t)lo | ((uint64_t)hi << 32);
}

// Count (WRITE=false) or bitvector + count (WRITE=true) of one chunk per workgroup.
// rows_per_chunk is a multiple of kWaves * 64 * V * kUnroll.
// SUM=true accumulates the matching values instead of counting them (SIMD512::sum).
//
// The block iterations that lie wholly inside the chunk run software-pipelined over
// two register sets: iteration i+1's loads are issued before iteration i's bitvector
// stores.  gfx950 retires loads and stores through one in-order vmcnt, so a wait for a
// load also waits for every older store; issued in this order, the wait for i+1's
// loads never waits for i's stores.  Loads are raw buffer loads over the chunk (one
// 32-bit lane offset + a uniform offset; the prefetch past the last iteration reads
// 0 from the bounds check and is not used).  A ragged chunk end (only the last chunk
// of a column) takes the element-wise tail path.
template <typename T, bool WRITE, bool SUM>
struct PredicateTile {
    static constexpr uint32_t V = 16 / sizeof(T);  // rows per lane per load
    static constexpr uint32_t LPW = 64 / V;        // lanes per 64-row word
    static constexpr uint32_t FULL = (1u << V) - 1u;
    static constexpr uint64_t STEP = (uint64_t)kWaves * 64 * V;  // rows per block per load round

    // masks, counts (or sums) and bitvector words of kUnroll loads starting at row `base`.
    // FULL_TILE: every row is inside the column, and all LPW lanes of a group store
    // their (identical) word — no branch around the store, so the compiler's vmcnt
    // accounting sees a fixed number of stores between the prefetch and its wait.
    template <bool FULL_TILE>
    static __device__ __forceinline__ void process(const uint4 (&q)[kUnroll], const uint32_t (&valid)[kUnroll],
                                                   uint64_t base, uint64_t r1, uint64_t nwords, T lo, T hi,
                                                   uint64_t *__restrict__ bv, uint64_t &count,
                                                   uint64_t *win = nullptr, uint64_t win_word = 0) {
        const uint32_t lane = __lane_id();
        if constexpr (WRITE && FULL_TILE && LPW == (uint32_t)kUnroll) {
            // one word per lane (u8 codes: kUnroll rounds x 16 words = 64 words per
            // wave): each round's word is assembled in its LPW-lane group, whose every
            // lane holds it, and lane j of a group keeps round j's word (a select, no
            // cross-lane move; the ds_bpermute pair per round that gathered them before
            // measured equal, 0.913-0.917 vs 0.919-0.922 ms on one box), so the wave
            // stores its 64 words with one 8-byte store per
            // lane — 16-word runs of the four rounds — instead of kUnroll stores in
            // which LPW lanes write the same word
            const uint32_t mine = lane % LPW;
            uint64_t w = 0;
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const uint32_t m = match_mask<T>(q[u], lo, hi, valid[u]);
                count += __popc(m);
                const uint64_t x = group_or<LPW>((uint64_t)m << (V * (lane % LPW)));
                if (mine == (uint32_t)u) w = x;
            }
            const uint64_t word = (base + mine * STEP) / 64 + lane / LPW;
            if (win) {  // staged in the workgroup's LDS window (k_predicate flushes it)
                win[word - win_word] = w;
                return;
            }
            // non-temporal: 0.957 vs 0.986 ms at 2^32 codes (the redundant-lane stores of
            // the loop below measured 20 % slower non-temporal)
            __builtin_nontemporal_store(w, bv + word);
            return;
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const uint32_t m = match_mask<T>(q[u], lo, hi, valid[u]);
            if (SUM) count += match_sum<T>(q[u], m);
            else count += __popc(m);
            if (WRITE) {
                const uint64_t x = group_or<LPW>((uint64_t)m << (V * (lane % LPW)));
                const uint64_t word = (base + u * STEP) / 64 + lane / LPW;
                // (a non-temporal word store measured 20 % slower, one lane per group
                // storing 2 % slower)
                if (FULL_TILE && win) {  // staged in the workgroup's LDS window
                    if ((lane % LPW) == 0) win[word - win_word] = x;
                } else if (FULL_TILE) bv[word] = x;
                else if ((lane % LPW) == 0 && word < nwords && (base + u * STEP) < r1) bv[word] = x;
            }
        }
    }
};

#ifndef SGXAMD_BV_BURST
#define SGXAMD_BV_BURST 1
#endif
#ifndef SGXAMD_BV_I32
#define SGXAMD_BV_I32 1
#endif
template <typename T, bool WRITE, bool SUM = false>
__global__ __launch_bounds__(kBlock) void k_predicate(const T *__restrict__ in, uint64_t n, T lo, T hi,
                                                      uint64_t rows_per_chunk, uint64_t *__restrict__ bv,
                                                      uint64_t *__restrict__ chunk_counts) {
    using PT = PredicateTile<T, WRITE, SUM>;
    constexpr uint32_t V = PT::V, FULL = PT::FULL;
    constexpr uint64_t STEP = PT::STEP;
    constexpr uint64_t ITER = STEP * kUnroll;  // rows per block iteration
    __shared__ uint64_t red[kWaves];
    // bitvectors: the words of BW block iterations are staged in LDS and written in one
    // burst per window (16-B non-temporal stores, consecutive lanes on consecutive
    // addresses) instead of one store per wave and iteration between the column's
    // reads.  uint8 at 2^32 codes, 1 %, on one box (profiles/r03q9_bitvector_window_ab.log):
    // direct stores 0.92 ms; windows of 8 / 16 / 32 / 40 / 64 / 72 iterations 0.90 /
    // 0.89 / 0.83 / 0.77 / 0.74 / 0.76 ms (64: 128 KiB of LDS, one workgroup per CU; with
    // 1,024 or 4,096 workgroups 0.75-0.76 / 0.73); int32 2^30: 0.765-0.776 -> 0.748-0.759
    // with 64 iterations (32 KiB), 0.704-0.713 with 128 (64 KiB: a 2^30-row chunk in one
    // window; profiles/r03q12_wide_bitvector_window_ab.log)
    constexpr bool BURST = WRITE && SGXAMD_BV_BURST && (SGXAMD_BV_I32 || PT::LPW == (uint32_t)kUnroll);
#ifndef SGXAMD_BV_WIN
#define SGXAMD_BV_WIN 64
#endif
#ifndef SGXAMD_BV_WIN_WIDE
#define SGXAMD_BV_WIN_WIDE 128
#endif
    constexpr uint32_t BW = sizeof(T) == 1 ? SGXAMD_BV_WIN : SGXAMD_BV_WIN_WIDE;  // iterations (16/32-bit codes)
    constexpr uint32_t WIN = BURST ? BW * (uint32_t)(ITER / 64) : 1;
    __shared__ uint64_t win[WIN];
    const uint32_t lane = __lane_id(), wave = threadIdx.x / kWave;
    const uint64_t r0 = (uint64_t)blockIdx.x * rows_per_chunk;
    const uint64_t r1 = (r0 + rows_per_chunk < n) ? r0 + rows_per_chunk : n;
    const uint64_t nwords = (n + 63) / 64;
    const uint64_t nfull = (r1 - r0) / ITER;
    const uint64_t full_end = r0 + nfull * ITER;
    uint64_t count = 0;
    if (nfull > 0) {
        // chunks hold far fewer than 2^32 bytes (geometry(): n / 2048 rows)
        const __amdgpu_buffer_rsrc_t rs = make_rsrc(in + r0, (uint32_t)((full_end - r0) * sizeof(T)));
        const uint32_t voff = (uint32_t)(((uint64_t)wave * 64 * V + (uint64_t)lane * V) * sizeof(T));
        uint32_t valid[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) valid[u] = FULL;
        uint4 qa[kUnroll], qb[kUnroll];
        auto load = [&](uint4(&q)[kUnroll], uint64_t it) {
#pragma unroll
            for (int u = 0; u < kUnroll; ++u)
                q[u] = buf_ld_nt_u128(rs, voff, (uint32_t)((it * ITER + u * STEP) * sizeof(T)));
            __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of the stores that follow
        };
        // an empty asm that reads a register set forces its wait at that point, in
        // straight-line code right after the other set's prefetch (otherwise the
        // compiler's wait analysis merges the loop back-edge into a vmcnt(0))
        auto wait_for = [](const uint4(&q)[kUnroll]) {
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) asm volatile("" ::"v"(q[u].x), "v"(q[u].y), "v"(q[u].z), "v"(q[u].w));
        };
        const uint64_t wbase = r0 + (uint64_t)wave * 64 * V;
        uint64_t *const wp = BURST ? win : nullptr;
        const auto win_word = [&](uint64_t it) { return (r0 + (it / BW) * BW * ITER) / 64; };
        // after iteration it: a full window (or the last iteration) goes out in one burst
        const auto flush = [&](uint64_t it) {
            if constexpr (BURST) {
                if ((it + 1) % BW != 0 && it + 1 != nfull) return;
                __syncthreads();
                typedef unsigned long long u64x2_t __attribute__((ext_vector_type(2)));
                const uint32_t nw = (uint32_t)(it % BW + 1) * (uint32_t)(ITER / 64);
                u64x2_t *dst = reinterpret_cast<u64x2_t *>(bv + win_word(it));
                const u64x2_t *src = reinterpret_cast<const u64x2_t *>(win);
                for (uint32_t i = threadIdx.x; i < nw / 2; i += kBlock) __builtin_nontemporal_store(src[i], dst + i);
                __syncthreads();
            }
        };
        // iterations in pairs, no branch between a prefetch and its wait (LLVM would sink
        // a prefetch whose result is dead on an early-exit path below the next stores)
        load(qa, 0);
        load(qb, 1);
        wait_for(qa);
        const uint64_t npairs = nfull / 2;
        for (uint64_t p = 0; p < npairs; ++p) {
            const uint64_t it = 2 * p;
            PT::template process<true>(qa, valid, wbase + it * ITER, r1, nwords, lo, hi, bv, count, wp, win_word(it));
            load(qa, it + 2);
            wait_for(qb);
            PT::template process<true>(qb, valid, wbase + (it + 1) * ITER, r1, nwords, lo, hi, bv, count, wp,
                                       win_word(it + 1));
            flush(it + 1);
            load(qb, it + 3);
            wait_for(qa);
        }
        if (nfull & 1) {
            PT::template process<true>(qa, valid, wbase + (nfull - 1) * ITER, r1, nwords, lo, hi, bv, count, wp,
                                       win_word(nfull - 1));
            flush(nfull - 1);
        }
    }
    // ragged end of the last chunk: fewer than ITER rows, element loads at the very end
    for (uint64_t base = full_end + (uint64_t)wave * 64 * V; base < r1; base += ITER) {
        uint4 q[kUnroll];
        uint32_t valid[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const uint64_t row = base + u * STEP + (uint64_t)lane * V;
            if (row + V <= r1) {
                q[u] = ld_nt(reinterpret_cast<const uint4 *>(in + row));
                valid[u] = FULL;
            } else if (row < r1) {  // element loads packed like a uint4
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
        PT::template process<false>(q, valid, base, r1, nwords, lo, hi, bv, count);
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

// LDS writes of a wave made visible to the other lanes of the same wave (no block
// barrier: the staging area below is private to its wave).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// SIMD512::explicit_index_scan (SIMD512.cpp:152-208) gathers the matches of row r from
// the u64 index vector index_compressed[i + j] (block i = r / 64, sub-block j = (r % 64) / 8),
// lane r % 8: entry 8 * (r / 64 + (r % 64) / 8) + r % 8, restated as written.
__device__ __forceinline__ uint64_t explicit_pos(uint64_t r) { return 8 * (r / 64 + (r % 64) / 8) + r % 8; }

// Output value of a selected row: its index (MODE 0), value (1), dictionary value (2) or
// explicit index entry (3; aux = the index array of aux_len entries, an out-of-range
// entry reads 0 and sets bit 2 of *err).
template <typename T, typename OutT, int MODE>
__device__ __forceinline__ OutT select_value(uint64_t row, const T *__restrict__ in, const int64_t *__restrict__ aux,
                                             uint64_t aux_len, uint32_t *err) {
    if constexpr (MODE == 0) return (OutT)row;
    else if constexpr (MODE == 1) return (OutT)in[row];
    else if constexpr (MODE == 2) return (OutT)aux[in[row]];
    else {
        const uint64_t q = explicit_pos(row);
        if (q < aux_len) return (OutT)aux[q];
        atomicOr(err, 2u);
        return (OutT)0;
    }
}

constexpr uint32_t kStage = 1024;  // staged outputs per wave and round (u32 row offsets, 4 KiB)

// ------------------------------------------------------- one-pass selection ---
// Index / value / dictionary output in ONE pass over the column (implicit_index_scan,
// scan and dict_scan_* of SIMD512.cpp:91-150, 251-287, 289-629): the column is read
// once and the outputs written once; the bitvector never leaves LDS.
//
// Chunks of kSelChunk rows are claimed in order through a ticket counter, so every
// chunk below a workgroup's own has been claimed by a workgroup that is already
// running.  Per chunk:
//   1. predicate over the chunk into an LDS bitvector (one 64-row word per 64 rows,
//      assembled across the LPW lanes of a 64-row group as in k_predicate) + count;
//   2. decoupled look-back by the first wave (common.hpp lookback_exclusive): the
//      chunk's count is published at once, the predecessors are read 64 at a time
//      back to the nearest inclusive prefix, and the chunk's own inclusive prefix is
//      published; a predecessor that has not counted yet is polled again — it is
//      already running, so the wait ends;
//   3. the LDS bitvector expanded at the chunk's exclusive prefix: each wave expands a
//      contiguous quarter of the words (one block barrier for the quarters' offsets,
//      1.77 vs 1.82 ms at the uint8 10 % shape with the waves interleaved per 64-word
//      step and a barrier per step), 64 words (4096 rows) per step, one word per lane;
//      a lane writes the row offsets of
//      its set bits into the wave's LDS staging area at its exclusive word-popcount
//      prefix, then lane j writes the wave's j-th, (j+64)-th, ... output (every store
//      instruction covers 64 consecutive output slots; dense steps stage in rounds of
//      kStage).
// The chunk that ends the column writes the total.
constexpr uint32_t kSelChunk = 65536;  // rows per chunk of 32-bit values (8 KiB LDS bitvector)
// uint16 codes take 131,072 rows per chunk (the same 256 KiB of input)
// (uint8: 131,072 rows, 16 KiB of LDS bitvector, five workgroups per CU: 1.77 ms at the
// reference's 2^32-code 10 % shape against 1.81 with 65,536 and 1.97 with 262,144 rows)
template <typename T>
constexpr uint32_t sel_chunk() { return sizeof(T) == 1 ? 2 * kSelChunk : kSelChunk * (uint32_t)(4 / sizeof(T)); }

#ifndef SGXAMD_SEL_ABLATE
#define SGXAMD_SEL_ABLATE 0
#endif
template <typename T, typename OutT, int MODE>
__global__ __launch_bounds__(kBlock) void k_select(const T *__restrict__ in, uint64_t n, T lo, T hi,
                                                   uint32_t *__restrict__ ticket, uint64_t *__restrict__ status,
                                                   OutT *__restrict__ out, uint64_t cap,
                                                   const int64_t *__restrict__ dict, uint64_t aux_len,
                                                   uint64_t *__restrict__ total) {
    constexpr uint32_t V = 16 / sizeof(T), LPW = 64 / V, FULL = (1u << V) - 1u;
    constexpr uint32_t CH = sel_chunk<T>(), NWORD = CH / 64;
    constexpr int U = 8;  // 16-B loads in flight per lane (uint8: 4 or 16 measured equal)
    __shared__ uint64_t bits[NWORD];
    constexpr uint32_t STG = kStage;
    __shared__ uint32_t stage_s[kWaves][STG];
    __shared__ uint32_t wtot_s[kWaves];
    __shared__ uint64_t red[kWaves];
    __shared__ uint32_t chunk_s;
    __shared__ uint64_t excl_s;
    const uint32_t lane = __lane_id(), wave = threadIdx.x / kWave;
    if (threadIdx.x == 0) chunk_s = atomicAdd(ticket, 1u);
    __syncthreads();
    // uniform by construction; readfirstlane keeps the chunk's buffer resource in SGPRs
    // (read from LDS it stayed a VGPR value, and every buffer load became a waterfall loop)
    const uint32_t c = (uint32_t)__builtin_amdgcn_readfirstlane((int)chunk_s);
    const uint64_t r0 = (uint64_t)c * CH;
    if (r0 >= n) return;  // (the grid has exactly one workgroup per chunk)
    const uint64_t r1 = min<uint64_t>(r0 + CH, n);
    const uint32_t nw = (uint32_t)((r1 - r0 + 63) / 64);

    // 1. predicate -> LDS bitvector + count
    uint64_t count = 0;
    constexpr uint32_t STEP = kWaves * 64 * V;  // rows per block per load round
    static_assert(CH % (U * STEP) == 0, "whole load rounds per chunk");
    if (r1 - r0 == CH) {
        // a whole chunk (every chunk but the column's last): raw buffer loads over the
        // chunk, no per-load bounds branches
        const __amdgpu_buffer_rsrc_t rs = make_rsrc(in + r0, CH * (uint32_t)sizeof(T));
        const uint32_t voff = (wave * 64 * V + lane * V) * (uint32_t)sizeof(T);
        for (uint32_t it = 0; it < CH / (U * STEP); ++it) {
            uint4 q[U];
#pragma unroll
            for (int u = 0; u < U; ++u) q[u] = buf_ld_nt_u128(rs, voff, (it * U + u) * STEP * (uint32_t)sizeof(T));
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t m = match_mask<T>(q[u], lo, hi, FULL);
                count += __popc(m);
                const uint64_t x = group_or<LPW>((uint64_t)m << (V * (lane % LPW)));
                const uint32_t row = (it * U + u) * STEP + wave * 64 * V + lane * V;  // chunk-relative
                if ((lane % LPW) == 0) bits[row / 64] = x;
            }
        }
    } else
    // wave-uniform loop: lanes past r1 read nothing and contribute empty masks, so every
    // lane takes part in the DPP word assembly
    for (uint64_t wbase = r0 + (uint64_t)wave * 64 * V; wbase < r1; wbase += U * STEP) {
        uint4 q[U];
        uint32_t valid[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t row = wbase + (uint64_t)u * STEP + (uint64_t)lane * V;
            if (row + V <= r1) {
                q[u] = ld_nt(reinterpret_cast<const uint4 *>(in + row));
                valid[u] = FULL;
            } else if (row < r1) {
                uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
                for (uint32_t j = 0; j < V; ++j) {
                    constexpr uint32_t B = 8 * sizeof(T);
                    constexpr uint32_t VM = B == 32 ? 0xFFFFFFFFu : ((1u << B) - 1u);
                    const uint32_t val = (row + j < r1) ? (uint32_t)in[row + j] : 0u;
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
        for (int u = 0; u < U; ++u) {
            const uint32_t m = match_mask<T>(q[u], lo, hi, valid[u]);
            count += __popc(m);
            const uint64_t x = group_or<LPW>((uint64_t)m << (V * (lane % LPW)));
            const uint64_t row = wbase + (uint64_t)u * STEP + (uint64_t)lane * V;
            // the group's first lane stores the word of its 64 rows (every word of the
            // chunk below nw has a first lane inside the chunk)
            if ((lane % LPW) == 0 && row < r1) bits[(row - r0) / 64] = x;
        }
    }
    count = wave_sum_u64(count);
    if (lane == 0) red[wave] = count;
    __syncthreads();
    uint64_t agg = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) agg += red[w];

    // 2. decoupled look-back (first wave)
    if (wave == 0) {
        const uint64_t excl = lookback_exclusive(status, c, agg, &ticket[1]);
        if (lane == 0) excl_s = excl;
    }
    __syncthreads();
    const uint64_t excl = excl_s;
    if (r1 == n && threadIdx.x == 0) *total = excl + agg;

    // 3. expand the LDS bitvector at the chunk's prefix
#if SGXAMD_SEL_ABLATE == 1  // development ablation: no expand
    return;
#endif
    // each wave expands a contiguous quarter of the chunk's words on its own (one block
    // barrier per chunk for the quarters' output offsets, wave-level syncs after it)
    const uint32_t qw = (nw + kWaves - 1) / kWaves;
    const uint32_t w0 = min(nw, wave * qw), w1 = min(nw, w0 + qw);
    uint32_t qc = 0;
    for (uint32_t wi = w0 + lane; wi < w1; wi += 64) qc += __popcll(bits[wi]);
    qc = wave_sum_u32(qc);
    if (lane == 0) wtot_s[wave] = qc;
    __syncthreads();
    uint64_t woff = excl;
    for (int w = 0; w < (int)wave; ++w) woff += wtot_s[w];
    uint32_t *stage = stage_s[wave];
    for (uint32_t wb = w0; wb < w1; wb += 64) {
        const uint32_t wi = wb + lane;
        const uint64_t x = wi < w1 ? bits[wi] : 0ull;
        const uint32_t cnt = __popcll(x);
        const uint32_t incl = wave_incl_scan_dpp_u32(cnt);
        const uint32_t ex = incl - cnt;
        const uint32_t wtot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        const uint64_t row0 = r0 + (uint64_t)wb * 64;
        if (wtot <= STG) {
            // the step's matches fit the staging area (every step below 1/4 density):
            // no staging rounds, and each 32-bit half of the word in its own bit loop
            // (v_ffbl_b32 + y &= y - 1 + one LDS store per set bit)
            // the set bits leave in groups of four (two ds_write2_b32 per group) after
            // a single and a pair that make the rest a multiple of four: a lane's loop
            // runs popcount / 4 times, and no write lands past its own slots (the
            // next lane's first slot is taken in the first round)
            uint32_t p = ex;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                uint32_t y = (uint32_t)(x >> (32 * h));
                const uint32_t base = lane * 64 + 32 * h;
                const uint32_t ch = __popc(y);
                if (ch & 1u) {
                    stage[p++] = base + (uint32_t)__builtin_ctz(y);
                    y &= y - 1;
                }
                if (ch & 2u) {
                    const uint32_t a = (uint32_t)__builtin_ctz(y);
                    y &= y - 1;
                    const uint32_t b = (uint32_t)__builtin_ctz(y);
                    y &= y - 1;
                    stage[p] = base + a;
                    stage[p + 1] = base + b;
                    p += 2;
                }
                while (y) {
                    uint32_t s[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        s[j] = base + (uint32_t)__builtin_ctz(y);
                        y &= y - 1;
                    }
#pragma unroll
                    for (int j = 0; j < 4; ++j) stage[p + j] = s[j];
                    p += 4;
                }
            }
            wave_lds_sync();
            // four staged offsets read per lane before their stores (one LDS wait per
            // four outputs instead of one per output)
            const bool fits = woff + wtot <= cap;
            for (uint32_t m0 = 0; m0 < wtot; m0 += 4 * 64) {
                uint32_t s[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) s[j] = stage[(m0 + j * 64 + lane) & (STG - 1)];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t m = m0 + j * 64 + lane;
                    const uint64_t o = woff + m;
                    if (m < wtot && (fits || o < cap) && SGXAMD_SEL_ABLATE != 2) {
                        const OutT v = select_value<T, OutT, MODE>(row0 + s[j], in, dict, aux_len, &ticket[1]);
                        __builtin_nontemporal_store(v, out + o);
                    }
                }
            }
            wave_lds_sync();
            woff += wtot;
            continue;
        }
        for (uint32_t s0 = 0; s0 < wtot; s0 += STG) {
            const uint32_t s1 = s0 + STG;
            if (ex < s1 && incl > s0) {
                uint64_t y = x;
                uint32_t p = ex;
                while (y) {
                    const uint32_t bit = (uint32_t)__builtin_ctzll(y);
                    y &= y - 1;
                    if (p >= s0 && p < s1) stage[p - s0] = lane * 64 + bit;
                    ++p;
                }
            }
            wave_lds_sync();
            const uint32_t nr = min(STG, wtot - s0);
            for (uint32_t m = lane; m < nr; m += 64) {
                const uint64_t row = row0 + stage[m];
                const uint64_t o = woff + s0 + m;
                if (o < cap && SGXAMD_SEL_ABLATE != 2) {
                    // non-temporal: the outputs are not re-read here (4 % faster than plain
                    // stores at C3; each lane storing its own matches instead of the staged,
                    // coalesced stores: 3.5 vs 1.8 ms at the uint8 10 % shape)
                    const OutT v = select_value<T, OutT, MODE>(row, in, dict, aux_len, &ticket[1]);
                    __builtin_nontemporal_store(v, out + o);
                }
            }
            wave_lds_sync();
        }
        woff += wtot;
    }
}

uint64_t select_chunks(uint64_t n) { return (n + kSelChunk - 1) / kSelChunk; }  // bound for every T

template <typename T, typename OutT, int MODE>
hipError_t launch_select(const T *in, uint64_t n, T lo, T hi, uint32_t *ticket, uint64_t *status, OutT *out,
                         uint64_t cap, uint64_t *total, hipStream_t s, const int64_t *dict, uint64_t aux_len) {
    const uint64_t nchunks = (n + sel_chunk<T>() - 1) / sel_chunk<T>();
    if (nchunks == 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(ticket, 0, 2 * sizeof(uint32_t), s);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(status, 0, nchunks * sizeof(uint64_t), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_select<T, OutT, MODE>), dim3((uint32_t)nchunks), dim3(kBlock), 0, s, in, n, lo, hi, ticket,
                       status, out, cap, dict, aux_len, total);
    return hipGetLastError();
}

#define SGX_SELECT_INST(T, OutT, MODE)                                                                         \
    template hipError_t launch_select<T, OutT, MODE>(const T *, uint64_t, T, T, uint32_t *, uint64_t *, OutT *, \
                                                     uint64_t, uint64_t *, hipStream_t, const int64_t *, \
                                                     uint64_t);
SGX_SELECT_INST(uint8_t, uint64_t, 0)
SGX_SELECT_INST(int32_t, uint64_t, 0)
SGX_SELECT_INST(uint8_t, uint32_t, 1)
SGX_SELECT_INST(int32_t, int32_t, 1)
SGX_SELECT_INST(uint8_t, uint64_t, 1)  // named by run<T, uint64_t>, never called
SGX_SELECT_INST(int32_t, uint64_t, 1)
SGX_SELECT_INST(uint8_t, int64_t, 2)
SGX_SELECT_INST(uint16_t, int64_t, 2)
SGX_SELECT_INST(uint32_t, int64_t, 2)
SGX_SELECT_INST(uint8_t, uint64_t, 3)
#undef SGX_SELECT_INST

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
