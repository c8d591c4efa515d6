// Shared host/device helpers for the MI355X (gfx950) kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

namespace sgxamd {

constexpr int kWave = 64;  // CDNA wavefront width (never 32)

// ---------------------------------------------------------------- device ---

// Streaming (non-temporal) 16-B / 8-B accesses: once-touched HBM data.  On gfx950
// the nt load path reads ~10 % faster than the default policy for a pure stream
// (tools/bw_lab), and nt stores help the partition scatter's 128-B granules.
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld_nt(const uint4 *p) {
    const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t *>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint64_t ld_nt(const uint64_t *p) { return __builtin_nontemporal_load(p); }

// Bijection blockIdx -> work item that gives each of the 8 XCDs (blocks are dealt to
// XCDs round-robin by blockIdx) one contiguous run of the n items, so neighbouring
// segments — which share partially written output lines — meet in the same L2.
__device__ __forceinline__ uint32_t xcd_contiguous(uint32_t b, uint32_t n) {
    constexpr uint32_t X = 8;
    const uint32_t q = n / X, r = n % X, x = b % X, i = b / X;
    return x < r ? x * (q + 1) + i : r * (q + 1) + (x - r) * q + i;
}

// Raw buffer resource over [base, base + bytes) (gfx9 dword3 for untyped dword access).
// Loads through it take a 32-bit per-lane offset and a uniform SGPR offset, so a
// streaming loop keeps no 64-bit per-lane addresses live, and out-of-range lanes
// read 0 (the hardware bounds check) instead of needing a tail path.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void *base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, (int)bytes, 0x00020000);
}
typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
// non-temporal 8-byte buffer load (aux bit 1 = nt)
__device__ __forceinline__ uint64_t buf_ld_nt_u64(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    const u32x2_t v = __builtin_amdgcn_raw_buffer_load_b64(r, (int)voff, (int)soff, 2);
    return ((uint64_t)v.y << 32) | v.x;
}
// non-temporal 16-byte buffer load
__device__ __forceinline__ uint4 buf_ld_nt_u128(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, (int)soff, 2);
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st_nt(uint64_t *p, uint64_t v) { __builtin_nontemporal_store(v, p); }
__device__ __forceinline__ void st_nt(uint32_t *p, uint32_t v) { __builtin_nontemporal_store(v, p); }

// c ? a : b as one v_cndmask_b32 (the compiler otherwise turns a select between two
// LDS addresses into exec-masked branches); the condition is the wave's lane mask
__device__ __forceinline__ uint32_t vsel(bool c, uint32_t a, uint32_t b) {
    const uint64_t m = __builtin_amdgcn_ballot_w64(c);
    uint32_t r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(b), "v"(a), "s"(m));
    return r;
}

__device__ __forceinline__ uint64_t lanemask_lt() {
    const uint32_t lane = __lane_id();
    return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

__device__ __forceinline__ uint32_t popc64(uint64_t x) { return __popcll(x); }

// Sum of a 64-bit value over the wave (result valid in every lane).
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
    return v;
}

// Largest 32-bit value over the wave (every lane gets it).
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = max(v, (uint32_t)__shfl_xor(v, off, kWave));
    return v;
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
    return v;
}

// Inclusive prefix sum over the wave on the VALU with DPP (no LDS round trips): a
// Kogge-Stone scan inside each 16-lane row (row_shr:1/2/4/8, lanes shifted in from
// outside the row read 0), then row_bcast:15 adds row 0's total to row 1 and row 2's to
// row 3, and row_bcast:31 adds lane 31's running total to rows 2 and 3 (GFX9 DPP).
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp_or0(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWS, 0xF, true);
}
__device__ __forceinline__ uint32_t wave_incl_scan_dpp_u32(uint32_t v) {
    v += dpp_or0<0x111, 0xF>(v);  // row_shr:1
    v += dpp_or0<0x112, 0xF>(v);  // row_shr:2
    v += dpp_or0<0x114, 0xF>(v);  // row_shr:4
    v += dpp_or0<0x118, 0xF>(v);  // row_shr:8
    v += dpp_or0<0x142, 0xA>(v);  // row_bcast:15 into rows 1 and 3
    v += dpp_or0<0x143, 0xC>(v);  // row_bcast:31 into rows 2 and 3
    return v;
}

// Inclusive prefix sum over the wave.
__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v) { return wave_incl_scan_dpp_u32(v); }

__device__ __forceinline__ uint64_t wave_incl_scan_u64(uint64_t v) {
    const uint32_t lane = __lane_id();
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
        uint64_t t = __shfl_up(v, off, kWave);
        if (lane >= (uint32_t)off) v += t;
    }
    return v;
}

// Block-wide exclusive scan of one u64 per thread (blockDim.x <= 1024, multiple of 64).
// `scratch` must hold blockDim.x / 64 + 1 entries.  Returns the exclusive prefix;
// *total receives the block sum.  Contains __syncthreads().
__device__ __forceinline__ uint64_t block_excl_scan_u64(uint64_t v, uint64_t *scratch, uint64_t *total) {
    const uint32_t lane = __lane_id();
    const uint32_t wave = threadIdx.x / kWave;
    const uint32_t nwaves = blockDim.x / kWave;
    uint64_t incl = wave_incl_scan_u64(v);
    if (lane == kWave - 1) scratch[wave] = incl;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t acc = 0;
        for (uint32_t w = 0; w < nwaves; ++w) {
            uint64_t t = scratch[w];
            scratch[w] = acc;
            acc += t;
        }
        scratch[nwaves] = acc;
    }
    __syncthreads();
    uint64_t r = scratch[wave] + incl - v;
    *total = scratch[nwaves];
    __syncthreads();
    return r;
}

// Block-wide max of one u64 per thread (every thread gets it); `scratch` holds
// blockDim.x / 64 entries.  Contains __syncthreads().
__device__ __forceinline__ uint64_t block_max_u64(uint64_t v, uint64_t *scratch) {
#pragma unroll
    for (int off = kWave / 2; off > 0; off >>= 1) {
        const uint64_t o = __shfl_xor(v, off, kWave);
        v = o > v ? o : v;
    }
    const uint32_t nwaves = blockDim.x / kWave;
    __syncthreads();
    if (__lane_id() == 0) scratch[threadIdx.x / kWave] = v;
    __syncthreads();
    uint64_t m = 0;
    for (uint32_t w = 0; w < nwaves; ++w) m = scratch[w] > m ? scratch[w] : m;
    __syncthreads();
    return m;
}

// ---------------------------------------------------- decoupled look-back ---
// Single-pass exclusive prefix over chunks claimed in order through a ticket counter
// (so every lower chunk belongs to a workgroup that is already running: the look-back
// cannot deadlock).  status[c] = kLbAgg | count as soon as chunk c is counted, then
// kLbIncl | inclusive prefix; zeroed before the launch.  Each status word is data and
// flag at once: one aligned 8-byte agent-scope relaxed store (sc1, write-through)
// publishes, agent-scope relaxed loads (sc1) poll (MI355X_MICROARCH.md visibility
// table, cdna_hip_programming.md Guideline 16 R2).
constexpr uint64_t kLbAgg = 1ull << 62, kLbIncl = 2ull << 62, kLbVal = kLbAgg - 1;

__device__ __forceinline__ uint64_t lb_load(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lb_store(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Called by ONE whole wave for chunk c with its count agg: publishes, walks back over
// the predecessors 64 at a time (summing aggregates back to the nearest inclusive
// prefix), publishes the inclusive prefix and returns the exclusive one in every lane.
// A poll that never completes (a predecessor cannot fail to publish: it is running)
// gives up after ~2^20 rounds and sets *fail instead of hanging the device.
__device__ __forceinline__ uint64_t lookback_exclusive(uint64_t *status, uint32_t c, uint64_t agg,
                                                       uint32_t *fail) {
    const uint32_t lane = __lane_id();
    if (c == 0) {
        if (lane == 0) lb_store(&status[0], kLbIncl | agg);
        return 0;
    }
    if (lane == 0) lb_store(&status[c], kLbAgg | agg);
    uint64_t excl = 0;
    int64_t hi_idx = (int64_t)c - 1;  // the window ends here
    while (true) {
        const int64_t j = hi_idx - (int64_t)lane;
        uint64_t st = j >= 0 ? lb_load(&status[j]) : kLbIncl;  // before chunk 0: prefix 0
        uint32_t spins = 0;
        while (__ballot(st == 0)) {
            __builtin_amdgcn_s_sleep(1);
            if (st == 0) st = lb_load(&status[j]);
            if (++spins == (1u << 20)) {
                if (lane == 0) atomicExch(fail, 1u);
                st = kLbIncl;
            }
        }
        const uint64_t incl_mask = __ballot((st & kLbIncl) != 0);
        // lanes up to and including the nearest inclusive predecessor
        const uint32_t stop = incl_mask ? (uint32_t)__builtin_ctzll(incl_mask) : 64u;
        excl += wave_sum_u64((lane <= stop && j >= 0) ? (st & kLbVal) : 0);
        if (incl_mask) break;
        hi_idx -= 64;
    }
    if (lane == 0) lb_store(&status[c], kLbIncl | (excl + agg));
    return excl;
}

// ------------------------------------------------------------------ host ---

// Thread-local error text, exposed through mi355_last_error().
void set_last_error(const std::string &msg);
const char *last_error();

}  // namespace sgxamd

// Evaluate a HIP call; on failure record the error and return MI355_ERR_HIP.
#define SGX_HIP(call)                                                                     \
    do {                                                                                  \
        hipError_t _e = (call);                                                           \
        if (_e != hipSuccess) {                                                           \
            ::sgxamd::set_last_error(std::string(#call) + ": " + hipGetErrorString(_e)); \
            return (_e == hipErrorOutOfMemory) ? MI355_ERR_OOM : MI355_ERR_HIP;          \
        }                                                                                 \
    } while (0)
