// HIP kernels of the MI355X radix hash join (gfx950 / CDNA4, wave64).
//
// The reference's CPU hot loops and what replaces them here:
//   partition_hist[_unrolled]   radix_join.cpp:617-654  -> k_hist
//   local/global prefix         radix_join.cpp:886-915  -> k_scan_cols / k_scan_digits / k_scan_regions
//   partition_copy[_unrolled]   radix_join.cpp:659-697  -> k_scatter (LDS counting sort per tile with
//                               64-B write combining, the SWWC variant at :961-1056)
//   bucket_chaining_join        radix_join.cpp:359-458  -> k_join (the same bucket chains in LDS,
//                               S streamed, one partial count per workgroup)
// Radix digits are taken as (key >> shift) & (F - 1) with the pass-1 digit in the
// low bits, exactly like HASH_BIT_MODULO(key, MASK, R) (:47) with R = shift.
// All work is integer; HBM bandwidth is the roofline.
#include <type_traits>

#include "common.hpp"
#include "rho_internal.hpp"

namespace sgxamd {
namespace rho {

constexpr int kWaves = kBlock / kWave;

// Development (SGXAMD_DEBUG_STAMPS, rho_host.cpp join_small): wall-clock stamps of the
// small join's workgroups, [kernel][stamp][workgroup] — 0: entry, 1: before the
// hand-off, 2: exit; null (the default) records nothing.
__device__ uint64_t *g_stamps = nullptr;
__device__ __forceinline__ void dbg_stamp(uint32_t kernel, uint32_t which) {
    uint64_t *p = g_stamps;
    if (p != nullptr && threadIdx.x == 0)
        p[(kernel * 3 + which) * kStampWgs + min(blockIdx.x, kStampWgs - 1)] = wall_clock64();
}
hipError_t set_debug_stamps(uint64_t *p) { return hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &p, sizeof(p)); }

// A uniform value kept in SGPRs.  readfirstlane returns int: each half goes through
// uint32_t, or a low word >= 2^31 would sign-extend over the high word (element
// indices past 2^31: test_max_size_pk_fk).
__device__ __forceinline__ uint64_t uni_u64(uint64_t v) {
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
    return ((uint64_t)hi << 32) | lo;
}

// Segment g -> [b, e) of the input and its region r.  Block-uniform; contains a
// __syncthreads() (every thread of the block must call it).
__device__ __forceinline__ bool seg_lookup(const SegMap &m, uint32_t g, uint32_t *lds_base, uint32_t &r,
                                           uint64_t &b, uint64_t &e) {
    if (m.reg_start == nullptr) {
        r = 0;
        b = (uint64_t)g * m.seg_size;
        e = b + m.seg_size;
        if (e > m.single_n) e = m.single_n;
        return b < e;
    }
    for (uint32_t i = threadIdx.x; i <= m.nreg; i += blockDim.x) lds_base[i] = m.seg_base[i];
    __syncthreads();
    if (g >= lds_base[m.nreg]) return false;
    uint32_t lo = 0, hi = m.nreg;  // largest lo with base[lo] <= g
    while (hi - lo > 1) {
        uint32_t mid = (lo + hi) >> 1;
        if (lds_base[mid] <= g) lo = mid; else hi = mid;
    }
    r = lo;
    const uint64_t rs = m.reg_start[r], rc = m.reg_count[r];
    b = rs + (uint64_t)(g - lds_base[r]) * m.seg_size;
    e = b + m.seg_size;
    if (e > rs + rc) e = rs + rc;
    return b < e;
}

__device__ __forceinline__ uint64_t hist_index(HistLayout layout, uint32_t g, uint32_t d, uint32_t F,
                                               uint32_t nseg_stride) {
    return layout == kDigitMajor ? (uint64_t)d * nseg_stride + g : (uint64_t)g * F + d;
}

// ------------------------------------------------------------------ hist ---
// Histogram of segment g's digits into LDS h[F] (zeroed here).  false: empty segment.
__device__ __forceinline__ bool hist_segment(const uint32_t *__restrict__ in_words, const SegMap &m, uint32_t g,
                                             uint32_t shift, uint32_t bits, uint32_t *h, uint32_t *sbase) {
    uint32_t r;
    uint64_t b, e;
    if (!seg_lookup(m, g, sbase, r, b, e)) return false;
    const uint32_t F = 1u << bits, mask = F - 1;
    for (uint32_t d = threadIdx.x; d < F; d += blockDim.x) h[d] = 0;
    __syncthreads();
    // 16-B non-temporal loads (two tuples per lane); an odd leading tuple first
    const uint64_t *in64 = reinterpret_cast<const uint64_t *>(in_words);
    uint64_t b2 = b;
    if ((b & 1) && b < e) {
        if (threadIdx.x == 0) atomicAdd(&h[(in_words[2 * b] >> shift) & mask], 1u);
        b2 = b + 1;
    }
    const uint4 *pairs = reinterpret_cast<const uint4 *>(in64 + b2);
    const uint64_t np = (e - b2) / 2;
    constexpr int U = 8;
    uint64_t i = threadIdx.x;
    for (; i + (U - 1) * kBlock < np; i += U * kBlock) {
        uint4 q[U];
#pragma unroll
        for (int u = 0; u < U; ++u) q[u] = ld_nt(pairs + i + u * kBlock);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            atomicAdd(&h[(q[u].x >> shift) & mask], 1u);
            atomicAdd(&h[(q[u].z >> shift) & mask], 1u);
        }
    }
    for (; i < np; i += kBlock) {
        const uint4 q = ld_nt(pairs + i);
        atomicAdd(&h[(q.x >> shift) & mask], 1u);
        atomicAdd(&h[(q.z >> shift) & mask], 1u);
    }
    if (((e - b2) & 1) && threadIdx.x == 0) atomicAdd(&h[(in_words[2 * (e - 1)] >> shift) & mask], 1u);
    __syncthreads();
    return true;
}

// Histograms of two consecutive segments of a single-region map (2g and 2g + 1, even
// starts) into h / h2 with both segments' 16-B loads in flight together (one memory round
// trip per step instead of one per segment).  false: both empty.  kmax: this thread's
// largest key seen (max-ed in).
__device__ __forceinline__ bool hist_two_segments(const uint32_t *__restrict__ in_words, const SegMap &m, uint32_t g,
                                                  uint32_t shift, uint32_t bits, uint32_t *h, uint32_t *h2,
                                                  uint32_t &kmax) {
    const uint64_t n = m.single_n, seg = m.seg_size;
    const uint64_t bA = min<uint64_t>(2ull * g * seg, n), eA = min<uint64_t>(bA + seg, n), eB = min<uint64_t>(eA + seg, n);
    if (bA >= eB) return false;
    const uint32_t F = 1u << bits, mask = F - 1;
    for (uint32_t d = threadIdx.x; d < F; d += blockDim.x) h[d] = h2[d] = 0;
    __syncthreads();
    const uint64_t *in64 = reinterpret_cast<const uint64_t *>(in_words);
    const uint4 *pa = reinterpret_cast<const uint4 *>(in64 + bA), *pb = reinterpret_cast<const uint4 *>(in64 + eA);
    const uint64_t npa = (eA - bA) / 2, npb = (eB - eA) / 2, np = npa > npb ? npa : npb;
    constexpr int U = 8;
    for (uint64_t i = threadIdx.x; i < np; i += U * kBlock) {
        uint4 qa[U], qb[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t k = i + u * kBlock;
            qa[u] = k < npa ? ld_nt(pa + k) : make_uint4(0, 0, 0, 0);
            qb[u] = k < npb ? ld_nt(pb + k) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t k = i + u * kBlock;
            if (k < npa) {
                atomicAdd(&h[(qa[u].x >> shift) & mask], 1u);
                atomicAdd(&h[(qa[u].z >> shift) & mask], 1u);
                kmax = max(kmax, max(qa[u].x, qa[u].z));
            }
            if (k < npb) {
                atomicAdd(&h2[(qb[u].x >> shift) & mask], 1u);
                atomicAdd(&h2[(qb[u].z >> shift) & mask], 1u);
                kmax = max(kmax, max(qb[u].x, qb[u].z));
            }
        }
    }
    if (threadIdx.x == 0) {  // odd trailing tuples (segments start at even offsets)
        if ((eA - bA) & 1) {
            const uint32_t k = in_words[2 * (eA - 1)];
            atomicAdd(&h[(k >> shift) & mask], 1u);
            kmax = max(kmax, k);
        }
        if ((eB - eA) & 1) {
            const uint32_t k = in_words[2 * (eB - 1)];
            atomicAdd(&h2[(k >> shift) & mask], 1u);
            kmax = max(kmax, k);
        }
    }
    __syncthreads();
    return true;
}

__global__ __launch_bounds__(kBlock) void k_hist(const uint32_t *__restrict__ in_words, SegMap m, uint32_t shift,
                                                 uint32_t bits, uint64_t *__restrict__ hist, HistLayout layout,
                                                 uint32_t nseg_stride) {
    __shared__ uint32_t h[kMaxF];
    __shared__ uint32_t sbase[kMaxF + 1];
    // XCD-contiguous segments for one-region passes (measured faster there, slower
    // over pass 2's many regions)
    const uint32_t g = layout == kDigitMajor ? xcd_contiguous(blockIdx.x, gridDim.x) : blockIdx.x;
    if (!hist_segment(in_words, m, g, shift, bits, h, sbase)) return;
    const uint32_t F = 1u << bits;
    for (uint32_t d = threadIdx.x; d < F; d += kBlock) hist[hist_index(layout, g, d, F, nseg_stride)] = h[d];
}

// ------------------------------------------- in-launch hand-off (last arriver) ---
// Counter form of cdna_hip_programming.md §6 Guideline 16: every wave drains its
// stores, the workgroup meets, one lane releases at agent scope and takes a ticket; the
// last of n arrivers acquires at agent scope before the workgroup reads what the others
// wrote.  The ticket is reset by the last arriver (atomic store) for the next call; the
// words start at zero (Context::sync, zeroed when allocated).  True in every thread of
// the last workgroup.
__device__ __forceinline__ bool arrive_last(uint64_t *ticket, uint64_t n, uint32_t *lds_flag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint64_t t = __hip_atomic_fetch_add(ticket, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool last = t == n - 1;
        if (last) {
            __hip_atomic_store(ticket, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        *lds_flag = last ? 1u : 0u;
    }
    __syncthreads();
    return *lds_flag != 0;
}

// The same over kSyncSpread groups (rho_internal.hpp): arrival idx (a segment or
// workgroup index < n) takes its group's sub-ticket (idx mod groups); the last of each
// group takes the ticket.  At most n / groups + groups serialised device atomics per
// address instead of n.
__device__ __forceinline__ bool arrive_last_spread(uint64_t *ticket, uint64_t n, uint32_t idx, uint32_t *lds_flag) {
    const uint32_t groups = n < kSyncSpread ? (uint32_t)n : kSyncSpread;
    if (groups <= 1) return arrive_last(ticket, n, lds_flag);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t grp = idx % groups;
        const uint64_t members = (n - grp + groups - 1) / groups;
        uint64_t *sub = ticket + kSyncSub + kNumTickets * grp;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        bool last = false;
        if (__hip_atomic_fetch_add(sub, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == members - 1) {
            __hip_atomic_store(sub, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // the group's writes (acquired) pass on with this workgroup's release
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (__hip_atomic_fetch_add(ticket, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == groups - 1) {
                __hip_atomic_store(ticket, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                last = true;
            }
        }
        *lds_flag = last ? 1u : 0u;
    }
    __syncthreads();
    return *lds_flag != 0;
}

__device__ __forceinline__ uint64_t ld_agent(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ----------------------------------------- one-launch histogram (small joins) ---
// For small one-pass joins: the histograms of R and S in ONE launch.  Segment g of a
// relation adds its digit counts to the relation's digit totals (this call's set, see
// launch_scatter_pair) with one device atomic per digit; the value returned is the
// segment's offset inside the digit (segments take their places in arrival order; the
// join count does not depend on the order inside a partition).  Nothing else: the digit
// starts (the scan of radix_join.cpp:901-914) are taken by the scatter's workgroups
// themselves, each for its own cursors, and the partition table and task list by one
// extra workgroup of the scatter -- no hand-off at the end of this launch (round 4 ran a
// relation ticket, the digit scan, a second ticket and the task list serially at its
// end: 12 of its 20 us, r04v stamps).
struct HistPairRel {
    const uint32_t *in;   // tuples as u32 words
    SegMap m;
    uint32_t grid;        // segments of the relation
    uint32_t shift;
    uint64_t *offs;       // [d][g] (stride grid): segment g's offset inside its copy of digit d
    uint64_t *tot;        // [kSyncSpread][kMaxF] digit totals, zero at entry
    uint64_t *kmax;       // (nullable) the relation's largest key, max-ed in (zero at entry)
};

__global__ __launch_bounds__(kBlock) void k_hist_pair(HistPairRel A, HistPairRel B, uint32_t bits,
                                                      uint64_t *__restrict__ t0) {
    __shared__ uint32_t h[kMaxF], h2[kMaxF];
    const bool isB = blockIdx.x >= A.grid;
    const HistPairRel &H = isB ? B : A;
    const uint32_t g = isB ? blockIdx.x - A.grid : blockIdx.x;  // segment g = scatter segments 2g, 2g + 1
    const uint32_t F = 1u << bits;
    if (blockIdx.x == 0 && threadIdx.x == 0) *t0 = wall_clock64();  // the call's start (small-join device span)
    dbg_stamp(0, 0);
    // segment g is two scatter segments (H.m's, halves 2g and 2g + 1: one tile each, so
    // that the scatter's workgroups each load, sort and write one tile): one histogram
    // each, their sum to the totals, the second half's offset after the first half's
    uint32_t km = 0;
    const bool any = hist_two_segments(H.in, H.m, g, H.shift, bits, h, h2, km);
    if (H.kmax) {  // one device atomic per workgroup (h2's words are free after the counts)
        km = wave_max_u32(km);
        __shared__ uint32_t wm[kBlock / kWave];
        if (__lane_id() == 0) wm[threadIdx.x / kWave] = km;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t m = 0;
            for (uint32_t w = 0; w < kBlock / kWave; ++w) m = max(m, wm[w]);
            if (m) __hip_atomic_fetch_max(H.kmax, (uint64_t)m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    uint64_t *tot_c = H.tot + (uint64_t)(g % kSyncSpread) * kMaxF;  // this segment's copy of the totals
    for (uint32_t d = threadIdx.x; d < F; d += kBlock) {
        const uint32_t a = any ? h[d] : 0u, v = a + (any ? h2[d] : 0u);
        const uint64_t off =
            v ? __hip_atomic_fetch_add(&tot_c[d], (uint64_t)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
        H.offs[(uint64_t)d * 2 * H.grid + 2 * g] = off;
        H.offs[(uint64_t)d * 2 * H.grid + 2 * g + 1] = off + a;
    }
    dbg_stamp(0, 1);
}

hipError_t launch_hist_pair(const row_t *R, const SegMap &mR, uint32_t gridR, const row_t *S, const SegMap &mS,
                            uint32_t gridS, uint32_t shift, uint32_t bits, uint64_t *offsR, uint64_t *offsS,
                            uint64_t *totR, uint64_t *totS, uint64_t *t0, hipStream_t s, uint64_t *kmaxR) {
    const HistPairRel A{reinterpret_cast<const uint32_t *>(R), mR, gridR, shift, offsR, totR, kmaxR};
    const HistPairRel B{reinterpret_cast<const uint32_t *>(S), mS, gridS, shift, offsS, totS, nullptr};
    hipLaunchKernelGGL(k_hist_pair, dim3(gridR + gridS), dim3(kBlock), 0, s, A, B, bits, t0);
    return hipGetLastError();
}

hipError_t launch_hist(const row_t *in, const SegMap &m, uint32_t grid, uint32_t shift, uint32_t bits,
                       uint64_t *hist, HistLayout layout, uint32_t nseg_stride, hipStream_t s) {
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL(k_hist, dim3(grid), dim3(kBlock), 0, s, reinterpret_cast<const uint32_t *>(in), m, shift,
                       bits, hist, layout, nseg_stride);
    return hipGetLastError();
}

// Pass-2 histogram over the digit side stream written by the pass-1 scatter: the same
// segments as the pass-2 scatter, one byte (the digit itself) per tuple instead of the
// 8-byte tuple.  16-B non-temporal loads (16 digits per lane, 4 in flight), an
// unaligned head and tail byte by byte; segment-major [g][F] output.
__global__ __launch_bounds__(kBlock) void k_hist_side(const uint8_t *__restrict__ side, SegMap m, uint32_t bits,
                                                      uint64_t *__restrict__ hist) {
    __shared__ uint32_t h[kMaxF];
    __shared__ uint32_t sbase[kMaxF + 1];
    const uint32_t g = blockIdx.x;
    uint32_t r;
    uint64_t b, e;
    if (!seg_lookup(m, g, sbase, r, b, e)) return;
    const uint32_t F = 1u << bits;
    for (uint32_t d = threadIdx.x; d < F; d += kBlock) h[d] = 0;
    __syncthreads();
    uint64_t a0 = (b + 15) & ~uint64_t(15);
    if (a0 > e) a0 = e;
    const uint64_t a1 = a0 + ((e - a0) & ~uint64_t(15));
    if (threadIdx.x < a0 - b) atomicAdd(&h[side[b + threadIdx.x]], 1u);
    if (threadIdx.x < e - a1) atomicAdd(&h[side[a1 + threadIdx.x]], 1u);
    const uint4 *v = reinterpret_cast<const uint4 *>(side + a0);
    const uint64_t nv = (a1 - a0) / 16;
    auto count16 = [&](const uint4 &q) {
        const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int j = 0; j < 16; ++j) atomicAdd(&h[__builtin_amdgcn_ubfe(w[j >> 2], (j & 3) * 8, 8)], 1u);
    };
    constexpr int U = 4;
    uint64_t i = threadIdx.x;
    for (; i + (U - 1) * kBlock < nv; i += U * kBlock) {
        uint4 q[U];
#pragma unroll
        for (int u = 0; u < U; ++u) q[u] = ld_nt(v + i + u * kBlock);
#pragma unroll
        for (int u = 0; u < U; ++u) count16(q[u]);
    }
    for (; i < nv; i += kBlock) count16(ld_nt(v + i));
    __syncthreads();
    for (uint32_t d = threadIdx.x; d < F; d += kBlock) hist[(uint64_t)g * F + d] = h[d];
}

hipError_t launch_hist_side(const uint8_t *side, const SegMap &m, uint32_t grid, uint32_t bits, uint64_t *hist,
                            hipStream_t s) {
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL(k_hist_side, dim3(grid), dim3(kBlock), 0, s, side, m, bits, hist);
    return hipGetLastError();
}

// ------------------------------------------------------------------ scans ---
// One block per digit column: exclusive prefix over the segments (in place).
// guard (nullable): nothing to do when *guard >> gshift fits 16 bits (the 4-byte pool
// repeated after a narrow pool that stood, PoolOut::guard).
__global__ __launch_bounds__(kBlock) void k_scan_cols(uint64_t *__restrict__ hist, uint32_t nseg,
                                                      uint64_t *__restrict__ totals,
                                                      const uint32_t *__restrict__ guard = nullptr,
                                                      uint32_t gshift = 0) {
    __shared__ uint64_t scratch[kWaves + 1];
    if (guard && ((*guard >> gshift) >> 16) == 0) return;
    uint64_t *col = hist + (uint64_t)blockIdx.x * nseg;
    uint64_t carry = 0;
    for (uint32_t base = 0; base < nseg; base += kBlock) {
        const uint32_t g = base + threadIdx.x;
        const uint64_t v = g < nseg ? col[g] : 0;
        uint64_t tot;
        const uint64_t ex = block_excl_scan_u64(v, scratch, &tot);
        if (g < nseg) col[g] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) totals[blockIdx.x] = carry;
}

// One block: digit starts from totals, and the segment table of the next pass.
__global__ __launch_bounds__(1024) void k_scan_digits(const uint64_t *__restrict__ totals, uint32_t F,
                                                      uint64_t *__restrict__ out_start,
                                                      uint64_t *__restrict__ out_count, uint64_t base,
                                                      uint32_t *__restrict__ next_seg_base,
                                                      uint64_t next_seg_size) {
    __shared__ uint64_t scratch[1024 / kWave + 1];
    const uint32_t d = threadIdx.x;
    const uint64_t v = d < F ? totals[d] : 0;
    uint64_t tot;
    const uint64_t ex = block_excl_scan_u64(v, scratch, &tot);
    if (d < F) {
        out_start[d] = base + ex;
        out_count[d] = v;
    }
    if (next_seg_base != nullptr) {
        const uint64_t ns = d < F ? (v + next_seg_size - 1) / next_seg_size : 0;
        uint64_t tot2;
        const uint64_t ex2 = block_excl_scan_u64(ns, scratch, &tot2);
        if (d < F) next_seg_base[d] = (uint32_t)ex2;
        if (d == 0) next_seg_base[F] = (uint32_t)tot2;
    }
}

hipError_t launch_scan_single(uint64_t *hist, uint32_t nseg, uint32_t bits, uint64_t *totals,
                              uint64_t *out_start, uint64_t *out_count, uint64_t base, uint32_t *next_seg_base,
                              uint64_t next_seg_size, hipStream_t s) {
    const uint32_t F = 1u << bits;
    hipLaunchKernelGGL(k_scan_cols, dim3(F), dim3(kBlock), 0, s, hist, nseg, totals);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const uint32_t threads = F < 64 ? 64 : F;
    hipLaunchKernelGGL(k_scan_digits, dim3(1), dim3(threads), 0, s, totals, F, out_start, out_count, base,
                       next_seg_base, next_seg_size);
    return hipGetLastError();
}

// One block per region.  Cursors for [g][d] and the partition table.  The region's
// segments are split among S = 512 / F threads per digit (tid = j * F + d), so the
// reads of one digit's column run in parallel instead of as one dependent chain.
// pad (the u16 wire's senders): every partition starts on a multiple of 8 elements --
// region r's partitions from round_up8(reg_start[r] + 8 F r), each taking round_up8(its
// count): at most 8 F P / F + 8 elements past the unpadded layout (wire_pad_slack).
__global__ __launch_bounds__(kMaxF) void k_scan_regions(uint64_t *__restrict__ hist,
                                                        const uint32_t *__restrict__ seg_base,
                                                        const uint64_t *__restrict__ reg_start, uint32_t F,
                                                        uint64_t *__restrict__ part_start,
                                                        uint64_t *__restrict__ part_count, uint32_t pad) {
    __shared__ uint64_t scratch[kMaxF / kWave + 1];
    __shared__ uint64_t part[kMaxF];   // [j][d]: sum of thread j's chunk, then its prefix inside d
    __shared__ uint64_t startd[kMaxF];
    const uint32_t r = blockIdx.x, tid = threadIdx.x;
    const uint32_t S = kMaxF / F, d = tid % F, j = tid / F;
    const uint32_t sb = seg_base[r], se = seg_base[r + 1];
    const uint64_t rs = reg_start[r];
    const uint32_t per = (se - sb + S - 1) / S;
    const uint32_t g0 = min(se, sb + j * per), g1 = min(se, g0 + per);
    // The first kKeep counts of the chunk stay in registers for the cursor pass below
    // (all of them at the bench's ~31 segments per region), so the column is read once.
    constexpr uint32_t kKeep = 12;
    uint64_t keep[kKeep];
    uint64_t sum = 0;
#pragma unroll
    for (uint32_t i = 0; i < kKeep; ++i) {
        keep[i] = g0 + i < g1 ? hist[(uint64_t)(g0 + i) * F + d] : 0;
        sum += keep[i];
    }
    for (uint32_t g = g0 + kKeep; g < g1; ++g) sum += hist[(uint64_t)g * F + d];
    part[tid] = sum;
    __syncthreads();
    uint64_t total = 0;
    if (j == 0) {
        for (uint32_t jj = 0; jj < S; ++jj) {
            const uint64_t t = part[jj * F + d];
            part[jj * F + d] = total;
            total += t;
        }
    }
    uint64_t tot;
    const uint64_t ex = block_excl_scan_u64(j == 0 ? (pad ? (total + 7) & ~7ull : total) : 0, scratch,
                                            &tot);  // digits are tids 0..F-1
    if (j == 0) {
        const uint64_t start = (pad ? (rs + 8ull * F * r + 7) & ~7ull : rs) + ex;
        startd[d] = start;
        part_start[(uint64_t)r * F + d] = start;
        part_count[(uint64_t)r * F + d] = total;
    }
    __syncthreads();
    uint64_t run = startd[d] + part[tid];
#pragma unroll
    for (uint32_t i = 0; i < kKeep; ++i)
        if (g0 + i < g1) {
            hist[(uint64_t)(g0 + i) * F + d] = run;
            run += keep[i];
        }
    for (uint32_t g = g0 + kKeep; g < g1; ++g) {
        const uint64_t c = hist[(uint64_t)g * F + d];
        hist[(uint64_t)g * F + d] = run;
        run += c;
    }
}

hipError_t launch_scan_regions(uint64_t *hist, const uint32_t *seg_base, const uint64_t *reg_start, uint32_t nreg,
                               uint32_t bits, uint64_t *part_start, uint64_t *part_count, hipStream_t s, bool pad) {
    const uint32_t F = 1u << bits;
    hipLaunchKernelGGL(k_scan_regions, dim3(nreg), dim3(kMaxF), 0, s, hist, seg_base, reg_start, F, part_start,
                       part_count, pad ? 1u : 0u);
    return hipGetLastError();
}

// --------------------------------------------------------------- scatter ---
// Partition copy of one segment per workgroup (partition_copy, radix_join.cpp:659-697),
// organised like the reference's software write-combining variant
// parallel_radix_partition_optimized (:961-1056): every digit keeps its unfinished
// 128-B output granule (kGran tuples) in LDS and only whole, aligned granules go to
// HBM, so no HBM line is written twice.  Per tile of NT * ITEMS tuples:
//   A. every tuple takes a slot of its digit with one LDS atomic (tile histogram and
//      in-tile rank at once; order inside a digit is arrival order, the join count
//      does not depend on it);
//   B. owner thread d: pending = carried + tile tuples of d; the prefix that ends on a
//      granule boundary is written now (w), the rest (r < kGran) is carried.  One
//      block scan gives the digit-sorted tile offsets and the granule descriptors;
//   C. the tile is placed digit-sorted in LDS (one LDS read of tbase[d] per tuple);
//   D. 16-lane groups write whole granules: carried tuples first, then the tile's;
//   E. 16-lane groups move each digit's new carries (< kGran) into its carry slots.
// The ablation measurements behind this layout (LDS-bound, not HBM-bound, with the
// carries in registers and four random metadata reads per tuple) are in DESIGN.md.
// The next tile's tuples are already loading while a tile is processed (two
// register sets).  The last carries of the segment are flushed at the end.
constexpr uint32_t kGran = 16;  // tuples per output granule = one 128-B line

// c ? *a : *b for two LDS elements with one read: the LDS address is selected, not the
// loaded value (a select between two loads becomes exec-masked branches, each with its
// own read and wait)
template <typename T>
__device__ __forceinline__ T lds_pick(bool c, const T *a, const T *b) {
    typedef __attribute__((address_space(3))) const T lds_t;
    const uint32_t pa = (uint32_t)(uintptr_t)(lds_t *)a, pb = (uint32_t)(uintptr_t)(lds_t *)b;
    return *(lds_t *)(uintptr_t)vsel(c, pa, pb);
}

#ifndef SGXAMD_POOL_GRAN  // pooled keys (4-byte pool): bytes per write granule, 128 or 256
#define SGXAMD_POOL_GRAN 128
#endif
// EXT: 0 = cursor output, contiguous input; 1 = pooled output (PoolOut); 2 = block-list
// input (the segment's list entries staged in ents).
// T: the element moved (uint64_t tuple, or uint32_t key of a count-only join).
// OB: bytes per element written (sizeof(T); 2: the pooled pass 1 of a narrow relation
// writes the keys' 16-bit residuals, k_scatter_pool's narrow variant).
template <int BITS, int ITEMS, int NT, int EXT = 0, typename T = uint64_t, int OB = (int)sizeof(T)>
struct ScatterLds {
    static constexpr uint32_t F = 1u << BITS;
    static constexpr uint32_t TILE = NT * ITEMS;
    static constexpr uint32_t NW = NT / kWave;
    // elements per write granule (128 B; the 4-byte key pool SGXAMD_POOL_GRAN)
    static constexpr uint32_t G = (EXT == 1 && sizeof(T) == 4 && OB == 4 ? SGXAMD_POOL_GRAN : 128) / OB;
    static constexpr uint32_t GPB = kBlk / G;       // granules per pool block
    static constexpr uint32_t MAXDESC = (TILE + (G - 1) * F) / G + F;
    union {
        uint32_t sbase[kMaxF + 1];  // segment table (only before the first tile)
        T tile[TILE];               // this tile's elements, digit-sorted
    };
    T carry[F * (G - 1)];             // digit d: slots [d*(G-1), (d+1)*(G-1))
    uint64_t pend[F];                 // global position of d's first pending (carried) tuple
    uint2 meta[F];                    // {tbase, c | r << 8 | w << 16} of the current tile
    uint32_t cnt[F];                  // tile histogram (phase A), zero between tiles
    uint32_t tbase[F];                // digit-sorted tile offset of d
    uint32_t gbase[F];                // first granule descriptor of d
    uint16_t desc[MAXDESC];           // granule j belongs to digit desc[j]
    uint32_t wt[NW][2];
    uint2 gaddr[EXT == 1 ? F : 1];    // pooled: {granule of d's first write in its current block,
                                      //          first granule of the blocks d took for this tile}
    uint64_t ents[EXT == 2 ? kPass2Ents : 1];  // block-list input: phys block | fill << 32
    uint32_t pool_next;               // pooled: blocks taken from the segment's pool
    uint32_t kmax;                    // pooled keys: the largest key of the segment
};

// Chain histograms (pooled pass 1 of keys, F2 > 0): every chain's histogram of pass-2
// digits, two u16 counts per LDS word, counted in phase C while the tile is in
// registers (replacing the digit side stream and the pass-2 histogram pass over it),
// stored as u32 [d][g][F2] at the segment's end.  A count wraps only in a chain of more
// than 65,535 elements (a heavily skewed digit); the pass-2 histogram (k_hist_chain)
// counts those chains from their keys (checking the chain records), so no flush sits in
// the scatter's loop, which has no register to spare.
struct ChainState {
    uint32_t *h2;   // LDS [F][F2 / 2]
    uint32_t *out;  // global [F][nseg][F2] (u32)
    uint32_t g, nseg, shift2;
};

// The table out, after the segment's last tile (not inlined: its registers stay out of
// the scatter's loop).
template <int F, int F2, int NT>
__device__ __noinline__ void chain_store(const uint32_t *h2, uint32_t *__restrict__ out, uint32_t g, uint32_t nseg) {
    for (uint32_t i = threadIdx.x; i < F * F2 / 2; i += NT) {
        const uint32_t d = i / (F2 / 2), j = i % (F2 / 2), w = h2[i];
        *reinterpret_cast<uint2 *>(out + ((uint64_t)d * nseg + g) * F2 + 2 * j) = make_uint2(w & 0xFFFFu, w >> 16);
    }
}

// The 4-byte pool's launches after a speculative narrow pool (po.guard: the relation's
// largest key; po.guard_shift: the residual shift): nothing to do when every residual fit
// 16 bits.
__device__ __forceinline__ bool pool_guard_skip(const PoolOut &po) {
    return po.guard != nullptr && ((*po.guard >> po.guard_shift) >> 16) == 0;
}

// Pooled output, per owner thread (digit): its chain's current block and length.
struct PoolState {
    uint32_t cur;
    uint32_t nb;
    uint32_t pool0;  // first block of the segment's pool
    uint32_t *binfo;
};

// Waves per SIMD that the LDS footprint allows (__launch_bounds__ second argument:
// k workgroups per CU of NT threads <=> k * NT / 256 waves per SIMD), so the
// register allocation never becomes the tighter occupancy limit.
#ifndef SGXAMD_POOL_MAXW  // pooled pass 1: waves per SIMD the register budget is cut for
#define SGXAMD_POOL_MAXW 4
#endif
template <int BITS, int ITEMS, int NT, int EXT = 0, typename T = uint64_t, int OB = (int)sizeof(T)>
constexpr int scatter_waves_per_simd() {
    constexpr int k = (160 * 1024) / (int)sizeof(ScatterLds<BITS, ITEMS, NT, EXT, T, OB>);
    constexpr int w = (k < 1 ? 1 : k) * NT / 256;
    // at most 4 waves/SIMD (128 VGPRs): fewer registers spill, and a scratch reload is
    // a vector-memory op whose wait would also wait for every store in flight
    constexpr int cap = EXT == 1 ? SGXAMD_POOL_MAXW : 4;
    return w < 1 ? 1 : (w > cap ? cap : w);
}

// One tile of the segment behind rsrc (byte offset soff of the tile); lanes past the
// segment end read 0 through the buffer bounds check.
template <int ITEMS, int NT>
__device__ __forceinline__ void load_tile(__amdgpu_buffer_rsrc_t rs, uint32_t soff, uint64_t (&dst)[ITEMS]) {
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) dst[k] = buf_ld_nt_u64(rs, threadIdx.x * 8u, soff + (uint32_t)(k * NT * 8));
}

// Element loads of T from an input of IS-byte elements (IS = 8 and T = uint32_t: the
// key word of each tuple; the cache lines fetched are the same).
template <typename T>
__device__ __forceinline__ T buf_ld_nt_t(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff);
template <>
__device__ __forceinline__ uint64_t buf_ld_nt_t<uint64_t>(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return buf_ld_nt_u64(r, voff, soff);
}
template <>
__device__ __forceinline__ uint32_t buf_ld_nt_t<uint32_t>(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(r, (int)voff, (int)soff, 2);
}
template <typename T, int IS, int ITEMS, int NT>
__device__ __forceinline__ void load_tile_t(__amdgpu_buffer_rsrc_t rs, uint32_t soff, T (&dst)[ITEMS]) {
#pragma unroll
    for (int k = 0; k < ITEMS; ++k)
        dst[k] = buf_ld_nt_t<T>(rs, threadIdx.x * (uint32_t)IS, soff + (uint32_t)(k * NT * IS));
}

// Block-wide exclusive scan of two u32 counters at once (one __syncthreads).
template <int NW>
__device__ __forceinline__ void block_scan2(uint32_t a, uint32_t b, uint32_t (&wt)[NW][2], uint32_t &ea,
                                            uint32_t &eb, uint32_t &ta, uint32_t &tb) {
    const uint32_t lane = __lane_id(), wave = threadIdx.x / kWave;
    const uint32_t ia = wave_incl_scan_u32(a), ib = wave_incl_scan_u32(b);
    if (lane == kWave - 1) {
        wt[wave][0] = ia;
        wt[wave][1] = ib;
    }
    __syncthreads();
    uint32_t pa = 0, pb = 0;
    ta = 0;
    tb = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        const uint32_t x = wt[w][0], y = wt[w][1];
        if (w < (int)wave) {
            pa += x;
            pb += y;
        }
        ta += x;
        tb += y;
    }
    ea = pa + ia - a;
    eb = pb + ib - b;
}

// Phases A-C of one tile: the tile ends up digit-sorted in L.tile (v is dead after).
// tn: valid tuples of the tile (items tid + k * NT < tn); with block-list input (EXT 2)
// a bit mask instead, bit k = item k valid.  ps: the owner thread's chain (EXT 1).
// FULL: every item is valid (no per-item checks; callers take it for full tiles).
template <int BITS, int ITEMS, int NT, int EXT = 0, typename T = uint64_t, bool FULL = false, int F2 = 0,
          int OB = (int)sizeof(T)>
__device__ __forceinline__ uint32_t scatter_tile_sort(ScatterLds<BITS, ITEMS, NT, EXT, T, OB> &L, uint64_t &pend,
                                                      uint32_t &carried, const T (&v)[ITEMS],
                                                      T *__restrict__ out, uint32_t tn, uint32_t shift,
                                                      uint64_t tbase_global, PoolState *ps = nullptr,
                                                      ChainState *cs = nullptr) {
    constexpr uint32_t F = 1u << BITS, mask = F - 1, NW = NT / kWave;
    constexpr uint32_t G = ScatterLds<BITS, ITEMS, NT, EXT, T, OB>::G, GPB = ScatterLds<BITS, ITEMS, NT, EXT, T, OB>::GPB;
    const uint32_t tid = threadIdx.x;
    const auto valid = [&](int k) { return FULL || (EXT == 2 ? ((tn >> k) & 1u) != 0 : tid + k * NT < tn); };
#ifdef SGXAMD_ABLATE_NOSORT  // development ablation (tools/part_bench): the memory pipeline alone
#pragma unroll
    for (int k = 0; k < ITEMS; ++k)
        if (valid(k)) st_nt(out + tbase_global + tid + k * NT, v[k]);
    return 0;
#endif
    (void)tbase_global;
    (void)ps;
    (void)cs;
    // A. slot of every tuple inside its digit (chain histograms: and its pass-2 digit's count)
    uint32_t slot[ITEMS];
#pragma unroll
    for (int k = 0; k < ITEMS; ++k)
        if (valid(k)) slot[k] = atomicAdd(&L.cnt[((uint32_t)v[k] >> shift) & mask], 1u);
    __syncthreads();
    // B. per digit: what is written now (w), what is carried on (r), granules touched (g)
    uint32_t t = 0, g = 0, w = 0, r = 0, c = 0;
    uint64_t p0 = 0;
    if (tid < F) {
        t = L.cnt[tid];
        L.cnt[tid] = 0;
        c = carried;
        p0 = pend;
        const uint64_t aligned = (p0 + c + t) & ~uint64_t(G - 1);
        if (aligned > p0) {
            w = (uint32_t)(aligned - p0);
            g = (uint32_t)(aligned / G - p0 / G);
        }
        r = c + t - w;
    }
    uint32_t tb, gb, ttot, gtot;
    block_scan2<NW>(t, g, L.wt, tb, gb, ttot, gtot);
    (void)ttot;
    if (tid < F) {
        uint32_t mx = tb;
        if constexpr (EXT == 1) {
            // pooled: pend is granule-aligned (only whole granules are written before the
            // segment's end).  g0 granules fill the current block, the rest go to nnew
            // fresh blocks of the pool, taken together (consecutive, so contiguous).
            const uint32_t off = (uint32_t)(p0 / G) & (GPB - 1);
            const uint32_t g0 = off ? min(g, GPB - off) : 0u;
            const uint32_t nnew = (g - g0 + GPB - 1) / GPB;
            uint32_t nb0 = 0;
            if (nnew) {
                nb0 = ps->pool0 + atomicAdd(&L.pool_next, nnew);
                for (uint32_t j = 0; j < nnew; ++j) ps->binfo[nb0 + j] = tid | (kBlk << 16);
            }
            L.gaddr[tid] = make_uint2(ps->cur * GPB + off, nb0 * GPB);
            mx |= g0 << 16;
            if (nnew) {
                ps->cur = nb0 + nnew - 1;
                ps->nb += nnew;
            }
        }
        L.tbase[tid] = tb;
        L.gbase[tid] = gb;
        L.meta[tid] = make_uint2(mx, c | (r << 8) | (w << 16));
        L.pend[tid] = p0;
        for (uint32_t j = 0; j < g; ++j) L.desc[gb + j] = (uint16_t)tid;
        pend = p0 + w;
        carried = r;
    }
    __syncthreads();
    // C. the tile, digit-sorted (chain histograms: each key's pass-2 digit counted here,
    // where its rank's register is free again; in phase A the count spilled registers)
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        if (valid(k)) {
            const uint32_t d = ((uint32_t)v[k] >> shift) & mask;
            L.tile[L.tbase[d] + slot[k]] = v[k];
            if constexpr (F2 > 0) {
                const uint32_t d2 = ((uint32_t)v[k] >> cs->shift2) & (uint32_t)(F2 - 1);
                atomicAdd(&cs->h2[d * (F2 / 2) + (d2 >> 1)], 1u << ((d2 & 1u) * 16u));
            }
        }
    }
    __syncthreads();
    return gtot;
}

// Phases D-E of the tile sorted by scatter_tile_sort (gtot = its granule count).
// The digit side stream's byte stores (non-temporal with SGXAMD_SIDE_NT).
#ifndef SGXAMD_SIDE_NT
#define SGXAMD_SIDE_NT 1
#endif
__device__ __forceinline__ void st_side(uint8_t *p, uint8_t v) {
#if SGXAMD_SIDE_NT
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}

// SIDE: every stored tuple's next-pass digit also goes to side[a] (a 16-lane group
// writes 16 consecutive bytes next to its 128-B granule).
// OB 2 (narrow pool): the elements written are the keys' residuals key >> rshift, u16.
template <int BITS, int ITEMS, int NT, bool SIDE, int EXT = 0, typename T = uint64_t, int OB = (int)sizeof(T)>
__device__ __forceinline__ void scatter_tile_write(ScatterLds<BITS, ITEMS, NT, EXT, T, OB> &L, T *__restrict__ out,
                                                   uint32_t gtot, uint8_t *__restrict__ side, uint32_t shift2,
                                                   uint32_t mask2, uint32_t rshift = 0) {
    constexpr uint32_t G = ScatterLds<BITS, ITEMS, NT, EXT, T, OB>::G;
    constexpr uint32_t F = 1u << BITS, NG = NT / G;
    constexpr uint32_t CS = G - 1;
    constexpr uint32_t TB = EXT == 1 ? 0xFFFFu : ~0u;  // tile offset bits of meta.x
#ifdef SGXAMD_ABLATE_NOSORT
    return;
#endif
    const uint32_t tid = threadIdx.x;
    // D. whole granules, G lanes (one 128-B line) per granule
    const uint32_t lane = tid & (G - 1), grp = tid / G;
    if constexpr (OB == 2) {
        // narrow pool (pooled, every granule whole): 16 lanes per 64-residual granule, four
        // consecutive keys per lane -- one 8-byte store of their residuals and one 4-byte
        // store of their next-pass digits
        static_assert(EXT == 1 && sizeof(T) == 4 && SIDE, "narrow pool: pooled keys with the side stream");
        constexpr uint32_t NG4 = NT / 16;
        const uint32_t l4 = 4 * (tid & 15);
        uint16_t *__restrict__ o16 = reinterpret_cast<uint16_t *>(out);
        for (uint32_t j = tid / 16; j < gtot; j += NG4) {
            const uint32_t d = L.desc[j];
            const uint2 m = L.meta[d];
            const uint32_t jj = j - L.gbase[d], cd = m.y & 0xFFu, tbx = m.x & TB;
            const uint64_t gv = *reinterpret_cast<const uint64_t *>(&L.gaddr[d]);
            const uint32_t g0 = m.x >> 16;
            const uint32_t gb = jj < g0 ? (uint32_t)gv + jj : (uint32_t)(gv >> 32) + (jj - g0);
            const uint64_t a = (uint64_t)gb * G + l4;
            const uint32_t q = jj * G + l4;
            uint32_t x[4];
#pragma unroll
            for (int i = 0; i < 4; ++i)
                x[i] = (uint32_t)lds_pick(q + i < cd, &L.carry[d * CS + q + i], &L.tile[tbx + q + i - cd]);
            const uint32_t r01 = ((x[0] >> rshift) & 0xFFFFu) | ((x[1] >> rshift) << 16);
            const uint32_t r23 = ((x[2] >> rshift) & 0xFFFFu) | ((x[3] >> rshift) << 16);
            st_nt(reinterpret_cast<uint64_t *>(o16 + a), (uint64_t)r01 | ((uint64_t)r23 << 32));
            *reinterpret_cast<uint32_t *>(side + a) = ((x[0] >> shift2) & mask2) | (((x[1] >> shift2) & mask2) << 8) |
                                                      (((x[2] >> shift2) & mask2) << 16) |
                                                      (((x[3] >> shift2) & mask2) << 24);
        }
    } else if constexpr (sizeof(T) == 4) {
        // keys: G / 2 lanes per granule, two consecutive keys per lane (one 8-byte store and
        // one 2-byte side store), half the rounds and metadata reads of one key per lane
        constexpr uint32_t LPG = G / 2, NG2 = NT / LPG;
        const uint32_t l2 = 2 * (tid & (LPG - 1)), grp2 = tid / LPG;
        // element q of d's run: its carries, then the tile's
        const auto elem = [&](uint32_t d, uint32_t q, uint32_t cd, uint32_t tbx) -> uint32_t {
            return (uint32_t)lds_pick(q < cd, &L.carry[d * CS + q], &L.tile[tbx + q - cd]);
        };
        // one granule's write: destination, its two keys, which of them are written
        struct GranW {
            uint64_t a;
            uint32_t x0, x1;
            bool v0, v1;
        };
        const auto gran = [&](uint32_t j) -> GranW {
            const uint32_t d = L.desc[j];
            const uint2 m = L.meta[d];
            const uint32_t jj = j - L.gbase[d], cd = m.y & 0xFFu, tbx = m.x & TB;
            GranW w;
            uint32_t q;
            if constexpr (EXT == 1) {
                // every granule whole; both block addresses in one 64-bit LDS read
                const uint64_t gv = *reinterpret_cast<const uint64_t *>(&L.gaddr[d]);
                const uint32_t g0 = m.x >> 16;
                const uint32_t gb = jj < g0 ? (uint32_t)gv + jj : (uint32_t)(gv >> 32) + (jj - g0);
                w.a = (uint64_t)gb * G + l2;
                q = jj * G + l2;
                w.v0 = w.v1 = true;
            } else {
                const uint64_t pd = L.pend[d];
                const uint32_t wd = m.y >> 16;
                w.a = (pd / G + jj) * G + l2;
                q = (uint32_t)(w.a - pd);  // wraps when a < pd
                w.v0 = w.a >= pd && q < wd;
                w.v1 = w.a + 1 >= pd && q + 1 < wd;
            }
            // reads of keys not written stay inside the digit's run (q = 0)
            w.x0 = elem(d, w.v0 ? q : 0u, cd, tbx);
            w.x1 = elem(d, w.v1 ? q + 1 : 0u, cd, tbx);
            return w;
        };
        const auto put = [&](const GranW &w) {
            if (w.v0 && w.v1) {
                st_nt(reinterpret_cast<uint64_t *>(out + w.a), (uint64_t)w.x0 | ((uint64_t)w.x1 << 32));
                if (SIDE)
                    *reinterpret_cast<uint16_t *>(side + w.a) =
                        (uint16_t)(((w.x0 >> shift2) & mask2) | (((w.x1 >> shift2) & mask2) << 8));
            } else if (w.v0 || w.v1) {
                const uint32_t o = w.v0 ? 0u : 1u, x = w.v0 ? w.x0 : w.x1;
                st_nt(reinterpret_cast<uint32_t *>(out + w.a + o), x);
                if (SIDE) st_side(side + w.a + o, (uint8_t)((x >> shift2) & mask2));
            }
        };
        // pooled pass 1: two granules per group and round, so that their LDS read
        // chains overlap (measured 1 % faster there, 0.5 % slower in the cursor pass 2)
        uint32_t j = grp2;
        if constexpr (EXT == 1)
            for (; j + NG2 < gtot; j += 2 * NG2) {
                const GranW w0 = gran(j), w1 = gran(j + NG2);
                put(w0);
                put(w1);
            }
        for (; j < gtot; j += NG2) put(gran(j));
    } else if constexpr (EXT == 1) {
        // pooled: every granule is whole (the digit's writes start granule-aligned); the
        // first g0 of d go to its current block, the rest to its fresh blocks
        for (uint32_t j = grp; j < gtot; j += NG) {
            const uint32_t d = L.desc[j];
            const uint2 m = L.meta[d];
            const uint2 ga = L.gaddr[d];
            const uint32_t jj = j - L.gbase[d], g0 = m.x >> 16, cd = m.y & 0xFFu;
            const uint32_t gran = jj < g0 ? ga.x + jj : ga.y + (jj - g0);
            const uint64_t a = (uint64_t)gran * G + lane;
            const uint32_t q = jj * G + lane;
            const T x = lds_pick(q < cd, &L.carry[d * CS + q], &L.tile[(m.x & TB) + q - cd]);
            st_nt(out + a, x);
            if (SIDE) st_side(side + a, (uint8_t)(((uint32_t)x >> shift2) & mask2));
        }
    } else
    for (uint32_t j = grp; j < gtot; j += NG) {
        const uint32_t d = L.desc[j];
        const uint2 m = L.meta[d];
        const uint64_t pd = L.pend[d];
        const uint32_t cd = m.y & 0xFFu, wd = m.y >> 16;
        const uint64_t a = (pd / G + (j - L.gbase[d])) * G + lane;
        const uint64_t q = a - pd;  // sequence position inside d (wraps when a < pd)
        const bool valid = a >= pd && q < wd;
        T x = 0;
        if (valid) {
            x = lds_pick(q < cd, &L.carry[d * CS + q], &L.tile[m.x + q - cd]);
#ifdef SGXAMD_ABLATE_NOSTORE  // development ablation: everything but the global stores
            if (x == (T)~0ull) out[0] = x;
#else
            st_nt(out + a, x);
#endif
        }
        // next-pass digit beside the tuple: the 16 lanes of a granule write 16
        // consecutive bytes (measured faster than gathering them into one 16-B store
        // per granule with DPP)
        if (SIDE && valid) st_side(side + a, (uint8_t)(((uint32_t)x >> shift2) & mask2));
    }
    __syncthreads();
    // E. new carries (the next tile's phase A touches only cnt; C/D come after barriers)
    for (uint32_t d = grp; d < F; d += NG) {
        const uint2 m = L.meta[d];
        const uint32_t cd = m.y & 0xFFu, rd = (m.y >> 8) & 0xFFu, wd = m.y >> 16;
        if (wd > 0) {
            if (lane < rd) L.carry[d * CS + lane] = L.tile[(m.x & TB) + wd - cd + lane];
        } else if (lane < rd - cd) {
            L.carry[d * CS + cd + lane] = L.tile[(m.x & TB) + lane];
        }
    }
}

// Scatter of segment g (the body of k_scatter; k_scatter_pair runs two relations' segments
// in one launch).
template <int BITS, int ITEMS, int NT, bool SIDE>
__device__ __forceinline__ void scatter_segment(ScatterLds<BITS, ITEMS, NT> &L, uint32_t g,
                                                const uint64_t *__restrict__ in, uint64_t *__restrict__ out,
                                                const SegMap &m, uint32_t shift, const uint64_t *__restrict__ cur_init,
                                                HistLayout layout, uint32_t nseg_stride,
                                                const uint64_t *__restrict__ digit_base, uint8_t *__restrict__ side,
                                                uint32_t shift2, uint32_t mask2) {
    constexpr uint32_t TILE = NT * ITEMS;
    constexpr uint32_t F = 1u << BITS, NG = NT / kGran, CS = kGran - 1;
    static_assert(F <= NT, "one owner thread per digit");
    uint32_t r;
    uint64_t b, e;
    if (!seg_lookup(m, g, L.sbase, r, b, e)) return;
    uint64_t pend = 0;
    uint32_t carried = 0;
    const uint32_t tid = threadIdx.x;
    if (tid < F) {
        pend = cur_init[hist_index(layout, g, tid, F, nseg_stride)] +
               (digit_base ? digit_base[(uint64_t)r * F + tid] : 0);
        L.cnt[tid] = 0;
    }
    __syncthreads();  // sbase (aliased with tile) is dead from here on
    // segments hold far fewer than 2^29 tuples (seg_size_for), so byte offsets fit 32 bits
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(in + b, (uint32_t)((e - b) * sizeof(uint64_t)));
    // Two tiles in flight: tile T+2 loads into T's registers as soon as T is sorted into
    // LDS, and T+1's registers are waited for right after that — before T's stores are
    // issued.  gfx950 retires loads and stores through one in-order vmcnt, so a wait for
    // a load also waits for every older store; placed here, the older stores are those of
    // tile T-1, issued a whole sort phase earlier, instead of the ones just issued.
    // Loads past the segment end read 0 (buffer bounds), so every load is unconditional
    // and the compiler sees a fixed count of loads between a load and its use.
    uint64_t va[ITEMS], vb[ITEMS];
    load_tile<ITEMS, NT>(rs, 0u, va);
    load_tile<ITEMS, NT>(rs, TILE * 8u, vb);
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) asm volatile("" ::"v"(va[k]));
    // Each sort reads registers that were waited for earlier in straight-line code, so
    // the compiler's wait analysis never merges a loop back-edge into a first use.
    uint32_t gt = scatter_tile_sort<BITS, ITEMS, NT>(L, pend, carried, va, out, (uint32_t)min<uint64_t>(TILE, e - b),
                                                     shift, b);
    for (uint64_t tb = b;; tb += 2 * TILE) {
        const uint32_t off = (uint32_t)((tb - b) * 8);
        // tile tb is sorted in LDS; vb holds (in flight) tile tb + TILE
        load_tile<ITEMS, NT>(rs, off + 2 * TILE * 8u, va);
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) asm volatile("" ::"v"(vb[k]));
        scatter_tile_write<BITS, ITEMS, NT, SIDE>(L, out, gt, side, shift2, mask2);
        if (tb + TILE >= e) break;
        gt = scatter_tile_sort<BITS, ITEMS, NT>(L, pend, carried, vb, out, (uint32_t)min<uint64_t>(TILE, e - tb - TILE),
                                                shift, tb + TILE);
        load_tile<ITEMS, NT>(rs, off + 3 * TILE * 8u, vb);
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) asm volatile("" ::"v"(va[k]));
        scatter_tile_write<BITS, ITEMS, NT, SIDE>(L, out, gt, side, shift2, mask2);
        if (tb + 2 * TILE >= e) break;
        gt = scatter_tile_sort<BITS, ITEMS, NT>(L, pend, carried, va, out,
                                                (uint32_t)min<uint64_t>(TILE, e - tb - 2 * TILE), shift, tb + 2 * TILE);
    }
    // flush the carried (partial) granules
    __syncthreads();
    if (tid < F) {
        L.pend[tid] = pend;
        L.cnt[tid] = carried;
    }
    __syncthreads();
    const uint32_t lane = tid & (kGran - 1);
    for (uint32_t d = tid / kGran; d < F; d += NG) {
        if (lane < L.cnt[d]) {
            const uint64_t x = L.carry[d * CS + lane];
            out[L.pend[d] + lane] = x;
            if (SIDE) side[L.pend[d] + lane] = (uint8_t)(((uint32_t)x >> shift2) & mask2);
        }
    }
}

template <int BITS, int ITEMS, int NT, bool SIDE>
__global__ __launch_bounds__(NT, (scatter_waves_per_simd<BITS, ITEMS, NT>())) void k_scatter(
    const uint64_t *__restrict__ in, uint64_t *__restrict__ out, SegMap m, uint32_t shift,
    const uint64_t *__restrict__ cur_init, HistLayout layout, uint32_t nseg_stride,
    const uint64_t *__restrict__ digit_base, uint8_t *__restrict__ side, uint32_t shift2, uint32_t mask2) {
    __shared__ ScatterLds<BITS, ITEMS, NT> L;
    scatter_segment<BITS, ITEMS, NT, SIDE>(L, xcd_contiguous(blockIdx.x, gridDim.x), in, out, m, shift, cur_init,
                                           layout, nseg_stride, digit_base, side, shift2, mask2);
}

// Both relations' one-pass scatters in one launch (small joins): workgroups
// [0, gridR) take R's segments, [gridR, gridR + gridS) S's, and the last one lays out the
// partitions.  A scatter workgroup first takes its cursor bases itself -- the digit starts
// of its segment's totals copy (an exclusive scan over the digits of this call's totals,
// complete since k_hist_pair's launch ended) -- so no workgroup waits on another.  The
// layout workgroup writes both relations' partition starts / counts and largest
// partitions, the build/probe task list (k_make_tasks's rule: the further S chunks of
// partitions above s_chunk), and zeroes the other set of totals, which the next call's
// histograms add into (the totals alternate between two sets per call: the scatters
// still read this call's set).
struct ScatterPairRel {
    const uint64_t *in;
    uint64_t *out;
    SegMap m;
    uint32_t grid;
    const uint64_t *offs;
    const uint64_t *tot;  // [kSyncSpread][kMaxF]: this call's digit totals (k_hist_pair)
    uint64_t *tot_next;   // the other set, zeroed for the next call
    uint64_t *start, *cnt;  // partition starts / counts (the build/probe's table)
};

// Digit totals of a relation, start[d] = the exclusive scan (F <= kMaxF, one block).
// base (optional) += the copies before copy c of each digit.
template <int NT>
__device__ __forceinline__ void pair_starts(const uint64_t *__restrict__ tot, uint32_t F, uint32_t c, uint64_t *start,
                                            uint64_t *count, uint64_t *scratch) {
    uint64_t carry = 0;
    for (uint32_t d0 = 0; d0 < F; d0 += NT) {
        const uint32_t d = d0 + threadIdx.x;
        uint64_t v = 0, before = 0;
#pragma unroll
        for (uint32_t k = 0; k < kSyncSpread; ++k) {
            const uint64_t x = d < F ? tot[(uint64_t)k * kMaxF + d] : 0ull;
            before += k < c ? x : 0ull;
            v += x;
        }
        uint64_t t;
        const uint64_t ex = block_excl_scan_u64(v, scratch, &t);
        if (d < F) {
            start[d] = carry + ex + before;
            if (count) count[d] = v;
        }
        carry += t;
    }
}

template <int BITS, int ITEMS, int NT>
__global__ __launch_bounds__(NT, (scatter_waves_per_simd<BITS, ITEMS, NT>())) void k_scatter_pair(
    ScatterPairRel A, ScatterPairRel B, uint32_t shift, uint64_t *__restrict__ over, uint32_t over_cap,
    uint64_t *__restrict__ meta, uint64_t s_chunk, uint64_t *__restrict__ kmax_next) {
    __shared__ ScatterLds<BITS, ITEMS, NT> L;
    __shared__ uint64_t base[1u << BITS];
    __shared__ uint64_t scratch[NT / kWave + 1];
    constexpr uint32_t F = 1u << BITS;
    if (blockIdx.x == A.grid + B.grid) {  // the layout workgroup
        uint64_t *cR = reinterpret_cast<uint64_t *>(L.tile), *cS = cR + F;  // (the tile space: no scatter here)
        pair_starts<NT>(A.tot, F, 0, A.start, cR, scratch);
        pair_starts<NT>(B.tot, F, 0, B.start, cS, scratch);
        __syncthreads();
        uint64_t base_over = 0, mr = 0, ms = 0;
        for (uint32_t p0 = 0; p0 < F; p0 += NT) {
            const uint32_t p = p0 + threadIdx.x;
            const uint64_t nR = p < F ? cR[p] : 0, nS = p < F ? cS[p] : 0;
            if (p < F) {
                A.cnt[p] = nR;
                B.cnt[p] = nS;
            }
            mr = nR > mr ? nR : mr;
            ms = nS > ms ? nS : ms;
            const uint64_t k = (nR == 0 || nS <= s_chunk) ? 0 : (nS + s_chunk - 1) / s_chunk - 1;
            uint64_t t;
            const uint64_t ex = base_over + block_excl_scan_u64(k, scratch, &t);
            for (uint64_t j = 0; j < k && ex + j < over_cap; ++j) over[ex + j] = p | ((j + 1) << 32);
            base_over += t;
        }
        mr = block_max_u64(mr, scratch);
        ms = block_max_u64(ms, scratch);
        if (threadIdx.x == 0) {
            meta[0] = mr;
            meta[1] = ms;
            meta[2] = base_over;  // n_over (u32, low word; the high word is 0)
        }
        for (uint32_t i = threadIdx.x; i < kSyncSpread * kMaxF; i += NT) {
            A.tot_next[i] = 0;
            B.tot_next[i] = 0;
        }
        if (kmax_next && threadIdx.x == 0) *kmax_next = 0;  // the next call's largest R key
        return;
    }
    const bool isB = blockIdx.x >= A.grid;
    const ScatterPairRel &P = isB ? B : A;
    const uint32_t g = isB ? blockIdx.x - A.grid : blockIdx.x;
    dbg_stamp(1, 0);
    pair_starts<NT>(P.tot, F, g % kSyncSpread, base, nullptr, scratch);
    __syncthreads();
    scatter_segment<BITS, ITEMS, NT, false>(L, g, P.in, P.out, P.m, shift, P.offs, kDigitMajor, P.grid, base, nullptr,
                                            0, 0);
    dbg_stamp(1, 2);
}

hipError_t launch_scatter_pair(const row_t *R, row_t *outR, const SegMap &mR, uint32_t gridR, const uint64_t *offsR,
                               const uint64_t *totR, uint64_t *totR_next, uint64_t *startR, uint64_t *cntR,
                               const row_t *S, row_t *outS, const SegMap &mS, uint32_t gridS, const uint64_t *offsS,
                               const uint64_t *totS, uint64_t *totS_next, uint64_t *startS, uint64_t *cntS,
                               uint32_t shift, uint32_t bits, uint64_t *over, uint32_t over_cap, uint64_t *meta,
                               uint64_t s_chunk, hipStream_t s, uint64_t *kmax_next) {
    constexpr int ITEMS = kScatterItems, NT = kScatterThreads;
    const ScatterPairRel A{reinterpret_cast<const uint64_t *>(R), reinterpret_cast<uint64_t *>(outR), mR, gridR,
                           offsR, totR, totR_next, startR, cntR};
    const ScatterPairRel B{reinterpret_cast<const uint64_t *>(S), reinterpret_cast<uint64_t *>(outS), mS, gridS,
                           offsS, totS, totS_next, startS, cntS};
    const dim3 grid(gridR + gridS + 1);
#define PAIR_CASE(BB)                                                                                       \
    case BB:                                                                                                \
        if constexpr (sizeof(ScatterLds<BB, ITEMS, NT>) + (8u << BB) + 8 * (NT / kWave + 1) <= 160 * 1024 &&  \
                      (1 << BB) <= NT) {                                                                     \
            hipLaunchKernelGGL((k_scatter_pair<BB, ITEMS, NT>), grid, dim3(NT), 0, s, A, B, shift, over,       \
                               over_cap, meta, s_chunk, kmax_next);                                         \
            break;                                                                                          \
        } else {                                                                                            \
            return hipErrorInvalidValue;                                                                    \
        }
    switch (bits) {
        PAIR_CASE(0)
        PAIR_CASE(1)
        PAIR_CASE(2)
        PAIR_CASE(3)
        PAIR_CASE(4)
        PAIR_CASE(5)
        PAIR_CASE(6)
        PAIR_CASE(7)
        PAIR_CASE(8)
        PAIR_CASE(9)
        default:
            return hipErrorInvalidValue;
    }
#undef PAIR_CASE
    return hipGetLastError();
}

template <int ITEMS, int NT>
hipError_t launch_scatter_items(const uint64_t *in, uint64_t *out, const SegMap &m, uint32_t grid, uint32_t shift,
                                uint32_t bits, const uint64_t *cursors, HistLayout layout, uint32_t nseg_stride,
                                const uint64_t *digit_base, hipStream_t s, const DigitSide *ds = nullptr) {
    uint8_t *side = ds ? ds->side : nullptr;
    const uint32_t shift2 = ds ? ds->shift2 : 0, mask2 = ds ? (1u << ds->bits2) - 1u : 0;
#define SCATTER_CASE(B)                                                                                  \
    case B:                                                                                              \
        if constexpr (sizeof(ScatterLds<B, ITEMS, NT>) <= 160 * 1024 && (1 << B) <= NT) {                  \
            if (side)                                                                                    \
                hipLaunchKernelGGL((k_scatter<B, ITEMS, NT, true>), dim3(grid), dim3(NT), 0, s, in, out, m, \
                                   shift, cursors, layout, nseg_stride, digit_base, side, shift2, mask2); \
            else                                                                                         \
                hipLaunchKernelGGL((k_scatter<B, ITEMS, NT, false>), dim3(grid), dim3(NT), 0, s, in, out, m, \
                                   shift, cursors, layout, nseg_stride, digit_base, side, shift2, mask2); \
            break;                                                                                       \
        } else {                                                                                         \
            return hipErrorInvalidValue;                                                                 \
        }
    switch (bits) {
        SCATTER_CASE(0)
        SCATTER_CASE(1)
        SCATTER_CASE(2)
        SCATTER_CASE(3)
        SCATTER_CASE(4)
        SCATTER_CASE(5)
        SCATTER_CASE(6)
        SCATTER_CASE(7)
        SCATTER_CASE(8)
        SCATTER_CASE(9)
        default:
            return hipErrorInvalidValue;
    }
#undef SCATTER_CASE
    return hipGetLastError();
}

hipError_t launch_scatter(const row_t *in, row_t *out, const SegMap &m, uint32_t grid, uint32_t shift,
                          uint32_t bits, const uint64_t *cursors, HistLayout layout, uint32_t nseg_stride,
                          const uint64_t *digit_base, const DigitSide *ds, hipStream_t s) {
    if (grid == 0) return hipSuccess;
    const uint64_t *i64 = reinterpret_cast<const uint64_t *>(in);
    uint64_t *o64 = reinterpret_cast<uint64_t *>(out);
    return launch_scatter_items<kScatterItems, kScatterThreads>(i64, o64, m, grid, shift, bits, cursors, layout,
                                                                nseg_stride, digit_base, s, ds);
}

// ------------------------------------------------ pooled pass 1, block-list pass 2 ---
// Two-pass plans without a pass-1 histogram (rho_internal.hpp PoolOut).  Pass 1
// (EXT 1): the same tile sort and write combining, but a digit's granules go to a chain
// of kBlk-tuple blocks taken from the workgroup's own pool (one LDS atomic per new
// block) instead of to cursors from a histogram + scan, so the relation is read once.
// Pass 2 (EXT 2): a segment is up to kPass2Ents blocks of one region; a tile is
// TILE / kBlk whole blocks, item k of thread t being tuple (t mod kBlk) of block
// k * NT / kBlk + t / kBlk — uniform per wave, so each item loads through a buffer
// resource over its block (lanes past the block's fill read 0 and are masked out).

// Tile loads of a block-list segment (entries staged in LDS); returns the valid mask
// (bit k: item k of this lane) and, in bit 31, whether the whole tile is full.
// in: the pass-1 output, IS-byte elements.
template <typename T, int IS, int ITEMS, int NT, int BITS>
__device__ __forceinline__ uint32_t load_tile_blk(const char *__restrict__ in,
                                                  const ScatterLds<BITS, ITEMS, NT, 2, T> &L, uint32_t nent,
                                                  uint32_t e0, T (&dst)[ITEMS]) {
    static_assert(NT % kBlk == 0, "a wave reads inside one block");
    constexpr uint32_t BPT = ITEMS * (NT / kBlk);  // blocks per tile
    static_assert(BPT <= kWave, "one list entry per lane");
    const uint32_t o = threadIdx.x & (kBlk - 1), lane = __lane_id();
    const uint32_t h = __builtin_amdgcn_readfirstlane(threadIdx.x >> kBlkShift);
    // the tile's list entries, one per lane (LDS broadcast-free, one read)
    const uint64_t en = (lane < BPT && e0 + lane < nent) ? L.ents[e0 + lane] : 0ull;
    const uint32_t en_lo = (uint32_t)en, en_hi = (uint32_t)(en >> 32);
    // all blocks present and full: every item valid (the common case)
    const bool full = __ballot(lane < BPT && en_hi != kBlk) == 0;
    uint32_t vm = 0;
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        const uint32_t idx = (uint32_t)k * (NT / kBlk) + h;
        const uint32_t phys = __builtin_amdgcn_readlane(en_lo, idx);
        const uint32_t fill = __builtin_amdgcn_readlane(en_hi, idx);
        const __amdgpu_buffer_rsrc_t rs = make_rsrc(in + (uint64_t)phys * (kBlk * IS), fill * (uint32_t)IS);
        dst[k] = buf_ld_nt_t<T>(rs, o * (uint32_t)IS, 0u);
        if (!full) vm |= (o < fill ? 1u : 0u) << k;
    }
    // bit 31: the whole tile is full — workgroup-uniform (every wave sees the same
    // entries), unlike the per-lane masks, so callers may branch on it around barriers
    static_assert(ITEMS < 31, "bit 31 is the full-tile flag");
    return full ? (0x80000000u | ((1u << ITEMS) - 1u)) : vm;
}

// EXT 0: contiguous segment g of `in` -> `out` at the cursors cur_init (layout, stride,
//        + digit_base), as scatter_segment (the keys-only shard partition).
// EXT 1: contiguous segment g of `in` -> pooled output (po), digit side stream.
// EXT 2: block-list segment g (list) -> `out` at the segment-major cursors cur_init.
// T: the element written (tuple or key); IS: the input element size in bytes.
template <int BITS, int ITEMS, int NT, int EXT, typename T, int IS, int F2 = 0, int OB = (int)sizeof(T)>
__device__ __forceinline__ void scatter_segment_ext(ScatterLds<BITS, ITEMS, NT, EXT, T, OB> &L, uint32_t g,
                                                    const char *__restrict__ in, T *__restrict__ out,
                                                    const SegMap &m, uint32_t shift,
                                                    const uint64_t *__restrict__ cur_init,
                                                    const uint64_t *__restrict__ list, const PoolOut &po,
                                                    uint8_t *__restrict__ side, uint32_t shift2, uint32_t mask2,
                                                    HistLayout layout = kSegMajor, uint32_t nseg_stride = 0,
                                                    const uint64_t *__restrict__ digit_base = nullptr,
                                                    ChainState *cs = nullptr) {
    using LdsT = ScatterLds<BITS, ITEMS, NT, EXT, T, OB>;
    constexpr uint32_t TILE = NT * ITEMS, BPT = TILE / kBlk;
    constexpr uint32_t F = 1u << BITS, G = LdsT::G, GPB = LdsT::GPB, NG = NT / G, CS = G - 1;
    constexpr bool SIDE = EXT == 1 && F2 == 0;  // chain histograms replace the side stream
    static_assert(F2 == 0 || (EXT == 1 && sizeof(T) == 4), "chain histograms: pooled keys");
    static_assert(F <= NT, "one owner thread per digit");
    static_assert(sizeof(T) <= IS, "elements are the input elements or their key words");
    uint32_t r;
    uint64_t b, e;
    if (!seg_lookup(m, g, L.sbase, r, b, e)) return;
    uint64_t pend = 0;
    uint32_t carried = 0;
    const uint32_t tid = threadIdx.x;
    const uint32_t gp = EXT == 1 ? g + po.g0 : g;  // pooled: the segment's id among all launches' segments
    PoolState ps{0u, 0u, EXT == 1 ? gp * po.pool_blocks : 0u, po.binfo};
    if (tid < F) {
        if constexpr (EXT != 1)
            pend = cur_init[hist_index(layout, g, tid, F, nseg_stride)] +
                   (digit_base ? digit_base[(uint64_t)r * F + tid] : 0);
        L.cnt[tid] = 0;
    }
    if (tid == 0) {
        L.pool_next = 0;
        L.kmax = 0;
    }
    if constexpr (F2 > 0) {
        for (uint32_t i = tid; i < F * F2 / 2; i += NT) cs->h2[i] = 0;
    }
    uint32_t nent = 0;
    if constexpr (EXT == 2) {
        nent = (uint32_t)(e - b);  // <= kPass2Ents (the plan's segment size)
        for (uint32_t i = tid; i < nent; i += NT) L.ents[i] = list[b + i];
    }
    __syncthreads();  // sbase (aliased with tile) is dead from here on
    const uint32_t ntiles = EXT == 2 ? (nent + BPT - 1) / BPT : (uint32_t)((e - b + TILE - 1) / TILE);
    // (EXT 1) segments hold far fewer than 2^29 elements, so byte offsets fit 32 bits
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(in + b * IS, EXT == 2 ? 0u : (uint32_t)((e - b) * IS));
    const auto load = [&](uint32_t ti, T(&dst)[ITEMS]) -> uint32_t {
        if constexpr (EXT == 2) {
            return load_tile_blk<T, IS, ITEMS, NT, BITS>(in, L, nent, ti * BPT, dst);
        } else {
            load_tile_t<T, IS, ITEMS, NT>(rs, ti * TILE * (uint32_t)IS, dst);
            return 0u;
        }
    };
    const auto tn_of = [&](uint32_t ti, uint32_t vm) -> uint32_t {
        if constexpr (EXT == 2) return vm;
        return (uint32_t)min<uint64_t>(TILE, e - b - (uint64_t)ti * TILE);
    };
    // full tiles (all but the segment's last in pass 1; tiles without a partial block in
    // pass 2) sort without per-item validity checks.  The test must be uniform over the
    // workgroup (the sort has barriers): tn itself with contiguous input, the loader's
    // full-tile bit with block-list input (the per-lane masks differ).
    const auto is_full = [&](uint32_t tn) -> bool {
        if constexpr (EXT == 2) return (tn >> 31) != 0;
        return tn == TILE;
    };
    // (pooled pass 1, EXT 1, keeps one sort copy: a full-tile copy spills 3-5 VGPRs there)
    const auto sort = [&](T(&v)[ITEMS], uint32_t tn) -> uint32_t {
        if (EXT != 1 && is_full(tn))
            return scatter_tile_sort<BITS, ITEMS, NT, EXT, T, true, 0, OB>(L, pend, carried, v, out, tn, shift, 0, &ps);
        return scatter_tile_sort<BITS, ITEMS, NT, EXT, T, false, F2, OB>(L, pend, carried, v, out, tn, shift, 0, &ps,
                                                                         cs);
    };
    // pooled keys: the largest key of the segment (lanes past its end load 0): whether
    // pass 2 may write 16-bit residuals (k_sort_blk), and the build/probe's table size
    constexpr bool KOR = EXT == 1 && sizeof(T) == 4;
    uint32_t kmax = 0;
    const auto key_max = [&](const T(&v)[ITEMS]) {
        if constexpr (KOR) {
#pragma unroll
            for (int k = 0; k < ITEMS; ++k) kmax = max(kmax, (uint32_t)v[k]);
        }
    };
    // the two-tiles-in-flight pipeline of scatter_segment
    T va[ITEMS], vb[ITEMS];
    uint32_t ma = load(0, va);
    uint32_t mb = load(1, vb);
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) asm volatile("" ::"v"(va[k]));
    key_max(va);
    uint32_t gt = sort(va, tn_of(0, ma));
    for (uint32_t ti = 0;; ti += 2) {
        ma = load(ti + 2, va);
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) asm volatile("" ::"v"(vb[k]));
        scatter_tile_write<BITS, ITEMS, NT, SIDE, EXT, T, OB>(L, out, gt, side, shift2, mask2, po.rshift);
        if (ti + 1 >= ntiles) break;
        key_max(vb);
        gt = sort(vb, tn_of(ti + 1, mb));
        mb = load(ti + 3, vb);
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) asm volatile("" ::"v"(va[k]));
        scatter_tile_write<BITS, ITEMS, NT, SIDE, EXT, T, OB>(L, out, gt, side, shift2, mask2, po.rshift);
        if (ti + 2 >= ntiles) break;
        key_max(va);
        gt = sort(va, tn_of(ti + 2, ma));
    }
    if (KOR && kmax) atomicMax(&L.kmax, kmax);
    // flush the carried (partial) granules; pooled: close every chain
    __syncthreads();
    if (tid < F) {
        if constexpr (EXT == 1) {
            uint32_t gran = 0;
            if (carried) {
                const uint32_t off = (uint32_t)(pend / G) & (GPB - 1);
                if (off == 0) {  // the chain is empty or its block is full
                    ps.cur = ps.pool0 + atomicAdd(&L.pool_next, 1u);
                    ++ps.nb;
                }
                gran = ps.cur * GPB + off;
            }
            const uint64_t Tn = pend + carried;  // elements of digit tid in this segment
            if (ps.nb) po.binfo[ps.cur] = tid | ((uint32_t)(Tn - (uint64_t)(ps.nb - 1) * kBlk) << 16);
            po.cnt[(uint64_t)tid * po.nseg + gp] = ((uint64_t)ps.nb << 40) | Tn;
            L.pend[tid] = (uint64_t)gran * G;
        } else {
            L.pend[tid] = pend;
        }
        L.cnt[tid] = carried;
    }
    __syncthreads();
    if (EXT == 1 && tid == 0) {
        po.used[gp] = L.pool_next;
        if (KOR && po.kmax) po.kmax[gp] = L.kmax;
    }
    const uint32_t lane = tid & (G - 1);
    for (uint32_t d = tid / G; d < F; d += NG) {
        if (lane < L.cnt[d]) {
            const T x = L.carry[d * CS + lane];
            if constexpr (OB == 2)  // narrow pool: the residual
                reinterpret_cast<uint16_t *>(out)[L.pend[d] + lane] = (uint16_t)((uint32_t)x >> po.rshift);
            else
                out[L.pend[d] + lane] = x;
            if (SIDE) side[L.pend[d] + lane] = (uint8_t)(((uint32_t)x >> shift2) & mask2);
        }
    }
    if constexpr (F2 > 0) chain_store<F, F2, NT>(cs->h2, cs->out, gp, cs->nseg);
}

// OB 2: the narrow pool (keys' residuals, u16), written speculatively: the relation's
// largest key (kmax, folded by launch_pool_layout) tells afterwards whether every residual
// fit; if not, the launches are repeated as a 4-byte pool, guarded by po.guard (they
// return at once when the narrow pool stood).
template <int BITS, int ITEMS, int NT, typename T, int IS, int F2 = 0, int OB = (int)sizeof(T)>
__global__ __launch_bounds__(NT, (scatter_waves_per_simd<BITS, ITEMS, NT, 1, T, OB>())) void k_scatter_pool(
    const char *__restrict__ in, T *__restrict__ out, SegMap m, uint32_t shift, PoolOut po,
    uint8_t *__restrict__ side, uint32_t shift2, uint32_t mask2, uint32_t *__restrict__ chain) {
    __shared__ ScatterLds<BITS, ITEMS, NT, 1, T, OB> L;
    if (pool_guard_skip(po)) return;
    const uint32_t g = xcd_contiguous(blockIdx.x, gridDim.x);
    if constexpr (F2 > 0) {
        __shared__ uint32_t h2[(1u << BITS) * F2 / 2];
        ChainState cs{h2, chain, g + po.g0, po.nseg, shift2};
        scatter_segment_ext<BITS, ITEMS, NT, 1, T, IS, F2>(L, g, in, out, m, shift, nullptr, nullptr, po, side, shift2,
                                                           mask2, kSegMajor, 0, nullptr, &cs);
    } else {
        scatter_segment_ext<BITS, ITEMS, NT, 1, T, IS, 0, OB>(L, g, in, out, m, shift, nullptr, nullptr, po, side,
                                                              shift2, mask2);
    }
}

// The one-pass scatter with cursors (k_scatter) writing the key words of the tuples.
template <int BITS, int ITEMS, int NT>
__global__ __launch_bounds__(NT, (scatter_waves_per_simd<BITS, ITEMS, NT, 0, uint32_t>())) void k_scatter_keys(
    const char *__restrict__ in, uint32_t *__restrict__ out, SegMap m, uint32_t shift,
    const uint64_t *__restrict__ cursors, HistLayout layout, uint32_t nseg_stride,
    const uint64_t *__restrict__ digit_base) {
    __shared__ ScatterLds<BITS, ITEMS, NT, 0, uint32_t> L;
    const PoolOut none{};
    scatter_segment_ext<BITS, ITEMS, NT, 0, uint32_t, 8>(L, xcd_contiguous(blockIdx.x, gridDim.x), in, out, m, shift,
                                                         cursors, nullptr, none, nullptr, 0, 0, layout, nseg_stride,
                                                         digit_base);
}

template <int BITS, int ITEMS, int NT, typename T>
__global__ __launch_bounds__(NT, (scatter_waves_per_simd<BITS, ITEMS, NT, 2, T>())) void k_scatter_blk(
    const char *__restrict__ in, const uint64_t *__restrict__ list, T *__restrict__ out, SegMap m, uint32_t shift,
    const uint64_t *__restrict__ cursors) {
    __shared__ ScatterLds<BITS, ITEMS, NT, 2, T> L;
    const PoolOut none{};
    scatter_segment_ext<BITS, ITEMS, NT, 2, T, (int)sizeof(T)>(L, blockIdx.x, in, out, m, shift, cursors, list, none,
                                                               nullptr, 0, 0);
}

// ----------------------------------------- pass 2 of key partitions as an LDS sort ---
// radix_cluster (:715-761) / the pass-2 partition_copy over the block list of a
// segment, for 4-byte keys: each tile of TILE keys is counting-sorted by its pass-2
// digit in LDS and written straight to the final partitions at the segment's cursors
// (the pass-2 histogram + scan: cursors[g * F + d]).  Per key: one LDS atomic (rank),
// one LDS read + write (placement), one LDS read of the sorted key and one 8-byte
// read of its digit's offset, one 4-byte store; no carries and no granule
// descriptors (k_scatter_blk's write combining).  The consecutive tiles of a segment
// continue the same digit runs, so a line split between two tiles is completed by the
// same workgroup moments later (in its XCD's L2); only the runs' ends at segment
// boundaries are written as partial lines by two workgroups.  The next tile's keys
// load while a tile is sorted and written (two register sets).
// List entries staged in LDS: a segment of up to kSortEnts blocks (kPass2Ents); longer
// segments read their entries from the list itself.
constexpr uint32_t kSortEnts = 1024;
template <int BITS, int NT, int ITEMS>
struct SortBlkLds {
    static constexpr uint32_t F = 1u << BITS, TILE = NT * ITEMS;
    union {
        uint32_t sbase[kMaxF + 1];  // segment table (seg_lookup, before the first tile)
        uint32_t sorted[TILE];      // the tile's keys, digit-sorted
    };
    uint64_t ents[kSortEnts];   // the segment's block list: physical block | fill << 32
    uint64_t dbase[F];          // next output position of digit d in this segment
    uint64_t off[F];            // destination of sorted position q with digit d: off[d] + q
    uint32_t cnt[F];            // tile histogram (phase A), zero between tiles
    uint32_t start[F];          // digit-sorted tile offset of d
    uint32_t wsum[NT / kWave + 1];
};

// Geometry (compile-time variants through scripts/build_variant.sh + ab_lib.sh, r03v-x):
// 1024 threads x 16 keys = 16,384-key tiles, one workgroup per CU (4 waves per SIMD,
// 128 VGPRs), phase D fully unrolled: 0.529-0.554 ms per 2^28 keys on three boxes
// against 0.585-0.63 for 512 x 16 with three workgroups per CU (the longer digit runs
// per tile -- 128 keys, 512 B -- leave fewer partial lines and per-tile steps).  Larger
// tiles spill (24 keys per thread: 0.94 ms); two 1024-thread workgroups per CU without
// the next-tile prefetch (64 VGPRs), or with the ranks taken by a second LDS atomic in
// phase C, measured equal (0.52-0.55); 512-key segments (SGXAMD_PASS2_ENTS=512) 0.54-0.57.
#ifndef SGXAMD_SORT_NT
#define SGXAMD_SORT_NT 512
#endif
#ifndef SGXAMD_SORT_ITEMS
#define SGXAMD_SORT_ITEMS 32
#endif
#ifndef SGXAMD_SORT_WGS
#define SGXAMD_SORT_WGS 2
#endif
#ifndef SGXAMD_SORT_UNROLL
#define SGXAMD_SORT_UNROLL 16
#endif
#ifndef SGXAMD_SORT_CRANK
#define SGXAMD_SORT_CRANK 1
#endif
// NAR: narrow partitions — every key's residual above the radix bits fits 16 bits (the
// relation's largest key from pass 1), so the output holds those u16 residuals.  The kernel
// picks the body once (one copy of the loop each, no store branches inside it).
template <int BITS, int NT, int ITEMS, bool NAR>
__device__ __forceinline__ void sort_blk_body(SortBlkLds<BITS, NT, ITEMS> &L, const uint32_t *__restrict__ in,
                                              const uint64_t *__restrict__ list, uint32_t *__restrict__ out, SegMap m,
                                              uint32_t shift, const uint64_t *__restrict__ cursors) {
    using LdsT = SortBlkLds<BITS, NT, ITEMS>;
    constexpr uint32_t F = LdsT::F, TILE = LdsT::TILE, BPT = TILE / kBlk, mask = F - 1, NW = NT / kWave;
    constexpr uint32_t WPB = kBlk / kWave;  // waves per block row: item u of wave w reads block u * (NT / kBlk) + w / WPB
    static_assert(TILE % kBlk == 0 && NT % kBlk == 0 && F <= NT && ITEMS <= 32 && TILE <= 65536, "tile geometry");
    const uint32_t tid = threadIdx.x, lane = __lane_id(), wave = tid / kWave;
    const uint32_t g = blockIdx.x;
    const uint32_t rshift = shift + BITS;
    uint16_t *__restrict__ out16 = reinterpret_cast<uint16_t *>(out);
    uint32_t r;
    uint64_t b, e;
    if (!seg_lookup(m, g, L.sbase, r, b, e)) return;
    const uint32_t nent = (uint32_t)(e - b);
    const bool big = nent > kSortEnts;  // workgroup-uniform
    if (!big)
        for (uint32_t i = tid; i < nent; i += NT) L.ents[i] = list[b + i];
    if (tid < F) {
        L.dbase[tid] = cursors[(uint64_t)g * F + tid];
        L.cnt[tid] = 0;
    }
    __syncthreads();  // sbase (aliased with sorted) is dead from here on
    const uint32_t ntiles = (nent + BPT - 1) / BPT;
    const uint32_t o = tid & (kBlk - 1);
    const uint32_t h = __builtin_amdgcn_readfirstlane(wave / WPB);
    // tile ti's keys: item u = element o of block u * (NT / kBlk) + h of the tile
    // (one block per wave and item, through a buffer resource over its fill: lanes past
    // it read 0 and are masked out); returns the valid mask (bit u: item u)
    const auto load = [&](uint32_t ti, uint32_t(&k)[ITEMS]) -> uint32_t {
        uint32_t vm = 0;
#pragma unroll
        for (int u = 0; u < (int)ITEMS; ++u) {
            const uint32_t idx = ti * BPT + (uint32_t)u * (NT / kBlk) + h;
            // one address per wave: a broadcast
            const uint64_t en = idx < nent ? (big ? list[b + idx] : L.ents[idx]) : 0ull;
            const uint32_t phys = __builtin_amdgcn_readfirstlane((uint32_t)en);
            const uint32_t fill = __builtin_amdgcn_readfirstlane((uint32_t)(en >> 32));
            const __amdgpu_buffer_rsrc_t rs = make_rsrc(in + (uint64_t)phys * kBlk, fill * 4u);
            k[u] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, (int)(o * 4u), 0, 2);
            vm |= (o < fill ? 1u : 0u) << u;
        }
        return vm;
    };
    const auto sort_write = [&](const uint32_t(&k)[ITEMS], uint32_t vm) {
#if SGXAMD_ABLATE_SORT2 == 1  // development ablation: the tile's keys copied in load order (no sort)
        {
            const uint64_t base = ((uint64_t)g * 4 * TILE) % (1ull << 27);
#pragma unroll
            for (int u = 0; u < (int)ITEMS; ++u)
                if ((vm >> u) & 1u) out[base + tid + (uint32_t)u * NT] = k[u];
            return;
        }
#endif
        // A. rank of every key inside its digit (tile histogram at once); SGXAMD_SORT_CRANK:
        // the histogram alone (no returned ranks: no rank registers across the scan), the
        // ranks taken in C from the digit starts
#if SGXAMD_SORT_CRANK
#pragma unroll
        for (int u = 0; u < (int)ITEMS; ++u)
            if ((vm >> u) & 1u) atomicAdd(&L.cnt[(k[u] >> shift) & mask], 1u);
#else
        uint32_t rd[ITEMS];
#pragma unroll
        for (int u = 0; u < (int)ITEMS; ++u) {
            const uint32_t d = (k[u] >> shift) & mask;
            rd[u] = ((vm >> u) & 1u) ? (atomicAdd(&L.cnt[d], 1u) | (d << 16)) : 0u;
        }
#endif
        __syncthreads();
        // B. digit starts (block scan over F counters), destinations, next cursors
        uint32_t c = 0, incl = 0;
        if (tid < F) {
            c = L.cnt[tid];
            incl = wave_incl_scan_u32(c);
            if (lane == kWave - 1 || tid == F - 1) L.wsum[wave] = incl;
        }
        __syncthreads();
        if (tid < F) {
            uint32_t pre = 0;
            for (uint32_t w = 0; w < wave; ++w) pre += L.wsum[w];
            const uint32_t st = pre + incl - c;
            L.start[tid] = st;
            const uint64_t db = L.dbase[tid];
            L.off[tid] = db - st;
            L.dbase[tid] = db + c;
            L.cnt[tid] = 0;
            if (tid == F - 1) L.wsum[NW] = st + c;  // the tile's valid keys
        }
        __syncthreads();
        // C. the tile, digit-sorted
#if SGXAMD_SORT_CRANK
#pragma unroll
        for (int u = 0; u < (int)ITEMS; ++u)
            if ((vm >> u) & 1u) L.sorted[atomicAdd(&L.start[(k[u] >> shift) & mask], 1u)] = k[u];
#else
#pragma unroll
        for (int u = 0; u < (int)ITEMS; ++u)
            if ((vm >> u) & 1u) L.sorted[L.start[rd[u] >> 16] + (rd[u] & 0xFFFFu)] = k[u];
#endif
        __syncthreads();
        // D. sorted position q -> off[d] + q: consecutive lanes, consecutive addresses
        const uint32_t tn = L.wsum[NW];
        if constexpr (NAR) {
#pragma unroll SGXAMD_SORT_UNROLL
            for (int u = 0; u < (int)ITEMS; ++u) {
                const uint32_t q = tid + (uint32_t)u * NT;
                if (q < tn) {
                    const uint32_t x = L.sorted[q];
                    out16[L.off[(x >> shift) & mask] + q] = (uint16_t)(x >> rshift);
                }
            }
            return;
        }
#pragma unroll SGXAMD_SORT_UNROLL
        for (int u = 0; u < (int)ITEMS; ++u) {
            const uint32_t q = tid + (uint32_t)u * NT;
            if (q < tn) {
                const uint32_t x = L.sorted[q];
                // a plain (write-back) store: the lines a store leaves partial are
                // completed in L2 by the next wave or tile, not sent to HBM in pieces
#if SGXAMD_ABLATE_SORT2 == 2  // development ablation: the sort without its stores
                if (x == 0xFFFFFFFFu) out[L.off[(x >> shift) & mask] + q] = x;
#else
                out[L.off[(x >> shift) & mask] + q] = x;
#endif
            }
        }
        // the next tile's phase A touches only cnt (zeroed in B); its C comes after a barrier
    };
    uint32_t ka[ITEMS], kb[ITEMS];
    uint32_t ma = load(0, ka);
    for (uint32_t ti = 0;; ti += 2) {
        const uint32_t mb = load(ti + 1, kb);  // past the last tile: no blocks, all masked
#pragma unroll
        for (int u = 0; u < (int)ITEMS; ++u) asm volatile("" ::"v"(ka[u]));
        sort_write(ka, ma);
        if (ti + 1 >= ntiles) break;
        ma = load(ti + 2, ka);
#pragma unroll
        for (int u = 0; u < (int)ITEMS; ++u) asm volatile("" ::"v"(kb[u]));
        sort_write(kb, mb);
        if (ti + 2 >= ntiles) break;
    }
}

template <int BITS, int NT, int ITEMS>
__global__ __launch_bounds__(NT, NT * SGXAMD_SORT_WGS / 256) void k_sort_blk(const uint32_t *__restrict__ in, const uint64_t *__restrict__ list,
                                                    uint32_t *__restrict__ out, SegMap m, uint32_t shift,
                                                    const uint64_t *__restrict__ cursors,
                                                    const uint32_t *__restrict__ narrow, uint32_t skip_narrow) {
    __shared__ SortBlkLds<BITS, NT, ITEMS> L;
    if (narrow != nullptr && ((*narrow >> (shift + BITS)) >> 16) == 0) {
        if (skip_narrow) return;  // k_place_seg, launched beside it, places them
        sort_blk_body<BITS, NT, ITEMS, true>(L, in, list, out, m, shift, cursors);
        return;
    }
    sort_blk_body<BITS, NT, ITEMS, false>(L, in, list, out, m, shift, cursors);
}

#ifndef SGXAMD_PLACE_WGS  // workgroups per CU of k_place_seg (its LDS holds a segment)
#define SGXAMD_PLACE_WGS (SGXAMD_PASS2_ENTS <= 128 ? 2 : 1)
#endif
#ifndef SGXAMD_PLACE_NT
#define SGXAMD_PLACE_NT (1024 / SGXAMD_PLACE_WGS)
#endif
#ifndef SGXAMD_PLACE_U  // 16-byte loads (4 keys) per thread and tile
#define SGXAMD_PLACE_U 2
#endif
#ifndef SGXAMD_PLACE_NT_STORE  // non-temporal 16-byte stores of the runs
#define SGXAMD_PLACE_NT_STORE 1
#endif
#ifndef SGXAMD_PLACE_XCD  // consecutive segments on one XCD (their shared partial lines meet in one L2)
#define SGXAMD_PLACE_XCD 1
#endif
// Pass 2 of narrow key partitions as one placement per segment (k_place_seg, round 5).
// radix_cluster (radix_join.cpp:715-761) scatters a region by its pass-2 digit at
// cursors from a histogram; here the pass-2 histogram (k_hist_side_blk, over the digit
// side stream) already holds every segment's digit counts -- k_scan_regions turned them
// into the segment's cursors in place, and the counts come back as the difference of
// two consecutive segments' cursors (the region's last segment: its partition ends) --
// so the segment's digit-sorted layout is known before its first key is read.  Each key
// is placed as it arrives: one LDS add (its slot in its digit's run) and one 2-byte LDS
// store of its residual; after the segment's last key, the runs leave for their
// partitions with consecutive lanes on consecutive addresses.  Against k_sort_blk's
// per-16,384-key tile sort (a histogram pass, a scan, a placement and a sorted read per
// tile, four barriers): no per-tile histogram or scan, two barriers per segment, three
// LDS accesses per key instead of five, and digit runs of a whole segment (65,536 keys:
// 512 on average, 1 KiB of output) instead of a tile's (128).
// The segment's residuals are staged in LDS (kPass2Ents * 256 u16: 128 KiB at 256
// blocks, one workgroup per CU; 64 KiB at 128 blocks, two).  Only narrow relations
// (16-bit residuals); k_sort_blk, launched beside it, takes the others.
template <int BITS, int NT>
struct PlaceLds {
    static constexpr uint32_t F = 1u << BITS;
    // d's run sits at st[d] inside a slot range of round_up8(count + 7) u16 that starts
    // on a multiple of 8, with st[d] = dst[d] mod 8: the run's 16-byte pieces in LDS are
    // the 16-byte pieces of its destination (whole-line copies)
    static constexpr uint32_t CAP = kPass2Ents * kBlk + 14 * F;
    union alignas(16) {
        uint32_t sbase[kMaxF + 1];  // segment table (seg_lookup, before the first key)
        uint16_t res[CAP];          // the segment's residuals, digit-sorted
    };
    uint64_t ents[kPass2Ents];  // the segment's block list: physical block | fill << 32
    uint64_t dst[F];            // output position of digit d's run
    uint32_t pos[F];            // next free slot of d's run in res
    uint32_t st[F];             // run start of d in res
    uint32_t pb[F + 1];         // d's slot range starts (non-decreasing); pb[F] = the slots in use
    uint32_t cnt[F];
    uint32_t wsum[NT / kWave];
    uint32_t last;              // the segment is its region's last
};

// I16: the input is a narrow pool (k_scatter_pool OB 2): u16 residuals, the digits in the
// side stream beside them; else 4-byte keys.
// A wide relation (a residual past 16 bits: known on the device only) takes the tile
// sort itself (sort_blk_body over the 4-byte keys, NT x 16384 / NT keys per tile, 4-byte
// keys written to out as u32), so that no k_sort_blk launch waits beside it (round 6:
// one launch less per relation; k_sort_blk's own geometry, 512 x 32 with two workgroups
// per CU, measured 0.487 against 0.53-0.55 ms for this one, r03v-x / r05c).
template <int BITS, int NT>
union PlaceOrSortLds {
    PlaceLds<BITS, NT> p;
    SortBlkLds<BITS, NT, 16384 / NT> w;
};
template <int BITS, int NT, int U, bool I16>
__global__ __launch_bounds__(NT, NT *SGXAMD_PLACE_WGS / 256) void k_place_seg(
    const uint32_t *__restrict__ in, const uint8_t *__restrict__ side, const uint64_t *__restrict__ list,
    uint16_t *__restrict__ out, SegMap m, uint32_t shift, const uint64_t *__restrict__ cursors,
    const uint64_t *__restrict__ part_start, const uint64_t *__restrict__ part_count,
    const uint32_t *__restrict__ narrow) {
    using LdsT = PlaceLds<BITS, NT>;
    constexpr uint32_t F = LdsT::F, mask = F - 1, NW = NT / kWave;
    constexpr uint32_t BPT = NW * U;  // blocks per tile: U per wave, one 16-byte load per lane each
    static_assert(kBlk == 4 * kWave && F <= NT, "placement geometry");
    __shared__ PlaceOrSortLds<BITS, NT> LU;
    LdsT &L = LU.p;
    if (narrow == nullptr) return;
    if (((*narrow >> (shift + BITS)) >> 16) != 0) {  // wide: the 4-byte keys' tile sort
        sort_blk_body<BITS, NT, 16384 / NT, false>(LU.w, in, list, reinterpret_cast<uint32_t *>(out), m, shift,
                                                   cursors);
        return;
    }
    const uint32_t tid = threadIdx.x, lane = __lane_id(), wave = tid / kWave, g = SGXAMD_PLACE_XCD ? xcd_contiguous(blockIdx.x, gridDim.x) : blockIdx.x;
    const uint32_t rshift = shift + BITS;
    uint32_t r;
    uint64_t b, e;
    if (!seg_lookup(m, g, L.sbase, r, b, e)) return;
    const uint32_t nent = (uint32_t)(e - b);  // <= kPass2Ents (fixed-size segments)
    if (tid == 0) L.last = g + 1 == L.sbase[r + 1] ? 1u : 0u;
    for (uint32_t i = tid; i < nent; i += NT) L.ents[i] = list[b + i];
    __syncthreads();  // (last and ents; sbase is dead after the next barrier)
    // the segment's digit counts: the next segment's cursors (or the partition ends) less
    // its own; a block scan of the slot ranges gives the runs' starts
    uint32_t c = 0, slots = 0, incl = 0;
    uint64_t cur = 0;
    if (tid < F) {
        cur = cursors[(uint64_t)g * F + tid];
        const uint64_t nxt = L.last ? part_start[(uint64_t)r * F + tid] + part_count[(uint64_t)r * F + tid]
                                    : cursors[(uint64_t)(g + 1) * F + tid];
        c = (uint32_t)(nxt - cur);
        slots = c ? (c + 7 + 7) & ~7u : 0u;
        L.dst[tid] = cur;
        L.cnt[tid] = c;
        incl = wave_incl_scan_u32(slots);
        if (lane == kWave - 1 || tid == F - 1) L.wsum[wave] = incl;
    }
    __syncthreads();
    if (tid < F) {
        uint32_t pre = 0;
        for (uint32_t w = 0; w < wave; ++w) pre += L.wsum[w];
        L.pb[tid] = pre + incl - slots;
        L.st[tid] = L.pos[tid] = pre + incl - slots + (uint32_t)(cur & 7);
        if (tid == F - 1) L.pb[F] = pre + incl;
    }
    const uint32_t ntiles = (nent + BPT - 1) / BPT;
    // tile ti: item u of wave w = block ti * BPT + u * NW + w, lane l its keys 4l..4l+3
    // (a buffer resource over the block's fill: keys past it read 0 and are masked out)
    // (I16: .x/.y the four residuals, .z their four digits)
    const auto load = [&](uint32_t ti, uint4(&k)[U]) -> uint32_t {
        uint32_t vm = 0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t idx = ti * BPT + (uint32_t)u * NW + wave;
            const uint64_t en = idx < nent ? L.ents[idx] : 0ull;  // one address per wave: a broadcast
            const uint32_t phys = __builtin_amdgcn_readfirstlane((uint32_t)en);
            const uint32_t fill = __builtin_amdgcn_readfirstlane((uint32_t)(en >> 32));
            if constexpr (I16) {
                // (ranges rounded up to whole dwords: the bounds check is per dword, and the
                // elements past the fill are masked out)
                const uint16_t *b16 = reinterpret_cast<const uint16_t *>(in) + (uint64_t)phys * kBlk;
                const uint64_t r = buf_ld_nt_u64(make_rsrc(b16, (fill * 2u + 3u) & ~3u), lane * 8u, 0);
                const uint32_t dg = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(
                    make_rsrc(side + (uint64_t)phys * kBlk, (fill + 3u) & ~3u), (int)(lane * 4u), 0, 2);
                k[u] = make_uint4((uint32_t)r, (uint32_t)(r >> 32), dg, 0u);
            } else {
                k[u] = buf_ld_nt_u128(make_rsrc(in + (uint64_t)phys * kBlk, fill * 4u), lane * 16u, 0);
            }
            const uint32_t f = fill > 4 * lane ? min(fill - 4 * lane, 4u) : 0u;
            vm |= ((1u << f) - 1u) << (4 * u);
        }
        return vm;
    };
    const auto place = [&](const uint4(&k)[U], uint32_t vm) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if constexpr (I16) {
                const uint32_t rr[2] = {k[u].x, k[u].y};
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if ((vm >> (4 * u + j)) & 1u)
                        L.res[atomicAdd(&L.pos[(k[u].z >> (8 * j)) & mask], 1u)] =
                            (uint16_t)(rr[j >> 1] >> (16 * (j & 1)));
            } else {
                const uint32_t w[4] = {k[u].x, k[u].y, k[u].z, k[u].w};
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if ((vm >> (4 * u + j)) & 1u)
                        L.res[atomicAdd(&L.pos[(w[j] >> shift) & mask], 1u)] = (uint16_t)(w[j] >> rshift);
            }
        }
    };
    uint4 ka[U], kb[U];
    uint32_t ma = load(0, ka);
    __syncthreads();  // the runs' starts (pos) are set
    for (uint32_t ti = 0;; ti += 2) {
        const uint32_t mb = load(ti + 1, kb);  // past the last tile: no blocks, all masked
#pragma unroll
        for (int u = 0; u < U; ++u) asm volatile("" ::"v"(ka[u].x), "v"(ka[u].y), "v"(ka[u].z), "v"(ka[u].w));
        place(ka, ma);
        if (ti + 1 >= ntiles) break;
        ma = load(ti + 2, ka);
#pragma unroll
        for (int u = 0; u < U; ++u) asm volatile("" ::"v"(kb[u].x), "v"(kb[u].y), "v"(kb[u].z), "v"(kb[u].w));
        place(kb, mb);
        if (ti + 2 >= ntiles) break;
    }
    __syncthreads();  // the segment is placed
    // the runs out: wave w takes slots [w C, (w + 1) C) (C a multiple of 8) and copies the
    // part of every run inside them: its 16-byte pieces one per lane (ds_read_b128, a
    // 16-byte store on a 16-byte boundary of the output), the up to 7 keys before the
    // first and after the last piece one per lane.  Run bounds are wave-uniform.
    const uint32_t total = L.pb[F];
    const uint32_t C = ((total + NW - 1) / NW + 7) & ~7u;
    const uint32_t q0 = wave * C, q1 = min(total, q0 + C);
    if (q0 >= q1) return;
    uint32_t lo = 0, hi = F;  // the first run that may reach into [q0, q1): the last d with pb[d] <= q0
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (L.pb[mid] <= q0) lo = mid; else hi = mid;
    }
    for (uint32_t d = __builtin_amdgcn_readfirstlane(lo); d < F; ++d) {
        if (__builtin_amdgcn_readfirstlane(L.pb[d]) >= q1) break;
        const uint32_t rs = __builtin_amdgcn_readfirstlane(L.st[d]);
        const uint32_t re = rs + __builtin_amdgcn_readfirstlane(L.cnt[d]);
        const uint32_t a = max(rs, q0), z = min(re, q1);
        if (a >= z) continue;
        // slot q -> output dst[d] + q - rs (o[q] below); o[8k] is 16-byte aligned
        uint16_t *o = out + uni_u64(L.dst[d]);
        o -= rs;
        const uint32_t a8 = min((a + 7) & ~7u, z), z8 = max(z & ~7u, a8);
        if (lane < a8 - a) o[a + lane] = L.res[a + lane];
        if (lane < z - z8) o[z8 + lane] = L.res[z8 + lane];
        for (uint32_t q = a8 + 8 * lane; q < z8; q += 8 * kWave) {
#if SGXAMD_PLACE_NT_STORE
            __builtin_nontemporal_store(*reinterpret_cast<const u32x4_t *>(&L.res[q]),
                                        reinterpret_cast<u32x4_t *>(o + q));
#else
            *reinterpret_cast<uint4 *>(o + q) = *reinterpret_cast<const uint4 *>(&L.res[q]);
#endif
        }
    }
}

// Elements per thread per tile: 8 tuples (32 KiB tiles); keys: 12 in the pooled pass 1
// (24 KiB tiles; 16 spill 17-19 VGPRs at the 128-register cap), 16 in the block-list
// pass 2 (larger tiles amortise the per-tile work: 0.75 -> 0.69 ms per 2^28 keys).
#ifndef SGXAMD_KEY_ITEMS
#define SGXAMD_KEY_ITEMS 12
#endif
#ifndef SGXAMD_POOL_NT  // pooled pass 1: threads per workgroup
#define SGXAMD_POOL_NT kScatterThreads
#endif
#ifndef SGXAMD_KEY_ITEMS_BLK
#define SGXAMD_KEY_ITEMS_BLK 16
#endif
template <typename T, int EXT>
constexpr int items_of() {
    return sizeof(T) == 8 ? kScatterItems : (EXT == 2 ? SGXAMD_KEY_ITEMS_BLK : SGXAMD_KEY_ITEMS);
}

template <typename T, int IS>
hipError_t launch_scatter_pool_t(const void *in, void *out, const SegMap &m, uint32_t grid, uint32_t shift,
                                 uint32_t bits, const PoolOut &po, const DigitSide &ds, hipStream_t s,
                                 uint32_t *chain) {
    constexpr int ITEMS = items_of<T, 1>(), NT = SGXAMD_POOL_NT;
    const char *ib = static_cast<const char *>(in);
    T *o = static_cast<T *>(out);
    const uint32_t mask2 = (1u << ds.bits2) - 1u;
    if (chain) {  // chain histograms (keys, chain_hist_supported): 7-bit pass 1, 6- or 7-bit pass 2
        if constexpr (sizeof(T) == 4) {
            if (bits == 7 && ds.bits2 == 7)
                hipLaunchKernelGGL((k_scatter_pool<7, ITEMS, NT, T, IS, 128>), dim3(grid), dim3(NT), 0, s, ib, o, m,
                                   shift, po, nullptr, ds.shift2, mask2, chain);
            else if (bits == 7 && ds.bits2 == 6)
                hipLaunchKernelGGL((k_scatter_pool<7, ITEMS, NT, T, IS, 64>), dim3(grid), dim3(NT), 0, s, ib, o, m,
                                   shift, po, nullptr, ds.shift2, mask2, chain);
            else
                return hipErrorInvalidValue;
            return hipGetLastError();
        }
        return hipErrorInvalidValue;
    }
    if (po.narrow16) {  // the narrow pool: keys with the side stream, up to 8-bit digits
        if constexpr (sizeof(T) == 4) {
            if (!ds.side || po.guard) return hipErrorInvalidValue;
#define NPOOL_CASE(B)                                                                                          \
    case B:                                                                                                    \
        hipLaunchKernelGGL((k_scatter_pool<B, ITEMS, NT, T, IS, 0, 2>), dim3(grid), dim3(NT), 0, s, ib, o, m, \
                           shift, po, ds.side, ds.shift2, mask2, nullptr);                                     \
        break;
            switch (bits) {
                NPOOL_CASE(1)
                NPOOL_CASE(2)
                NPOOL_CASE(3)
                NPOOL_CASE(4)
                NPOOL_CASE(5)
                NPOOL_CASE(6)
                NPOOL_CASE(7)
                default:
                    return hipErrorInvalidValue;
            }
#undef NPOOL_CASE
            return hipGetLastError();
        }
        return hipErrorInvalidValue;
    }
#define POOL_CASE(B)                                                                                             \
    case B:                                                                                                      \
        if constexpr (sizeof(ScatterLds<B, ITEMS, NT, 1, T>) <= 160 * 1024 && (1 << B) <= NT) {                   \
            hipLaunchKernelGGL((k_scatter_pool<B, ITEMS, NT, T, IS>), dim3(grid), dim3(NT), 0, s, ib, o, m, shift, \
                               po, ds.side, ds.shift2, mask2, nullptr);                                          \
            break;                                                                                               \
        } else {                                                                                                 \
            return hipErrorInvalidValue;                                                                         \
        }
    switch (bits) {
        POOL_CASE(1)
        POOL_CASE(2)
        POOL_CASE(3)
        POOL_CASE(4)
        POOL_CASE(5)
        POOL_CASE(6)
        POOL_CASE(7)
        POOL_CASE(8)
        POOL_CASE(9)
        default:
            return hipErrorInvalidValue;
    }
#undef POOL_CASE
    return hipGetLastError();
}

hipError_t launch_scatter_pool(const void *in, uint32_t in_size, void *out, uint32_t out_size, const SegMap &m,
                               uint32_t grid, uint32_t shift, uint32_t bits, const PoolOut &po, const DigitSide &ds,
                               hipStream_t s, uint32_t *chain) {
    if (grid == 0) return hipSuccess;
    if (in_size == 8 && out_size == 8 && !chain)
        return launch_scatter_pool_t<uint64_t, 8>(in, out, m, grid, shift, bits, po, ds, s, nullptr);
    if (in_size == 8 && out_size == 4)
        return launch_scatter_pool_t<uint32_t, 8>(in, out, m, grid, shift, bits, po, ds, s, chain);
    if (in_size == 4 && out_size == 4)
        return launch_scatter_pool_t<uint32_t, 4>(in, out, m, grid, shift, bits, po, ds, s, chain);
    return hipErrorInvalidValue;
}

bool chain_hist_supported(uint32_t bits1, uint32_t bits2) { return bits1 == 7 && (bits2 == 6 || bits2 == 7); }

// SGXAMD_SORT2 (development A/B switch, read once): 1 (default) = key partitions' pass 2
// as the LDS counting sort k_sort_blk; 0 = the write-combining k_scatter_blk.
// 2^28 keys per relation: 0.53-0.55 ms (16,384-key tiles, r03v-x) vs 0.585-0.60 for
// k_scatter_blk (alternating on one box, r03u).
bool sort2_enabled() {
    static const bool on = [] {
        const char *e = std::getenv("SGXAMD_SORT2");
        return !(e && std::atoi(e) == 0);
    }();
    return on;
}
// SGXAMD_PLACE (development A/B switch, read once): 1 (default) = narrow relations' pass
// 2 as the segment placement k_place_seg; 0 = k_sort_blk's tile sort.
bool place_enabled() {
    static const bool on = [] {
        const char *e = std::getenv("SGXAMD_PLACE");
        return !(e && std::atoi(e) == 0);
    }();
    return on;
}
template <typename T>
hipError_t launch_scatter_blk_t(const void *in, const uint64_t *list, void *out, const SegMap &m, uint32_t grid,
                                uint32_t shift, uint32_t bits, const uint64_t *cursors, hipStream_t s,
                                const uint32_t *narrow, const uint64_t *part_start, const uint64_t *part_count,
                                const uint8_t *side16) {
    if constexpr (sizeof(T) == 4) {
        if (sort2_enabled()) {
            const uint32_t *ik = static_cast<const uint32_t *>(in);
            uint32_t *ok = static_cast<uint32_t *>(out);
            // narrow relations: k_place_seg (fixed-size segments with their partition
            // ends); k_sort_blk then returns at once for them (the width is known on the
            // device only)
            const bool place = narrow && part_start && part_count && place_enabled();
            if (side16 && !place) return hipErrorInvalidValue;  // a narrow pool is read by k_place_seg only
            // the placements' 16-byte run copies assume that residual 8k of `out` sits on a
            // 16-byte boundary (each u16-wire destination's pass 2 starts on one)
            if (place && (reinterpret_cast<uintptr_t>(out) & 15u) != 0) return hipErrorInvalidValue;
            const uint32_t skip = place ? 1u : 0u;
#define SORT_CASE(B)                                                                                              \
    case B:                                                                                                       \
        if (place && side16)                                                                                      \
            hipLaunchKernelGGL((k_place_seg<B, SGXAMD_PLACE_NT, SGXAMD_PLACE_U, true>), dim3(grid),             \
                               dim3(SGXAMD_PLACE_NT), 0, s, ik, side16, list, reinterpret_cast<uint16_t *>(out), m, \
                               shift, cursors, part_start, part_count, narrow);                                   \
        else if (place)                                                                                           \
            hipLaunchKernelGGL((k_place_seg<B, SGXAMD_PLACE_NT, SGXAMD_PLACE_U, false>), dim3(grid),            \
                               dim3(SGXAMD_PLACE_NT), 0, s, ik, nullptr, list, reinterpret_cast<uint16_t *>(out), \
                               m, shift, cursors, part_start, part_count, narrow);                                \
        if (!place) /* (k_place_seg sorts a wide relation itself) */                                             \
            hipLaunchKernelGGL((k_sort_blk<B, SGXAMD_SORT_NT, SGXAMD_SORT_ITEMS>), dim3(grid), dim3(SGXAMD_SORT_NT), 0, \
                               s, ik, list, ok, m, shift, cursors, narrow, skip);                                 \
        break;
            switch (bits) {
                SORT_CASE(1)
                SORT_CASE(2)
                SORT_CASE(3)
                SORT_CASE(4)
                SORT_CASE(5)
                SORT_CASE(6)
                SORT_CASE(7)
                SORT_CASE(8)
                default:
                    return hipErrorInvalidValue;
            }
#undef SORT_CASE
            return hipGetLastError();
        }
    }
    constexpr int ITEMS = items_of<T, 2>(), NT = kScatterThreads;
    const char *ib = static_cast<const char *>(in);
    T *o = static_cast<T *>(out);
#define BLK_CASE(B)                                                                                                \
    case B:                                                                                                        \
        hipLaunchKernelGGL((k_scatter_blk<B, ITEMS, NT, T>), dim3(grid), dim3(NT), 0, s, ib, list, o, m, shift, \
                           cursors);                                                                               \
        break;
    switch (bits) {
        BLK_CASE(1)
        BLK_CASE(2)
        BLK_CASE(3)
        BLK_CASE(4)
        BLK_CASE(5)
        BLK_CASE(6)
        BLK_CASE(7)
        BLK_CASE(8)
        default:
            return hipErrorInvalidValue;
    }
#undef BLK_CASE
    return hipGetLastError();
}

hipError_t launch_scatter_keys(const row_t *in, uint32_t *out, const SegMap &m, uint32_t grid, uint32_t shift,
                               uint32_t bits, const uint64_t *cursors, HistLayout layout, uint32_t nseg_stride,
                               const uint64_t *digit_base, hipStream_t s) {
    if (grid == 0) return hipSuccess;
    constexpr int ITEMS = items_of<uint32_t, 0>(), NT = kScatterThreads;
    const char *ib = reinterpret_cast<const char *>(in);
#define KEYS_CASE(B)                                                                                            \
    case B:                                                                                                     \
        hipLaunchKernelGGL((k_scatter_keys<B, ITEMS, NT>), dim3(grid), dim3(NT), 0, s, ib, out, m, shift, cursors, \
                           layout, nseg_stride, digit_base);                                                    \
        break;
    switch (bits) {
        KEYS_CASE(1)
        KEYS_CASE(2)
        KEYS_CASE(3)
        KEYS_CASE(4)
        KEYS_CASE(5)
        KEYS_CASE(6)
        KEYS_CASE(7)
        KEYS_CASE(8)
        default:
            return hipErrorInvalidValue;
    }
#undef KEYS_CASE
    return hipGetLastError();
}

hipError_t launch_scatter_blk(const void *in, const uint64_t *list, void *out, uint32_t elem_size, const SegMap &m,
                              uint32_t grid, uint32_t shift, uint32_t bits, const uint64_t *cursors, hipStream_t s,
                              const uint32_t *narrow, const uint64_t *part_start, const uint64_t *part_count,
                              const uint8_t *side16) {
    if (grid == 0) return hipSuccess;
    // narrow residuals: key partitions through k_sort_blk / k_place_seg only
    if (narrow && !(elem_size == 4 && sort2_enabled())) return hipErrorInvalidValue;
    if (elem_size == 8)
        return launch_scatter_blk_t<uint64_t>(in, list, out, m, grid, shift, bits, cursors, s, nullptr, nullptr,
                                              nullptr, nullptr);
    if (elem_size == 4)
        return launch_scatter_blk_t<uint32_t>(in, list, out, m, grid, shift, bits, cursors, s, narrow, part_start,
                                              part_count, side16);
    return hipErrorInvalidValue;
}

// One block: from the column-scanned chain records (totals[d] = blocks << 40 | tuples)
// the pass-2 output layout of every region (tuple starts / counts), its block-list
// base / length and the pass-2 segment table (kPass2Ents blocks per segment).
__global__ __launch_bounds__(1024) void k_pool_layout(const uint64_t *__restrict__ totals, uint32_t F,
                                                      uint64_t *__restrict__ start, uint64_t *__restrict__ count,
                                                      uint64_t *__restrict__ lbase, uint64_t *__restrict__ lcount,
                                                      uint32_t *__restrict__ seg_base, uint32_t nseg,
                                                      uint32_t *__restrict__ kmax,
                                                      const uint32_t *__restrict__ guard, uint32_t gshift) {
    __shared__ uint64_t scratch[1024 / kWave + 1];
    __shared__ uint32_t kmax_all;
    if (guard && ((*guard >> gshift) >> 16) == 0) return;
    const uint32_t d = threadIdx.x;
    if (d == 0) kmax_all = 0;
    const uint64_t v = d < F ? totals[d] : 0;
    const uint64_t tup = v & ((1ull << 40) - 1), blk = v >> 40;
    uint64_t tot;
    const uint64_t ex_t = block_excl_scan_u64(tup, scratch, &tot);
    const uint64_t ex_b = block_excl_scan_u64(blk, scratch, &tot);
    const uint64_t ns = (blk + kPass2Ents - 1) / kPass2Ents;  // kPass2Ents-block segments
    const uint64_t ex_s = block_excl_scan_u64(ns, scratch, &tot);
    if (d < F) {
        start[d] = ex_t;
        count[d] = tup;
        lbase[d] = ex_b;
        lcount[d] = blk;
        seg_base[d] = (uint32_t)ex_s;
    }
    if (d == 0) seg_base[F] = (uint32_t)tot;
    if (kmax) {  // the relation's largest key into kmax[nseg]
        uint32_t x = 0;
        for (uint32_t i = d; i < nseg; i += blockDim.x) x = max(x, kmax[i]);
        if (x) atomicMax(&kmax_all, x);
        __syncthreads();
        if (d == 0) kmax[nseg] = kmax_all;
    }
}

hipError_t launch_pool_layout(uint64_t *cnt, uint32_t nseg, uint32_t bits, uint64_t *totals, uint64_t *start,
                              uint64_t *count, uint64_t *lbase, uint64_t *lcount, uint32_t *seg_base, hipStream_t s,
                              uint32_t *kmax, const uint32_t *guard, uint32_t gshift) {
    const uint32_t F = 1u << bits;
    hipLaunchKernelGGL(k_scan_cols, dim3(F), dim3(kBlock), 0, s, cnt, nseg, totals, guard, gshift);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const uint32_t threads = F < 64 ? 64 : F;
    hipLaunchKernelGGL(k_pool_layout, dim3(1), dim3(threads), 0, s, totals, F, start, count, lbase, lcount, seg_base,
                       nseg, kmax, guard, gshift);
    return hipGetLastError();
}

// One workgroup per pass-1 segment: its pool's blocks into the regions' block lists
// (position = the region's base + the segment's prefix of blocks in that region + a
// rank taken with an LDS atomic; the order inside a region does not matter).
__global__ __launch_bounds__(kBlock) void k_block_list(PoolOut po, const uint64_t *__restrict__ lbase,
                                                       uint64_t *__restrict__ list, uint32_t F) {
    __shared__ uint32_t rank[kMaxF];
    __shared__ uint64_t pre[kMaxF];  // the segment's first list position per digit
    if (pool_guard_skip(po)) return;
    const uint32_t g = blockIdx.x;
    for (uint32_t d = threadIdx.x; d < F; d += kBlock) {
        rank[d] = 0;
        pre[d] = lbase[d] + (po.cnt[(uint64_t)d * po.nseg + g] >> 40);
    }
    __syncthreads();
    const uint32_t used = po.used[g], base = g * po.pool_blocks;
    // eight block infos per thread in flight at once (the loop was a chain of dependent
    // global loads: 13.7 us per 2^28-key relation, r04p)
    constexpr int U = 8;
    for (uint32_t k0 = threadIdx.x; k0 < used; k0 += U * kBlock) {
        uint32_t info[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t k = k0 + u * kBlock;
            info[u] = k < used ? po.binfo[base + k] : 0u;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t k = k0 + u * kBlock;
            if (k < used) {
                const uint32_t d = info[u] & 0xFFFFu;
                const uint32_t rk = atomicAdd(&rank[d], 1u);
                list[pre[d] + rk] = (uint64_t)(base + k) | ((uint64_t)(info[u] >> 16) << 32);
            }
        }
    }
}

hipError_t launch_block_list(const PoolOut &po, const uint64_t *lbase, uint64_t *list, uint32_t bits, hipStream_t s) {
    if (po.nseg == 0) return hipSuccess;
    hipLaunchKernelGGL(k_block_list, dim3(po.nseg), dim3(kBlock), 0, s, po, lbase, list, 1u << bits);
    return hipGetLastError();
}

// k_pool_layout folded into the block list (round 6: one launch less per relation): every
// workgroup scans the F <= 256 digit totals for the regions' list bases itself (one digit
// per thread), and workgroup 0 also writes the pass-2 layout -- region tuple starts /
// counts, list bases / lengths, the kPass2Ents-block segment table -- and the relation's
// largest key, as k_pool_layout does.
__global__ __launch_bounds__(kBlock) void k_block_list_l(PoolOut po, const uint64_t *__restrict__ totals, uint32_t F,
                                                         uint64_t *__restrict__ start, uint64_t *__restrict__ count,
                                                         uint64_t *__restrict__ lbase, uint64_t *__restrict__ lcount,
                                                         uint32_t *__restrict__ seg_base, uint64_t *__restrict__ list) {
    __shared__ uint32_t rank[kBlock];
    __shared__ uint64_t pre[kBlock];  // the segment's first list position per digit
    __shared__ uint64_t scratch[kBlock / kWave + 1];
    __shared__ uint32_t kmax_all;
    if (pool_guard_skip(po)) return;
    constexpr uint64_t M40 = (1ull << 40) - 1;
    const uint32_t g = blockIdx.x, d = threadIdx.x;
    if (d == 0) kmax_all = 0;
    const uint64_t v = d < F ? totals[d] : 0;
    const uint64_t c = d < F ? po.cnt[(uint64_t)d * po.nseg + g] : 0;
    const uint64_t blk = v >> 40;
    uint64_t tot;
    const uint64_t ex_b = block_excl_scan_u64(blk, scratch, &tot);
    if (d < F) {
        rank[d] = 0;
        pre[d] = ex_b + (c >> 40);
    }
    if (g == 0) {  // (workgroup-uniform) the layout
        const uint64_t tup = v & M40, ns = (blk + kPass2Ents - 1) / kPass2Ents;
        const uint64_t ex_t = block_excl_scan_u64(tup, scratch, &tot);
        uint64_t nsegs;
        const uint64_t ex_s = block_excl_scan_u64(ns, scratch, &nsegs);
        if (d < F) {
            start[d] = ex_t;
            count[d] = tup;
            lbase[d] = ex_b;
            lcount[d] = blk;
            seg_base[d] = (uint32_t)ex_s;
        }
        if (d == 0) seg_base[F] = (uint32_t)nsegs;
        if (po.zero8 && d < 8) po.zero8[d] = 0;
        if (po.kmax) {  // the segments' largest keys -> the relation's, kmax[nseg]
            uint32_t x = 0;
            for (uint32_t i = d; i < po.nseg; i += kBlock) x = max(x, po.kmax[i]);
            if (x) atomicMax(&kmax_all, x);
            __syncthreads();
            if (d == 0) po.kmax[po.nseg] = kmax_all;
        }
    }
    __syncthreads();
    const uint32_t used = po.used[g], base = g * po.pool_blocks;
    constexpr int U = 8;
    for (uint32_t k0 = threadIdx.x; k0 < used; k0 += U * kBlock) {
        uint32_t info[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t k = k0 + u * kBlock;
            info[u] = k < used ? po.binfo[base + k] : 0u;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t k = k0 + u * kBlock;
            if (k < used) {
                const uint32_t dd = info[u] & 0xFFFFu;
                const uint32_t rk = atomicAdd(&rank[dd], 1u);
                list[pre[dd] + rk] = (uint64_t)(base + k) | ((uint64_t)(info[u] >> 16) << 32);
            }
        }
    }
}

hipError_t launch_pool_layout_list(const PoolOut &po, uint32_t bits, uint64_t *totals, uint64_t *start,
                                   uint64_t *count, uint64_t *lbase, uint64_t *lcount, uint32_t *seg_base,
                                   uint64_t *list, hipStream_t s) {
    const uint32_t F = 1u << bits;
    if (po.zero8 && (F > kBlock || po.nseg == 0)) {  // (no k_block_list_l workgroup 0 to zero them)
        hipError_t e = hipMemsetAsync(po.zero8, 0, 8 * sizeof(uint64_t), s);
        if (e != hipSuccess) return e;
    }
    if (F > kBlock) {  // (a pass-1 digit past 8 bits: the separate layout workgroup)
        hipError_t e = launch_pool_layout(po.cnt, po.nseg, bits, totals, start, count, lbase, lcount, seg_base, s,
                                          po.kmax, po.guard, po.guard_shift);
        if (e != hipSuccess) return e;
        return launch_block_list(po, lbase, list, bits, s);
    }
    hipLaunchKernelGGL(k_scan_cols, dim3(F), dim3(kBlock), 0, s, po.cnt, po.nseg, totals, po.guard, po.guard_shift);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || po.nseg == 0) return e;
    hipLaunchKernelGGL(k_block_list_l, dim3(po.nseg), dim3(kBlock), 0, s, po, totals, F, start, count, lbase, lcount,
                       seg_base, list);
    return hipGetLastError();
}

// Pass-2 histogram of up to 128 digits with one private counter row per lane: the two
// u16 counts of digits 2p and 2p+1 for lane l sit in word p * 64 + l, so the lanes of
// an atomic hit distinct words in distinct banks (4-byte LDS atomics bank on (a/4) mod 32
// per 32-lane group); lane l of the four waves shares a row.  A row counts at most
// 4 waves x 16 keys per block x (segment blocks / 16) per lane (1024 at kPass2Ents = 256,
// 8192 at 2048), inside a u16.  A shared 128-bin histogram spent 70 % of its LDS cycles
// in bank conflicts (SQ counters, r02t); the private rows take 5-10 % off the kernel
// (0.096 -> 0.087 ms per 2^28 keys), the list entries staged in LDS with the next
// step's digit bytes in flight another 18-20 % (0.087 -> 0.071): the kernel was bound
// by its two dependent loads per step more than by the LDS.
constexpr uint32_t kLaneHistF = 128;
#ifndef SGXAMD_HSIDE_U
#define SGXAMD_HSIDE_U 4
#endif
__device__ __forceinline__ void hist_side_lanes(const uint8_t *__restrict__ side, const uint64_t *__restrict__ list,
                                                uint64_t b, uint64_t e, uint32_t F, uint64_t *__restrict__ out) {
    static_assert(kPass2Ents <= 4096, "u16 lane counters");
    constexpr uint32_t W = kLaneHistF / 2 * kWave;
    __shared__ uint32_t hp[W];
    __shared__ uint64_t ents[kPass2Ents];  // the segment's list entries, one coalesced read
    const uint32_t tid = threadIdx.x, lane = __lane_id();
    const uint32_t ne = (uint32_t)(e - b);  // <= kPass2Ents (pass-2 segments)
    for (uint32_t i = tid; i < W; i += kBlock) hp[i] = 0;
    for (uint32_t i = tid; i < ne; i += kBlock) ents[i] = list[b + i];
    __syncthreads();
    const uint32_t grp = tid / 16, l = tid % 16;
    constexpr int U = SGXAMD_HSIDE_U;  // blocks per 16-lane group and step
    constexpr uint32_t SPAN = 16 * U;
    // one step: the 16-B digit pieces of U blocks per group (entries past ne load nothing)
    const auto load_step = [&](uint32_t i0, uint4 (&q)[U], uint32_t (&nv)[U]) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t i = i0 + grp + 16 * u;
            nv[u] = 0;
            q[u] = make_uint4(0, 0, 0, 0);
            if (i < ne) {
                const uint64_t en = ents[i];
                const uint32_t fill = (uint32_t)(en >> 32), lo = l * 16;
                nv[u] = fill > lo ? min(16u, fill - lo) : 0u;
                if (nv[u]) q[u] = ld_nt(reinterpret_cast<const uint4 *>(side + (uint64_t)(uint32_t)en * kBlk) + l);
            }
        }
    };
    const auto count_step = [&](const uint4 (&q)[U], const uint32_t (&nv)[U]) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t w[4] = {q[u].x, q[u].y, q[u].z, q[u].w};
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const uint32_t d = __builtin_amdgcn_ubfe(w[j >> 2], (j & 3) * 8, 8);
                if ((uint32_t)j < nv[u]) atomicAdd(&hp[(d >> 1) * kWave + lane], 1u << ((d & 1u) * 16u));
            }
        }
    };
    // two register sets: the next step's loads are in flight while a step is counted
    uint4 q0[U], q1[U];
    uint32_t n0[U], n1[U];
    load_step(0, q0, n0);
    for (uint32_t i0 = 0; i0 < ne; i0 += 2 * SPAN) {
        load_step(i0 + SPAN, q1, n1);
        count_step(q0, n0);
        load_step(i0 + 2 * SPAN, q0, n0);
        count_step(q1, n1);
    }
    __syncthreads();
    for (uint32_t d = tid; d < F; d += kBlock) {
        uint32_t c = 0;
        for (uint32_t k = 0; k < kWave; ++k)  // rotated rows: the 32 lanes of a read hit 32 banks
            c += (hp[(d >> 1) * kWave + ((k + d) & (kWave - 1))] >> ((d & 1u) * 16u)) & 0xFFFFu;
        out[d] = c;
    }
}

// Pass-2 histogram of a block-list segment from the digit side stream: 16 lanes per
// block (16 B each: a block's kBlk digit bytes), 16 blocks per step, 4 steps in flight.
__global__ __launch_bounds__(kBlock) void k_hist_side_blk(const uint8_t *__restrict__ side,
                                                          const uint64_t *__restrict__ list, SegMap m, uint32_t bits,
                                                          uint64_t *__restrict__ hist) {
    static_assert(kBlk == 256, "16 lanes x 16 B per block");
    __shared__ uint32_t h[kMaxF];
    __shared__ uint32_t sbase[kMaxF + 1];
    const uint32_t g = blockIdx.x;
    uint32_t r;
    uint64_t b, e;
    if (!seg_lookup(m, g, sbase, r, b, e)) return;
    const uint32_t F = 1u << bits;
    const uint32_t grp = threadIdx.x / 16, l = threadIdx.x % 16;
    constexpr int U = 4;
    if (F <= kLaneHistF && e - b <= kPass2Ents) {  // workgroup-uniform
        hist_side_lanes(side, list, b, e, F, hist + (uint64_t)g * F);
        return;
    }
    for (uint32_t d = threadIdx.x; d < F; d += kBlock) h[d] = 0;
    __syncthreads();
    for (uint64_t i0 = b; i0 < e; i0 += 16 * U) {
        uint4 q[U];
        uint32_t nv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = i0 + grp + 16 * u;
            nv[u] = 0;
            q[u] = make_uint4(0, 0, 0, 0);
            if (i < e) {
                const uint64_t en = list[i];
                const uint32_t fill = (uint32_t)(en >> 32), lo = l * 16;
                nv[u] = fill > lo ? min(16u, fill - lo) : 0u;
                if (nv[u]) q[u] = ld_nt(reinterpret_cast<const uint4 *>(side + (uint64_t)(uint32_t)en * kBlk) + l);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t w[4] = {q[u].x, q[u].y, q[u].z, q[u].w};
#pragma unroll
            for (int j = 0; j < 16; ++j)
                if ((uint32_t)j < nv[u]) atomicAdd(&h[__builtin_amdgcn_ubfe(w[j >> 2], (j & 3) * 8, 8)], 1u);
        }
    }
    __syncthreads();
    for (uint32_t d = threadIdx.x; d < F; d += kBlock) hist[(uint64_t)g * F + d] = h[d];
}

hipError_t launch_hist_side_blk(const uint8_t *side, const uint64_t *list, const SegMap &m, uint32_t grid,
                                uint32_t bits, uint64_t *hist, hipStream_t s) {
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL(k_hist_side_blk, dim3(grid), dim3(kBlock), 0, s, side, list, m, bits, hist);
    return hipGetLastError();
}

// Pass-2 histogram of a block-list segment from the chain histograms (no side stream).
// Region r's list holds its chains one after another (chain j = pass-1 segment j's
// blocks of digit r, k_block_list), so a segment of kPass2Ents blocks is whole chains
// plus at most a cut chain at either end.  The whole chains' digit counts are summed
// from the chain histograms pass 1 stored; a cut chain's part is counted from its keys,
// or, when the part outside the segment is the smaller, the chain's histogram less that
// part (counted from its keys); a chain of more than 65,535 elements, whose u16 counts
// may have wrapped, always from its keys.  Uniform 2^28-key relations: about 16 whole
// chains (8 KiB of histograms) and 8 blocks of keys on average per segment, instead of
// its 64 KiB of side-stream bytes, and 2,048 LDS atomics instead of 65,536.
constexpr uint32_t kHistChainRanges = 8;  // cut / wrapped chain parts per segment (<= 2 + kPass2Ents / 256)
static_assert(kPass2Ents <= 1024, "k_hist_chain's range table");
// One wave per segment (F2 <= 128): a 2^28-key relation's 4,224 segments are all
// resident at once, and a segment's work is four dependent round trips -- the segment
// table; the region's chain records; the whole chains' histogram rows (16 B per lane,
// F2 / 4 lanes a row) with the cut chains' list entries; their keys.  256-thread
// workgroups (three rounds of eight per CU) took 0.035 ms per relation against 0.031
// (profiles/r06p_hist_chain_wave_ab.log).
constexpr int kHcU = 8;  // chain records per lane per step (512 chains in one step)
__global__ __launch_bounds__(kWave, 5) void k_hist_chain(const uint64_t *__restrict__ rec,
                                                           const uint64_t *__restrict__ tot, uint32_t nseg,
                                                           const uint32_t *__restrict__ chain,
                                                           const uint64_t *__restrict__ list,
                                                           const uint32_t *__restrict__ keys, SegMap m,
                                                           uint32_t shift2, uint32_t bits2,
                                                           uint64_t *__restrict__ hist) {
    constexpr uint64_t M40 = (1ull << 40) - 1;
    __shared__ uint32_t sbase[kMaxF + 1];
    __shared__ uint32_t h[kLaneHistF];
    __shared__ uint32_t good[kHistChainMaxSegs / 32];
    __shared__ uint32_t rg[kHistChainRanges][3];  // [p0, p1) region-local, subtract
    __shared__ uint32_t jlo, jhi, nrg;
    const uint32_t g = blockIdx.x, lane = threadIdx.x;
    const uint32_t F1 = m.nreg, F2 = 1u << bits2, mask2 = F2 - 1;
    for (uint32_t i = lane; i <= F1; i += kWave) sbase[i] = m.seg_base[i];
    for (uint32_t i = lane; i < F2; i += kWave) h[i] = 0;
    for (uint32_t i = lane; i < (nseg + 31) / 32; i += kWave) good[i] = 0;
    if (lane == 0) {
        jlo = 0xFFFFFFFFu;
        jhi = 0;
        nrg = 0;
    }
    __syncthreads();
    if (g >= sbase[F1]) return;  // wave-uniform
    uint32_t r = 0, hi = F1;     // largest r with sbase[r] <= g
    while (hi - r > 1) {
        const uint32_t mid = (r + hi) >> 1;
        if (sbase[mid] <= g) r = mid; else hi = mid;
    }
    const uint64_t lb0 = m.reg_start[r], lcnt = m.reg_count[r], tr = tot[r];
    const uint64_t lb = (uint64_t)(g - sbase[r]) * kPass2Ents, le = min(lb + kPass2Ents, lcnt);
    const uint64_t *rc = rec + (uint64_t)r * nseg;
    // the region's chains against [lb, le): whole ones (histogram rows), cut ones (ranges)
    for (uint32_t j0 = 0; j0 < nseg; j0 += kWave * kHcU) {
        uint64_t v0[kHcU], v1[kHcU];
#pragma unroll
        for (int u = 0; u < kHcU; ++u) {
            const uint32_t j = j0 + u * kWave + lane;
            v0[u] = j < nseg ? rc[j] : 0ull;
            v1[u] = j + 1 < nseg ? rc[j + 1] : tr;
        }
#pragma unroll
        for (int u = 0; u < kHcU; ++u) {
            const uint32_t j = j0 + u * kWave + lane;
            const uint64_t a0 = v0[u] >> 40, a1 = v1[u] >> 40;
            const uint64_t p0 = max(a0, lb), p1 = min(a1, le);
            if (j >= nseg || p0 >= p1) continue;
            const bool exact = (v1[u] & M40) - (v0[u] & M40) <= 65535;  // its histogram did not wrap
            const bool whole = a0 >= lb && a1 <= le;
            // a chain cut at one end of the segment whose part outside is the smaller:
            // its histogram less the outside part (counted from its keys)
            const bool sub = exact && !whole && (a0 >= lb || a1 <= le) && (a1 - a0) - (p1 - p0) < p1 - p0;
            if ((whole && exact) || sub) {
                atomicOr(&good[j / 32], 1u << (j % 32));
                atomicMin(&jlo, j);
                atomicMax(&jhi, j);
            }
            if (!(whole && exact)) {
                const uint32_t k = atomicAdd(&nrg, 1u);
                if (k < kHistChainRanges) {
                    rg[k][0] = (uint32_t)(sub ? (a0 < lb ? a0 : le) : p0);
                    rg[k][1] = (uint32_t)(sub ? (a0 < lb ? lb : a1) : p1);
                    rg[k][2] = sub ? 1u : 0u;
                }
            }
        }
    }
    __syncthreads();
    const uint32_t nr = min(nrg, kHistChainRanges);
    uint32_t nb = 0;
    for (uint32_t k = 0; k < nr; ++k) nb += rg[k][1] - rg[k][0];
    // block i of the ranges -> its list position (region-local) | subtract << 31, or ~0
    const auto pos_of = [&](uint32_t i) -> uint32_t {
        for (uint32_t k = 0; k < nr; ++k) {
            const uint32_t w = rg[k][1] - rg[k][0];
            if (i < w) return (rg[k][0] + i) | (rg[k][2] << 31);
            i -= w;
        }
        return 0xFFFFFFFFu;
    };
    constexpr int U = 8;  // cut blocks per step
    uint64_t en[U];
    uint32_t inc[U];  // 1, or -1 for a subtracted part
#pragma unroll
    for (int u = 0; u < U; ++u) {  // the first step's list entries, in flight with the rows below
        const uint32_t p = pos_of((uint32_t)u);
        en[u] = p != 0xFFFFFFFFu ? list[lb0 + (p & 0x7FFFFFFFu)] : 0ull;
        inc[u] = p != 0xFFFFFFFFu && (p >> 31) ? 0xFFFFFFFFu : 1u;
    }
    // whole chains: F2 / 4 lanes per histogram row, 256 / F2 rows per load
    {
        const uint32_t lpr = F2 / 4, rpi = kWave / lpr, sub = lane / lpr, dq = lane % lpr;
        const uint32_t *ch = chain + (uint64_t)r * nseg * F2 + 4 * dq;
        uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
        if (jlo <= jhi) {
            for (uint32_t j0 = jlo + sub; j0 <= jhi; j0 += U * rpi) {
                uint4 c[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t j = j0 + u * rpi;
                    c[u] = j <= jhi && ((good[j / 32] >> (j % 32)) & 1u)
                               ? *reinterpret_cast<const uint4 *>(ch + (uint64_t)j * F2)
                               : make_uint4(0, 0, 0, 0);
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    s0 += c[u].x;
                    s1 += c[u].y;
                    s2 += c[u].z;
                    s3 += c[u].w;
                }
            }
        }
        if (s0) atomicAdd(&h[4 * dq], s0);
        if (s1) atomicAdd(&h[4 * dq + 1], s1);
        if (s2) atomicAdd(&h[4 * dq + 2], s2);
        if (s3) atomicAdd(&h[4 * dq + 3], s3);
    }
    // cut parts from their keys: a lane 4 keys of each block
    for (uint32_t i0 = 0; i0 < nb; i0 += U) {
        if (i0) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t p = pos_of(i0 + u);
                en[u] = p != 0xFFFFFFFFu ? list[lb0 + (p & 0x7FFFFFFFu)] : 0ull;
                inc[u] = p != 0xFFFFFFFFu && (p >> 31) ? 0xFFFFFFFFu : 1u;
            }
        }
        uint4 q[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t fill = i0 + u < nb ? (uint32_t)(en[u] >> 32) : 0u;
            q[u] = lane * 4 < fill ? ld_nt(reinterpret_cast<const uint4 *>(keys + (uint64_t)(uint32_t)en[u] * kBlk) + lane)
                                   : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t fill = i0 + u < nb ? (uint32_t)(en[u] >> 32) : 0u;
            const uint32_t w[4] = {q[u].x, q[u].y, q[u].z, q[u].w};
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (lane * 4 + j < fill) atomicAdd(&h[(w[j] >> shift2) & mask2], inc[u]);
        }
    }
    __syncthreads();
    for (uint32_t d = lane; d < F2; d += kWave) hist[(uint64_t)g * F2 + d] = h[d];
}

hipError_t launch_hist_chain(const uint64_t *cnt, const uint64_t *tot, uint32_t nseg, const uint32_t *chain,
                             const uint64_t *list, const uint32_t *keys, const SegMap &m, uint32_t grid,
                             uint32_t shift2, uint32_t bits2, uint64_t *hist, hipStream_t s) {
    if (nseg > kHistChainMaxSegs || bits2 < 2 || bits2 > 7) return hipErrorInvalidValue;
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL(k_hist_chain, dim3(grid), dim3(kWave), 0, s, cnt, tot, nseg, chain, list, keys, m, shift2,
                       bits2, hist);
    return hipGetLastError();
}

// ------------------------------------------------------------ build+probe ---
// bucket_chaining_join (radix_join.cpp:359-458) per task, in LDS.  A task is a
// partition p and one chunk of at most kSChunk of its S tuples: S partitions
// larger than kSChunk (skew, e.g. a Zipf hot key) are split over several tasks so
// that no single workgroup is left with a hot partition (the reference has no
// skew handling, prj_params.h:69-71).  Task t < P is (p = t, chunk 0); the extra
// chunks of large partitions follow as overflow entries {p, chunk}.
//
// For an R chunk of nrc <= RCAP tuples: N = nextpow2(nrc) bucket heads, bucket of a
// key = HASH_BIT_MODULO(key, (N-1) << bits, bits) = (key >> bits) & (N-1) exactly as
// the reference (:374-378, :388); keys[] and 16-bit next[] hold the chains with
// 1-based positions (:393 "we start pos's from 1").  The build links tuple i with
// one LDS atomic exchange on its bucket head (chain order differs from the
// reference's serial build; the count does not).  The probe walks every chain and
// counts key equality (:429-436).  Each thread handles U = RCAP / BLOCK tuples at
// a time; their chain walks advance in lockstep so the LDS reads of independent
// tuples overlap.  Partitions whose R side exceeds RCAP are built chunk by chunk
// with the task's S chunk re-probed per R chunk.
//
// MODE kJoinCount     one partial count per workgroup (count-only join);
// MODE kJoinTaskCount one count per task (first pass of materialisation);
// MODE kJoinWrite     every match as an output_triple_t {key, R payload, S payload}
//                     (radix_join.cpp:437-446) at task_off[t] + a task-local slot
//                     taken with one LDS atomic per wave and chain step.

// Count-mode reduction in the join launch itself (replaces k_reduce), for small joins:
// every workgroup with a task adds its count into ONE 64-bit device word together with
// its arrival -- (1 << 48) | count, one atomic -- after adding its build / probe ticks
// (two 32-bit halves of a second word, waited for first), and the workgroup whose atomic
// returns n - 1 arrivals is the last: it holds the total (the returned sum + its own
// count), reads the ticks, resets both words for the next call and writes the result.
// No per-workgroup count slots, release fences, second ticket or final summation
// (round 4: a ticket of 256 arrivals, then the last workgroup summing the slots: 3.3 +
// 2.2 us of the 2^20 join, r05n stamps).  counts / cyc: this workgroup's count and
// ticks at [blockIdx.x] / [2 blockIdx.x .. + 1] (written by its thread 0).
__device__ __forceinline__ void join_reduce_last(const uint64_t *__restrict__ counts, const uint64_t *__restrict__ cyc,
                                                 uint64_t *__restrict__ result, uint64_t *__restrict__ ticket,
                                                 uint64_t *red, uint64_t tasks) {
    (void)red;
    // workgroups without a task (blockIdx >= tasks) do not arrive
    const uint64_t n = tasks < gridDim.x ? tasks : gridDim.x;
    if ((blockIdx.x >= n && n > 0) || threadIdx.x != 0) return;
    const uint64_t na = n > 0 ? n : gridDim.x;  // < 2^16 (small-join grids)
    // two levels: workgroup b arrives at group b mod kJoinGroups (one word pair per group:
    // arrivals << 48 | counts, and ticks), the last arrival of a group carries the group's
    // sums to the top pair; at most n / kJoinGroups + kJoinGroups atomics queue on one
    // address (each ~14 ns: 256 arrivals on one word took 3.6 us)
    constexpr uint64_t M48 = (1ull << 48) - 1;
    const uint32_t G = na < kJoinGroups ? (uint32_t)na : kJoinGroups;
    const uint32_t grp = blockIdx.x % G;
    const uint64_t members = (na - grp + G - 1) / G;
    uint64_t *gsum = ticket + (kSyncJoinGrp - kSyncTicketJoin) + 2 * grp, *gtick = gsum + 1;
    uint64_t *sumw = ticket + (kSyncJoinSum - kSyncTicketJoin);
    uint64_t *tickw = ticket + (kSyncJoinTicks - kSyncTicketJoin);
    const uint64_t acc = counts[blockIdx.x];
    // (per workgroup far below 2^32 ticks: the halves never carry into each other)
    uint64_t tk = cyc ? ((uint64_t)(uint32_t)cyc[2 * blockIdx.x] << 32) | (uint32_t)cyc[2 * blockIdx.x + 1] : 0ull;
    if (cyc) {
        tk += __hip_atomic_fetch_add(gtick, tk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // performed before the arrival below
    }
    dbg_stamp(3, 0);
    uint64_t old = __hip_atomic_fetch_add(gsum, (1ull << 48) | acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((old >> 48) != members - 1) return;
    // the group's last: every member's ticks were added before its arrival
    const uint64_t gs = (old & M48) + acc;
    if (cyc) tk = __hip_atomic_fetch_add(gtick, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(gsum, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(gtick, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cyc) {
        (void)__hip_atomic_fetch_add(tickw, tk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    old = __hip_atomic_fetch_add(sumw, (1ull << 48) | gs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((old >> 48) != G - 1) return;
    const uint64_t t = (old & M48) + gs;
    tk = cyc ? __hip_atomic_fetch_add(tickw, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
    __hip_atomic_store(sumw, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(tickw, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t tb = tk >> 32, tp = tk & 0xFFFFFFFFull;
    dbg_stamp(3, 1);
    result[0] = t;
    if (cyc) {
        result[4] = tb;
        result[5] = tp;
    }
    // the call's result block in mapped host memory (kSyncHostResult): all six words
    // (result[1..3] come from the launches before this one), the device span, then the
    // done flag the host spins on -- the kernel's last memory operation (the kernel's end
    // releases it; one system fence orders the words before it)
    volatile uint64_t *h = reinterpret_cast<volatile uint64_t *>(ticket[kSyncHostResult - kSyncTicketJoin]);
    if (h) {
        h[0] = t;
        h[1] = result[1];
        h[2] = result[2];
        h[3] = result[3];
        h[4] = tb;
        h[5] = tp;
        h[kHostJoinSpan] = wall_clock64() - ticket[kSyncT0 - kSyncTicketJoin];
        __threadfence_system();
        h[kHostJoinDone] = 1;
    }
    dbg_stamp(3, 2);
}

__device__ __forceinline__ void tmatch_add(uint64_t &m, bool hit) { m += hit ? 1u : 0u; }

__device__ __forceinline__ void decode_task(uint64_t t, uint64_t P, const uint64_t *__restrict__ over, uint64_t &p,
                                            uint64_t &chunk) {
    if (t < P) {
        p = t;
        chunk = 0;
    } else {
        const uint64_t e = over[t - P];
        p = e & 0xFFFFFFFFull;
        chunk = e >> 32;
    }
}

// LDS of one build/probe workgroup: exactly 10 * RCAP bytes when counting (4
// workgroups per CU at RCAP 4096), + 4 * RCAP of R payloads when writing.  The
// reduction slots reuse the bucket heads, which are dead after each probe.
template <int RCAP, int MODE, int NW>
struct JoinLds {
    union {
        __attribute__((aligned(16))) uint32_t head[RCAP];
        uint64_t red[NW + 2];
    };
    uint32_t keys[RCAP];
    uint16_t next[RCAP];
};
template <int RCAP, int NW>
struct JoinLds<RCAP, kJoinWrite, NW> {
    union {
        __attribute__((aligned(16))) uint32_t head[RCAP];
        uint64_t red[NW + 2];
    };
    uint32_t keys[RCAP];
    uint16_t next[RCAP];
    uint32_t rpay[RCAP];
    uint32_t cursor;
};

// KS: u32 words per partitioned element (2: row_t tuples; 1: packed keys, counting only).
// DIRECT (counting; small joins): task_off holds R's largest key (one u64; the unused
// output offsets of a counting launch).  When every R residual (key >> hash_shift) is
// below 2 RCAP, a chunk is counted in a direct table instead of the chain table: one u16
// counter per residual (two per head word), R's keys add 1, S's keys read their
// residual's counter (residuals identify keys inside a partition: the low hash_shift
// bits are the partition's).  One LDS atomic per R key and one read per S key instead of
// the chain's exchange, two stores, and the walk.
template <int RCAP, int MODE, int BLOCK = kBlock, int KS = 2, bool DIRECT = false>
__global__ __launch_bounds__(BLOCK) void k_join(const uint64_t *__restrict__ R, const uint64_t *__restrict__ S,
                                                 const uint64_t *__restrict__ r_start,
                                                 const uint64_t *__restrict__ r_count,
                                                 const uint64_t *__restrict__ s_start,
                                                 const uint64_t *__restrict__ s_count, uint64_t P,
                                                 const uint64_t *__restrict__ over,
                                                 const uint32_t *__restrict__ n_over, uint32_t hash_shift, uint64_t s_chunk,
                                                 uint64_t *__restrict__ counts,
                                                 const uint64_t *__restrict__ task_off,
                                                 output_triple_t *__restrict__ out, uint64_t *__restrict__ cyc,
                                                 uint64_t *__restrict__ red_result, uint64_t *__restrict__ red_ticket) {
    constexpr int U = RCAP / BLOCK, NW = BLOCK / kWave;
    static_assert(KS == 2 || MODE != kJoinWrite, "materialisation needs the payloads");
    __shared__ JoinLds<RCAP, MODE, NW> L;
    const uint32_t *Rk = reinterpret_cast<const uint32_t *>(R), *Sk = reinterpret_cast<const uint32_t *>(S);
    const uint32_t tid = threadIdx.x, lane = __lane_id();
    dbg_stamp(2, 0);
    const uint64_t T = P + *n_over;
    uint64_t matches = 0;
    uint64_t bcyc = 0, pcyc = 0;  // build / probe wall-clock ticks of this workgroup
    static_assert(!DIRECT || MODE == kJoinCount, "the direct table counts");
    // residuals in use (u16 counters): 0 = the chain table
    const uint32_t tlim = DIRECT && (task_off[0] >> hash_shift) < 2ull * RCAP
                              ? (uint32_t)(task_off[0] >> hash_shift) + 1u : 0u;
    for (uint64_t t = blockIdx.x; t < T; t += gridDim.x) {
        uint64_t p, chunk;
        decode_task(t, P, over, p, chunk);
        const uint64_t nR = r_count[p], nSp = s_count[p];
        const uint64_t s_lo = chunk * s_chunk;
        const uint64_t nS = (nR == 0 || s_lo >= nSp) ? 0 : min<uint64_t>(nSp - s_lo, s_chunk);
        uint64_t tmatch = 0;
        if constexpr (MODE == kJoinWrite) {
            if (tid == 0) L.cursor = 0;
        }
        if (nS > 0) {
            const uint64_t *rp = R + r_start[p];
            const uint64_t *sp = S + s_start[p] + s_lo;
            for (uint64_t rc = 0; rc < nR; rc += RCAP) {
                const uint64_t c_build = wall_clock64();
                const uint32_t nrc = (uint32_t)((nR - rc) < RCAP ? (nR - rc) : RCAP);
                uint32_t N = 1;
                while (N < nrc) N <<= 1;  // NEXT_POW_2(numR)
                const uint32_t hmask = N - 1;
                uint64_t kr[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t i = tid + u * BLOCK;
                    if constexpr (KS == 1)
                        kr[u] = i < nrc ? __builtin_nontemporal_load(Rk + r_start[p] + rc + i) : 0u;
                    else
                        kr[u] = i < nrc ? ld_nt(rp + rc + i) : 0ull;
                }
                if (DIRECT && tlim) {
                    for (uint32_t i = tid; i < (tlim + 1) / 2; i += BLOCK) L.head[i] = 0;
                    __syncthreads();
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const uint32_t i = tid + u * BLOCK;
                        if (i < nrc) {
                            const uint32_t r = (uint32_t)kr[u] >> hash_shift;
                            atomicAdd(&L.head[r >> 1], 1u << ((r & 1u) * 16u));
                        }
                    }
                    __syncthreads();
                    const uint64_t c_probe = wall_clock64();
                    bcyc += c_probe - c_build;
                    for (uint64_t s0 = 0; s0 < nS; s0 += RCAP) {
                        uint32_t ks[U];
#pragma unroll
                        for (int u = 0; u < U; ++u) {
                            const uint64_t i = s0 + tid + u * BLOCK;
                            if constexpr (KS == 1)
                                ks[u] = i < nS ? __builtin_nontemporal_load(Sk + s_start[p] + s_lo + i) : 0u;
                            else
                                ks[u] = i < nS ? __builtin_nontemporal_load(reinterpret_cast<const uint32_t *>(sp + i)) : 0u;
                        }
#pragma unroll
                        for (int u = 0; u < U; ++u) {
                            const uint64_t i = s0 + tid + u * BLOCK;
                            const uint32_t r = ks[u] >> hash_shift;
                            if (i < nS && r < tlim) tmatch += (L.head[r >> 1] >> ((r & 1u) * 16u)) & 0xFFFFu;
                        }
                    }
                    __syncthreads();
                    pcyc += wall_clock64() - c_probe;
                    continue;
                }
                for (uint32_t i = tid; i < (N + 3) / 4; i += BLOCK)
                    reinterpret_cast<uint4 *>(L.head)[i] = make_uint4(0, 0, 0, 0);
                __syncthreads();
#pragma unroll
                for (int u = 0; u < U; ++u) {  // BUILD-LOOP (:407-411)
                    const uint32_t i = tid + u * BLOCK;
                    if (i < nrc) {
                        const uint32_t k = (uint32_t)kr[u];
                        L.keys[i] = k;
                        if constexpr (MODE == kJoinWrite) L.rpay[i] = (uint32_t)(kr[u] >> 32);
                        const uint32_t prev = atomicExch(&L.head[(k >> hash_shift) & hmask], i + 1);
                        L.next[i] = (uint16_t)prev;
                    }
                }
                __syncthreads();
                const uint64_t c_probe = wall_clock64();
                bcyc += c_probe - c_build;
                for (uint64_t s0 = 0; s0 < nS; s0 += RCAP) {  // PROBE-LOOP (:429-436)
                    uint32_t ks[U], cur[U];
                    uint32_t sv[MODE == kJoinWrite ? U : 1];
                    if constexpr (MODE == kJoinWrite) {
#pragma unroll
                        for (int u = 0; u < U; ++u) {
                            const uint64_t i = s0 + tid + u * BLOCK;
                            const uint64_t x = i < nS ? ld_nt(sp + i) : 0ull;
                            ks[u] = (uint32_t)x;
                            sv[u] = (uint32_t)(x >> 32);
                        }
                    } else {
#pragma unroll
                        for (int u = 0; u < U; ++u) {
                            const uint64_t i = s0 + tid + u * BLOCK;
                            if constexpr (KS == 1)
                                ks[u] = i < nS ? __builtin_nontemporal_load(Sk + s_start[p] + s_lo + i) : 0u;
                            else
                                ks[u] = i < nS ? __builtin_nontemporal_load(reinterpret_cast<const uint32_t *>(sp + i)) : 0u;
                        }
                    }
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const uint64_t i = s0 + tid + u * BLOCK;
                        cur[u] = i < nS ? L.head[(ks[u] >> hash_shift) & hmask] : 0u;
                    }
                    bool more = true;
                    while (more) {
                        more = false;
#pragma unroll
                        for (int u = 0; u < U; ++u) {
                            if constexpr (MODE == kJoinWrite) {
                                // ballot over the active lanes, one LDS atomic per wave
                                bool m = false;
                                uint32_t e = 0;
                                if (cur[u]) {
                                    e = cur[u] - 1;
                                    m = L.keys[e] == ks[u];
                                }
                                // the chain-walk loop diverges: lanes whose chains ended have left
                                // it, so the slot is taken by the lowest still-active lane
                                const uint64_t bal = __ballot(m);
                                if (bal) {
                                    const int leader = __ffsll((unsigned long long)__ballot(1)) - 1;
                                    uint32_t base = 0;
                                    if ((int)lane == leader) base = atomicAdd(&L.cursor, (uint32_t)__popcll(bal));
                                    base = __shfl(base, leader, kWave);
                                    if (m) {
                                        const uint64_t o = task_off[t] + base + __popcll(bal & lanemask_lt());
                                        uint32_t *w = reinterpret_cast<uint32_t *>(out + o);
                                        w[0] = ks[u];
                                        w[1] = L.rpay[e];
                                        w[2] = sv[u];
                                    }
                                }
                                if (cur[u]) {
                                    cur[u] = L.next[e];
                                    more |= cur[u] != 0;
                                }
                            } else if (cur[u] != 0) {
                                const uint32_t e = cur[u] - 1;
                                tmatch += (L.keys[e] == ks[u]);
                                cur[u] = L.next[e];
                                more |= cur[u] != 0;
                            }
                        }
                    }
                }
                __syncthreads();
                pcyc += wall_clock64() - c_probe;
            }
        }
        if constexpr (MODE == kJoinTaskCount) {
            const uint64_t wsum = wave_sum_u64(tmatch);
            __syncthreads();  // red aliases head
            if (lane == 0) L.red[tid / kWave] = wsum;
            __syncthreads();
            if (tid == 0) {
                uint64_t acc = 0;
                for (int w = 0; w < NW; ++w) acc += L.red[w];
                counts[t] = acc;
            }
            __syncthreads();
        } else if constexpr (MODE == kJoinWrite) {
            __syncthreads();  // the task's cursor is re-armed only after every wave wrote
        }
        matches += tmatch;
    }
    if constexpr (MODE == kJoinCount) {
        matches = wave_sum_u64(matches);
        __syncthreads();
        if (lane == 0) L.red[tid / kWave] = matches;
        __syncthreads();
        if (tid == 0) {
            uint64_t acc = 0;
            for (int w = 0; w < NW; ++w) acc += L.red[w];
            counts[blockIdx.x] = acc;
        }
    }
    if (cyc && tid == 0) {
        cyc[2 * blockIdx.x] = bcyc;
        cyc[2 * blockIdx.x + 1] = pcyc;
    }
    dbg_stamp(2, 1);
    if constexpr (MODE == kJoinCount) {
        if (red_ticket) join_reduce_last(counts, cyc, red_result, red_ticket, L.red, T);
    }
    dbg_stamp(2, 2);
}

// ------------------------------ 16,384-key counting table with exchange links (X) ---
// bucket_chaining_join (:359-458) for counting joins with one LDS word per bucket and
// one per R key, each a link that carries the tag of the entry it points to:
//   head[b]  = (i + 1) | tag(i) << 16 for the last R key i inserted into bucket b, 0 = empty;
//   link[i]  = head[b] as it was before i was inserted (the next entry and its tag).
// The build is one LDS exchange and one LDS store per R key (no compare-and-swap
// retries: a 32-bit head is swapped whole); a chain step of the probe is one LDS read,
// which yields the next entry's index and tag together, so a probe costs 1 + chain
// length reads (the 80 KiB tagged table reads head, tag and next: 1 + 2 x chain).
// link is indexed by the 1-based entry, so a finished walk (w = 0) reads link[0] = 0 and
// every chain step is branch-free.
// Tags are the 16 key bits above the bucket bits: with hash_shift + log2 N + 16 >= 32
// they are all remaining key bits and tag equality is key equality; otherwise a tag
// match is confirmed against the R key (an L2 hit).  128 KiB per table: one 1,024-thread
// workgroup per CU, so the keys stream in strips of UP per thread with the next strip's
// buffer loads in flight while one is inserted or probed, across task boundaries (the
// 80 KiB table instead overlaps two workgroups' phases).
template <int RCAP, int NW>
struct JoinLdsX {
    union {
        struct {
            uint32_t head[RCAP];
            uint32_t link[RCAP + 1];  // 1-based: link[0] = 0, the end of every chain, is never written
        };
        // narrow relations (x_step DIRECT): the count of R keys per 16-bit residual, two
        // u16 counters per word (a chunk holds at most RCAP <= 65535 keys: no carry)
        uint32_t cnt2[1u << 15];
    };
    static_assert(RCAP <= 65535 && 2 * RCAP >= (1u << 15), "direct count table inside the chain table");
    uint64_t red[NW + 2];
    uint32_t nxt[3];  // task tickets (SGXAMD_JOIN_TICKETS): successors of tasks j (nxt[j & 1]), a skip
};

__device__ __forceinline__ uint32_t key_tag16(uint32_t k, uint32_t tshift) {
    return tshift >= 32 ? 0u : ((k >> tshift) & 0xFFFFu);
}

// Workgroup-uniform position in the workgroup's stream of key strips: task t (grid
// stride), its R chunk rc, phase 0 (R keys, build) or 1 (S keys, probe), strip offset;
// r_base / s_base: the element index of the task's R chunk / S range.
struct XCursor {
    uint64_t t, nR, nS, rc, off, r_base, s_base;
    uint32_t phase;
    uint32_t j;  // the workgroup's task ordinal (task tickets)
};


// Task order: grid stride, or (SGXAMD_JOIN_TICKETS, tick != null) task tickets: a
// workgroup's first task is blockIdx.x, each later one the next value of a device
// counter (+ gridDim.x), so that workgroups take tasks as they finish (Zipf: a few
// partitions hold 33x the mean S, and a static stride leaves some workgroups with far
// more than others).  The ticket for task j's successor is taken by thread 0 when the
// cursor enters task j and lands in LDS (nxt[j & 1]) before task j's first build strip,
// whose barriers publish it; the cursor reads it when it leaves task j.
#ifndef SGXAMD_JOIN_TICKETS
#define SGXAMD_JOIN_TICKETS 0
#endif
struct XTasks {
    const uint64_t *r_start, *r_count, *s_start, *s_count, *over;
    uint64_t P, T, s_chunk;
    uint32_t *tick;  // null: grid stride
    uint32_t *nxt;   // LDS: JoinLdsX::nxt
};

template <int RCAP>
__device__ __forceinline__ uint32_t x_nrc(const XCursor &c) {
    const uint64_t d = c.nR - c.rc;
    return d < (uint64_t)RCAP ? (uint32_t)d : (uint32_t)RCAP;
}

// the first task at or after c.t with work (c.t >= T: none); with tickets, tkv (thread
// 0) receives the ticket of its successor
__device__ __forceinline__ void x_seek(XCursor &c, const XTasks &k, uint32_t &tkv) {
    for (; c.t < k.T;) {
        uint64_t p, chunk;
        // tickets take the further S chunks of the large partitions first (position
        // c.t < n_over: over[c.t]), then the partitions: the largest tasks start first
        // instead of finishing last
        uint64_t t = uni_u64(c.t);
#if SGXAMD_JOIN_TICKETS
        if (k.tick != nullptr) t = t < k.T - k.P ? k.P + t : t - (k.T - k.P);
#endif
        decode_task(t, k.P, k.over, p, chunk);
        p = uni_u64(p);
        chunk = uni_u64(chunk);
        const uint64_t nR = uni_u64(k.r_count[p]), nSp = uni_u64(k.s_count[p]);
        const uint64_t s_lo = chunk * k.s_chunk;
        const uint64_t rem = nSp > s_lo ? nSp - s_lo : 0;
        const uint64_t nS = nR == 0 ? 0 : (rem < k.s_chunk ? rem : k.s_chunk);
        if (nS) {
            c.nR = nR;
            c.nS = nS;
            c.rc = 0;
            c.off = 0;
            c.phase = 0;
            c.r_base = uni_u64(k.r_start[p]);
            c.s_base = uni_u64(k.s_start[p]) + s_lo;
#if SGXAMD_JOIN_TICKETS
            if (k.tick != nullptr && threadIdx.x == 0) tkv = atomicAdd(k.tick, 1u);
#endif
            return;
        }
#if SGXAMD_JOIN_TICKETS
        if (k.tick != nullptr) {  // a task without work (no R or no S tuples): the next ticket now
            __syncthreads();
            if (threadIdx.x == 0) k.nxt[2] = atomicAdd(k.tick, 1u) + gridDim.x;
            __syncthreads();
            c.t = (uint32_t)__builtin_amdgcn_readfirstlane(k.nxt[2]);
            continue;
        }
#endif
        c.t += gridDim.x;
    }
}

template <int RCAP, uint32_t STRIP>
__device__ __forceinline__ void x_advance(XCursor &c, const XTasks &k, uint32_t &tkv) {
    c.off += STRIP;
    if (c.phase == 0) {
        if (c.off >= x_nrc<RCAP>(c)) {
            c.phase = 1;
            c.off = 0;
        }
    } else if (c.off >= c.nS) {
        c.rc += RCAP;
        c.off = 0;
        c.phase = 0;
        if (c.rc >= c.nR) {
#if SGXAMD_JOIN_TICKETS
            c.t = k.tick != nullptr ? (uint32_t)__builtin_amdgcn_readfirstlane(k.nxt[c.j & 1]) : c.t + gridDim.x;
#else
            c.t += gridDim.x;
#endif
            ++c.j;
            x_seek(c, k, tkv);
        }
    }
}

// The strip's keys through a buffer resource over exactly its elements: lanes past the
// end read 0 (hardware bounds check, applied to the VGPR offset, which therefore holds
// the whole offset), so every load is issued unconditionally and the wait for a strip
// never covers the loads of the strip after it.
// The keys arrive as their residuals above the radix bits (key >> hash_shift; NR / NS:
// R's / S's partitions hold them as u16, launch_scatter_blk's narrow partitions).
template <int RCAP, int BLOCK, int UP, int KS, bool NR, bool NS>
__device__ __forceinline__ void x_load(const XCursor &c, const XTasks &k, const uint32_t *rkeys,
                                       const uint32_t *skeys, uint32_t hash_shift, uint32_t (&v)[UP]) {
    constexpr uint32_t STRIP = BLOCK * UP;
    uint64_t base = 0, n = 0;
    const uint32_t *src = rkeys;
    if (c.t < k.T) {
        if (c.phase == 0) {
            base = c.r_base + c.rc + c.off;
            n = x_nrc<RCAP>(c) - c.off;
        } else {
            src = skeys;
            base = c.s_base + c.off;
            n = c.nS - c.off;
        }
    }
    const uint32_t cnt = n < STRIP ? (uint32_t)n : STRIP;
    // (NR == NS: one width for both phases, no branch between the loads and their use)
    const bool nar = NR == NS ? NR : (c.phase == 0 ? NR : NS);
    if (nar) {
        const __amdgpu_buffer_rsrc_t rs = make_rsrc(reinterpret_cast<const uint16_t *>(src) + base, cnt * 2u);
#pragma unroll
        for (int u = 0; u < UP; ++u)
            v[u] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(rs, (int)((threadIdx.x + u * BLOCK) * 2u), 0, 2);
    } else {
        const __amdgpu_buffer_rsrc_t rs = make_rsrc(src + base * KS, cnt * 4u * KS);
#pragma unroll
        for (int u = 0; u < UP; ++u)
            v[u] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, (int)((threadIdx.x + u * BLOCK) * 4u * KS), 0, 2) >>
                   hash_shift;
    }
}

// One strip: clear the table at a chunk's first R strip, insert (phase 0) or probe
// (phase 1) the strip's keys; a barrier after a chunk's last R strip (nx: the strip
// after this one).  Returns the strip's matches (this thread).
// k: residuals (x_load); rbits: the residuals' width (16 when both relations are narrow,
// else 32 - hash_shift).  The bucket is HASH_BIT_MODULO(key, N-1 << bits, bits) = the
// residual's low lgN bits, the tag its next 16.
// DIRECT (either relation narrow): the residuals that can match lie below 2^16, so the
// table has one bucket per residual value — every chain holds one key value, and the
// count a probe takes from it is the chain's length: the table keeps that length (a u16
// counter per residual, cnt2) instead of the chain.  Build: one LDS add per R key;
// probe: one LDS read per S key; a residual at or above 2^16 (the wide relation's)
// matches nothing on the narrow side and is skipped.
#ifndef SGXAMD_JOIN_DIRECT  // development A/B: 0 keeps the chain table for narrow relations
#define SGXAMD_JOIN_DIRECT 1
#endif
#ifndef SGXAMD_ABLATE_JOIN
#define SGXAMD_ABLATE_JOIN 0
#endif
template <int RCAP, int BLOCK, int UP, int KS, bool NR, bool NS = false>
__device__ __forceinline__ uint32_t x_step(JoinLdsX<RCAP, BLOCK / kWave> &L, const XCursor &c, const XCursor &nx,
                                           const uint32_t (&k)[UP], const uint32_t *rkeys, uint32_t hash_shift,
                                           uint32_t rbits, uint32_t tlim, uint64_t &cyc2) {
    const uint32_t tid = threadIdx.x;
    const uint64_t c0 = wall_clock64();
    const uint32_t nrc = x_nrc<RCAP>(c);
    // (DIRECT: tlim = the counters in use, 2^(the narrower relation's residual bits): a
    // residual at or above it matches nothing; only their words are cleared per chunk)
    if constexpr (SGXAMD_JOIN_DIRECT && (NR || NS)) {
        uint32_t m = 0;
        if (c.phase == 0) {
            if (c.off == 0) {
                __syncthreads();  // the previous chunk's probe is done with the table
#if SGXAMD_ABLATE_JOIN != 1  // development ablation 1: no clear (wrong counts)
                for (uint32_t i = tid; i < (tlim + 7) / 8; i += BLOCK)
                    reinterpret_cast<uint4 *>(L.cnt2)[i] = make_uint4(0, 0, 0, 0);
#endif
                __syncthreads();
            }
            const uint32_t lim = nrc - (uint32_t)c.off;
#pragma unroll
            for (int u = 0; u < UP; ++u) {
                const uint32_t r = k[u];
#if SGXAMD_ABLATE_JOIN == 2  // development ablation 2: plain stores instead of the adds (wrong counts)
                if (tid + u * BLOCK < lim && r < tlim) L.cnt2[r >> 1] = r;
#elif SGXAMD_ABLATE_JOIN == 3  // development ablation 3: no table writes (wrong counts)
                if (tid + u * BLOCK < lim && r == 0xFFFFFFFFu) L.cnt2[r >> 1] = r;
#else
                if (tid + u * BLOCK < lim && r < tlim) atomicAdd(&L.cnt2[r >> 1], 1u << ((r & 1u) << 4));
#endif
            }
            if (nx.phase != 0 || nx.t != c.t || nx.rc != c.rc) __syncthreads();  // the chunk's table is complete
        } else {
            const uint64_t lim = c.nS - c.off;
#pragma unroll
            for (int u = 0; u < UP; ++u) {
                const uint32_t r = k[u];
                const bool ok = tid + u * BLOCK < lim && r < tlim;
                const uint32_t w = L.cnt2[(ok ? r : 0u) >> 1];
                m += ok ? (w >> ((r & 1u) << 4)) & 0xFFFFu : 0u;
            }
        }
        cyc2 = wall_clock64() - c0;
        return m;
    }
    const uint32_t lgN = nrc <= 1 ? 0u : 32u - __builtin_clz(nrc - 1);  // N = NEXT_POW_2(numR)
    const uint32_t hmask = (1u << lgN) - 1;
    const uint32_t tshift = lgN;
    uint32_t m = 0;
    if (c.phase == 0) {  // BUILD-LOOP (:407-411)
        if (c.off == 0) {
            __syncthreads();  // the previous chunk's probe is done with the table
            for (uint32_t i = tid; i < ((1u << lgN) + 3) / 4; i += BLOCK)
                reinterpret_cast<uint4 *>(L.head)[i] = make_uint4(0, 0, 0, 0);
            __syncthreads();
        }
        const uint32_t lim = nrc - (uint32_t)c.off;
        if (lim >= BLOCK * UP) {  // a full strip: every exchange in flight before the link stores
            uint32_t old[UP];
#pragma unroll
            for (int u = 0; u < UP; ++u) {
                const uint32_t i = (uint32_t)c.off + tid + u * BLOCK;
                old[u] = atomicExch(&L.head[k[u] & hmask], (i + 1) | (key_tag16(k[u], tshift) << 16));
            }
#pragma unroll
            for (int u = 0; u < UP; ++u) L.link[(uint32_t)c.off + tid + u * BLOCK + 1] = old[u];
        } else {
#pragma unroll
            for (int u = 0; u < UP; ++u) {
                const uint32_t j = tid + u * BLOCK;
                if (j < lim) {
                    const uint32_t i = (uint32_t)c.off + j;
                    L.link[i + 1] = atomicExch(&L.head[k[u] & hmask], (i + 1) | (key_tag16(k[u], tshift) << 16));
                }
            }
        }
        if (nx.phase != 0 || nx.t != c.t || nx.rc != c.rc) __syncthreads();  // the chunk's table is complete
    } else {  // PROBE-LOOP (:429-436)
        const uint64_t lim = c.nS - c.off;
        uint32_t w[UP];
#pragma unroll
        for (int u = 0; u < UP; ++u) {
            const uint32_t h = L.head[k[u] & hmask];
            w[u] = vsel(tid + u * BLOCK < lim, h, 0u);
        }
        if (tshift + 16 >= rbits) {
            // the tag is every remaining key bit: chain steps without branches, all UP link
            // reads in flight at once (a finished walk re-reads link[0], a broadcast)
            bool more = true;
            while (more) {
                more = false;
#pragma unroll
                for (int u = 0; u < UP; ++u) {
                    const uint32_t x = w[u];
                    m += (x != 0 && (x >> 16) == key_tag16(k[u], tshift)) ? 1u : 0u;
                    w[u] = L.link[x & 0xFFFFu];
                    more |= w[u] != 0;
                }
            }
        } else {  // a tag match is confirmed against the R key's residual (an L2 hit)
            const uint32_t *rkc = rkeys + (c.r_base + c.rc) * KS;
            const uint16_t *rkc16 = reinterpret_cast<const uint16_t *>(rkeys) + (c.r_base + c.rc);
            bool more = true;
            while (more) {
                more = false;
#pragma unroll
                for (int u = 0; u < UP; ++u) {
                    if (w[u] != 0) {
                        const uint32_t e = w[u] & 0xFFFFu;
                        if ((w[u] >> 16) == key_tag16(k[u], tshift) &&
                            (NR ? (uint32_t)rkc16[e - 1] : rkc[KS * (e - 1)] >> hash_shift) == k[u])
                            ++m;
                        w[u] = L.link[e];
                        more |= w[u] != 0;
                    }
                }
            }
        }
    }
    cyc2 = wall_clock64() - c0;
    return m;
}

// Keys per thread per strip when both relations are narrow (2-byte keys: the same bytes
// in flight per strip as 8 four-byte keys at 16)
#ifndef SGXAMD_JOIN_UP_NARROW
#define SGXAMD_JOIN_UP_NARROW 16
#endif
// The kernel body for one pair of key widths (NR / NS: R / S hold u16 residuals); the
// kernel picks it once, from the relations' largest keys, so no branch sits inside the loop.
template <int RCAP, int BLOCK, int UP, int KS, bool NR, bool NS>
__device__ __forceinline__ void join_x_body(
    JoinLdsX<RCAP, BLOCK / kWave> &L, const uint64_t *__restrict__ R, const uint64_t *__restrict__ S,
    const uint64_t *__restrict__ r_start, const uint64_t *__restrict__ r_count, const uint64_t *__restrict__ s_start,
    const uint64_t *__restrict__ s_count, uint64_t P, const uint64_t *__restrict__ over,
    const uint32_t *__restrict__ n_over, uint32_t hash_shift, uint64_t s_chunk, uint64_t *__restrict__ counts,
    uint64_t *__restrict__ cyc, uint64_t *__restrict__ red_result, uint64_t *__restrict__ red_ticket,
    uint32_t ncounts, uint32_t *__restrict__ tickets, uint32_t tlim) {
    constexpr int NW = BLOCK / kWave;
    constexpr uint32_t STRIP = BLOCK * UP;
    const uint32_t rbits = NR && NS ? 16u : 32u - hash_shift;
    const uint32_t tid = threadIdx.x, lane = __lane_id();
    const XTasks tk{r_start, r_count, s_start, s_count, over, P, uni_u64(P + *n_over), s_chunk, tickets, L.nxt};
    const uint32_t *rkeys = reinterpret_cast<const uint32_t *>(R);
    const uint32_t *skeys = reinterpret_cast<const uint32_t *>(S);
    uint64_t matches = 0, bcyc = 0, pcyc = 0;
    if (tid == 0) L.link[0] = 0;  // visible after the first build strip's barriers
    uint32_t tkv = 0;  // thread 0: the ticket of the current task's successor (in flight)
    // before the first build strip of a task: its successor's ticket into LDS (the
    // strip's barriers publish it; the ticket was taken a strip earlier, and the wait
    // for this strip's keys, issued after it, has already covered it)
    const auto publish = [&](const XCursor &c) {
#if SGXAMD_JOIN_TICKETS
        if (tk.tick != nullptr && tid == 0 && c.t < tk.T && c.phase == 0 && c.rc == 0 && c.off == 0)
            L.nxt[c.j & 1] = tkv + gridDim.x;
#else
        (void)c;
#endif
    };

    XCursor ca{(uint64_t)blockIdx.x, 0, 0, 0, 0, 0, 0, 0, 0}, cb{};
    x_seek(ca, tk, tkv);
    uint32_t ka[UP], kb[UP];
    x_load<RCAP, BLOCK, UP, KS, NR, NS>(ca, tk, rkeys, skeys, hash_shift, ka);
    // two register sets, the loop unrolled by two so that no set is ever copied (a copy
    // of a set still in flight would wait for it); the empty asm uses wait for a set
    // right after the next set's loads are issued, in straight-line code, where the
    // compiler's wait count is exactly UP
    while (ca.t < tk.T) {
        cb = ca;
        x_advance<RCAP, STRIP>(cb, tk, tkv);
        x_load<RCAP, BLOCK, UP, KS, NR, NS>(cb, tk, rkeys, skeys, hash_shift, kb);
#pragma unroll
        for (int u = 0; u < UP; ++u) asm volatile("" ::"v"(ka[u]));
        publish(ca);
        uint64_t dt;
        matches += x_step<RCAP, BLOCK, UP, KS, NR, NS>(L, ca, cb, ka, rkeys, hash_shift, rbits, tlim, dt);
        bcyc += ca.phase == 0 ? dt : 0;
        pcyc += ca.phase == 0 ? 0 : dt;
        if (cb.t >= tk.T) break;
        ca = cb;
        x_advance<RCAP, STRIP>(ca, tk, tkv);
        x_load<RCAP, BLOCK, UP, KS, NR, NS>(ca, tk, rkeys, skeys, hash_shift, ka);
#pragma unroll
        for (int u = 0; u < UP; ++u) asm volatile("" ::"v"(kb[u]));
        publish(cb);
        matches += x_step<RCAP, BLOCK, UP, KS, NR, NS>(L, cb, ca, kb, rkeys, hash_shift, rbits, tlim, dt);
        bcyc += cb.phase == 0 ? dt : 0;
        pcyc += cb.phase == 0 ? 0 : dt;
    }
    matches = wave_sum_u64(matches);
    __syncthreads();
    if (lane == 0) L.red[tid / kWave] = matches;
    __syncthreads();
    if (tid == 0) {
        uint64_t acc = 0;
        for (int w = 0; w < NW; ++w) acc += L.red[w];
        counts[blockIdx.x] = acc;
    }
    if (cyc && tid == 0) {
        cyc[2 * blockIdx.x] = bcyc;
        cyc[2 * blockIdx.x + 1] = pcyc;
    }
    // the grid is one workgroup per CU; the caller's count slots past it read as 0
    for (uint32_t i = gridDim.x + blockIdx.x * BLOCK + tid; i < ncounts; i += gridDim.x * BLOCK) {
        counts[i] = 0;
        if (cyc) cyc[2 * i] = cyc[2 * i + 1] = 0;
    }
    if (red_ticket) join_reduce_last(counts, cyc, red_result, red_ticket, L.red, tk.T);
}

// k_reduce folded into k_join_x (its workgroups are few -- one per CU -- and, on narrow
// relations, idle): every workgroup arrives on res[7] after its slots are written; the
// last sums the ncounts count slots and tick pairs (k_join_n's or k_join_x's) into
// res[0] / [4] / [5].  Called by every thread of the workgroup.
// x_fold_sum: the sums alone, by one workgroup (the narrow relations' path, whose count
// slots an earlier launch, k_join_n, wrote: workgroup 0 sums them while the others return,
// instead of every workgroup arriving on the ticket -- 256 device atomics on one word).
// host (nullable): mapped host memory that also receives the result block's words 0..6
// (the caller then needs no copy of them after the stream synchronisation).
template <int BLOCK>
__device__ __forceinline__ void x_fold_sum(const uint64_t *__restrict__ counts, const uint64_t *__restrict__ cyc,
                                           uint32_t ncounts, uint64_t *__restrict__ res, uint64_t *red,
                                           uint64_t *host);
template <int BLOCK>
__device__ __forceinline__ void x_fold_reduce(const uint64_t *__restrict__ counts, const uint64_t *__restrict__ cyc,
                                              uint32_t ncounts, uint64_t *__restrict__ res, uint64_t *red,
                                              uint64_t *host) {
    __shared__ uint32_t last;
    __syncthreads();  // this workgroup's slot writes are issued
    if (threadIdx.x == 0) {
        __threadfence();
        last = atomicAdd(reinterpret_cast<unsigned long long *>(&res[7]), 1ull) == gridDim.x - 1 ? 1u : 0u;
    }
    __syncthreads();
    if (!last) return;
    __threadfence();
    x_fold_sum<BLOCK>(counts, cyc, ncounts, res, red, host);
}
template <int BLOCK>
__device__ __forceinline__ void x_fold_sum(const uint64_t *__restrict__ counts, const uint64_t *__restrict__ cyc,
                                           uint32_t ncounts, uint64_t *__restrict__ res, uint64_t *red,
                                           uint64_t *host) {
    constexpr uint32_t NW = BLOCK / kWave;
    uint64_t c = 0, b = 0, p = 0;
    for (uint32_t i = threadIdx.x; i < ncounts; i += BLOCK) {
        c += __hip_atomic_load(&counts[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cyc) {
            b += __hip_atomic_load(&cyc[2 * i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            p += __hip_atomic_load(&cyc[2 * i + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    c = wave_sum_u64(c);
    b = wave_sum_u64(b);
    p = wave_sum_u64(p);
    const uint32_t w = threadIdx.x / kWave;
    __syncthreads();  // (red: the join body's last use is done)
    if (__lane_id() == 0) {
        red[w] = c;
        red[NW + w] = b;
        red[2 * NW + w] = p;
    }
    __syncthreads();
    const uint32_t tid = threadIdx.x;
    if (tid < 3) {
        uint64_t t = 0;
        for (uint32_t k = 0; k < NW; ++k) t += red[tid * NW + k];
        if (tid == 0) res[0] = t;
        else if (cyc) res[3 + tid] = t;
        if (host && (tid == 0 || cyc)) host[tid == 0 ? 0 : 3 + tid] = t;
    } else if (host && tid >= kWave && tid < kWave + 7) {
        // the words earlier launches wrote (largest partitions, extra tasks, the widths)
        const uint32_t w = tid - kWave;
        if (!(w == 0 || (cyc && (w == 4 || w == 5))))
            host[w] = __hip_atomic_load(&res[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (host) __threadfence_system();
}

template <int RCAP, int BLOCK, int UP, int KS = 1>
__global__ __launch_bounds__(BLOCK, 1) void k_join_x(
    const uint64_t *__restrict__ R, const uint64_t *__restrict__ S, const uint64_t *__restrict__ r_start,
    const uint64_t *__restrict__ r_count, const uint64_t *__restrict__ s_start, const uint64_t *__restrict__ s_count,
    uint64_t P, const uint64_t *__restrict__ over, const uint32_t *__restrict__ n_over, uint32_t hash_shift,
    uint64_t s_chunk, uint64_t *__restrict__ counts, uint64_t *__restrict__ cyc, uint64_t *__restrict__ red_result,
    uint64_t *__restrict__ red_ticket, uint32_t ncounts, uint32_t *__restrict__ tickets,
    const uint32_t *__restrict__ narrow_r, const uint32_t *__restrict__ narrow_s, uint32_t skip_narrow,
    uint64_t *__restrict__ fold, uint64_t *fold_host) {
    __shared__ JoinLdsX<RCAP, BLOCK / kWave> L;
    // (the same test as k_sort_blk's, which wrote the partitions)
    const bool nr = narrow_r != nullptr && ((*narrow_r >> hash_shift) >> 16) == 0;
    const bool ns = narrow_s != nullptr && ((*narrow_s >> hash_shift) >> 16) == 0;
    if (skip_narrow && (nr || ns)) {  // k_join_n, launched beside it, joined them
        if (fold && blockIdx.x == 0)
            x_fold_sum<BLOCK>(counts, cyc, ncounts, fold, reinterpret_cast<uint64_t *>(L.head), fold_host);
        return;
    }
    // the direct table's counters: residuals below 2^(the fewest residual bits of a narrow
    // relation; 16 for a wide one) — BASELINE config 2's keys 1..2^28 over 14 bits: 2^14
    const auto res_bits = [&](bool n, const uint32_t *kmax) -> uint32_t {
        const uint32_t x = n ? (*kmax >> hash_shift) : 0xFFFFu;
        return x ? 32u - (uint32_t)__builtin_clz(x) : 0u;
    };
#ifdef SGXAMD_JOIN_FULL_TABLE  // development A/B: all 2^16 counters
    const uint32_t tlim = 1u << 16;
#else
    const uint32_t tlim = 1u << min(res_bits(nr, narrow_r), res_bits(ns, narrow_s));
#endif
    // the widths taken, for the caller's statistics (the ticket word's high half, zeroed by
    // launch_make_tasks)
    if (tickets && blockIdx.x == 0 && threadIdx.x == 0) tickets[1] = 1u | (nr ? 2u : 0u) | (ns ? 4u : 0u);
#define JOIN_X_BODY_U(U, A, B)                                                                                     \
    join_x_body<RCAP, BLOCK, U, KS, A, B>(L, R, S, r_start, r_count, s_start, s_count, P, over, n_over, hash_shift, \
                                          s_chunk, counts, cyc, red_result, red_ticket, ncounts, tickets, tlim)
#define JOIN_X_BODY(A, B) JOIN_X_BODY_U(UP, A, B)
    if constexpr (KS == 1) {
        if (nr && ns) JOIN_X_BODY_U(SGXAMD_JOIN_UP_NARROW, true, true);
        else if (nr) JOIN_X_BODY(true, false);
        else if (ns) JOIN_X_BODY(false, true);
        else JOIN_X_BODY(false, false);
    } else {
        JOIN_X_BODY(false, false);
    }
#undef JOIN_X_BODY
#undef JOIN_X_BODY_U
    if (fold) x_fold_reduce<BLOCK>(counts, cyc, ncounts, fold, reinterpret_cast<uint64_t *>(L.head), fold_host);
}

// ------------------------------------------- narrow build/probe (round 5) ---
// k_join_n: bucket_chaining_join (radix_join.cpp:359-458) over narrow partitions as a
// direct count table (x_step DIRECT's table: one counter per residual, since a chain of
// the one-bucket-per-residual table holds one key value and a probe counts its length),
// with an LDS footprint sized to the residuals instead of k_join_x's 128 KiB chain
// table, and one task per workgroup: two to four workgroups share a CU, so one task's
// clear and barriers overlap another's loads (k_join_x, one workgroup per CU, left the
// CU's memory queue idle at every per-chunk clear and build->probe barrier).
//
// Table: kNarrowCap counters (2^14 + 64: BASELINE config 2's keys 1..2^28 over 14 radix
// bits leave residuals 0..2^14 -- the relations' largest keys, pass 1's kmax words, give
// the bound) and two dump slots: DR takes the R keys that do not go into the table
// (outside the strip, or, in the general body, outside the window), DS -- never written
// -- is the counter the S keys outside read (0).  C16: u16 counters, two per word
// (a chunk holds at most kBigRcap keys: no carry into the neighbour).
//
// Keys stream in strips of L 16-byte loads per thread (8 u16 residuals or 4 u32 keys per
// load), through a buffer resource from the 16-byte boundary at or below the range's
// first key; lanes whose 16 bytes straddle the range's ends replace the keys outside it
// with the dump slot (only the first and last strip check, a branch only those lanes
// take), so the loops themselves hold no per-key test.
//
// Fast body (both relations narrow, every residual below kNarrowCap): per key one LDS
// add (build) or one LDS read (probe) and its address.  General body (one relation
// wide, or residuals up to 2^16): the matching residual range [0, lim) (the narrow
// relations' largest residual + 1) in windows of kNarrowCap, each key mapped to its
// window's counter or the dump slot; the strips of a chunk are read once per window.
constexpr uint32_t kNarrowCap = (1u << 14) + 64;

template <int BLOCK, bool C16>
struct JoinLdsN {
    static constexpr uint32_t DR = kNarrowCap, DS = C16 ? kNarrowCap + 2 : kNarrowCap + 1;
    static constexpr uint32_t WORDS = ((C16 ? kNarrowCap / 2 + 2 : kNarrowCap + 2) + 3) & ~3u;
    uint32_t cnt[WORDS];
    uint64_t red[BLOCK / kWave];
};

// One relation's range of a task: 16-byte aligned byte base, the keys before the range
// start inside the first 16 bytes (h), the keys (n), strips of SB bytes.
struct NRange {
    const char *p;
    uint32_t h, n, strips, bytes;
};

template <int ESZ, uint32_t SB>
__device__ __forceinline__ NRange n_range(const void *keys, uint64_t first, uint32_t n) {
    const uint64_t b = first * ESZ, a = b & ~15ull;
    NRange r;
    r.p = static_cast<const char *>(keys) + a;
    r.h = (uint32_t)(b - a) / ESZ;
    r.n = n;
    // whole 16-byte units (the buffers hold at least 15 bytes past any range: the
    // partitions of |X| keys sit in a buffer of 8 |X| bytes)
    r.bytes = ((r.h + n) * ESZ + 15u) & ~15u;
    r.strips = (r.bytes + SB - 1) / SB;
    return r;
}

// (bytes = 0: no strip, every load reads 0; issued all the same, so that no branch
// stands between a strip's loads and the wait for them)
template <int BLOCK, int L>
__device__ __forceinline__ void n_load(const char *p, uint32_t bytes, uint32_t k, uint4 (&v)[L]) {
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(p, bytes);
#pragma unroll
    for (int j = 0; j < L; ++j)
        v[j] = buf_ld_nt_u128(rs, (k * (uint32_t)(BLOCK * L) + threadIdx.x + (uint32_t)j * BLOCK) * 16u, 0);
}

// The u16 residuals of one 16-byte load outside [h, h + n) (element q0 = the load's
// first) replaced by the dump slot D (a u16 value: kNarrowCap + 2 < 2^16).
__device__ __forceinline__ void n_fix16(uint4 &w, uint32_t q0, uint32_t h, uint32_t n, uint32_t D) {
    uint32_t c[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const bool lo = q0 + 2 * i - h < n, hi = q0 + 2 * i + 1 - h < n;
        c[i] = (lo ? c[i] & 0xFFFFu : D) | (hi ? c[i] & 0xFFFF0000u : D << 16);
    }
    w = make_uint4(c[0], c[1], c[2], c[3]);
}

template <bool C16>
__device__ __forceinline__ void n_add(uint32_t *cnt, uint32_t k) {
    if constexpr (C16) atomicAdd(&cnt[k >> 1], 1u << ((k & 1u) << 4));
    else atomicAdd(&cnt[k], 1u);
}
template <bool C16>
__device__ __forceinline__ uint32_t n_get(const uint32_t *cnt, uint32_t k) {
    if constexpr (C16) return reinterpret_cast<const uint16_t *>(cnt)[k];
    else return cnt[k];
}

// One strip of a relation: build (BUILD: adds) or probe (returns the matches).
// NAR: u16 residuals; else u32 keys (residual = key >> hash_shift).  GEN: the general
// body's window mapping (wb: the window's first residual, wl: its counters in use).
// PC (pieces, the u16 wire's S side): load j of this lane holds nv[j] valid residuals
// (its first ones), whatever r says.
template <int BLOCK, int L, bool C16, bool NAR, bool BUILD, bool GEN, bool PC = false>
__device__ __forceinline__ uint32_t n_strip(uint32_t *cnt, const NRange &r, uint32_t k, uint4 (&v)[L],
                                            uint32_t hash_shift, uint32_t wb, uint32_t wl,
                                            const uint32_t *nv = nullptr) {
    constexpr uint32_t KPL = NAR ? 8 : 4;
    constexpr uint32_t D = BUILD ? JoinLdsN<BLOCK, C16>::DR : JoinLdsN<BLOCK, C16>::DS;
    static_assert(!PC || (NAR && !BUILD), "pieces: the S side's u16 residuals");
    // the strip's first and last units may straddle the range's ends (uniform test)
    const uint32_t u0 = k * (uint32_t)(BLOCK * L);
    const bool edge = (k == 0 && r.h != 0) || (u0 + BLOCK * L) * KPL > r.h + r.n;
    uint32_t m = 0;
#pragma unroll
    for (int j = 0; j < L; ++j) {
        const uint32_t q0 = PC ? 0u : (u0 + threadIdx.x + (uint32_t)j * BLOCK) * KPL;
        const uint32_t h = PC ? 0u : r.h, n = PC ? nv[j] : r.n;
        if constexpr (!GEN) {  // (both narrow, every residual inside the table)
            if (PC ? n < KPL : (edge && (q0 < r.h || q0 + KPL > r.h + r.n))) n_fix16(v[j], q0, h, n, D);
            const uint32_t c[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t a = c[i] & 0xFFFFu, b = c[i] >> 16;
                if constexpr (BUILD) {
                    n_add<C16>(cnt, a);
                    n_add<C16>(cnt, b);
                } else {
                    m += n_get<C16>(cnt, a) + n_get<C16>(cnt, b);
                }
            }
        } else {
            const uint32_t c[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
#pragma unroll
            for (int i = 0; i < (int)KPL; ++i) {
                const uint32_t key = NAR ? ((c[i / 2] >> ((i & 1) * 16)) & 0xFFFFu) : (c[i] >> hash_shift);
                const uint32_t x = key - wb;
                const uint32_t e = (q0 + (uint32_t)i - h < n && x < wl) ? x : D;
                if constexpr (BUILD) n_add<C16>(cnt, e);
                else m += n_get<C16>(cnt, e);
            }
        }
    }
    return m;
}

// The u16 wire's S side read in place (round 6): partition p of S is
// G pieces, one per sender, each starting on a 16-byte unit of the receive buffer (the
// senders pad every partition to 8 residuals, multi_host.cpp); a task's S chunk is a range
// of units in the partition's unit space (its pieces' units back to back).  Lane unit u
// finds its piece by comparing u with the pieces' first units (G <= kPieceMax, unrolled:
// the arrays stay in SGPRs) and loads its 16 bytes; its valid residuals are the piece's
// keys left (at most 8).  Replaces the gather into contiguous partitions (k_wire_gather).
constexpr uint32_t kPieceMax = 8;
struct SPieces {
    __amdgpu_buffer_rsrc_t rs;  // the receive buffer of residuals
    uint32_t u0, nu, G;         // the chunk's first unit (partition unit space), its units, pieces
    uint32_t up[kPieceMax];     // first unit of piece q in the partition's unit space
    uint32_t ub[kPieceMax];     // piece q's first unit in the receive buffer
    uint32_t nk[kPieceMax];     // its keys
};

template <int BLOCK, int L>
__device__ __forceinline__ void n_load_pieces(const SPieces &sp, uint32_t k, uint4 (&v)[L], uint32_t (&nv)[L]) {
#pragma unroll
    for (int j = 0; j < L; ++j) {
        const uint32_t i = k * (uint32_t)(BLOCK * L) + threadIdx.x + (uint32_t)j * BLOCK;  // unit of the chunk
        const uint32_t u = sp.u0 + i;
        uint32_t up = sp.up[0], ub = sp.ub[0], nk = sp.nk[0];
#pragma unroll
        for (uint32_t q = 1; q < kPieceMax; ++q) {
            const bool in = q < sp.G && u >= sp.up[q];
            up = in ? sp.up[q] : up;
            ub = in ? sp.ub[q] : ub;
            nk = in ? sp.nk[q] : nk;
        }
        const uint32_t r = u - up, left = nk > 8 * r ? nk - 8 * r : 0u;
        const bool ok = i < sp.nu;
        nv[j] = ok ? min(left, 8u) : 0u;
        // (a unit past the chunk reads 0 through the buffer bounds)
        v[j] = buf_ld_nt_u128(sp.rs, ok ? (ub + r) * 16u : 0xFFFFFFF0u, 0);
    }
}

// One task (a partition's S chunk): per R chunk of kBigRcap keys and per window, clear,
// build from R's strips, probe S's strips; the strips of one (chunk, window) pass are
// one sequence with the next strip's loads in flight while one is processed.
// PC: S is the u16 wire's pieces (sp), not the contiguous range [s_base, + nS).
template <int BLOCK, int L, bool C16, bool NR, bool NS, bool GEN, bool PC = false>
__device__ __forceinline__ uint64_t join_n_task(JoinLdsN<BLOCK, C16> &Ls, const void *rk, const void *sk,
                                                uint64_t r_base, uint64_t nR, uint64_t s_base, uint32_t nS,
                                                uint32_t hash_shift, uint32_t lim, uint64_t &bt, uint64_t &pt,
                                                const SPieces *sp = nullptr) {
    constexpr uint32_t SB = BLOCK * L * 16u;
    constexpr int ER = NR ? 2 : 4, ES = NS ? 2 : 4;
    static_assert(!PC || NS, "pieces hold u16 residuals");
    const uint32_t nwin = GEN ? (lim + kNarrowCap - 1) / kNarrowCap : 1u;
    const NRange sr = PC ? NRange{nullptr, 0u, 0u, 0u, 0u} : n_range<ES, SB>(sk, s_base, nS);
    const uint32_t s_strips = PC ? (sp->nu + BLOCK * L - 1) / (BLOCK * L) : sr.strips;
    uint64_t m = 0;
    bool first = true;
    for (uint64_t rc = 0; rc < nR; rc += kBigRcap) {
        const NRange rr = n_range<ER, SB>(rk, r_base + rc, (uint32_t)min(nR - rc, (uint64_t)kBigRcap));
        const uint32_t nsr = rr.strips, ns = nsr + s_strips;
        for (uint32_t w = 0; w < nwin; ++w) {
            const uint32_t wb = w * kNarrowCap, wl = GEN ? min(kNarrowCap, lim - wb) : kNarrowCap;
            const uint64_t t0 = wall_clock64();
            uint4 va[L], vb[L];
            uint32_t nva[L], nvb[L];
            const auto load = [&](uint32_t i, uint4(&v)[L], uint32_t(&nv)[L]) {
                const bool isr = i < nsr;
                if constexpr (PC) {
                    if (!isr) {  // (uniform)
                        n_load_pieces<BLOCK, L>(*sp, i < ns ? i - nsr : 0xFFFFu, v, nv);
                        return;
                    }
                }
                n_load<BLOCK, L>(isr ? rr.p : sr.p, isr ? rr.bytes : (i < ns ? sr.bytes : 0u), isr ? i : i - nsr, v);
            };
            uint64_t tb = t0;
            const auto step = [&](uint32_t i, uint4(&v)[L], const uint32_t(&nv)[L]) {
                if (i < nsr) {
                    n_strip<BLOCK, L, C16, NR, true, GEN>(Ls.cnt, rr, i, v, hash_shift, wb, wl);
                    if (i + 1 == nsr) {
                        __syncthreads();  // the table is complete
                        tb = wall_clock64();
                    }
                } else {
                    m += n_strip<BLOCK, L, C16, NS, false, GEN, PC>(Ls.cnt, sr, i - nsr, v, hash_shift, wb, wl, nv);
                }
            };
            load(0, va, nva);
            if (!first) __syncthreads();  // the previous pass's probe is done with the table
            first = false;
            for (uint32_t i = threadIdx.x; i < JoinLdsN<BLOCK, C16>::WORDS / 4; i += BLOCK)
                reinterpret_cast<uint4 *>(Ls.cnt)[i] = make_uint4(0, 0, 0, 0);
            __syncthreads();
            // two register sets, the loop unrolled by two (no copy of a set in flight)
            for (uint32_t i = 0;; i += 2) {
                load(i + 1, vb, nvb);
#pragma unroll
                for (int j = 0; j < L; ++j) asm volatile("" ::"v"(va[j].x), "v"(va[j].y), "v"(va[j].z), "v"(va[j].w));
                step(i, va, nva);
                if (i + 1 >= ns) break;
                load(i + 2, va, nva);
#pragma unroll
                for (int j = 0; j < L; ++j) asm volatile("" ::"v"(vb[j].x), "v"(vb[j].y), "v"(vb[j].z), "v"(vb[j].w));
                step(i + 1, vb, nvb);
                if (i + 2 >= ns) break;
            }
            bt += tb - t0;
            pt += wall_clock64() - tb;
        }
    }
    return m;
}

// Geometry: BLOCK threads, L 16-byte loads per thread and strip, C16 u16 counters,
// WPC workgroups per CU (occupancy hint).
#ifndef SGXAMD_JN_BLOCK
#define SGXAMD_JN_BLOCK 256
#endif
#ifndef SGXAMD_JN_L
#define SGXAMD_JN_L 4
#endif
#ifndef SGXAMD_JN_C16
#define SGXAMD_JN_C16 1
#endif
#ifndef SGXAMD_JN_WPC
#define SGXAMD_JN_WPC 4
#endif

// grid = an upper bound of the tasks (P + over_cap - 1); workgroup t takes task t
// (decode_task: the partitions, then the further S chunks of large ones).  Counts and
// build / probe ticks go to slot t mod nslots (device atomics, the slots zeroed by
// launch_make_tasks).  Nothing to do unless a relation is narrow (k_join_x, launched
// beside it, takes that case).
template <int BLOCK, int L, bool C16>
__global__ __launch_bounds__(BLOCK, BLOCK *SGXAMD_JN_WPC / 256) void k_join_n(
    const void *__restrict__ R, const void *__restrict__ S, const uint64_t *__restrict__ r_start,
    const uint64_t *__restrict__ r_count, const uint64_t *__restrict__ s_start, const uint64_t *__restrict__ s_count,
    uint64_t P, const uint64_t *__restrict__ over, const uint32_t *__restrict__ n_over, uint32_t hash_shift,
    uint64_t s_chunk, uint64_t *__restrict__ counts, uint64_t *__restrict__ cyc, uint32_t nslots,
    uint32_t *__restrict__ tickets, const uint32_t *__restrict__ narrow_r, const uint32_t *__restrict__ narrow_s) {
    __shared__ JoinLdsN<BLOCK, C16> Ls;
    // the largest residual of each relation (k_sort_blk's test: narrow below 2^16)
    const uint32_t xr = narrow_r ? (*narrow_r >> hash_shift) : 0xFFFFFFFFu;
    const uint32_t xs = narrow_s ? (*narrow_s >> hash_shift) : 0xFFFFFFFFu;
    const bool nr = xr < 0x10000u, ns = xs < 0x10000u;
    if (!nr && !ns) return;
    if (tickets && blockIdx.x == 0 && threadIdx.x == 0) tickets[1] = 1u | (nr ? 2u : 0u) | (ns ? 4u : 0u);
    const uint64_t t = blockIdx.x;
    if (t >= P + *n_over) return;
    uint64_t p, chunk;
    decode_task(t, P, over, p, chunk);
    const uint64_t nR = r_count[p], nSp = s_count[p];
    const uint64_t s_lo = chunk * s_chunk;
    const uint64_t rem = nSp > s_lo ? nSp - s_lo : 0;
    const uint32_t nS = nR == 0 ? 0u : (uint32_t)(rem < s_chunk ? rem : s_chunk);
    if (nS == 0) return;
    const uint64_t rb = r_start[p], sb = s_start[p] + s_lo;
    // the residuals that can match: [0, lim), lim = the narrow relations' smallest
    // (largest residual + 1)
    const uint32_t lim = min(nr ? xr + 1 : 0xFFFFFFFFu, ns ? xs + 1 : 0xFFFFFFFFu);
    uint64_t bt = 0, pt = 0, m;
    if (nr && ns && xr < kNarrowCap && xs < kNarrowCap)
        m = join_n_task<BLOCK, L, C16, true, true, false>(Ls, R, S, rb, nR, sb, nS, hash_shift, lim, bt, pt);
    else if (nr && ns)
        m = join_n_task<BLOCK, L, C16, true, true, true>(Ls, R, S, rb, nR, sb, nS, hash_shift, lim, bt, pt);
    else if (nr)
        m = join_n_task<BLOCK, L, C16, true, false, true>(Ls, R, S, rb, nR, sb, nS, hash_shift, lim, bt, pt);
    else
        m = join_n_task<BLOCK, L, C16, false, true, true>(Ls, R, S, rb, nR, sb, nS, hash_shift, lim, bt, pt);
    m = wave_sum_u64(m);
    if (__lane_id() == 0) Ls.red[threadIdx.x / kWave] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t acc = 0;
        for (int w = 0; w < BLOCK / kWave; ++w) acc += Ls.red[w];
        const uint32_t slot = (uint32_t)(t % nslots);
        if (acc) atomicAdd((unsigned long long *)&counts[slot], (unsigned long long)acc);
        if (cyc) {
            atomicAdd((unsigned long long *)&cyc[2 * slot], (unsigned long long)bt);
            atomicAdd((unsigned long long *)&cyc[2 * slot + 1], (unsigned long long)pt);
        }
    }
}

// k_join_n over the u16 wire's S pieces (join_n_task PC): task t = (partition p, S chunk
// of s_chunk / 8 units of p's unit space).  piece_ub / piece_nk [p * G + q]: piece (p,
// q)'s first unit in the receive buffer s16 and its keys; s_units8[p] = 8 x p's units
// (the task list's S sizes, launch_make_tasks).  Both relations are narrow here (the
// u16 wire's plan).
template <int BLOCK, int L, bool C16>
__global__ __launch_bounds__(BLOCK, BLOCK *SGXAMD_JN_WPC / 256) void k_join_np(
    const void *__restrict__ R, const uint16_t *__restrict__ s16, uint32_t s_bytes,
    const uint64_t *__restrict__ r_start, const uint64_t *__restrict__ r_count, const uint32_t *__restrict__ piece_ub,
    const uint32_t *__restrict__ piece_nk, uint32_t G, const uint64_t *__restrict__ s_units8, uint64_t P,
    const uint64_t *__restrict__ over, const uint32_t *__restrict__ n_over, uint32_t hash_shift, uint64_t s_chunk,
    uint64_t *__restrict__ counts, uint64_t *__restrict__ cyc, uint32_t nslots, uint32_t *__restrict__ tickets,
    const uint32_t *__restrict__ narrow_r, const uint32_t *__restrict__ narrow_s) {
    __shared__ JoinLdsN<BLOCK, C16> Ls;
    const uint32_t xr = *narrow_r >> hash_shift, xs = *narrow_s >> hash_shift;
    if (xr >= 0x10000u || xs >= 0x10000u) return;  // (the plan guarantees both)
    if (tickets && blockIdx.x == 0 && threadIdx.x == 0) tickets[1] = 1u | 2u | 4u;
    const uint64_t t = blockIdx.x;
    if (t >= P + *n_over) return;
    uint64_t p, chunk;
    decode_task(t, P, over, p, chunk);
    const uint64_t nR = r_count[p];
    const uint32_t units = (uint32_t)(s_units8[p] / 8), cu = (uint32_t)(s_chunk / 8);
    const uint32_t u0 = (uint32_t)chunk * cu;
    const uint32_t nu = u0 < units ? min(cu, units - u0) : 0u;
    if (nR == 0 || nu == 0) return;
    SPieces sp;
    sp.rs = make_rsrc(s16, s_bytes);
    sp.u0 = u0;
    sp.nu = nu;
    sp.G = G;
    uint32_t at = 0;
#pragma unroll
    for (uint32_t q = 0; q < kPieceMax; ++q) {
        const uint32_t nk = q < G ? piece_nk[p * G + q] : 0u;
        sp.up[q] = at;
        sp.ub[q] = q < G ? piece_ub[p * G + q] : 0u;
        sp.nk[q] = nk;
        at += (nk + 7) / 8;
    }
    const uint32_t lim = min(xr, xs) + 1;
    uint64_t bt = 0, pt = 0, m;
    if (xr < kNarrowCap && xs < kNarrowCap)
        m = join_n_task<BLOCK, L, C16, true, true, false, true>(Ls, R, nullptr, r_start[p], nR, 0, 0, hash_shift, lim,
                                                                bt, pt, &sp);
    else
        m = join_n_task<BLOCK, L, C16, true, true, true, true>(Ls, R, nullptr, r_start[p], nR, 0, 0, hash_shift, lim,
                                                               bt, pt, &sp);
    m = wave_sum_u64(m);
    if (__lane_id() == 0) Ls.red[threadIdx.x / kWave] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t acc = 0;
        for (int w = 0; w < BLOCK / kWave; ++w) acc += Ls.red[w];
        const uint32_t slot = (uint32_t)(t % nslots);
        if (acc) atomicAdd((unsigned long long *)&counts[slot], (unsigned long long)acc);
        if (cyc) {
            atomicAdd((unsigned long long *)&cyc[2 * slot], (unsigned long long)bt);
            atomicAdd((unsigned long long *)&cyc[2 * slot + 1], (unsigned long long)pt);
        }
    }
}

// ------------------------------------------------------- histogram join (RHT) ---
// histogram_join (radix_join.cpp:463-612), the build/probe of RHT (:1645-1648), per
// task in LDS.  For an R chunk of nrc tuples: Nhist = max(nextpow2(nrc) / 4, 4)
// buckets (get_hist_size :462-467), bucket = HASH_BIT_MODULO(key, (Nhist-1) << bits,
// bits); an LDS histogram (one atomic per tuple, which is also the tuple's rank in
// its bucket), an exclusive scan into bucket offsets (:520-524), and the R keys
// re-ordered bucket-contiguous in LDS (:527-561).  The probe compares each S key
// with its bucket's contiguous run [off[b], off[b+1]) (:574-600).  The reference's
// unrolled re-order tail drops the "+ 1" of the bucket index (:556-560); that slip
// is not restated here, every R tuple lands in its own bucket.
template <int RCAP, int MODE, int NW = kWaves>
struct HistJoinLds {
    static constexpr int NB = RCAP / 4;  // max buckets of one chunk
    uint32_t off[NB + 1];
    uint32_t keys[RCAP];
    uint32_t rpay[MODE == kJoinWrite ? RCAP : 1];
    uint32_t cursor;
    uint64_t red[NW + 2];
};

// Element i of a partitioned relation: an 8-byte tuple (KS 2) or a 4-byte key (KS 1,
// counting joins over key partitions; the payload half reads as 0).
template <int KS>
__device__ __forceinline__ uint64_t ld_elem_nt(const uint64_t *base, uint64_t i) {
    if constexpr (KS == 2) return ld_nt(base + i);
    else return __builtin_nontemporal_load(reinterpret_cast<const uint32_t *>(base) + i);
}

// BLOCK threads per table: kBlock (256) for tables up to 8192 tuples; 1024 for the
// 16,384-key counting table (80 KiB: keys + 4,097 bucket offsets, two workgroups per CU),
// which probes in strips of 8 S keys per thread to stay within 64 VGPRs.
template <int RCAP, int MODE, int KS = 2, int BLOCK = kBlock>
__global__ __launch_bounds__(BLOCK) void k_join_hist(const uint64_t *__restrict__ R, const uint64_t *__restrict__ S,
                                                      const uint64_t *__restrict__ r_start,
                                                      const uint64_t *__restrict__ r_count,
                                                      const uint64_t *__restrict__ s_start,
                                                      const uint64_t *__restrict__ s_count, uint64_t P,
                                                      const uint64_t *__restrict__ over,
                                                      const uint32_t *__restrict__ n_over, uint32_t hash_shift, uint64_t s_chunk,
                                                      uint64_t *__restrict__ counts,
                                                      const uint64_t *__restrict__ task_off,
                                                      output_triple_t *__restrict__ out, uint64_t *__restrict__ cyc,
                                                      uint64_t *__restrict__ red_result,
                                                      uint64_t *__restrict__ red_ticket) {
    static_assert(KS == 2 || MODE == kJoinCount, "key partitions carry no payloads");
    constexpr int NW = BLOCK / kWave;
    constexpr int U = RCAP / BLOCK;
    constexpr int UP = (BLOCK == kBlock || U < 8) ? U : 8;  // S keys per thread and probe strip
    constexpr int NB = HistJoinLds<RCAP, MODE, NW>::NB;
    // R elements held across the histogram scan: the key (and the payload when writing)
    using RT = typename std::conditional<MODE == kJoinWrite, uint64_t, uint32_t>::type;
    __shared__ HistJoinLds<RCAP, MODE, NW> L;
    __shared__ uint64_t scan_scratch[NW + 1];
    const uint32_t tid = threadIdx.x, lane = __lane_id();
    const uint64_t T = P + *n_over;
    uint64_t matches = 0;
    uint64_t bcyc = 0, pcyc = 0;  // build / probe wall-clock ticks of this workgroup
    for (uint64_t t = blockIdx.x; t < T; t += gridDim.x) {
        uint64_t p, chunk;
        decode_task(t, P, over, p, chunk);
        const uint64_t nR = r_count[p], nSp = s_count[p];
        const uint64_t s_lo = chunk * s_chunk;
        const uint64_t nS = (nR == 0 || s_lo >= nSp) ? 0 : min<uint64_t>(nSp - s_lo, s_chunk);
        uint64_t tmatch = 0;
        if constexpr (MODE == kJoinWrite) {
            if (tid == 0) L.cursor = 0;
        }
        if (nS > 0) {
            const uint64_t r0 = r_start[p], sb = s_start[p] + s_lo;
            for (uint64_t rc = 0; rc < nR; rc += RCAP) {
                const uint64_t c_build = wall_clock64();
                const uint32_t nrc = (uint32_t)((nR - rc) < RCAP ? (nR - rc) : RCAP);
                uint32_t N = 1;
                while (N < nrc) N <<= 1;
                uint32_t nh = N >> 2;
                if (nh < 4) nh = 4;  // get_hist_size
                const uint32_t hmask = nh - 1;
                RT kr[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t i = tid + u * BLOCK;
                    kr[u] = i < nrc ? (RT)ld_elem_nt<KS>(R, r0 + rc + i) : (RT)0;
                }
                for (uint32_t i = tid; i <= nh; i += BLOCK) L.off[i] = 0;
                __syncthreads();
                uint32_t slot[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {  // HISTOGRAM CREATION (:489-517)
                    const uint32_t i = tid + u * BLOCK;
                    if (i < nrc) slot[u] = atomicAdd(&L.off[((uint32_t)kr[u] >> hash_shift) & hmask], 1u);
                }
                __syncthreads();
                {  // prefix sum on histogram (:520-524): thread tid owns buckets [tid*E, tid*E + E)
                    const uint32_t E = (nh + BLOCK - 1) / BLOCK;
                    uint32_t loc[NB / BLOCK > 0 ? NB / BLOCK : 1];
                    uint32_t sum = 0;
                    for (uint32_t j = 0; j < E; ++j) {
                        const uint32_t b = tid * E + j;
                        const uint32_t c = b < nh ? L.off[b] : 0u;
                        loc[j] = sum;
                        sum += c;
                    }
                    uint64_t tot;
                    const uint32_t base = (uint32_t)block_excl_scan_u64(sum, scan_scratch, &tot);
                    for (uint32_t j = 0; j < E; ++j) {
                        const uint32_t b = tid * E + j;
                        if (b < nh) L.off[b] = base + loc[j];
                    }
                    if (tid == 0) L.off[nh] = (uint32_t)tot;
                }
                __syncthreads();
#pragma unroll
                for (int u = 0; u < U; ++u) {  // BUILD PHASE: re-order (:527-561)
                    const uint32_t i = tid + u * BLOCK;
                    if (i < nrc) {
                        const uint32_t pos = L.off[((uint32_t)kr[u] >> hash_shift) & hmask] + slot[u];
                        L.keys[pos] = (uint32_t)kr[u];
                        if constexpr (MODE == kJoinWrite) L.rpay[pos] = (uint32_t)(kr[u] >> 32);
                    }
                }
                __syncthreads();
                const uint64_t c_probe = wall_clock64();
                bcyc += c_probe - c_build;
                for (uint64_t s0 = 0; s0 < nS; s0 += (uint64_t)UP * BLOCK) {  // PROBE PHASE (:570-600)
                    uint32_t ks[UP], j[UP], end[UP];
                    uint32_t sv[MODE == kJoinWrite ? UP : 1];
#pragma unroll
                    for (int u = 0; u < UP; ++u) {
                        const uint64_t i = s0 + tid + u * BLOCK;
                        const uint64_t x = i < nS ? ld_elem_nt<KS>(S, sb + i) : 0ull;
                        ks[u] = (uint32_t)x;
                        if constexpr (MODE == kJoinWrite) sv[u] = (uint32_t)(x >> 32);
                    }
#pragma unroll
                    for (int u = 0; u < UP; ++u) {
                        const uint64_t i = s0 + tid + u * BLOCK;
                        const uint32_t b = (ks[u] >> hash_shift) & hmask;
                        j[u] = i < nS ? L.off[b] : 0u;
                        end[u] = i < nS ? L.off[b + 1] : 0u;
                    }
                    bool more = true;
                    while (more) {
                        more = false;
#pragma unroll
                        for (int u = 0; u < UP; ++u) {
                            if constexpr (MODE == kJoinWrite) {
                                const bool live = j[u] < end[u];
                                const bool m = live && L.keys[j[u]] == ks[u];
                                const uint64_t bal = __ballot(m);
                                if (bal) {
                                    const int leader = __ffsll((unsigned long long)__ballot(1)) - 1;
                                    uint32_t base = 0;
                                    if ((int)lane == leader) base = atomicAdd(&L.cursor, (uint32_t)__popcll(bal));
                                    base = __shfl(base, leader, kWave);
                                    if (m) {
                                        const uint64_t o = task_off[t] + base + __popcll(bal & lanemask_lt());
                                        uint32_t *w = reinterpret_cast<uint32_t *>(out + o);
                                        w[0] = ks[u];
                                        w[1] = L.rpay[j[u]];
                                        w[2] = sv[u];
                                    }
                                }
                                if (live) {
                                    ++j[u];
                                    more |= j[u] < end[u];
                                }
                            } else if (j[u] < end[u]) {
                                tmatch += (L.keys[j[u]] == ks[u]);
                                ++j[u];
                                more |= j[u] < end[u];
                            }
                        }
                    }
                }
                __syncthreads();
                pcyc += wall_clock64() - c_probe;
            }
        }
        if constexpr (MODE == kJoinTaskCount) {
            const uint64_t wsum = wave_sum_u64(tmatch);
            if (lane == 0) L.red[tid / kWave] = wsum;
            __syncthreads();
            if (tid == 0) {
                uint64_t acc = 0;
                for (int w = 0; w < NW; ++w) acc += L.red[w];
                counts[t] = acc;
            }
            __syncthreads();
        } else if constexpr (MODE == kJoinWrite) {
            __syncthreads();
        }
        matches += tmatch;
    }
    if constexpr (MODE == kJoinCount) {
        matches = wave_sum_u64(matches);
        if (lane == 0) L.red[tid / kWave] = matches;
        __syncthreads();
        if (tid == 0) {
            uint64_t acc = 0;
            for (int w = 0; w < NW; ++w) acc += L.red[w];
            counts[blockIdx.x] = acc;
        }
    }
    if (cyc && tid == 0) {
        cyc[2 * blockIdx.x] = bcyc;
        cyc[2 * blockIdx.x + 1] = pcyc;
    }
    if constexpr (MODE == kJoinCount) {
        if (red_ticket) join_reduce_last(counts, cyc, red_result, red_ticket, L.red, T);
    }
}

// RHT counting join (histogram_join :463-612) with 16,384-key tables in 72 KiB, two
// 1,024-thread workgroups per CU: the R keys of a chunk re-ordered bucket-contiguous
// (keys[16384], 64 KiB), bucket offsets as u16 (<= 16,384; 8 KiB), and the histogram's
// u32 counters in the keys' space until the scan has turned them into offsets.  The
// planner then gives RHT the same 14-bit plan as RHO at 2^28 with one table per
// partition (the 8192-tuple table builds each partition in two chunks and probes every
// S key twice).  8 waves per SIMD (64 VGPRs).  Each thread keeps its 16 R keys and their in-bucket ranks (two u16 per
// register) across the scan; the probe walks strips of 8 S keys per thread.
template <int KS>
__global__ __launch_bounds__(1024, 8) void k_join_hist_big(
    const uint64_t *__restrict__ R, const uint64_t *__restrict__ S, const uint64_t *__restrict__ r_start,
    const uint64_t *__restrict__ r_count, const uint64_t *__restrict__ s_start, const uint64_t *__restrict__ s_count,
    uint64_t P, const uint64_t *__restrict__ over, const uint32_t *__restrict__ n_over, uint32_t hash_shift,
    uint64_t s_chunk, uint64_t *__restrict__ counts, uint64_t *__restrict__ cyc, uint64_t *__restrict__ red_result,
    uint64_t *__restrict__ red_ticket) {
    constexpr int RCAP = kBigRcap, BLOCK = 1024, NW = BLOCK / kWave, U = RCAP / BLOCK, UP = 8, NB = RCAP / 4;
    struct Lds {
        union {
            uint32_t hist[NB];  // bucket counters (histogram creation, :489-517)
            uint32_t keys[RCAP];
        };
        uint16_t off[NB + 1];
        uint64_t red[NW + 2];  // block scan scratch, then the reduction
    };
    __shared__ Lds L;
    const uint32_t tid = threadIdx.x, lane = __lane_id();
    const uint64_t T = P + *n_over;
    uint64_t matches = 0, bcyc = 0, pcyc = 0;
    for (uint64_t t = blockIdx.x; t < T; t += gridDim.x) {
        uint64_t p, chunk;
        decode_task(uni_u64(t), P, over, p, chunk);
        p = uni_u64(p);
        chunk = uni_u64(chunk);
        const uint64_t nR = uni_u64(r_count[p]), nSp = uni_u64(s_count[p]);
        const uint64_t s_lo = chunk * s_chunk;
        const uint64_t nS = (nR == 0 || s_lo >= nSp) ? 0 : min<uint64_t>(nSp - s_lo, s_chunk);
        if (nS == 0) continue;
        const uint64_t r0 = uni_u64(r_start[p]), sb = uni_u64(s_start[p]) + s_lo;
        for (uint64_t rc = 0; rc < nR; rc += RCAP) {
            const uint64_t c_build = wall_clock64();
            const uint32_t nrc = (uint32_t)((nR - rc) < RCAP ? (nR - rc) : RCAP);
            uint32_t N = 1;
            while (N < nrc) N <<= 1;
            const uint32_t nh = N >> 2 < 4 ? 4u : N >> 2;  // get_hist_size
            const uint32_t hmask = nh - 1;
            // buffer loads over the chunk: the whole offset in the VGPR (the hardware range
            // check covers the VGPR offset, not the SGPR one), 0 past the chunk's end
            const __amdgpu_buffer_rsrc_t rr =
                make_rsrc(reinterpret_cast<const uint32_t *>(R) + (r0 + rc) * KS, nrc * 4u * KS);
            uint32_t kr[U];
#pragma unroll
            for (int u = 0; u < U; ++u)
                kr[u] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rr, (int)((tid + u * BLOCK) * 4u * KS), 0, 2);
            __syncthreads();  // the previous chunk's probe is done with keys / off
            for (uint32_t i = tid; i < nh; i += BLOCK) L.hist[i] = 0;
            __syncthreads();
            uint32_t slot2[U / 2];  // in-bucket ranks, two u16 per register
            const auto ranks = [&](auto full) {  // HISTOGRAM CREATION (:489-517)
#pragma unroll
                for (int u = 0; u < U; u += 2) {
                    const uint32_t i = tid + u * BLOCK;
                    const uint32_t a =
                        (full || i < nrc) ? atomicAdd(&L.hist[(kr[u] >> hash_shift) & hmask], 1u) : 0u;
                    const uint32_t b =
                        (full || i + BLOCK < nrc) ? atomicAdd(&L.hist[(kr[u + 1] >> hash_shift) & hmask], 1u) : 0u;
                    slot2[u / 2] = a | (b << 16);
                }
            };
            // a full chunk (every chunk at 2^28) without per-item exec masks
            if (nrc == (uint32_t)RCAP) ranks(std::true_type{});
            else ranks(std::false_type{});
            __syncthreads();
            {  // prefix sum on histogram (:520-524): thread tid owns buckets [tid*E, tid*E + E)
                const uint32_t E = (nh + BLOCK - 1) / BLOCK;
                uint32_t loc[NB / BLOCK];
                uint32_t sum = 0;
#pragma unroll
                for (uint32_t j = 0; j < (uint32_t)(NB / BLOCK); ++j) {
                    const uint32_t b = tid * E + j;
                    const uint32_t c = (j < E && b < nh) ? L.hist[b] : 0u;
                    loc[j] = sum;
                    sum += c;
                }
                uint64_t tot;
                const uint32_t base = (uint32_t)block_excl_scan_u64(sum, L.red, &tot);
#pragma unroll
                for (uint32_t j = 0; j < (uint32_t)(NB / BLOCK); ++j) {
                    const uint32_t b = tid * E + j;
                    if (j < E && b < nh) L.off[b] = (uint16_t)(base + loc[j]);
                }
                if (tid == 0) L.off[nh] = (uint16_t)nrc;
            }
            __syncthreads();  // hist is dead: its space takes the keys
            // the bucket addresses are recomputed here rather than kept from the histogram
            // atomics across the scan (16 more live registers: spills at 64 VGPRs)
#pragma unroll
            for (int u = 0; u < U; ++u) asm volatile("" : "+v"(kr[u]));
#pragma unroll
            for (int u = 0; u < U; ++u) {  // BUILD PHASE: re-order (:527-561)
                const uint32_t i = tid + u * BLOCK;
                if (i < nrc) {
                    const uint32_t sl = (slot2[u / 2] >> ((u & 1) * 16)) & 0xFFFFu;
                    L.keys[L.off[(kr[u] >> hash_shift) & hmask] + sl] = kr[u];
                }
            }
            __syncthreads();
            const uint64_t c_probe = wall_clock64();
            bcyc += c_probe - c_build;
            for (uint64_t s0 = 0; s0 < nS; s0 += (uint64_t)UP * BLOCK) {  // PROBE PHASE (:570-600)
                const uint32_t lim = (uint32_t)min<uint64_t>(nS - s0, (uint64_t)UP * BLOCK);
                const __amdgpu_buffer_rsrc_t rs =
                    make_rsrc(reinterpret_cast<const uint32_t *>(S) + (sb + s0) * KS, lim * 4u * KS);
                uint32_t ks[UP], j[UP], end[UP];
#pragma unroll
                for (int u = 0; u < UP; ++u)
                    ks[u] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, (int)((tid + u * BLOCK) * 4u * KS), 0, 2);
#pragma unroll
                for (int u = 0; u < UP; ++u) {
                    const uint32_t i = tid + u * BLOCK;
                    const uint32_t b = (ks[u] >> hash_shift) & hmask;
                    j[u] = i < lim ? L.off[b] : 0u;
                    end[u] = i < lim ? L.off[b + 1] : 0u;
                }
                bool more = true;
                while (more) {
                    more = false;
#pragma unroll
                    for (int u = 0; u < UP; ++u) {
                        if (j[u] < end[u]) {
                            matches += (L.keys[j[u]] == ks[u]);
                            ++j[u];
                            more |= j[u] < end[u];
                        }
                    }
                }
            }
            pcyc += wall_clock64() - c_probe;
        }
    }
    matches = wave_sum_u64(matches);
    __syncthreads();
    if (lane == 0) L.red[tid / kWave] = matches;
    __syncthreads();
    if (tid == 0) {
        uint64_t acc = 0;
        for (int w = 0; w < NW; ++w) acc += L.red[w];
        counts[blockIdx.x] = acc;
    }
    if (cyc && tid == 0) {
        cyc[2 * blockIdx.x] = bcyc;
        cyc[2 * blockIdx.x + 1] = pcyc;
    }
    if (red_ticket) join_reduce_last(counts, cyc, red_result, red_ticket, L.red, T);
}

// Multiprocessors of the current device: k_join_x runs one workgroup per CU.
uint32_t cu_count() {
    static const uint32_t n = [] {
        int dev = 0, v = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
            v = 256;
        return (uint32_t)v;
    }();
    return n;
}

// SGXAMD_JOIN_N (development A/B switch, read once): 1 (default) = narrow relations'
// build/probe in k_join_n (one task per workgroup, the table sized to the residuals);
// 0 = k_join_x's direct table (one workgroup per CU).
bool narrow_join_enabled() {
    static const bool on = [] {
        const char *e = std::getenv("SGXAMD_JOIN_N");
        return !(e && std::atoi(e) == 0);
    }();
    return on;
}

// Counting build/probe over packed keys (key-only partitions, KS = 1).
hipError_t launch_join_keys(const void *R, const void *S, const uint64_t *r_start, const uint64_t *r_count,
                            const uint64_t *s_start, const uint64_t *s_count, uint64_t P, const uint64_t *over,
                            const uint32_t *n_over, uint32_t hash_shift, uint32_t rcap, uint64_t s_chunk,
                            uint32_t grid, int mode, int algo, uint64_t *counts, uint64_t *cyc, hipStream_t s,
                            const JoinReduce *reduce, uint32_t *tickets, const uint32_t *narrow_r,
                            const uint32_t *narrow_s, uint32_t tasks_max, uint64_t *fold, uint64_t *fold_host) {
    if (mode != kJoinCount) return hipErrorInvalidValue;
    if (fold && (reduce || algo != kAlgoChaining || rcap != kBigRcap)) return hipErrorNotSupported;
    // narrow partitions are read by the 16,384-key chaining table only
    if ((narrow_r || narrow_s) && !(algo == kAlgoChaining && rcap == kBigRcap)) return hipErrorInvalidValue;
    const uint64_t *R64 = static_cast<const uint64_t *>(R);
    const uint64_t *S64 = static_cast<const uint64_t *>(S);
    uint64_t *rres = reduce ? reduce->result : nullptr;
    uint64_t *rtick = reduce ? reduce->ticket : nullptr;
    if (algo == kAlgoHistogram) {
#define HIST_KEYS_CASE(RC)                                                                                   \
    case RC:                                                                                                 \
        hipLaunchKernelGGL((k_join_hist<RC, kJoinCount, 1>), dim3(grid), dim3(kBlock), 0, s, R64, S64,      \
                           r_start, r_count, s_start, s_count, P, over, n_over, hash_shift, s_chunk, counts, \
                           nullptr, nullptr, cyc, rres, rtick);                                              \
        break;
        switch (rcap) {
            HIST_KEYS_CASE(2048)
            HIST_KEYS_CASE(4096)
            HIST_KEYS_CASE(8192)
            case kBigRcap:
                hipLaunchKernelGGL(k_join_hist_big<1>, dim3(grid), dim3(1024), 0, s, R64, S64, r_start, r_count,
                                   s_start, s_count, P, over, n_over, hash_shift, s_chunk, counts, cyc, rres, rtick);
                break;
            default:
                return hipErrorInvalidValue;
        }
#undef HIST_KEYS_CASE
        return hipGetLastError();
    }
    if (algo != kAlgoChaining) return hipErrorInvalidValue;
    if (rcap == kBigRcap) {  // one workgroup per CU (128 KiB table), strips of 8 keys per thread
        // narrow relations: k_join_n, one task per workgroup (tasks_max of them), its
        // counts and ticks added into the grid's slots (zeroed by launch_make_tasks);
        // k_join_x takes the join only when neither relation is narrow (the width is
        // known on the device only: both are launched, one returns at once)
        const bool nar = (narrow_r || narrow_s) && narrow_join_enabled();
        if (nar) {
            if (reduce) return hipErrorInvalidValue;
            hipLaunchKernelGGL((k_join_n<SGXAMD_JN_BLOCK, SGXAMD_JN_L, SGXAMD_JN_C16 != 0>),
                               dim3(std::max<uint32_t>(tasks_max, 1)), dim3(SGXAMD_JN_BLOCK), 0, s, R, S, r_start,
                               r_count, s_start, s_count, P, over, n_over, hash_shift, s_chunk, counts, cyc, grid,
                               tickets, narrow_r, narrow_s);
            const hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL((k_join_x<kBigRcap, 1024, 8, 1>), dim3(std::min<uint32_t>(grid, cu_count())), dim3(1024), 0,
                           s, R64, S64, r_start, r_count, s_start, s_count, P, over, n_over, hash_shift, s_chunk, counts,
                           cyc, rres, rtick, grid, tickets, narrow_r, narrow_s, nar ? 1u : 0u, fold, fold ? fold_host : nullptr);
        return hipGetLastError();
    }
#define KEYS_CASE(RC)                                                                                                   case RC:                                                                                                                hipLaunchKernelGGL((k_join<RC, kJoinCount, kBlock, 1>), dim3(grid), dim3(kBlock), 0, s, R64, S64, r_start,                            r_count, s_start, s_count, P, over, n_over, hash_shift, s_chunk, counts, nullptr, nullptr,                             cyc, rres, rtick);                                                                               break;
    switch (rcap) {
        KEYS_CASE(2048)
        KEYS_CASE(4096)
        KEYS_CASE(8192)
        default:
            return hipErrorInvalidValue;
    }
#undef KEYS_CASE
    return hipGetLastError();
}

hipError_t launch_join_pieces(const void *R, const uint64_t *r_start, const uint64_t *r_count, const uint16_t *s16,
                              uint64_t s_bytes, const WirePieces &w, uint64_t P, const uint64_t *over,
                              const uint32_t *n_over, uint32_t hash_shift, uint64_t s_chunk, uint32_t grid,
                              uint32_t tasks_max, uint64_t *counts, uint64_t *cyc, uint32_t *tickets,
                              const uint32_t *narrow_r, const uint32_t *narrow_s, uint64_t *fold, hipStream_t s) {
    static_assert(kPieceMaxG == kPieceMax, "one bound");
    if (w.G == 0 || w.G > kPieceMax || s_bytes > 0xFFFFFFF0ull || (s_chunk & 7) || !narrow_r || !narrow_s)
        return hipErrorInvalidValue;
    hipLaunchKernelGGL((k_join_np<SGXAMD_JN_BLOCK, SGXAMD_JN_L, SGXAMD_JN_C16 != 0>), dim3(std::max<uint32_t>(tasks_max, 1)),
                       dim3(SGXAMD_JN_BLOCK), 0, s, R, s16, (uint32_t)s_bytes, r_start, r_count, w.ub, w.nk, w.G,
                       w.units8, P, over, n_over, hash_shift, s_chunk, counts, cyc, grid, tickets, narrow_r, narrow_s);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    // the count reduction (k_join_x returns at once on narrow relations; its workgroups sum
    // the slots)
    const uint64_t *R64 = static_cast<const uint64_t *>(R);
    hipLaunchKernelGGL((k_join_x<kBigRcap, 1024, 8, 1>), dim3(std::min<uint32_t>(grid, cu_count())), dim3(1024), 0, s,
                       R64, reinterpret_cast<const uint64_t *>(s16), r_start, r_count, r_start, r_count, P, over,
                       n_over, hash_shift, s_chunk, counts, cyc, nullptr, nullptr, grid, tickets, narrow_r, narrow_s,
                       1u, fold, nullptr);
    return hipGetLastError();
}

hipError_t launch_join(const row_t *R, const row_t *S, const uint64_t *r_start, const uint64_t *r_count,
                       const uint64_t *s_start, const uint64_t *s_count, uint64_t P, const uint64_t *over,
                       const uint32_t *n_over, uint32_t hash_shift, uint32_t rcap, uint64_t s_chunk, uint32_t grid,
                       int mode, int algo, uint64_t *counts, const uint64_t *task_off, output_triple_t *out,
                       uint64_t *cyc, hipStream_t s, const JoinReduce *reduce, int key_stride, uint32_t *tickets,
                       const uint32_t *narrow_r, const uint32_t *narrow_s, uint32_t tasks_max,
                       const uint64_t *small_kmax, uint64_t *fold, uint64_t *fold_host) {
    if (key_stride == 1)
        return launch_join_keys(R, S, r_start, r_count, s_start, s_count, P, over, n_over, hash_shift, rcap, s_chunk,
                                grid, mode, algo, counts, cyc, s, reduce, tickets, narrow_r, narrow_s, tasks_max, fold,
                                fold_host);
    if (fold && (mode != kJoinCount || reduce || algo == kAlgoHistogram || rcap != kBigRcap))
        return hipErrorNotSupported;
    if (narrow_r || narrow_s) return hipErrorInvalidValue;
    const uint64_t *R64 = reinterpret_cast<const uint64_t *>(R);
    const uint64_t *S64 = reinterpret_cast<const uint64_t *>(S);
    uint64_t *rres = (reduce && mode == kJoinCount) ? reduce->result : nullptr;
    uint64_t *rtick = (reduce && mode == kJoinCount) ? reduce->ticket : nullptr;
#define JOIN_LAUNCH(K, RC, MD)                                                                             \
    hipLaunchKernelGGL((K<RC, MD>), dim3(grid), dim3(kBlock), 0, s, R64, S64, r_start, r_count, s_start,    \
                       s_count, P, over, n_over, hash_shift, s_chunk, counts, task_off, out, cyc, rres, rtick)
#define JOIN_MODES(K, RC)                                                    \
    case RC:                                                                 \
        if (mode == kJoinCount) JOIN_LAUNCH(K, RC, kJoinCount);              \
        else if (mode == kJoinTaskCount) JOIN_LAUNCH(K, RC, kJoinTaskCount); \
        else JOIN_LAUNCH(K, RC, kJoinWrite);                                 \
        break;
    if (algo == kAlgoHistogram) {
        switch (rcap) {
            JOIN_MODES(k_join_hist, 2048)
            JOIN_MODES(k_join_hist, 4096)
            JOIN_MODES(k_join_hist, 8192)
            case kBigRcap:  // the 16,384-tuple table: counting only
                if (mode != kJoinCount) return hipErrorInvalidValue;
                hipLaunchKernelGGL(k_join_hist_big<2>, dim3(grid), dim3(1024), 0, s, R64, S64, r_start, r_count,
                                   s_start, s_count, P, over, n_over, hash_shift, s_chunk, counts, cyc, rres, rtick);
                break;
            default:
                return hipErrorInvalidValue;
        }
    } else if (rcap == kBigRcap) {
        // the 16,384-tuple counting table (k_join_x: 128 KiB, one workgroup per CU;
        // plain counting only, the materialising table carries 4 B more per tuple)
        if (mode != kJoinCount) return hipErrorInvalidValue;
        hipLaunchKernelGGL((k_join_x<kBigRcap, 1024, 8, 2>), dim3(std::min<uint32_t>(grid, cu_count())), dim3(1024), 0,
                           s, R64, S64, r_start, r_count, s_start, s_count, P, over, n_over, hash_shift, s_chunk, counts,
                           cyc, rres, rtick, grid, tickets, nullptr, nullptr, 0u, fold, fold ? fold_host : nullptr);
    } else if (mode == kJoinCount && grid <= 512 && rcap <= 4096) {
        // few tasks (small joins: one workgroup per CU at most): 1,024 threads per table
        // instead of 256, so that a CU holds 16 waves to hide the load latencies
#define JOIN_WIDE(RC)                                                                                        \
    case RC:                                                                                                 \
        if (small_kmax) /* the direct table where R's residuals allow (task_off: R's largest key) */       \
            hipLaunchKernelGGL((k_join<RC, kJoinCount, 1024, 2, true>), dim3(grid), dim3(1024), 0, s, R64,    \
                               S64, r_start, r_count, s_start, s_count, P, over, n_over, hash_shift, s_chunk, \
                               counts, small_kmax, out, cyc, rres, rtick);                                    \
        else                                                                                                 \
            hipLaunchKernelGGL((k_join<RC, kJoinCount, 1024>), dim3(grid), dim3(1024), 0, s, R64, S64,        \
                               r_start, r_count, s_start, s_count, P, over, n_over, hash_shift, s_chunk,      \
                               counts, task_off, out, cyc, rres, rtick);                                      \
        break;
        switch (rcap) {
            JOIN_WIDE(2048)
            JOIN_WIDE(4096)
            default:
                return hipErrorInvalidValue;
        }
#undef JOIN_WIDE
    } else {
        switch (rcap) {
            JOIN_MODES(k_join, 2048)
            JOIN_MODES(k_join, 4096)
            JOIN_MODES(k_join, 8192)
            default:
                return hipErrorInvalidValue;
        }
    }
#undef JOIN_MODES
#undef JOIN_LAUNCH
    return hipGetLastError();
}

// Overflow tasks: the S chunks 1.. of every partition whose S side exceeds kSChunk
// (and whose R side is not empty).
__global__ __launch_bounds__(kBlock) void k_make_tasks(const uint64_t *__restrict__ r_count,
                                                       const uint64_t *__restrict__ s_count, uint64_t P,
                                                       uint64_t *__restrict__ over, uint32_t over_cap,
                                                       uint32_t *__restrict__ n_over, uint64_t *__restrict__ max_rs,
                                                       uint64_t s_chunk, uint64_t *__restrict__ zero,
                                                       uint64_t *__restrict__ zero2, uint32_t nzero) {
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < nzero; i += gridDim.x * kBlock) {
        zero[i] = 0;
        zero2[2 * i] = zero2[2 * i + 1] = 0;
    }
    uint64_t mr = 0, ms = 0;  // largest partitions (diagnostics), folded into this pass over the counts
    for (uint64_t p = blockIdx.x * (uint64_t)kBlock + threadIdx.x; p < P; p += (uint64_t)gridDim.x * kBlock) {
        const uint64_t nS = s_count[p], nR = r_count[p];
        mr = nR > mr ? nR : mr;
        ms = nS > ms ? nS : ms;
        if (nR == 0 || nS <= s_chunk) continue;
        const uint32_t k = (uint32_t)((nS + s_chunk - 1) / s_chunk) - 1;
        const uint32_t base = atomicAdd(n_over, k);
        for (uint32_t j = 0; j < k && base + j < over_cap; ++j) over[base + j] = p | ((uint64_t)(j + 1) << 32);
    }
    {  // one pair of device atomics per workgroup
        __shared__ uint64_t red[2][kWaves];
#pragma unroll
        for (int off = kWave / 2; off > 0; off >>= 1) {
            const uint64_t a = __shfl_xor(mr, off, kWave), b = __shfl_xor(ms, off, kWave);
            mr = a > mr ? a : mr;
            ms = b > ms ? b : ms;
        }
        if (__lane_id() == 0) {
            red[0][threadIdx.x / kWave] = mr;
            red[1][threadIdx.x / kWave] = ms;
        }
        __syncthreads();
        if (threadIdx.x < 2) {
            uint64_t m = 0;
            for (int w = 0; w < kWaves; ++w) m = red[threadIdx.x][w] > m ? red[threadIdx.x][w] : m;
            if (m) atomicMax((unsigned long long *)&max_rs[threadIdx.x], (unsigned long long)m);
        }
    }
}

hipError_t launch_make_tasks(const uint64_t *r_count, const uint64_t *s_count, uint64_t P, uint64_t *over,
                             uint32_t over_cap, uint64_t *meta, uint64_t s_chunk, hipStream_t s, uint64_t *zero,
                             uint64_t *zero2, uint32_t nzero, bool zeroed) {
    // meta = result + 1 of the join's 8-word, 256-byte aligned result block: the whole
    // block in one aligned fill (meta's 48 bytes alone, 8-byte aligned, took three fill
    // kernels: head, body and tail -- 13.7 us per join in the r05g trace); none when R's
    // pass-1 layout zeroed it (round 6, PoolOut::zero8)
    if (!zeroed) {
        hipError_t e = hipMemsetAsync(meta - 1, 0, 8 * sizeof(uint64_t), s);
        if (e != hipSuccess) return e;
    }
    uint32_t *n_over = reinterpret_cast<uint32_t *>(meta + 2);
    uint64_t blocks = (P + kBlock - 1) / kBlock;
    if (blocks > 1024) blocks = 1024;
    hipLaunchKernelGGL(k_make_tasks, dim3((uint32_t)blocks), dim3(kBlock), 0, s, r_count, s_count, P, over, over_cap,
                       n_over, meta, s_chunk, zero, zero2, zero && zero2 ? nzero : 0u);
    return hipGetLastError();
}

// One block: exclusive scan of n u64 values (task counts -> output offsets), total in *total.
__global__ __launch_bounds__(1024) void k_excl_scan(const uint64_t *__restrict__ in, const uint32_t *__restrict__ n_extra,
                                                    uint64_t n_base, uint64_t *__restrict__ out,
                                                    uint64_t *__restrict__ total) {
    __shared__ uint64_t scratch[1024 / kWave + 1];
    const uint64_t n = n_base + (n_extra ? *n_extra : 0);
    uint64_t carry = 0;
    for (uint64_t b = 0; b < n; b += 1024) {
        const uint64_t i = b + threadIdx.x;
        const uint64_t v = i < n ? in[i] : 0;
        uint64_t tot;
        const uint64_t ex = block_excl_scan_u64(v, scratch, &tot);
        if (i < n) out[i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) *total = carry;
}

// Tests: one thread holding a stream for a while (multi_host.cpp's exchange delay,
// SGXAMD_DEBUG_EXCHANGE_DELAY_US, so that a consumer missing its wait reads early).
__global__ void k_spin(uint64_t ticks) {
    const uint64_t t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(16);
}

hipError_t launch_spin(uint32_t us, hipStream_t s) {
    int dev = 0, khz = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0)
        khz = 100000;
    hipLaunchKernelGGL(k_spin, dim3(1), dim3(1), 0, s, (uint64_t)us * (uint64_t)khz / 1000);
    return hipGetLastError();
}

hipError_t launch_excl_scan(const uint64_t *in, const uint32_t *n_extra, uint64_t n_base, uint64_t *out,
                            uint64_t *total, hipStream_t s) {
    hipLaunchKernelGGL(k_excl_scan, dim3(1), dim3(1024), 0, s, in, n_extra, n_base, out, total);
    return hipGetLastError();
}

// ---------------------------------------------------------------- reduce ---
// out[0] = sum of the n partial counts (skipped when v is null); with cyc: out[4] /
// out[5] = the build / probe ticks summed over the ncyc join workgroups.
__global__ __launch_bounds__(kBlock) void k_reduce(const uint64_t *__restrict__ v, uint32_t n,
                                                   uint64_t *__restrict__ out, const uint64_t *__restrict__ cyc,
                                                   uint32_t ncyc) {
    __shared__ uint64_t red[3][kWaves];
    uint64_t acc = 0, b = 0, p = 0;
    if (v)
        for (uint32_t i = threadIdx.x; i < n; i += kBlock) acc += v[i];
    if (cyc)
        for (uint32_t i = threadIdx.x; i < ncyc; i += kBlock) {
            b += cyc[2 * i];
            p += cyc[2 * i + 1];
        }
    acc = wave_sum_u64(acc);
    b = wave_sum_u64(b);
    p = wave_sum_u64(p);
    if (__lane_id() == 0) {
        red[0][threadIdx.x / kWave] = acc;
        red[1][threadIdx.x / kWave] = b;
        red[2][threadIdx.x / kWave] = p;
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        uint64_t t = 0;
        for (int w = 0; w < kWaves; ++w) t += red[threadIdx.x][w];
        if (threadIdx.x == 0 && v) out[0] = t;
        if (threadIdx.x > 0 && cyc) out[3 + threadIdx.x] = t;
    }
}

hipError_t launch_reduce(const uint64_t *partials, uint32_t n, uint64_t *result, const uint64_t *cyc, uint32_t ncyc,
                         hipStream_t s) {
    hipLaunchKernelGGL(k_reduce, dim3(1), dim3(kBlock), 0, s, partials, n, result, cyc, ncyc);
    return hipGetLastError();
}

}  // namespace rho
}  // namespace sgxamd
