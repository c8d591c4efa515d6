// HIP kernels of the MI355X radix hash join (gfx950 / CDNA4, wave64).
//
// The reference's CPU hot loops and what replaces them here:
//   partition_hist[_unrolled]   radix_join.cpp:617-654  -> k_hist
//   local/global prefix         radix_join.cpp:886-915  -> k_scan_cols / k_scan_digits / k_scan_regions
//   partition_copy[_unrolled]   radix_join.cpp:659-697  -> k_scatter (stable LDS multisplit, the
//                               GPU analogue of the SWWC variant at :961-1056)
//   bucket_chaining_join        radix_join.cpp:359-458  -> k_join (LDS linear-probing table per
//                               partition, S streamed, one partial count per workgroup)
// Radix digits are taken as (key >> shift) & (F - 1) with the pass-1 digit in the
// low bits, exactly like HASH_BIT_MODULO(key, MASK, R) (:47) with R = shift.
// All work is integer; HBM bandwidth is the roofline.
#include "common.hpp"
#include "rho_internal.hpp"

namespace sgxamd {
namespace rho {

constexpr int kWaves = kBlock / kWave;

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
__global__ __launch_bounds__(kBlock) void k_hist(const uint32_t *__restrict__ in_words, SegMap m, uint32_t shift,
                                                 uint32_t bits, uint64_t *__restrict__ hist, HistLayout layout,
                                                 uint32_t nseg_stride) {
    __shared__ uint32_t h[kMaxF];
    __shared__ uint32_t sbase[kMaxF + 1];
    const uint32_t g = blockIdx.x;
    uint32_t r;
    uint64_t b, e;
    if (!seg_lookup(m, g, sbase, r, b, e)) return;
    const uint32_t F = 1u << bits, mask = F - 1;
    for (uint32_t d = threadIdx.x; d < F; d += kBlock) h[d] = 0;
    __syncthreads();
    constexpr int U = 8;
    uint64_t i = b + threadIdx.x;
    for (; i + (U - 1) * kBlock < e; i += U * kBlock) {
        uint32_t k[U];
#pragma unroll
        for (int u = 0; u < U; ++u) k[u] = in_words[2 * (i + u * kBlock)];
#pragma unroll
        for (int u = 0; u < U; ++u) atomicAdd(&h[(k[u] >> shift) & mask], 1u);
    }
    for (; i < e; i += kBlock) atomicAdd(&h[(in_words[2 * i] >> shift) & mask], 1u);
    __syncthreads();
    for (uint32_t d = threadIdx.x; d < F; d += kBlock) hist[hist_index(layout, g, d, F, nseg_stride)] = h[d];
}

hipError_t launch_hist(const row_t *in, const SegMap &m, uint32_t grid, uint32_t shift, uint32_t bits,
                       uint64_t *hist, HistLayout layout, uint32_t nseg_stride, hipStream_t s) {
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL(k_hist, dim3(grid), dim3(kBlock), 0, s, reinterpret_cast<const uint32_t *>(in), m, shift,
                       bits, hist, layout, nseg_stride);
    return hipGetLastError();
}

// ------------------------------------------------------------------ scans ---
// One block per digit column: exclusive prefix over the segments (in place).
__global__ __launch_bounds__(kBlock) void k_scan_cols(uint64_t *__restrict__ hist, uint32_t nseg,
                                                      uint64_t *__restrict__ totals) {
    __shared__ uint64_t scratch[kWaves + 1];
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

// One block per region, one thread per digit: cursors for [g][d] and the partition table.
__global__ __launch_bounds__(kMaxF) void k_scan_regions(uint64_t *__restrict__ hist,
                                                        const uint32_t *__restrict__ seg_base,
                                                        const uint64_t *__restrict__ reg_start, uint32_t F,
                                                        uint64_t *__restrict__ part_start,
                                                        uint64_t *__restrict__ part_count) {
    __shared__ uint64_t scratch[kMaxF / kWave + 1];
    const uint32_t r = blockIdx.x, d = threadIdx.x;
    const uint32_t sb = seg_base[r], se = seg_base[r + 1];
    uint64_t run = 0;
    if (d < F) {
        for (uint32_t g = sb; g < se; ++g) {
            const uint64_t c = hist[(uint64_t)g * F + d];
            hist[(uint64_t)g * F + d] = run;
            run += c;
        }
    }
    uint64_t tot;
    const uint64_t ex = block_excl_scan_u64(d < F ? run : 0, scratch, &tot);
    if (d < F) {
        const uint64_t start = reg_start[r] + ex;
        for (uint32_t g = sb; g < se; ++g) hist[(uint64_t)g * F + d] += start;
        part_start[(uint64_t)r * F + d] = start;
        part_count[(uint64_t)r * F + d] = run;
    }
}

hipError_t launch_scan_regions(uint64_t *hist, const uint32_t *seg_base, const uint64_t *reg_start, uint32_t nreg,
                               uint32_t bits, uint64_t *part_start, uint64_t *part_count, hipStream_t s) {
    const uint32_t F = 1u << bits;
    const uint32_t threads = F < 64 ? 64 : F;
    hipLaunchKernelGGL(k_scan_regions, dim3(nreg), dim3(threads), 0, s, hist, seg_base, reg_start, F, part_start,
                       part_count);
    return hipGetLastError();
}

// --------------------------------------------------------------- scatter ---
// Stable multisplit of tiles of kTile tuples.  Wave w owns tile rows
// [w*64*ITEMS, (w+1)*64*ITEMS); item k of lane l is row w*64*ITEMS + k*64 + l, so
// (wave, item, lane) order is input order.  Equal-digit peers in a wave are found
// with one ballot per digit bit; per-wave LDS counters give stable ranks; the tile
// is reordered by digit in LDS and written as contiguous per-digit runs that
// continue where the previous tile of this workgroup stopped.
template <int ITEMS>
__global__ __launch_bounds__(kBlock) void k_scatter(const uint64_t *__restrict__ in, uint64_t *__restrict__ out,
                                                    SegMap m, uint32_t shift, uint32_t bits,
                                                    const uint64_t *__restrict__ cur_init, HistLayout layout,
                                                    uint32_t nseg_stride, const uint64_t *__restrict__ digit_base) {
    constexpr int TILE = kBlock * ITEMS;
    __shared__ uint32_t sbase[kMaxF + 1];
    __shared__ uint32_t wcnt[kWaves][kMaxF];
    __shared__ uint32_t tcnt[kMaxF];
    __shared__ uint32_t toff[kMaxF];
    __shared__ uint64_t cursor[kMaxF];
    __shared__ uint64_t scratch[kWaves + 1];
    __shared__ uint64_t stage[TILE];

    const uint32_t g = blockIdx.x;
    uint32_t r;
    uint64_t b, e;
    if (!seg_lookup(m, g, sbase, r, b, e)) return;
    const uint32_t F = 1u << bits, mask = F - 1;
    const uint32_t tid = threadIdx.x, lane = __lane_id(), wave = tid / kWave;
    for (uint32_t d = tid; d < F; d += kBlock)
        cursor[d] = cur_init[hist_index(layout, g, d, F, nseg_stride)] +
                    (digit_base ? digit_base[(uint64_t)r * F + d] : 0);

    const uint64_t lt = lanemask_lt();
    for (uint64_t tb = b; tb < e; tb += TILE) {
        const uint32_t tn = (uint32_t)((e - tb) < (uint64_t)TILE ? (e - tb) : (uint64_t)TILE);
        for (uint32_t i = tid; i < kWaves * F; i += kBlock) (&wcnt[0][0])[(i / F) * kMaxF + (i % F)] = 0;
        uint64_t v[ITEMS];
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            const uint32_t li = wave * kWave * ITEMS + k * kWave + lane;
            v[k] = li < tn ? in[tb + li] : 0ull;
        }
        __syncthreads();
        uint32_t dig[ITEMS], rank[ITEMS];
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            const uint32_t li = wave * kWave * ITEMS + k * kWave + lane;
            const bool valid = li < tn;
            const uint32_t d = valid ? (((uint32_t)v[k] >> shift) & mask) : 0u;
            uint64_t peers = __ballot(valid);
            for (uint32_t bit = 0; bit < bits; ++bit) {
                const bool set = (d >> bit) & 1u;
                const uint64_t bb = __ballot(set);
                peers &= set ? bb : ~bb;
            }
            uint32_t rk = 0;
            if (valid) {
                const uint32_t old = wcnt[wave][d];
                const uint64_t below = peers & lt;
                rk = old + popc64(below);
                if (below == 0) wcnt[wave][d] = old + popc64(peers);
            }
            dig[k] = d;
            rank[k] = rk;
        }
        __syncthreads();
        // per digit: exclusive prefix across waves (in place) and the tile count
        for (uint32_t d = tid; d < F; d += kBlock) {
            uint32_t acc = 0;
#pragma unroll
            for (int w = 0; w < kWaves; ++w) {
                const uint32_t t = wcnt[w][d];
                wcnt[w][d] = acc;
                acc += t;
            }
            tcnt[d] = acc;
        }
        __syncthreads();
        // exclusive scan over digits (F <= 2 * kBlock): two digits per thread
        {
            const uint32_t d0 = 2 * tid, d1 = 2 * tid + 1;
            const uint32_t c0 = d0 < F ? tcnt[d0] : 0u, c1 = d1 < F ? tcnt[d1] : 0u;
            uint64_t tot;
            const uint64_t ex = block_excl_scan_u64((uint64_t)c0 + c1, scratch, &tot);
            if (d0 < F) toff[d0] = (uint32_t)ex;
            if (d1 < F) toff[d1] = (uint32_t)ex + c0;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            const uint32_t li = wave * kWave * ITEMS + k * kWave + lane;
            if (li < tn) stage[toff[dig[k]] + wcnt[wave][dig[k]] + rank[k]] = v[k];
        }
        __syncthreads();
        for (uint32_t i = tid; i < tn; i += kBlock) {
            const uint64_t x = stage[i];
            const uint32_t d = ((uint32_t)x >> shift) & mask;
            out[cursor[d] + (i - toff[d])] = x;
        }
        __syncthreads();
        for (uint32_t d = tid; d < F; d += kBlock) cursor[d] += tcnt[d];
        __syncthreads();
    }
}

hipError_t launch_scatter(const row_t *in, row_t *out, const SegMap &m, uint32_t grid, uint32_t shift,
                          uint32_t bits, const uint64_t *cursors, HistLayout layout, uint32_t nseg_stride,
                          const uint64_t *digit_base, hipStream_t s) {
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL(k_scatter<kScatterItems>, dim3(grid), dim3(kBlock), 0, s,
                       reinterpret_cast<const uint64_t *>(in), reinterpret_cast<uint64_t *>(out), m, shift, bits,
                       cursors, layout, nseg_stride, digit_base);
    return hipGetLastError();
}

// ------------------------------------------------------------ build+probe ---
// One partition per loop iteration.  R keys go into an LDS linear-probing table of
// T = nextpow2(2 |R_chunk|) slots (load factor <= 1/2); R chunks larger than
// TMAX / 2 are built one after another and S is re-probed per chunk.  Duplicate R
// keys occupy separate slots, so a probe counts every equal key in its cluster,
// which is what walking the reference's bucket chain does (:429-436).  The slot
// of a key is its bits above the radix bits, HASH_BIT_MODULO(key, (N-1)<<bits, bits)
// of bucket_chaining_join (:378,:388).  A key equal to the empty marker is counted
// on the side.
template <int TMAX>
__global__ __launch_bounds__(kBlock) void k_join(const uint32_t *__restrict__ Rw, const uint32_t *__restrict__ Sw,
                                                 const uint64_t *__restrict__ r_start,
                                                 const uint64_t *__restrict__ r_count,
                                                 const uint64_t *__restrict__ s_start,
                                                 const uint64_t *__restrict__ s_count, uint64_t P,
                                                 uint32_t hash_shift, uint64_t *__restrict__ partials) {
    __shared__ __attribute__((aligned(16))) uint32_t table[TMAX];
    __shared__ uint32_t s_empty;
    __shared__ uint64_t red[kWaves];
    constexpr uint32_t RCAP = TMAX / 2;
    constexpr int U = 4;
    const uint32_t tid = threadIdx.x;
    uint64_t matches = 0;
    for (uint64_t p = blockIdx.x; p < P; p += gridDim.x) {
        const uint64_t nR = r_count[p], nS = s_count[p];
        if (nR == 0 || nS == 0) continue;
        const uint64_t rb = r_start[p], sb = s_start[p];
        for (uint64_t rc = 0; rc < nR; rc += RCAP) {
            const uint32_t nrc = (uint32_t)((nR - rc) < RCAP ? (nR - rc) : RCAP);
            uint32_t T = 64;
            while (T < 2 * nrc) T <<= 1;
            const uint32_t tmask = T - 1;
            for (uint32_t i = tid; i < T / 4; i += kBlock)
                reinterpret_cast<uint4 *>(table)[i] = make_uint4(kEmptyKey, kEmptyKey, kEmptyKey, kEmptyKey);
            if (tid == 0) s_empty = 0;
            __syncthreads();
            // build
            const uint32_t *rk = Rw + 2 * (rb + rc);
            for (uint32_t i = tid; i < nrc; i += kBlock) {
                const uint32_t k = rk[2 * i];
                if (k == kEmptyKey) {
                    atomicAdd(&s_empty, 1u);
                    continue;
                }
                uint32_t h = (k >> hash_shift) & tmask;
                while (atomicCAS(&table[h], kEmptyKey, k) != kEmptyKey) h = (h + 1) & tmask;
            }
            __syncthreads();
            const uint32_t n_empty = s_empty;
            // probe
            const uint32_t *sk = Sw + 2 * sb;
            uint64_t i = tid;
            for (; i + (U - 1) * kBlock < nS; i += U * kBlock) {
                uint32_t k[U];
#pragma unroll
                for (int u = 0; u < U; ++u) k[u] = sk[2 * (i + u * kBlock)];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    if (k[u] == kEmptyKey) {
                        matches += n_empty;
                        continue;
                    }
                    uint32_t h = (k[u] >> hash_shift) & tmask;
                    uint32_t t;
                    while ((t = table[h]) != kEmptyKey) {
                        matches += (t == k[u]);
                        h = (h + 1) & tmask;
                    }
                }
            }
            for (; i < nS; i += kBlock) {
                const uint32_t k = sk[2 * i];
                if (k == kEmptyKey) {
                    matches += n_empty;
                    continue;
                }
                uint32_t h = (k >> hash_shift) & tmask;
                uint32_t t;
                while ((t = table[h]) != kEmptyKey) {
                    matches += (t == k);
                    h = (h + 1) & tmask;
                }
            }
            __syncthreads();
        }
    }
    matches = wave_sum_u64(matches);
    if (__lane_id() == 0) red[tid / kWave] = matches;
    __syncthreads();
    if (tid == 0) {
        uint64_t acc = 0;
        for (int w = 0; w < kWaves; ++w) acc += red[w];
        partials[blockIdx.x] = acc;
    }
}

hipError_t launch_join(const row_t *R, const row_t *S, const uint64_t *r_start, const uint64_t *r_count,
                       const uint64_t *s_start, const uint64_t *s_count, uint64_t P, uint32_t hash_shift,
                       uint32_t table_slots, uint32_t grid, uint64_t *partials, hipStream_t s) {
    const uint32_t *Rw = reinterpret_cast<const uint32_t *>(R);
    const uint32_t *Sw = reinterpret_cast<const uint32_t *>(S);
    switch (table_slots) {
        case 4096:
            hipLaunchKernelGGL(k_join<4096>, dim3(grid), dim3(kBlock), 0, s, Rw, Sw, r_start, r_count, s_start,
                               s_count, P, hash_shift, partials);
            break;
        case 8192:
            hipLaunchKernelGGL(k_join<8192>, dim3(grid), dim3(kBlock), 0, s, Rw, Sw, r_start, r_count, s_start,
                               s_count, P, hash_shift, partials);
            break;
        case 16384:
            hipLaunchKernelGGL(k_join<16384>, dim3(grid), dim3(kBlock), 0, s, Rw, Sw, r_start, r_count, s_start,
                               s_count, P, hash_shift, partials);
            break;
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------- reduce ---
__global__ __launch_bounds__(kBlock) void k_reduce(const uint64_t *__restrict__ v, uint32_t n,
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

hipError_t launch_reduce(const uint64_t *partials, uint32_t n, uint64_t *result, hipStream_t s) {
    hipLaunchKernelGGL(k_reduce, dim3(1), dim3(kBlock), 0, s, partials, n, result);
    return hipGetLastError();
}

__global__ __launch_bounds__(kBlock) void k_max(const uint64_t *__restrict__ v, uint64_t n,
                                                uint64_t *__restrict__ out) {
    __shared__ uint64_t red[kWaves];
    uint64_t acc = 0;
    for (uint64_t i = threadIdx.x; i < n; i += kBlock) acc = v[i] > acc ? v[i] : acc;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t t = __shfl_xor(acc, off, kWave);
        acc = t > acc ? t : acc;
    }
    if (__lane_id() == 0) red[threadIdx.x / kWave] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = 0;
        for (int w = 0; w < kWaves; ++w) t = red[w] > t ? red[w] : t;
        *out = t;
    }
}

hipError_t launch_max(const uint64_t *v, uint64_t n, uint64_t *result, hipStream_t s) {
    hipLaunchKernelGGL(k_max, dim3(1), dim3(kBlock), 0, s, v, n, result);
    return hipGetLastError();
}

}  // namespace rho
}  // namespace sgxamd
