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
// Partition copy of one segment per workgroup (partition_copy, radix_join.cpp:659-697),
// organised like the reference's software write-combining variant
// parallel_radix_partition_optimized (:961-1056): every digit keeps its unfinished
// output segment (SEGT tuples, 128 B) and only whole, aligned segments go to HBM.
// Thread d owns digit d: its pending carry (< SEGT tuples) and its write cursor
// live in that thread's registers, not in LDS.  Per tile of NT * ITEMS tuples:
//   1. each tuple takes a slot of its digit with one LDS atomic (tile histogram and
//      in-tile rank at once; order inside a digit is arrival order, the join count
//      does not depend on it);
//   2. per digit: pending = carried tuples + this tile's tuples; the prefix that ends
//      on a segment boundary is written, the rest (< SEGT tuples) is carried on;
//   3. tuples are placed in LDS as [all written tuples, digit-major | new carries]
//      and the written block goes out with consecutive lanes on consecutive addresses.
// The next tile's tuples are already loading while a tile is processed (two
// register sets).  The last carries of the segment are flushed at the end.
template <int BITS, int ITEMS, int NT, int SEGT>
struct ScatterLds {
    static constexpr uint32_t F = 1u << BITS;
    static constexpr uint32_t TILE = NT * ITEMS;
    static constexpr uint32_t NW = NT / kWave;
    uint32_t cnt[F];     // tile count -> sequence position of the tile's first tuple of d
    uint32_t cbase[F];   // stage index of sequence position 0 of d in the carry block (minus wcount)
    uint32_t wbase[F];   // stage index of sequence position 0 of d in the write block
    uint32_t wcount[F];  // tuples of d written this tile
    uint64_t ob[F];      // output base of d: global position = ob[d] + stage index
    uint32_t wtot[NW][2];
    union {
        uint32_t sbase[kMaxF + 1];  // segment table (only before the first tile)
        uint64_t stage[TILE + (SEGT - 1) * F];
    };
};

template <int ITEMS, int NT>
__device__ __forceinline__ void load_tile(const uint64_t *__restrict__ in, uint64_t tb, uint64_t e,
                                          uint64_t (&dst)[ITEMS]) {
    constexpr uint32_t TILE = NT * ITEMS;
    if (tb + TILE <= e) {
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) dst[k] = __builtin_nontemporal_load(in + tb + threadIdx.x + k * NT);
    } else {
        const uint32_t tn = (uint32_t)(e - tb);
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            const uint32_t li = threadIdx.x + k * NT;
            dst[k] = li < tn ? in[tb + li] : 0ull;
        }
    }
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

// Per-digit state held in the registers of the digit's owner thread.
template <int SEGT>
struct DigitState {
    uint64_t pend;           // global position of the first pending tuple
    uint32_t c;              // carried tuples
    uint64_t carry[SEGT - 1];
};

template <int BITS, int ITEMS, int NT, int SEGT>
__device__ __forceinline__ void scatter_tile(ScatterLds<BITS, ITEMS, NT, SEGT> &L, DigitState<SEGT> &ds,
                                             const uint64_t (&v)[ITEMS], uint64_t *__restrict__ out, uint32_t tn,
                                             uint32_t shift) {
    constexpr uint32_t F = 1u << BITS, mask = F - 1;
    const uint32_t tid = threadIdx.x;
    const bool owner = tid < F;  // thread tid owns digit tid
    // 1. slot of every tuple inside its digit
    uint32_t slot[ITEMS];
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        if (tid + k * NT < tn) slot[k] = atomicAdd(&L.cnt[((uint32_t)v[k] >> shift) & mask], 1u);
    }
    __syncthreads();
    // 2. per digit: what is written now, what is carried on
    uint32_t w = 0, r = 0, c = 0;
    if (owner) {
        const uint32_t t = L.cnt[tid];
        c = ds.c;
        const uint64_t end = ds.pend + c + t;
        const uint64_t aligned = end & ~uint64_t(SEGT - 1);
        w = aligned > ds.pend ? (uint32_t)(aligned - ds.pend) : 0u;
        r = c + t - w;
    }
    uint32_t we, re, W, R;
    block_scan2(w, r, L.wtot, we, re, W, R);
    if (owner) {
        L.wbase[tid] = we;
        L.cbase[tid] = W + re - w;
        L.wcount[tid] = w;
        L.ob[tid] = ds.pend - we;
        L.cnt[tid] = c;  // sequence position of the tile's first tuple
        // old carries open the digit's sequence
#pragma unroll
        for (int s = 0; s < SEGT - 1; ++s)
            if ((uint32_t)s < c) L.stage[(uint32_t)s < w ? we + s : W + re - w + s] = ds.carry[s];
        ds.pend += w;
        ds.c = r;
    }
    __syncthreads();
    // 3. place the tile's tuples behind the carries
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        if (tid + k * NT < tn) {
            const uint32_t d = ((uint32_t)v[k] >> shift) & mask;
            const uint32_t s = L.cnt[d] + slot[k];
            L.stage[s < L.wcount[d] ? L.wbase[d] + s : L.cbase[d] + s] = v[k];
        }
    }
    __syncthreads();
    // 4. write whole segments; collect the new carries; reset the counters
    for (uint32_t i = tid; i < W; i += NT) {
        const uint64_t x = L.stage[i];
        out[L.ob[((uint32_t)x >> shift) & mask] + i] = x;
    }
    if (owner) {
#pragma unroll
        for (int s = 0; s < SEGT - 1; ++s)
            if ((uint32_t)s < r) ds.carry[s] = L.stage[W + re + s];
        L.cnt[tid] = 0;
    }
    __syncthreads();
}

template <int BITS, int ITEMS, int NT, int SEGT>
__global__ __launch_bounds__(NT) void k_scatter(const uint64_t *__restrict__ in, uint64_t *__restrict__ out,
                                                SegMap m, uint32_t shift, const uint64_t *__restrict__ cur_init,
                                                HistLayout layout, uint32_t nseg_stride,
                                                const uint64_t *__restrict__ digit_base) {
    constexpr uint32_t TILE = NT * ITEMS;
    constexpr uint32_t F = 1u << BITS;
    static_assert(F <= NT, "one owner thread per digit");
    __shared__ ScatterLds<BITS, ITEMS, NT, SEGT> L;
    const uint32_t g = blockIdx.x;
    uint32_t r;
    uint64_t b, e;
    if (!seg_lookup(m, g, L.sbase, r, b, e)) return;
    DigitState<SEGT> ds;
    ds.c = 0;
    ds.pend = 0;
    const uint32_t tid = threadIdx.x;
    if (tid < F) {
        ds.pend = cur_init[hist_index(layout, g, tid, F, nseg_stride)] +
                  (digit_base ? digit_base[(uint64_t)r * F + tid] : 0);
        L.cnt[tid] = 0;
    }
    __syncthreads();  // sbase (aliased with stage) is dead from here on
    uint64_t va[ITEMS], vb[ITEMS];
    load_tile<ITEMS, NT>(in, b, e, va);
    for (uint64_t tb = b; tb < e; tb += 2 * TILE) {
        if (tb + TILE < e) load_tile<ITEMS, NT>(in, tb + TILE, e, vb);
        scatter_tile<BITS, ITEMS, NT, SEGT>(L, ds, va, out, (uint32_t)min<uint64_t>(TILE, e - tb), shift);
        if (tb + TILE >= e) break;
        const uint64_t t2 = tb + TILE;
        if (t2 + TILE < e) load_tile<ITEMS, NT>(in, t2 + TILE, e, va);
        scatter_tile<BITS, ITEMS, NT, SEGT>(L, ds, vb, out, (uint32_t)min<uint64_t>(TILE, e - t2), shift);
    }
    // flush the carried (partial) segments
    if (tid < F) {
#pragma unroll
        for (int s = 0; s < SEGT - 1; ++s)
            if ((uint32_t)s < ds.c) out[ds.pend + s] = ds.carry[s];
    }
}

template <int ITEMS, int NT, int SEGT>
hipError_t launch_scatter_items(const uint64_t *in, uint64_t *out, const SegMap &m, uint32_t grid, uint32_t shift,
                                uint32_t bits, const uint64_t *cursors, HistLayout layout, uint32_t nseg_stride,
                                const uint64_t *digit_base, hipStream_t s) {
#define SCATTER_CASE(B)                                                                                    \
    case B:                                                                                                \
        if constexpr (sizeof(ScatterLds<B, ITEMS, NT, SEGT>) <= 160 * 1024 && (1 << B) <= NT) {             \
            hipLaunchKernelGGL((k_scatter<B, ITEMS, NT, SEGT>), dim3(grid), dim3(NT), 0, s, in, out, m, shift, \
                               cursors, layout, nseg_stride, digit_base);                                  \
            break;                                                                                         \
        } else {                                                                                           \
            return hipErrorInvalidValue;                                                                   \
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
                          const uint64_t *digit_base, hipStream_t s) {
    if (grid == 0) return hipSuccess;
    const uint64_t *i64 = reinterpret_cast<const uint64_t *>(in);
    uint64_t *o64 = reinterpret_cast<uint64_t *>(out);
    if (bits > 8)  // 512 digit owners: 512-thread workgroups with the same tile size, 64-B granules (LDS)
        return launch_scatter_items<kTile / 512, 512, 8>(i64, o64, m, grid, shift, bits, cursors, layout,
                                                         nseg_stride, digit_base, s);
    return launch_scatter_items<kScatterItems, kScatterThreads, kScatterSegTuples>(
        i64, o64, m, grid, shift, bits, cursors, layout, nseg_stride, digit_base, s);
}

// ------------------------------------------------------------ build+probe ---
// bucket_chaining_join (radix_join.cpp:359-458) per partition, in LDS.  For an R
// chunk of nrc <= RCAP tuples: N = nextpow2(nrc) bucket heads, bucket of a key =
// HASH_BIT_MODULO(key, (N-1) << bits, bits) = (key >> bits) & (N-1) exactly as
// the reference (:374-378, :388); keys[] and 16-bit next[] hold the chains with
// 1-based positions (:393 "we start pos's from 1").  The build links tuple i with
// one LDS atomic exchange on its bucket head (chain order differs from the
// reference's serial build; the count does not).  The probe walks every chain and
// counts key equality (:429-436).  Each thread handles U = RCAP / kBlock tuples at
// a time; their chain walks advance in lockstep so the LDS reads of independent
// tuples overlap.  Partitions whose R side exceeds RCAP are built chunk by chunk
// with S re-probed per chunk.  One partial count per workgroup.
template <int RCAP>
__global__ __launch_bounds__(kBlock) void k_join(const uint32_t *__restrict__ Rw, const uint32_t *__restrict__ Sw,
                                                 const uint64_t *__restrict__ r_start,
                                                 const uint64_t *__restrict__ r_count,
                                                 const uint64_t *__restrict__ s_start,
                                                 const uint64_t *__restrict__ s_count, uint64_t P,
                                                 uint32_t hash_shift, uint64_t *__restrict__ partials) {
    constexpr int U = RCAP / kBlock;
    __shared__ __attribute__((aligned(16))) uint32_t head[RCAP];
    __shared__ uint32_t keys[RCAP];
    __shared__ uint16_t next[RCAP];
    uint64_t *red = reinterpret_cast<uint64_t *>(head);  // reused after the last table (keeps LDS = 10 * RCAP)
    const uint32_t tid = threadIdx.x;
    uint64_t matches = 0;
    for (uint64_t p = blockIdx.x; p < P; p += gridDim.x) {
        const uint64_t nR = r_count[p], nS = s_count[p];
        if (nR == 0 || nS == 0) continue;
        const uint64_t rb = r_start[p], sb = s_start[p];
        for (uint64_t rc = 0; rc < nR; rc += RCAP) {
            const uint32_t nrc = (uint32_t)((nR - rc) < RCAP ? (nR - rc) : RCAP);
            uint32_t N = 1;
            while (N < nrc) N <<= 1;  // NEXT_POW_2(numR)
            const uint32_t hmask = N - 1;
            const uint32_t *rk = Rw + 2 * (rb + rc);
            uint32_t kr[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t i = tid + u * kBlock;
                kr[u] = i < nrc ? rk[2 * i] : 0u;
            }
            for (uint32_t i = tid; i < (N + 3) / 4; i += kBlock)
                reinterpret_cast<uint4 *>(head)[i] = make_uint4(0, 0, 0, 0);
            __syncthreads();
#pragma unroll
            for (int u = 0; u < U; ++u) {  // BUILD-LOOP (:407-411)
                const uint32_t i = tid + u * kBlock;
                if (i < nrc) {
                    keys[i] = kr[u];
                    const uint32_t prev = atomicExch(&head[(kr[u] >> hash_shift) & hmask], i + 1);
                    next[i] = (uint16_t)prev;
                }
            }
            __syncthreads();
            const uint32_t *sk = Sw + 2 * sb;
            for (uint64_t s0 = 0; s0 < nS; s0 += RCAP) {  // PROBE-LOOP (:429-436)
                uint32_t ks[U], cur[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint64_t i = s0 + tid + u * kBlock;
                    ks[u] = i < nS ? sk[2 * i] : 0u;
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint64_t i = s0 + tid + u * kBlock;
                    cur[u] = i < nS ? head[(ks[u] >> hash_shift) & hmask] : 0u;
                }
                bool more = true;
                while (more) {
                    more = false;
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        if (cur[u]) {
                            const uint32_t e = cur[u] - 1;
                            matches += (keys[e] == ks[u]);
                            cur[u] = next[e];
                            more |= cur[u] != 0;
                        }
                    }
                }
            }
            __syncthreads();
        }
    }
    matches = wave_sum_u64(matches);
    __syncthreads();
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
                       uint32_t rcap, uint32_t grid, uint64_t *partials, hipStream_t s) {
    const uint32_t *Rw = reinterpret_cast<const uint32_t *>(R);
    const uint32_t *Sw = reinterpret_cast<const uint32_t *>(S);
    switch (rcap) {
        case 2048:
            hipLaunchKernelGGL(k_join<2048>, dim3(grid), dim3(kBlock), 0, s, Rw, Sw, r_start, r_count, s_start,
                               s_count, P, hash_shift, partials);
            break;
        case 4096:
            hipLaunchKernelGGL(k_join<4096>, dim3(grid), dim3(kBlock), 0, s, Rw, Sw, r_start, r_count, s_start,
                               s_count, P, hash_shift, partials);
            break;
        case 8192:
            hipLaunchKernelGGL(k_join<8192>, dim3(grid), dim3(kBlock), 0, s, Rw, Sw, r_start, r_count, s_start,
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
