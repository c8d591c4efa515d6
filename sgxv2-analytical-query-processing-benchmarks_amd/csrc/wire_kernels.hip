// Multi-GPU exchange with 2-byte residuals on the wire (multi_host.cpp "u16 wire",
// DESIGN.md §5): the receiver's side.  Every sender partitioned the keys it sends this
// rank with this rank's plan (the local join's two passes over key bits [key_shift,
// key_shift + bits), pass 2 writing narrow residuals) and sent them grouped by
// partition, followed by its P partition counts and its largest key.  A partition's G
// pieces (one per sender) are gathered here into one contiguous partition, the layout
// the build/probe reads (part_start / part_count).  The reference fills its shared
// partition arrays the same way: every thread's slice lands at offsets from a
// cross-thread prefix sum over the slices' histograms (radix_join.cpp:897-915).
#include "common.hpp"
#include "rho_internal.hpp"

namespace sgxamd {
namespace rho {

namespace {

constexpr uint32_t kWireTile = 1024;  // partitions per tile (one thread each)
constexpr uint32_t kGatherBlock = 256;

// Scratch (u64 words from `w`): src [G][P] (a piece's offset inside its tile of its
// sender's run), dst [G][P] (where the piece lands), tsum [G][T] (the row's tile
// totals), tbase [G][T] (where a tile's pieces start in the receive buffer), pbase [T]
// (where a tile's partitions start in the output), valid [G] (u32).
struct WireScratch {
    uint64_t *src, *dst, *tsum, *tbase, *pbase;
    uint32_t *valid;
    __device__ WireScratch(uint64_t *w, uint32_t G, uint32_t P, uint32_t T)
        : src(w), dst(w + (uint64_t)G * P), tsum(dst + (uint64_t)G * P), tbase(tsum + (uint64_t)G * T),
          pbase(tbase + (uint64_t)G * T), valid(reinterpret_cast<uint32_t *>(pbase + T)) {}
};

// Grid (T, G): row q's counts in tile t, one per thread (coalesced), their exclusive
// scan (the pieces' offsets inside the tile) and the tile's total.
__global__ __launch_bounds__(kWireTile) void k_wire_rows(const uint64_t *__restrict__ cnt, uint32_t P, uint32_t T,
                                                         uint64_t *__restrict__ src, uint64_t *__restrict__ tsum) {
    __shared__ uint64_t scratch[kWireTile / kWave + 1];
    const uint32_t t = blockIdx.x, q = blockIdx.y, p = t * kWireTile + threadIdx.x;
    const uint64_t v = p < P ? cnt[(uint64_t)q * (P + 1) + p] : 0;
    uint64_t total;
    const uint64_t ex = block_excl_scan_u64(v, scratch, &total);
    if (p < P) src[(uint64_t)q * P + p] = ex;
    if (threadIdx.x == 0) tsum[(uint64_t)q * T + t] = total;
}

// One workgroup: a row is used only when its counts add up to the run the count
// exchange announced (bases.n[q]) -- a sender that failed after the
// count exchange sent zeroed or stale rows, and its pieces are left out (the final
// all-reduce reports the failure) instead of steering the gather and the build/probe
// outside the buffers.  Then the tiles' bases in the receive buffer per row, the
// partitions' tile totals over the valid rows and their exclusive scan, and *narrow =
// the largest key of the valid rows (the word the build/probe sizes its table by).
// T <= kWireTile (P <= 2^20).
__global__ __launch_bounds__(kWireTile) void k_wire_bases(const uint64_t *__restrict__ cnt, uint32_t G, uint32_t P,
                                                          uint32_t T, WireBases bases, uint64_t *__restrict__ w,
                                                          uint32_t *__restrict__ narrow) {
    __shared__ uint64_t scratch[kWireTile / kWave + 1];
    __shared__ uint32_t ok[kWireMaxG];
    const WireScratch sc(w, G, P, T);
    const uint32_t i = threadIdx.x;
    if (i < G) {
        uint64_t run = bases.b[i];
        for (uint32_t t = 0; t < T; ++t) {
            sc.tbase[(uint64_t)i * T + t] = run;
            run += sc.tsum[(uint64_t)i * T + t];
        }
        ok[i] = run == bases.b[i] + bases.n[i] ? 1u : 0u;
        sc.valid[i] = ok[i];
    }
    __syncthreads();
    // (T <= kWireTile: one tile total per thread)
    uint64_t v = 0;
    if (i < T)
        for (uint32_t q = 0; q < G; ++q)
            if (ok[q]) v += sc.tsum[(uint64_t)q * T + i];
    uint64_t total;
    const uint64_t ex = block_excl_scan_u64(v, scratch, &total);
    if (i < T) sc.pbase[i] = ex;
    if (i == 0) {
        uint64_t m = 0;
        for (uint32_t q = 0; q < G; ++q)
            if (ok[q]) m = max(m, cnt[(uint64_t)q * (P + 1) + P]);
        *narrow = (uint32_t)min<uint64_t>(m, 0xFFFFFFFFull);
    }
}

// Grid T: partition p's keys over the valid rows (pc), its start (ps: the tile's base +
// the exclusive scan inside the tile), and where each valid sender's piece lands (dst).
__global__ __launch_bounds__(kWireTile) void k_wire_parts(const uint64_t *__restrict__ cnt, uint32_t G, uint32_t P,
                                                          uint32_t T, uint64_t *__restrict__ w,
                                                          uint64_t *__restrict__ ps, uint64_t *__restrict__ pc) {
    __shared__ uint64_t scratch[kWireTile / kWave + 1];
    const WireScratch sc(w, G, P, T);
    const uint32_t t = blockIdx.x, p = t * kWireTile + threadIdx.x;
    const uint64_t stride = (uint64_t)P + 1;
    uint64_t v = 0;
    if (p < P)
        for (uint32_t q = 0; q < G; ++q)
            if (sc.valid[q]) v += cnt[q * stride + p];
    uint64_t total;
    const uint64_t start = sc.pbase[t] + block_excl_scan_u64(v, scratch, &total);
    if (p >= P) return;
    ps[p] = start;
    pc[p] = v;
    uint64_t d = start;
    for (uint32_t q = 0; q < G; ++q)
        if (sc.valid[q]) {
            sc.dst[(uint64_t)q * P + p] = d;
            d += cnt[q * stride + p];
        }
}

// One wave per piece (partition p, sender q), the pieces of one partition on
// consecutive waves (their destinations are consecutive).  Lanes copy consecutive
// residuals (128 B per wave and step).
__global__ __launch_bounds__(kGatherBlock) void k_wire_gather(const uint16_t *__restrict__ in,
                                                              const uint64_t *__restrict__ cnt, uint32_t G, uint32_t P,
                                                              uint32_t T, const uint64_t *__restrict__ w,
                                                              uint16_t *__restrict__ out) {
    const uint64_t wv = (uint64_t)blockIdx.x * (kGatherBlock / kWave) + threadIdx.x / kWave;
    if (wv >= (uint64_t)G * P) return;
    const WireScratch sc(const_cast<uint64_t *>(w), G, P, T);
    const uint32_t lane = __lane_id(), p = (uint32_t)(wv / G), q = (uint32_t)(wv % G);
    const uint64_t n = cnt[(uint64_t)q * (P + 1) + p];
    if (n == 0 || !sc.valid[q]) return;
    const uint64_t qp = (uint64_t)q * P + p;
    const uint16_t *s = in + sc.tbase[(uint64_t)q * T + p / kWireTile] + sc.src[qp];
    uint16_t *o = out + sc.dst[qp];
    for (uint64_t i = lane; i < n; i += kWave) o[i] = s[i];
}

}  // namespace

uint64_t wire_scratch_words(uint32_t G, uint32_t P) {
    const uint64_t T = (P + kWireTile - 1) / kWireTile;
    return 2ull * G * P + 2ull * G * T + T + (G + 1) / 2 + 1;
}

hipError_t launch_wire_merge(const uint16_t *in, const uint64_t *cnt, uint32_t G, uint32_t P, const WireBases &bases,
                             uint64_t *scratch, uint64_t *ps, uint64_t *pc, uint32_t *narrow, uint16_t *out,
                             hipStream_t s) {
    if (G == 0 || G > kWireMaxG || P == 0) return hipErrorInvalidValue;
    const uint32_t T = (P + kWireTile - 1) / kWireTile;
    if (T > kWireTile) return hipErrorInvalidValue;  // P <= 2^20
    hipLaunchKernelGGL(k_wire_rows, dim3(T, G), dim3(kWireTile), 0, s, cnt, P, T, scratch,
                       scratch + 2ull * G * P);
    hipLaunchKernelGGL(k_wire_bases, dim3(1), dim3(kWireTile), 0, s, cnt, G, P, T, bases, scratch, narrow);
    hipLaunchKernelGGL(k_wire_parts, dim3(T), dim3(kWireTile), 0, s, cnt, G, P, T, scratch, ps, pc);
    const uint64_t waves = (uint64_t)G * P, per = kGatherBlock / kWave;
    const uint64_t grid = (waves + per - 1) / per;
    if (grid > 0x7FFFFFFFull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_wire_gather, dim3((uint32_t)grid), dim3(kGatherBlock), 0, s, in, cnt, G, P, T, scratch, out);
    return hipGetLastError();
}

}  // namespace rho
}  // namespace sgxamd
