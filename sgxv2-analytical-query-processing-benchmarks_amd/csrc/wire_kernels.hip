// Multi-GPU exchange with 2-byte residuals on the wire (multi_host.cpp "u16 wire",
// DESIGN.md §5): the receiver's side.  Every sender partitioned the keys it sends this
// rank with this rank's plan (the local join's two passes over key bits [key_shift,
// key_shift + bits), pass 2 writing narrow residuals, every partition padded to 8
// residuals) and sent them grouped by partition, after a row of P partition counts, P
// partition starts (relative to its run, multiples of 8) and its largest key.  Since
// round 6 the build/probe reads partition p of S in place as its G pieces, one per
// sender (k_join_np): launch_wire_pieces only tabulates where each piece starts and how
// many keys it holds.  The gather of a partition's pieces into one contiguous partition
// (launch_wire_merge) remains for worlds above kPieceMax ranks.  The reference fills
// its shared partition arrays the same way: every thread's slice lands at offsets from a
// cross-thread prefix sum over the slices' histograms (radix_join.cpp:897-915).
#include "common.hpp"
#include "rho_internal.hpp"

namespace sgxamd {
namespace rho {

namespace {

constexpr uint32_t kWireTile = 1024;  // partitions per tile (one thread each)
constexpr uint32_t kGatherBlock = 256;

// Grid (T, G): row q's counts in tile t (coalesced), summed; the tile's largest end
// (start + count) of a piece.
__global__ __launch_bounds__(kWireTile) void k_wire_rows(const uint64_t *__restrict__ rows, uint32_t P, uint32_t T,
                                                         uint64_t *__restrict__ tsum, uint64_t *__restrict__ tend) {
    __shared__ uint64_t scratch[kWireTile / kWave + 1];
    const uint32_t t = blockIdx.x, q = blockIdx.y, p = t * kWireTile + threadIdx.x;
    const uint64_t *row = rows + (uint64_t)q * (2ull * P + 1);
    const uint64_t c = p < P ? row[p] : 0, e = p < P ? row[P + p] + c : 0;
    const uint64_t ce = block_max_u64(e, scratch);
    uint64_t total;
    (void)block_excl_scan_u64(c, scratch, &total);
    if (threadIdx.x == 0) {
        tsum[(uint64_t)q * T + t] = total;
        tend[(uint64_t)q * T + t] = ce;
    }
}

// One workgroup: row q is used only when its counts add up to the run the count exchange
// announced (bases.n[q]) and its pieces end inside the run's slot (bases.span) -- a
// sender that failed after the count exchange sent zeroed or stale rows, and its pieces
// are left out (the final all-reduce reports the failure) instead of steering the
// build/probe outside the buffers.  *narrow = the largest key of the valid rows (the
// word the build/probe sizes its table by).
__global__ __launch_bounds__(kWireMaxG) void k_wire_valid(const uint64_t *__restrict__ rows, uint32_t G, uint32_t P,
                                                          uint32_t T, WireBases bases, const uint64_t *__restrict__ tsum,
                                                          const uint64_t *__restrict__ tend,
                                                          uint32_t *__restrict__ valid, uint32_t *__restrict__ narrow) {
    __shared__ uint64_t kmax[kWireMaxG];
    const uint32_t q = threadIdx.x;
    kmax[q] = 0;
    if (q < G) {
        uint64_t run = 0, end = 0;
        for (uint32_t t = 0; t < T; ++t) {
            run += tsum[(uint64_t)q * T + t];
            end = max(end, tend[(uint64_t)q * T + t]);
        }
        const bool ok = run == bases.n[q] && end <= bases.span[q];
        valid[q] = ok ? 1u : 0u;
        if (ok) kmax[q] = rows[(uint64_t)q * (2ull * P + 1) + 2ull * P];
    }
    __syncthreads();
    if (q == 0) {
        uint64_t m = 0;
        for (uint32_t i = 0; i < G; ++i) m = max(m, kmax[i]);
        *narrow = (uint32_t)min<uint64_t>(m, 0xFFFFFFFFull);
    }
}

// Thread per partition p: its pieces [p][q] -- first unit of 8 residuals in the receive
// buffer and keys (0 for a row left out) -- its keys (pc) and 8 x its units (units8: the
// task list's S size).
__global__ __launch_bounds__(kWireTile) void k_wire_table(const uint64_t *__restrict__ rows, uint32_t G, uint32_t P,
                                                          WireBases bases, const uint32_t *__restrict__ valid,
                                                          uint32_t *__restrict__ ub, uint32_t *__restrict__ nk,
                                                          uint64_t *__restrict__ pc, uint64_t *__restrict__ units8) {
    const uint32_t p = blockIdx.x * kWireTile + threadIdx.x;
    if (p >= P) return;
    uint64_t keys = 0, units = 0;
    for (uint32_t q = 0; q < G; ++q) {
        const uint64_t *row = rows + (uint64_t)q * (2ull * P + 1);
        const bool ok = valid[q] != 0;
        const uint64_t c = ok ? row[p] : 0;
        ub[(uint64_t)p * G + q] = ok ? (uint32_t)((bases.b[q] + row[P + p]) / 8) : 0u;
        nk[(uint64_t)p * G + q] = (uint32_t)c;
        keys += c;
        units += (c + 7) / 8;
    }
    pc[p] = keys;
    units8[p] = 8 * units;
}

// Gather (worlds above kPieceMax): one wave per piece (partition p, sender q), the
// pieces of one partition on consecutive waves; lanes copy consecutive residuals.
__global__ __launch_bounds__(kGatherBlock) void k_wire_gather(const uint16_t *__restrict__ in, uint32_t G, uint32_t P,
                                                              const uint32_t *__restrict__ ub,
                                                              const uint32_t *__restrict__ nk,
                                                              const uint64_t *__restrict__ ps,
                                                              uint16_t *__restrict__ out) {
    const uint64_t wv = (uint64_t)blockIdx.x * (kGatherBlock / kWave) + threadIdx.x / kWave;
    if (wv >= (uint64_t)G * P) return;
    const uint32_t lane = __lane_id(), p = (uint32_t)(wv / G), q = (uint32_t)(wv % G);
    const uint64_t n = nk[(uint64_t)p * G + q];
    if (n == 0) return;
    uint64_t d = ps[p];
    for (uint32_t i = 0; i < q; ++i) d += nk[(uint64_t)p * G + i];
    const uint16_t *s = in + (uint64_t)ub[(uint64_t)p * G + q] * 8;
    for (uint64_t i = lane; i < n; i += kWave) out[d + i] = s[i];
}

// One block: ps = exclusive scan of pc over the P partitions.
__global__ __launch_bounds__(1024) void k_wire_starts(const uint64_t *__restrict__ pc, uint32_t P,
                                                      uint64_t *__restrict__ ps) {
    __shared__ uint64_t scratch[1024 / kWave + 1];
    uint64_t carry = 0;
    for (uint32_t b = 0; b < P; b += 1024) {
        const uint32_t i = b + threadIdx.x;
        const uint64_t v = i < P ? pc[i] : 0;
        uint64_t tot;
        const uint64_t ex = block_excl_scan_u64(v, scratch, &tot);
        if (i < P) ps[i] = carry + ex;
        carry += tot;
    }
}

uint64_t wire_tiles(uint32_t P) { return (P + kWireTile - 1) / kWireTile; }

}  // namespace

uint64_t wire_scratch_words(uint32_t G, uint32_t P) {
    // tile sums and ends, valid flags, the piece table (u32 [P][G] twice), units8 [P]
    return 2ull * G * wire_tiles(P) + (G + 1) / 2 + 1 + (uint64_t)G * P + P;
}

WirePieces wire_pieces_of(uint64_t *scratch, uint32_t G, uint32_t P) {
    const uint64_t T = wire_tiles(P);
    WirePieces w;
    w.ub = reinterpret_cast<uint32_t *>(scratch + 2ull * G * T + (G + 1) / 2 + 1);
    w.nk = w.ub + (uint64_t)G * P;
    w.units8 = reinterpret_cast<uint64_t *>(w.nk + (uint64_t)G * P);
    w.G = G;
    w.P = P;
    return w;
}

hipError_t launch_wire_pieces(const uint64_t *rows, uint32_t G, uint32_t P, const WireBases &bases, uint64_t *scratch,
                              uint64_t *pc, uint32_t *narrow, hipStream_t s) {
    if (G == 0 || G > kWireMaxG || P == 0) return hipErrorInvalidValue;
    const uint64_t T = wire_tiles(P);
    uint64_t *tsum = scratch, *tend = tsum + (uint64_t)G * T;
    uint32_t *valid = reinterpret_cast<uint32_t *>(tend + (uint64_t)G * T);
    hipLaunchKernelGGL(k_wire_rows, dim3((uint32_t)T, G), dim3(kWireTile), 0, s, rows, P, (uint32_t)T, tsum, tend);
    hipLaunchKernelGGL(k_wire_valid, dim3(1), dim3(kWireMaxG), 0, s, rows, G, P, (uint32_t)T, bases, tsum, tend, valid,
                       narrow);
    const WirePieces w = wire_pieces_of(scratch, G, P);
    hipLaunchKernelGGL(k_wire_table, dim3((uint32_t)T), dim3(kWireTile), 0, s, rows, G, P, bases, valid, w.ub, w.nk,
                       pc, w.units8);
    return hipGetLastError();
}

hipError_t launch_wire_merge(const uint16_t *in, const uint64_t *rows, uint32_t G, uint32_t P,
                             const WireBases &bases, uint64_t *scratch, uint64_t *ps, uint64_t *pc, uint32_t *narrow,
                             uint16_t *out, hipStream_t s) {
    hipError_t e = launch_wire_pieces(rows, G, P, bases, scratch, pc, narrow, s);
    if (e != hipSuccess) return e;
    const WirePieces w = wire_pieces_of(scratch, G, P);
    hipLaunchKernelGGL(k_wire_starts, dim3(1), dim3(1024), 0, s, pc, P, ps);
    const uint64_t waves = (uint64_t)G * P, per = kGatherBlock / kWave;
    const uint64_t grid = (waves + per - 1) / per;
    if (grid > 0x7FFFFFFFull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_wire_gather, dim3((uint32_t)grid), dim3(kGatherBlock), 0, s, in, G, P, w.ub, w.nk, ps, out);
    return hipGetLastError();
}

}  // namespace rho
}  // namespace sgxamd
