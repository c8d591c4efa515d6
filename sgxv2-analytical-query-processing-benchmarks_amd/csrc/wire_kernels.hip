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

constexpr uint32_t kWireBlock = 1024;
constexpr uint32_t kGatherBlock = 256;

// Workgroup q < G: src[q * P + p] = where sender q's piece of partition p starts in the
// receive buffer (bases.b[q] + the exclusive scan of q's counts).  Workgroup G: pc[p] =
// the partition's keys over all senders, ps = their exclusive scan, *narrow = the
// largest key of any sender (the word the build/probe sizes its direct count table by).
// cnt: G rows of P counts + the sender's largest key.  A row is used only when its
// counts add up to the run the count exchange announced (bases.b[q + 1] - bases.b[q]):
// a sender that failed after the count exchange sent zeros or stale counts, and its
// pieces are left out (the final all-reduce reports the failure) instead of steering
// the gather and the build/probe outside the buffers.  valid[q]: the verdict (both
// workgroups reach it from the same sums).  Thread t takes partitions [t C, (t + 1) C).
__global__ __launch_bounds__(kWireBlock) void k_wire_scan(const uint64_t *__restrict__ cnt, uint32_t G, uint32_t P,
                                                          WireBases bases, uint64_t *__restrict__ src,
                                                          uint32_t *__restrict__ valid, uint64_t *__restrict__ ps,
                                                          uint64_t *__restrict__ pc, uint32_t *__restrict__ narrow) {
    __shared__ uint64_t scratch[kWireBlock / kWave + 1];
    __shared__ uint32_t ok[kWireMaxG];
    const uint32_t q = blockIdx.x, t = threadIdx.x;
    const uint32_t C = (P + kWireBlock - 1) / kWireBlock;
    const uint32_t p0 = min(P, t * C), p1 = min(P, p0 + C);
    const uint64_t stride = (uint64_t)P + 1;
    uint64_t local = 0, total = 0;
    if (q < G) {
        const uint64_t *c = cnt + q * stride;
        for (uint32_t p = p0; p < p1; ++p) local += c[p];
        uint64_t run = bases.b[q] + block_excl_scan_u64(local, scratch, &total);
        for (uint32_t p = p0; p < p1; ++p) {
            src[(uint64_t)q * P + p] = run;
            run += c[p];
        }
        if (t == 0) valid[q] = total == bases.b[q + 1] - bases.b[q] ? 1u : 0u;
        return;
    }
    for (uint32_t r = 0; r < G; ++r) {
        local = 0;
        for (uint32_t p = p0; p < p1; ++p) local += cnt[r * stride + p];
        (void)block_excl_scan_u64(local, scratch, &total);
        if (t == 0) ok[r] = total == bases.b[r + 1] - bases.b[r] ? 1u : 0u;
    }
    __syncthreads();
    local = 0;
    for (uint32_t p = p0; p < p1; ++p) {
        uint64_t s = 0;
        for (uint32_t r = 0; r < G; ++r)
            if (ok[r]) s += cnt[r * stride + p];
        pc[p] = s;
        local += s;
    }
    uint64_t run = block_excl_scan_u64(local, scratch, &total);
    for (uint32_t p = p0; p < p1; ++p) {
        ps[p] = run;
        run += pc[p];
    }
    if (t == 0) {
        uint64_t m = 0;
        for (uint32_t r = 0; r < G; ++r)
            if (ok[r]) m = max(m, cnt[r * stride + P]);
        *narrow = (uint32_t)min<uint64_t>(m, 0xFFFFFFFFull);
    }
}

// One wave per piece (partition p, sender q), the pieces of one partition on
// consecutive waves (their destinations are consecutive): the piece lands at ps[p] +
// the pieces of the (valid) senders before q.  Lanes copy consecutive residuals (128 B
// per wave and step).
__global__ __launch_bounds__(kGatherBlock) void k_wire_gather(const uint16_t *__restrict__ in,
                                                              const uint64_t *__restrict__ cnt, uint32_t G, uint32_t P,
                                                              const uint64_t *__restrict__ src,
                                                              const uint32_t *__restrict__ valid,
                                                              const uint64_t *__restrict__ ps,
                                                              uint16_t *__restrict__ out) {
    const uint64_t w = (uint64_t)blockIdx.x * (kGatherBlock / kWave) + threadIdx.x / kWave;
    if (w >= (uint64_t)G * P) return;
    const uint32_t lane = __lane_id(), p = (uint32_t)(w / G), q = (uint32_t)(w % G);
    const uint64_t stride = (uint64_t)P + 1;
    const uint64_t n = cnt[q * stride + p];
    if (n == 0 || !valid[q]) return;
    uint64_t d = ps[p];
    for (uint32_t r = 0; r < q; ++r)
        if (valid[r]) d += cnt[r * stride + p];
    const uint16_t *s = in + src[(uint64_t)q * P + p];
    uint16_t *o = out + d;
    for (uint64_t i = lane; i < n; i += kWave) o[i] = s[i];
}

}  // namespace

hipError_t launch_wire_merge(const uint16_t *in, const uint64_t *cnt, uint32_t G, uint32_t P, const WireBases &bases,
                             uint64_t *src, uint64_t *ps, uint64_t *pc, uint32_t *narrow, uint16_t *out,
                             hipStream_t s) {
    if (G == 0 || G > kWireMaxG || P == 0) return hipErrorInvalidValue;
    uint32_t *valid = reinterpret_cast<uint32_t *>(src + (uint64_t)G * P);
    hipLaunchKernelGGL(k_wire_scan, dim3(G + 1), dim3(kWireBlock), 0, s, cnt, G, P, bases, src, valid, ps, pc,
                       narrow);
    const uint64_t waves = (uint64_t)G * P, per = kGatherBlock / kWave;
    const uint64_t grid = (waves + per - 1) / per;
    if (grid > 0x7FFFFFFFull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_wire_gather, dim3((uint32_t)grid), dim3(kGatherBlock), 0, s, in, cnt, G, P, src, valid, ps,
                       out);
    return hipGetLastError();
}

}  // namespace rho
}  // namespace sgxamd
