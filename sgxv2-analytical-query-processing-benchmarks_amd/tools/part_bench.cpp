// Partition-pass microbenchmark (development tool, not part of the library):
// times hist / scan / scatter of one relation of 2^LOG2N tuples against a plain
// copy kernel.  Build variants with -DSGXAMD_ABLATE_* to isolate costs.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../csrc/rho_kernels.hip"

using namespace sgxamd::rho;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void k_fill(uint64_t *p, uint64_t n, uint64_t seed) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t x = (i + seed) * 0x9E3779B97F4A7C15ull;
        x ^= x >> 29; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 32;
        p[i] = (x & 0xFFFFFFFFull) | (i << 32);
    }
}
__global__ void k_copy(const uint4 *__restrict__ a, uint4 *__restrict__ b, uint64_t n16) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x)
        b[i] = a[i];
}

hipError_t variant(int v, const uint64_t *in, uint64_t *out, const SegMap &m, uint32_t nseg, uint32_t bits,
                   const uint64_t *hist, uint32_t ns, const uint64_t *start) {
    switch (v) {
        case 0: return launch_scatter_items<8, 512>(in, out, m, nseg, 0, bits, hist, kDigitMajor, ns, start, 0);
        case 1: return launch_scatter_items<16, 256>(in, out, m, nseg, 0, bits, hist, kDigitMajor, ns, start, 0);
        case 2: return launch_scatter_items<8, 256>(in, out, m, nseg, 0, bits, hist, kDigitMajor, ns, start, 0);
        case 3: return launch_scatter_items<4, 512>(in, out, m, nseg, 0, bits, hist, kDigitMajor, ns, start, 0);
        case 4: return launch_scatter_items<8, 1024>(in, out, m, nseg, 0, bits, hist, kDigitMajor, ns, start, 0);
        case 5: return launch_scatter_items<16, 512>(in, out, m, nseg, 0, bits, hist, kDigitMajor, ns, start, 0);
        default: return launch_scatter_items<8, 512>(in, out, m, nseg, 0, bits, hist, kDigitMajor, ns, start, 0);
    }
}
static const int kVariantTile[] = {4096, 4096, 2048, 2048, 8192, 8192, 4096};  // tuples per tile

int main(int argc, char **argv) {
    const int log2n = argc > 1 ? atoi(argv[1]) : 28;
    const uint32_t bits = argc > 2 ? atoi(argv[2]) : 8;
    const int reps = 5;
    const int v = argc > 3 ? atoi(argv[3]) : 0;
    const uint64_t n = 1ull << log2n;
    uint64_t *in, *out, *hist, *tot, *start, *cnt;
    CK(hipMalloc(&in, n * 8)); CK(hipMalloc(&out, n * 8));
    const uint64_t T = kVariantTile[v];
    const uint64_t seg = std::max<uint64_t>(T, (n / 2048 + T - 1) / T * T);
    const uint32_t nseg = (n + seg - 1) / seg, F = 1u << bits;
    CK(hipMalloc(&hist, 8ull * F * nseg)); CK(hipMalloc(&tot, 8 * F)); CK(hipMalloc(&start, 8 * F)); CK(hipMalloc(&cnt, 8 * F));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, in, n, 7ull);
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    float ms;
    SegMap m{nullptr, nullptr, nullptr, 1, seg, n};
    auto t = [&](const char *name, auto fn, double bytes) {
        fn();
        CK(hipDeviceSynchronize());
        float best = 1e9, sum = 0;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(a)); fn(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
            CK(hipEventElapsedTime(&ms, a, b)); best = std::min(best, ms); sum += ms;
        }
        printf("%-14s best %8.4f ms  avg %8.4f ms  %7.1f GB/s\n", name, best, sum / reps, bytes / (best * 1e-3) / 1e9);
    };
    t("copy", [&] { hipLaunchKernelGGL(k_copy, dim3(8192), dim3(256), 0, 0, (const uint4 *)in, (uint4 *)out, n / 2); }, 16.0 * n);
    // one pass = hist -> scan (in place) -> scatter, re-run from scratch every rep
    hipEvent_t ev[4];
    for (auto &x : ev) CK(hipEventCreate(&x));
    std::vector<uint64_t> hs(F), hc(F);
    float th = 1e9, ts = 1e9, tc = 1e9;
    for (int r = 0; r <= reps; ++r) {
        CK(hipEventRecord(ev[0]));
        CK(launch_hist((const row_t *)in, m, nseg, 0, bits, hist, kDigitMajor, nseg, 0));
        CK(hipEventRecord(ev[1]));
        CK(launch_scan_single(hist, nseg, bits, tot, start, cnt, 0, nullptr, 0, 0));
        CK(hipEventRecord(ev[2]));
        CK(hipEventSynchronize(ev[2]));
        // guard: digit starts + counts must tile [0, n) before any scatter runs
        CK(hipMemcpy(hs.data(), start, 8 * F, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hc.data(), cnt, 8 * F, hipMemcpyDeviceToHost));
        uint64_t acc = 0;
        for (uint32_t d = 0; d < F; ++d) {
            if (hs[d] != acc) { printf("bad scan at digit %u\n", d); return 1; }
            acc += hc[d];
        }
        if (acc != n) { printf("bad scan total\n"); return 1; }
        CK(hipEventRecord(ev[2]));
        CK(variant(v, (const uint64_t *)in, (uint64_t *)out, m, nseg, bits, hist, nseg, start));
        CK(hipEventRecord(ev[3]));
        CK(hipEventSynchronize(ev[3]));
        if (r == 0) continue;
        CK(hipEventElapsedTime(&ms, ev[0], ev[1])); th = std::min(th, ms);
        CK(hipEventElapsedTime(&ms, ev[2], ev[3])); tc = std::min(tc, ms);
    }
    if (!getenv("NOVERIFY")) {   // verify the last scatter: a permutation of the input, every tuple inside its digit's bin
        std::vector<uint64_t> h(n);
        CK(hipMemcpy(h.data(), out, 8 * n, hipMemcpyDeviceToHost));
        std::vector<uint8_t> seen(n, 0);
        for (uint32_t d = 0; d < F; ++d)
            for (uint64_t j = hs[d]; j < hs[d] + hc[d]; ++j) {
                const uint64_t x = h[j];
                const uint64_t id = x >> 32;
                if ((uint32_t)(x & (F - 1)) != d || id >= n || seen[id]) { printf("VERIFY FAILED at %lu\n", (unsigned long)j); return 1; }
                seen[id] = 1;
            }
        printf("verify ok\n");
    }
    printf("%-14s best %8.4f ms  %7.1f GB/s\n", "hist", th, 8.0 * n / (th * 1e-3) / 1e9);
    printf("%-14s v%d best %8.4f ms  %7.1f GB/s\n", "scatter", v, tc, 16.0 * n / (tc * 1e-3) / 1e9);
    (void)ts;
    return 0;
}
