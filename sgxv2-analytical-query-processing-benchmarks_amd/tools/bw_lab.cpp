// HBM ceiling microbenchmark (development tool): read-only, write-only and copy
// kernels in several shapes, to know what a streaming kernel can reach on this
// MI355X before judging the partition kernels against it.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <int U, bool NT>
__global__ __launch_bounds__(256) void k_read(const v4u *__restrict__ a, uint64_t n16, uint32_t *out) {
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
    for (uint64_t base = blockIdx.x * 256ull * U + threadIdx.x; base < n16; base += stride) {
        v4u v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = base + u * 256;
            if (i < n16) v[u] = NT ? __builtin_nontemporal_load(a + i) : a[i]; else v[u] = v4u{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <int U, bool NT>
__global__ __launch_bounds__(256) void k_write(v4u *__restrict__ b, uint64_t n16) {
    const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
    for (uint64_t base = blockIdx.x * 256ull * U + threadIdx.x; base < n16; base += stride) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = base + u * 256;
            const v4u v = v4u{(uint32_t)i, 1, 2, 3};
            if (i < n16) { if (NT) __builtin_nontemporal_store(v, b + i); else b[i] = v; }
        }
    }
}

template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_copy(const v4u *__restrict__ a, v4u *__restrict__ b, uint64_t n16) {
    const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
    for (uint64_t base = blockIdx.x * 256ull * U + threadIdx.x; base < n16; base += stride) {
        v4u v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = base + u * 256;
            if (i < n16) v[u] = NTL ? __builtin_nontemporal_load(a + i) : a[i];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = base + u * 256;
            if (i < n16) { if (NTS) __builtin_nontemporal_store(v[u], b + i); else b[i] = v[u]; }
        }
    }
}

// Granule writes in the partition-pass pattern: each group of GL = GB/16 lanes writes
// one GB-byte granule; consecutive granules go to NS different sequential output
// streams, round-robin.
template <int GB, int NS, bool NTS>
__global__ __launch_bounds__(256) void k_gscatter(const v4u *__restrict__ a, v4u *__restrict__ b, uint64_t n16) {
    constexpr int GL = GB / 16;
    const uint64_t ngran = n16 / GL;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
        const uint64_t g = i / GL;
        const uint64_t dg = (g % NS) * (ngran / NS) + (g / NS);
        const v4u v = __builtin_nontemporal_load(a + i);
        if (dg < ngran) {
            if (NTS) __builtin_nontemporal_store(v, b + dg * GL + (i % GL)); else b[dg * GL + (i % GL)] = v;
        }
    }
}

// Half-line granules written by one workgroup: the block owns NS output streams and
// writes its data as 64-B halves, all lower halves first (one per stream), then, a
// phase later, the upper halves — the write pattern of a key/payload-split scatter
// whose 16-tuple granules fill 128-B lines in two steps.  NTS: non-temporal stores.
template <bool NTS>
__global__ __launch_bounds__(256) void k_halfpair(const v4u *__restrict__ a, v4u *__restrict__ b, uint64_t n16) {
    constexpr int NS = 256;               // streams (lines in flight) per block
    const uint64_t per_block = NS * 8;    // 16-B words per block step: NS lines of 128 B
    for (uint64_t base = (uint64_t)blockIdx.x * per_block; base < n16; base += (uint64_t)gridDim.x * per_block) {
        for (int half = 0; half < 2; ++half) {
            for (int w = threadIdx.x; w < NS * 4; w += 256) {   // 4 words = one 64-B half per stream
                const int line = w / 4, q = w % 4;
                // stream `line` of this block: lines spaced NS apart in the output (strided streams)
                const uint64_t dst = (base / 8 + (uint64_t)line) * 8 + half * 4 + q;
                const uint64_t src = base + half * NS * 4 + w;
                if (dst < n16 && src < n16) {
                    const v4u v = __builtin_nontemporal_load(a + src);
                    if (NTS) __builtin_nontemporal_store(v, b + dst); else b[dst] = v;
                }
            }
            __syncthreads();
        }
    }
}

// Read only the first H bytes of every 128-B line (blocked-SoA key column probe).
template <int H, bool NT>
__global__ __launch_bounds__(256) void k_read_half(const uint32_t *__restrict__ a, uint64_t nlines, uint32_t *out) {
    constexpr int WPL = H / 4;  // words read per line
    uint32_t acc = 0;
    const uint64_t nw = nlines * WPL;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < nw; i += (uint64_t)gridDim.x * 256) {
        const uint64_t w = (i / WPL) * 32 + (i % WPL);
        acc ^= NT ? __builtin_nontemporal_load(a + w) : a[w];
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char **argv) {
    const int log2n = argc > 1 ? atoi(argv[1]) : 31;  // bytes
    const uint64_t bytes = 1ull << log2n, n16 = bytes / 16;
    v4u *a, *b;
    uint32_t *o;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMalloc(&o, 64));
    CK(hipMemset(a, 1, bytes));
    CK(hipMemset(b, 2, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto t = [&](const char *name, double moved, auto fn) {
        fn();
        CK(hipDeviceSynchronize());
        float best = 1e9;
        for (int r = 0; r < 7; ++r) {
            CK(hipEventRecord(e0));
            fn();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = std::min(best, ms);
        }
        printf("%-28s %8.4f ms  %7.1f GB/s\n", name, best, moved / (best * 1e-3) / 1e9);
    };
    printf("-- granule scatter, grid 4096\n");
#define GS(GB, NS, NT) t(NT ? "gscatter " #GB "B x" #NS " nts" : "gscatter " #GB "B x" #NS, 2.0 * bytes, [&] { hipLaunchKernelGGL((k_gscatter<GB, NS, NT>), dim3(4096), dim3(256), 0, 0, a, b, n16); });
    GS(64, 256, false) GS(128, 256, false) GS(256, 256, false) GS(512, 256, false) GS(1024, 256, false)
    GS(128, 256, true) GS(256, 256, true) GS(512, 256, true)
    GS(128, 64, false) GS(128, 1024, false) GS(256, 1024, false) GS(256, 64, false)
    t("halfpair 64B plain", 2.0 * bytes, [&] { hipLaunchKernelGGL((k_halfpair<false>), dim3(4096), dim3(256), 0, 0, a, b, n16); });
    t("halfpair 64B nts", 2.0 * bytes, [&] { hipLaunchKernelGGL((k_halfpair<true>), dim3(4096), dim3(256), 0, 0, a, b, n16); });
    printf("-- partial-line reads, grid 4096 (GB/s counts the bytes of whole lines)\n");
    t("read full 128B/line nt", bytes, [&] { hipLaunchKernelGGL((k_read_half<128, true>), dim3(4096), dim3(256), 0, 0, (const uint32_t *)a, bytes / 128, o); });
    t("read 64B/line nt", bytes, [&] { hipLaunchKernelGGL((k_read_half<64, true>), dim3(4096), dim3(256), 0, 0, (const uint32_t *)a, bytes / 128, o); });
    t("read 64B/line", bytes, [&] { hipLaunchKernelGGL((k_read_half<64, false>), dim3(4096), dim3(256), 0, 0, (const uint32_t *)a, bytes / 128, o); });
    t("read 32B/line nt", bytes, [&] { hipLaunchKernelGGL((k_read_half<32, true>), dim3(4096), dim3(256), 0, 0, (const uint32_t *)a, bytes / 128, o); });
    if (argc > 2) return 0;
    for (int grid : {1024, 2048, 4096, 16384}) {
        printf("-- grid %d\n", grid);
        t("read U1", bytes, [&] { hipLaunchKernelGGL((k_read<1, false>), dim3(grid), dim3(256), 0, 0, a, n16, o); });
        t("read U4", bytes, [&] { hipLaunchKernelGGL((k_read<4, false>), dim3(grid), dim3(256), 0, 0, a, n16, o); });
        t("read U8", bytes, [&] { hipLaunchKernelGGL((k_read<8, false>), dim3(grid), dim3(256), 0, 0, a, n16, o); });
        t("read U4 nt", bytes, [&] { hipLaunchKernelGGL((k_read<4, true>), dim3(grid), dim3(256), 0, 0, a, n16, o); });
        t("write U4", bytes, [&] { hipLaunchKernelGGL((k_write<4, false>), dim3(grid), dim3(256), 0, 0, b, n16); });
        t("write U4 nt", bytes, [&] { hipLaunchKernelGGL((k_write<4, true>), dim3(grid), dim3(256), 0, 0, b, n16); });
        t("copy U1", 2.0 * bytes, [&] { hipLaunchKernelGGL((k_copy<1, false, false>), dim3(grid), dim3(256), 0, 0, a, b, n16); });
        t("copy U4", 2.0 * bytes, [&] { hipLaunchKernelGGL((k_copy<4, false, false>), dim3(grid), dim3(256), 0, 0, a, b, n16); });
        t("copy U8", 2.0 * bytes, [&] { hipLaunchKernelGGL((k_copy<8, false, false>), dim3(grid), dim3(256), 0, 0, a, b, n16); });
        t("copy U4 ntl", 2.0 * bytes, [&] { hipLaunchKernelGGL((k_copy<4, true, false>), dim3(grid), dim3(256), 0, 0, a, b, n16); });
        t("copy U4 ntl nts", 2.0 * bytes, [&] { hipLaunchKernelGGL((k_copy<4, true, true>), dim3(grid), dim3(256), 0, 0, a, b, n16); });
    }
    return 0;
}
