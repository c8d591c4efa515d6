// Small-join host overhead through the C ABI (no Python): wall time per
// mi355_rho_join_ex call on device-resident pk/fk relations, next to the HIP
// primitives such a call is made of.  Build: scripts/build_small_latency.sh.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "sgxamd/generator.h"
#include "sgxamd/rho.h"

__global__ void k_empty() {}

__global__ void k_flag(volatile uint64_t *h) {
    if (threadIdx.x == 0) {
        __threadfence_system();
        h[0] = 1;
        __threadfence_system();
    }
}

static double med(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

template <class F>
static double time_us(int reps, F f) {
    std::vector<double> t;
    for (int i = 0; i < reps; ++i) {
        const auto a = std::chrono::steady_clock::now();
        f();
        t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count());
    }
    return med(t);
}

int main(int argc, char **argv) {
    // "spin": hipDeviceScheduleSpin (process-wide; the library cannot choose it for its caller)
    if (argc > 1 && std::string(argv[1]) == "spin") (void)hipSetDeviceFlags(hipDeviceScheduleSpin);
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    void *d = nullptr;
    (void)hipMalloc(&d, 64);
    hipPointerAttribute_t pa;
    for (int i = 0; i < 50; ++i) {
        k_empty<<<1, 64, 0, s>>>();
        (void)hipStreamSynchronize(s);
    }
    printf("hipPointerGetAttributes      %6.2f us\n", time_us(200, [&] { (void)hipPointerGetAttributes(&pa, d); }));
    printf("hipStreamSynchronize (idle)  %6.2f us\n", time_us(200, [&] { (void)hipStreamSynchronize(s); }));
    printf("hipEventRecord               %6.2f us\n", time_us(200, [&] { (void)hipEventRecord(e0, s); }));
    (void)hipStreamSynchronize(s);
    printf("launch (async)               %6.2f us\n", time_us(200, [&] { k_empty<<<1, 64, 0, s>>>(); }));
    (void)hipStreamSynchronize(s);
    printf("launch + sync                %6.2f us\n", time_us(200, [&] {
               k_empty<<<1, 64, 0, s>>>();
               (void)hipStreamSynchronize(s);
           }));
    printf("3 launches + sync            %6.2f us\n", time_us(200, [&] {
               k_empty<<<1, 64, 0, s>>>();
               k_empty<<<1, 64, 0, s>>>();
               k_empty<<<1, 64, 0, s>>>();
               (void)hipStreamSynchronize(s);
           }));
    uint64_t *hf = nullptr, *df = nullptr;
    (void)hipHostMalloc(reinterpret_cast<void **>(&hf), 64, hipHostMallocMapped | hipHostMallocCoherent);
    (void)hipHostGetDevicePointer(reinterpret_cast<void **>(&df), hf, 0);
    auto spin = [&] {
        auto *v = reinterpret_cast<volatile uint64_t *>(hf);
        while (v[0] == 0) {
        }
    };
    printf("launch + mapped-flag spin    %6.2f us\n", time_us(200, [&] {
               hf[0] = 0;
               k_flag<<<1, 64, 0, s>>>(df);
               spin();
           }));
    (void)hipStreamSynchronize(s);
    printf("3 launches + flag spin       %6.2f us\n", time_us(200, [&] {
               hf[0] = 0;
               k_empty<<<1, 64, 0, s>>>();
               k_empty<<<1, 64, 0, s>>>();
               k_flag<<<1, 64, 0, s>>>(df);
               spin();
           }));
    (void)hipStreamSynchronize(s);
    printf("launch + flag spin + sync    %6.2f us\n", time_us(200, [&] {
               hf[0] = 0;
               k_flag<<<1, 64, 0, s>>>(df);
               spin();
               (void)hipStreamSynchronize(s);
           }));

    const char *lgs = std::getenv("SMALL_LGS");
    std::vector<int> sizes;
    for (const char *p = lgs ? lgs : "14,16,18,20"; *p;) {
        sizes.push_back(std::atoi(p));
        while (*p && *p != ',') ++p;
        if (*p) ++p;
    }
    for (int lg : sizes) {
        const uint64_t n = 1ull << lg;
        row_t *R = nullptr, *S = nullptr;
        if (hipMalloc(&R, n * sizeof(row_t)) != hipSuccess || hipMalloc(&S, n * sizeof(row_t)) != hipSuccess) return 1;
        mi355_gen_pk_dev(R, n, 0, n, 11111, s);
        mi355_gen_fk_dev(S, n, 0, n, 22222, s);
        (void)hipStreamSynchronize(s);
        for (int timing = 0; timing < 2; ++timing) {
            mi355_rho_opts o{};
            o.stream = s;
            o.timing = timing;
            mi355_rho_stats st{};
            for (int i = 0; i < 20; ++i) mi355_rho_join_ex(R, n, S, n, &o, &st);
            bool ok = true;
            std::vector<double> dev;
            const double w = time_us(200, [&] {
                ok &= mi355_rho_join_ex(R, n, S, n, &o, &st) == MI355_OK && st.matches == n;
                dev.push_back(st.ms_total * 1e3);
            });
            printf("2^%d timing=%d: wall median %6.1f us, device %6.1f us, host overhead %5.1f us, %s\n", lg, timing,
                   w, med(dev), w - med(dev), ok ? "exact" : "WRONG");
        }
        (void)hipFree(R);
        (void)hipFree(S);
    }
    return 0;
}
