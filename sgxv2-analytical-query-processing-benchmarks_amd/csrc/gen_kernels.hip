// Device-side synthetic data: relations of the reference's pk / fk shapes and
// scan columns, generated directly in HBM.
//
// The reference builds keys with a serial glibc-rand Knuth shuffle
// (generator.cpp:100-153), which cannot be split across GPUs.  Here row r of a
// relation gets perm(r) + 1 for a keyed bijection perm of [0, n) (cycle-walking
// over a 4-round multiply/xor-shift mix on ceil(log2 n) bits), so keys are still
// exactly a shuffled 1..n (pk) or shuffled copies of 1..maxid (fk) and any rank
// can generate any slice.  Match counts are therefore the reference's
// (pk ⋈ fk = |S|); the row order is a different (keyed) shuffle.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.hpp"
#include "runtime.hpp"
#include "sgxamd/generator.h"
#include "sgxamd/rho.h"

namespace sgxamd {
namespace gen {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

struct Perm {
    uint64_t n;
    uint32_t k;      // bits of the domain
    uint64_t mask;
    uint64_t mul[4];
    uint64_t add[4];
};

__device__ __forceinline__ uint64_t perm_round(const Perm &p, uint64_t x) {
    const uint32_t sh = p.k / 2 + 1;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        x = (x * p.mul[r]) & p.mask;
        x ^= x >> sh;
        x = (x + p.add[r]) & p.mask;
    }
    return x;
}

__device__ __forceinline__ uint64_t perm_apply(const Perm &p, uint64_t x) {
    if (p.n <= 1) return 0;
    do {
        x = perm_round(p, x);
    } while (x >= p.n);  // cycle walking: stays a bijection of [0, n)
    return x;
}

__device__ Perm make_perm(uint64_t n, uint64_t seed) {
    Perm p;
    p.n = n;
    uint32_t k = 1;
    while ((1ull << k) < n) ++k;
    p.k = k;
    p.mask = (k >= 64) ? ~0ull : ((1ull << k) - 1);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        p.mul[r] = (splitmix64(seed * 8 + 2 * r) | 1ull) & p.mask;
        if (p.mul[r] == 0) p.mul[r] = 1;
        p.add[r] = splitmix64(seed * 8 + 2 * r + 1) & p.mask;
    }
    return p;
}

__global__ void k_gen_pk(row_t *__restrict__ out, uint64_t count, uint64_t first, uint64_t n, uint64_t seed) {
    const Perm p = make_perm(n, seed);
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < count;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t r = first + i;
        row_t t;
        t.key = (uint32_t)(perm_apply(p, r) + 1);
        t.payload = (uint32_t)r;
        out[i] = t;
    }
}

__global__ void k_gen_fk(row_t *__restrict__ out, uint64_t count, uint64_t first, uint64_t maxid, uint64_t seed) {
    uint64_t cur_copy = ~0ull;
    Perm p{};
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < count;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t r = first + i;
        const uint64_t c = r / maxid;
        if (c != cur_copy) {
            p = make_perm(maxid, seed + 0x1000 * (c + 1));
            cur_copy = c;
        }
        row_t t;
        t.key = (uint32_t)(perm_apply(p, r % maxid) + 1);
        t.payload = (uint32_t)r;
        out[i] = t;
    }
}

template <typename T>
__global__ void k_gen_scan(T *__restrict__ out, uint64_t n, int mode, uint64_t seed) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = mode == 0 ? (T)(i & 255) : (T)splitmix64(seed ^ (i * 0xD6E8FEB86659FD93ull));
}

// ---- Zipf (genzipf.cpp:34-144) on the device.  LUT[i] = sum_{j<=i+1} 1/j^theta
// (unnormalised; draws compare against u * LUT[N-1] instead of dividing the LUT),
// built by a three-kernel scan with a fixed decomposition so every rank of a
// multi-GPU run builds the identical table; draws use a counter-based uniform
// (row r -> splitmix64) and the reference's binary search (:118-136); the
// alphabet permutation of 1..N (gen_alphabet :34-49) is the keyed bijection.
constexpr int kZipfThreads = 256;
constexpr int kZipfPerThread = 16;
constexpr uint64_t kZipfBlock = (uint64_t)kZipfThreads * kZipfPerThread;

__device__ __forceinline__ double block_incl_scan_f64(double v, double *sh) {
    const uint32_t lane = __lane_id(), wave = threadIdx.x / kWave;
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
        const double t = __shfl_up(v, off, kWave);
        if (lane >= (uint32_t)off) v += t;
    }
    if (lane == kWave - 1) sh[wave] = v;
    __syncthreads();
    double pre = 0.0;
    for (uint32_t w = 0; w < wave; ++w) pre += sh[w];
    __syncthreads();
    return v + pre;
}

__global__ __launch_bounds__(kZipfThreads) void k_zipf_lut_local(double *__restrict__ lut, uint64_t N, double theta,
                                                                 double *__restrict__ bsum) {
    __shared__ double sh[kZipfThreads / kWave];
    const uint64_t base = blockIdx.x * kZipfBlock + (uint64_t)threadIdx.x * kZipfPerThread;
    double v[kZipfPerThread];
    double run = 0.0;
#pragma unroll
    for (int j = 0; j < kZipfPerThread; ++j) {
        const uint64_t i = base + j;
        run += i < N ? pow((double)(i + 1), -theta) : 0.0;
        v[j] = run;
    }
    const double incl = block_incl_scan_f64(run, sh);
    const double pre = incl - run;
#pragma unroll
    for (int j = 0; j < kZipfPerThread; ++j)
        if (base + j < N) lut[base + j] = pre + v[j];
    if (threadIdx.x == kZipfThreads - 1) bsum[blockIdx.x] = incl;
}

// One block: block sums -> exclusive block offsets (in place).
__global__ __launch_bounds__(1024) void k_zipf_scan_blocks(double *__restrict__ bsum, uint64_t nb) {
    __shared__ double sh[1024 / kWave];
    __shared__ double tot;
    double carry = 0.0;
    for (uint64_t b = 0; b < nb; b += 1024) {
        const uint64_t i = b + threadIdx.x;
        const double x = i < nb ? bsum[i] : 0.0;
        const double incl = block_incl_scan_f64(x, sh);
        if (threadIdx.x == 1023) tot = incl;
        __syncthreads();
        if (i < nb) bsum[i] = carry + (incl - x);
        carry += tot;
        __syncthreads();
    }
}

__global__ __launch_bounds__(kZipfThreads) void k_zipf_lut_add(double *__restrict__ lut, uint64_t N,
                                                               const double *__restrict__ boff) {
    const double o = boff[blockIdx.x];
    const uint64_t base = blockIdx.x * kZipfBlock;
    for (uint32_t j = threadIdx.x; j < kZipfBlock; j += kZipfThreads)
        if (base + j < N) lut[base + j] += o;
}

__global__ void k_gen_zipf(row_t *__restrict__ out, uint64_t count, uint64_t first, const double *__restrict__ lut,
                           uint64_t N, uint64_t seed) {
    const Perm p = make_perm(N, seed ^ 0xA1FAB37ull);  // gen_alphabet: permutation of 1..N
    const double tot = lut[N - 1];
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < count;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t r = first + i;
        const double u = (double)(splitmix64(seed * 0x9E3779B97F4A7C15ull + r) >> 11) * 0x1.0p-53;
        const double target = u * tot;
        uint64_t pos;
        if (lut[0] >= target) {
            pos = 0;
        } else {
            uint64_t left = 0, right = N - 1;
            while (right - left > 1) {
                const uint64_t m = (left + right) / 2;
                if (lut[m] < target) left = m; else right = m;
            }
            pos = right;
        }
        row_t t;
        t.key = (uint32_t)(perm_apply(p, pos) + 1);
        t.payload = (uint32_t)r;
        out[i] = t;
    }
}

inline dim3 grid_for(uint64_t count) {
    uint64_t b = (count + 255) / 256;
    if (b > 8192) b = 8192;
    if (b == 0) b = 1;
    return dim3((uint32_t)b);
}

}  // namespace gen
}  // namespace sgxamd

using namespace sgxamd;

#define GEN_CHECK()                                                           \
    do {                                                                      \
        hipError_t _e = hipGetLastError();                                    \
        if (_e == hipSuccess) _e = hipStreamSynchronize(s);                   \
        if (_e != hipSuccess) {                                               \
            set_last_error(std::string("generator: ") + hipGetErrorString(_e)); \
            return MI355_ERR_HIP;                                             \
        }                                                                     \
        return MI355_OK;                                                      \
    } while (0)

static hipStream_t gen_stream(void *stream, int *status) {
    Context *ctx = current_context(status);
    if (!ctx) return nullptr;
    return thread_stream(ctx, stream);
}

extern "C" {

int mi355_gen_pk_dev(row_t *out, uint64_t count, uint64_t first, uint64_t n, uint64_t seed, void *stream) {
    if ((!out && count) || first + count > n) return MI355_ERR_INVALID;
    int st = 0;
    hipStream_t s = gen_stream(stream, &st);
    if (st) return st;
    if (!count) return MI355_OK;
    hipLaunchKernelGGL(gen::k_gen_pk, gen::grid_for(count), dim3(256), 0, s, out, count, first, n, seed);
    GEN_CHECK();
}

int mi355_gen_fk_dev(row_t *out, uint64_t count, uint64_t first, uint64_t maxid, uint64_t seed, void *stream) {
    if ((!out && count) || maxid == 0) return MI355_ERR_INVALID;
    int st = 0;
    hipStream_t s = gen_stream(stream, &st);
    if (st) return st;
    if (!count) return MI355_OK;
    hipLaunchKernelGGL(gen::k_gen_fk, gen::grid_for(count), dim3(256), 0, s, out, count, first, maxid, seed);
    GEN_CHECK();
}

int mi355_gen_zipf_dev(row_t *out, uint64_t count, uint64_t first, uint32_t alphabet_size, double theta,
                       uint64_t seed, void *stream) {
    if ((!out && count) || alphabet_size == 0 || !(theta >= 0.0)) return MI355_ERR_INVALID;
    int st = 0;
    hipStream_t s = gen_stream(stream, &st);
    if (st) return st;
    if (!count) return MI355_OK;
    const uint64_t N = alphabet_size;
    const uint64_t nb = (N + gen::kZipfBlock - 1) / gen::kZipfBlock;
    double *lut = nullptr, *bsum = nullptr;
    if (hipMalloc(&lut, N * sizeof(double)) != hipSuccess || hipMalloc(&bsum, nb * sizeof(double)) != hipSuccess) {
        (void)hipFree(lut);
        set_last_error("generator: Zipf LUT allocation failed");
        return MI355_ERR_OOM;
    }
    hipLaunchKernelGGL(gen::k_zipf_lut_local, dim3((uint32_t)nb), dim3(gen::kZipfThreads), 0, s, lut, N, theta, bsum);
    hipLaunchKernelGGL(gen::k_zipf_scan_blocks, dim3(1), dim3(1024), 0, s, bsum, nb);
    hipLaunchKernelGGL(gen::k_zipf_lut_add, dim3((uint32_t)nb), dim3(gen::kZipfThreads), 0, s, lut, N, bsum);
    hipLaunchKernelGGL(gen::k_gen_zipf, gen::grid_for(count), dim3(256), 0, s, out, count, first, lut, N, seed);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    (void)hipFree(lut);
    (void)hipFree(bsum);
    if (e != hipSuccess) {
        set_last_error(std::string("generator: ") + hipGetErrorString(e));
        return MI355_ERR_HIP;
    }
    return MI355_OK;
}

int mi355_gen_scan_u8_dev(uint8_t *out, size_t n, int mode, uint64_t seed, void *stream) {
    if (!out && n) return MI355_ERR_INVALID;
    int st = 0;
    hipStream_t s = gen_stream(stream, &st);
    if (st) return st;
    if (!n) return MI355_OK;
    hipLaunchKernelGGL(gen::k_gen_scan<uint8_t>, gen::grid_for(n), dim3(256), 0, s, out, (uint64_t)n, mode, seed);
    GEN_CHECK();
}

int mi355_gen_scan_i32_dev(int32_t *out, size_t n, int mode, uint64_t seed, void *stream) {
    if (!out && n) return MI355_ERR_INVALID;
    int st = 0;
    hipStream_t s = gen_stream(stream, &st);
    if (st) return st;
    if (!n) return MI355_OK;
    hipLaunchKernelGGL(gen::k_gen_scan<int32_t>, gen::grid_for(n), dim3(256), 0, s, out, (uint64_t)n, mode, seed);
    GEN_CHECK();
}

}  // extern "C"
