// TPC-H query kernels for gfx950: selections as order-preserving two-pass stream
// compaction, join-result transforms, Q19's result predicate, and the synthetic
// table generator.
//
// Selections (filters.hpp:118-138 + Q*Predicates.hpp): pass 1 reads only the
// predicate columns (16 consecutive rows per lane, 16-B vector loads) and keeps one
// bit per row (a u16 per lane) plus a count per workgroup; an exclusive
// scan of the counts gives each workgroup its output offset; pass 2 reads the
// bits and gathers the emitted columns of the matching rows only, writing them in
// input order — exactly the rows, in the order, the reference's scalar
// filter_table produces.
#include <hip/hip_runtime.h>

#include "common.hpp"
#include "tpch_gen.hpp"
#include "tpch_internal.hpp"

namespace sgxamd {
namespace tpch {

// ------------------------------------------------------------ predicates ---
// 16 consecutive elements of a column from row i0 (16-B non-temporal vector loads when
// the run is whole and aligned; element loads at the column's end).
template <typename T>
__device__ __forceinline__ void load16(const T *__restrict__ p, uint64_t i0, uint64_t n, T (&v)[16]) {
    constexpr int PER = 16 / (int)sizeof(T);
    static_assert(16 % sizeof(T) == 0, "element size divides 16 bytes");
    if (i0 + 16 <= n && (reinterpret_cast<uintptr_t>(p + i0) & 15) == 0) {
        const u32x4_t *q = reinterpret_cast<const u32x4_t *>(p + i0);
#pragma unroll
        for (int j = 0; j < 16 / PER; ++j) {
            const u32x4_t w = __builtin_nontemporal_load(q + j);
            __builtin_memcpy(&v[j * PER], &w, 16);
        }
    } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = i0 + k < n ? p[i0 + k] : T{};
    }
}

// Two row layouts per workgroup of 4096 rows.  kConsecutive (1- and 4-byte columns):
// lane t owns rows 16 t .. 16 t + 15, one 16-B load per 16 rows of a byte column, and
// mask16(i0, n) gives bit k = row i0 + k survives.  Otherwise (8-byte columns): lane t
// owns rows t + 256 k, each load instruction of a wave covers 512 contiguous bytes,
// and pred(i) tests one row.  emit(i): the row_t the reference's copy function writes.
struct Q3Customer {  // Q3Predicates.hpp:166-174
    static constexpr bool kConsecutive = true;  // narrow columns: 16 rows per lane
    FilterCols c;
    __device__ uint32_t mask16(uint64_t i0, uint64_t n) const {
        uint8_t m[16];
        load16(c.b0, i0, n, m);
        uint32_t bits = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) bits |= (uint32_t)(m[k] == TPCH_MKT_BUILDING) << k;
        return bits;
    }
    __device__ row_t emit(uint64_t i) const { return c.rows[i]; }
};
struct DateFilter {  // orders / lineitem date selections: lo <= d0 < hi (open ends as 0 / ~0)
    static constexpr bool kConsecutive = false;  // 8-byte column: row per lane
    FilterCols c;
    uint64_t lo, hi;
    __device__ bool pred(uint64_t i) const {
        const uint64_t d = c.d0[i];
        return d >= lo && d < hi;
    }
};
struct Q3Orders : DateFilter {  // :176-185  o_orderdate < 1995-03-15 -> {o_custkey, o_orderkey}
    __device__ row_t emit(uint64_t i) const { return row_t{c.keys[i], c.rows[i].key}; }
};
struct Q3Lineitem : DateFilter {  // :187-195  l_shipdate >= 1995-03-16 -> l_orderkey
    __device__ row_t emit(uint64_t i) const { return c.rows[i]; }
};
struct Q10Orders : DateFilter {  // Q10Predicates.hpp:26-35 -> {o_custkey, o_orderkey.payload}
    __device__ row_t emit(uint64_t i) const { return row_t{c.keys[i], c.rows[i].payload}; }
};
struct Q10Lineitem {  // :37-45
    static constexpr bool kConsecutive = true;  // narrow columns: 16 rows per lane
    FilterCols c;
    __device__ uint32_t mask16(uint64_t i0, uint64_t n) const {
        char f[16];
        load16(c.c0, i0, n, f);
        uint32_t bits = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) bits |= (uint32_t)(f[k] == TPCH_L_RETURNFLAG_R) << k;
        return bits;
    }
    __device__ row_t emit(uint64_t i) const { return c.rows[i]; }
};
struct Q12Lineitem {  // Q12Predicates.hpp:22-37  d0 = shipdate, d1 = commitdate, d2 = receiptdate
    static constexpr bool kConsecutive = false;  // three 8-byte columns: row per lane
    FilterCols c;
    __device__ bool pred(uint64_t i) const {
        const uint8_t m = c.b0[i];
        if (m != TPCH_L_SHIPMODE_MAIL && m != TPCH_L_SHIPMODE_SHIP) return false;
        const uint64_t ship = c.d0[i], commit = c.d1[i], receipt = c.d2[i];
        return commit < receipt && ship < commit && receipt >= TPCH_TIMESTAMP_1994_01_01_SECONDS &&
               receipt < TPCH_TIMESTAMP_1995_01_01_SECONDS;
    }
    __device__ row_t emit(uint64_t i) const { return c.rows[i]; }
};
struct Q19Part {  // Q19Predicates.hpp:40-55  b0 = brand, b1 = container, u0 = size
    static constexpr bool kConsecutive = true;  // narrow columns: 16 rows per lane
    FilterCols c;
    __device__ uint32_t mask16(uint64_t i0, uint64_t n) const {
        uint8_t b[16], k8[16];
        uint32_t sz[16];
        load16(c.b0, i0, n, b);
        load16(c.b1, i0, n, k8);
        load16(c.u0, i0, n, sz);
        uint32_t bits = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const bool ok = b[k] >= TPCH_P_BRAND_12 && b[k] <= TPCH_P_BRAND_34 && k8[k] >= TPCH_P_CONTAINER_SM_CASE &&
                            k8[k] <= TPCH_P_CONTAINER_LG_PKG && sz[k] >= 1 && sz[k] <= 15;
            bits |= (uint32_t)ok << k;
        }
        return bits;
    }
    __device__ row_t emit(uint64_t i) const { return c.rows[i]; }
};
struct Q19Lineitem {  // :27-38  -> {l_partkey, l_orderkey.payload}; b0 = shipmode, b1 = shipinstruct
    static constexpr bool kConsecutive = true;  // narrow columns: 16 rows per lane
    FilterCols c;
    __device__ uint32_t mask16(uint64_t i0, uint64_t n) const {
        float q[16];
        uint8_t m[16], ins[16];
        load16(c.f0, i0, n, q);
        load16(c.b0, i0, n, m);
        load16(c.b1, i0, n, ins);
        uint32_t bits = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const bool ok = q[k] >= 1.f && q[k] <= 30.f &&
                            (m[k] == TPCH_L_SHIPMODE_AIR || m[k] == TPCH_L_SHIPMODE_AIR_REG) &&
                            ins[k] == TPCH_L_SHIPINSTRUCT_DELIVER_IN_PERSON;
            bits |= (uint32_t)ok << k;
        }
        return bits;
    }
    __device__ row_t emit(uint64_t i) const { return row_t{c.keys[i], c.rows[i].payload}; }
};

// --------------------------------------------------------------- filters ---
template <class P>
__device__ __forceinline__ uint32_t lane_bits(const P &p, uint64_t n) {
    uint32_t bits = 0;
    if constexpr (P::kConsecutive) {
        const uint64_t i0 = (uint64_t)blockIdx.x * kFilterSeg + (uint64_t)threadIdx.x * kFilterItems;
        if (i0 < n) bits = p.mask16(i0, n);
    } else {
        const uint64_t base = (uint64_t)blockIdx.x * kFilterSeg + threadIdx.x;
#pragma unroll
        for (int k = 0; k < kFilterItems; ++k) {
            const uint64_t i = base + (uint64_t)k * kFilterThreads;
            if (i < n && p.pred(i)) bits |= 1u << k;
        }
    }
    return bits;
}

template <class P>
__global__ __launch_bounds__(kFilterThreads) void k_filter_mark(P p, uint64_t n, uint16_t *__restrict__ mask,
                                                                uint64_t *__restrict__ blk_count) {
    __shared__ uint32_t red[kFilterThreads / kWave];
    const uint32_t bits = lane_bits(p, n);
    mask[(uint64_t)blockIdx.x * kFilterThreads + threadIdx.x] = (uint16_t)bits;
    uint32_t c = __popc(bits);
    for (int o = kWave / 2; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if (__lane_id() == 0) red[threadIdx.x / kWave] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int w = 0; w < kFilterThreads / kWave; ++w) t += red[w];
        blk_count[blockIdx.x] = t;
    }
}

template <class P>
__global__ __launch_bounds__(kFilterThreads) void k_filter_emit(P p, uint64_t n, const uint16_t *__restrict__ mask,
                                                                const uint64_t *__restrict__ blk_off,
                                                                row_t *__restrict__ out) {
    constexpr int W = kFilterThreads / kWave;
    static_assert(kFilterItems * W == kWave, "one wave scans the (item, wave) counts");
    uint32_t bits = mask[(uint64_t)blockIdx.x * kFilterThreads + threadIdx.x];
    const uint64_t obase = blk_off[blockIdx.x];
    if constexpr (P::kConsecutive) {
        // lanes own consecutive row runs: the lane order is the row order
        __shared__ uint64_t scratch[W + 1];
        uint64_t tot;
        uint64_t o = obase + block_excl_scan_u64(__popc(bits), scratch, &tot);
        const uint64_t i0 = (uint64_t)blockIdx.x * kFilterSeg + (uint64_t)threadIdx.x * kFilterItems;
        while (bits) {
            const int k = __ffs(bits) - 1;
            bits &= bits - 1;
            out[o++] = p.emit(i0 + k);
        }
    } else {
        // rows of (item k, wave w) come in row order k-major, w-minor
        __shared__ uint32_t pre[kFilterItems * W];
        const uint32_t lane = __lane_id(), w = threadIdx.x / kWave;
#pragma unroll
        for (int k = 0; k < kFilterItems; ++k) {
            const uint64_t bal = __ballot((bits >> k) & 1u);
            if (lane == 0) pre[k * W + w] = (uint32_t)__popcll(bal);
        }
        __syncthreads();
        if (threadIdx.x < kWave) {
            const uint64_t v = pre[threadIdx.x];
            const uint64_t incl = wave_incl_scan_u64(v);
            pre[threadIdx.x] = (uint32_t)(incl - v);
        }
        __syncthreads();
        if (bits == 0) return;
        const uint64_t lt = (1ull << lane) - 1;
        const uint64_t base = (uint64_t)blockIdx.x * kFilterSeg + threadIdx.x;
#pragma unroll
        for (int k = 0; k < kFilterItems; ++k) {
            const bool b = (bits >> k) & 1u;
            const uint64_t bal = __ballot(b);
            if (b) out[obase + pre[k * W + w] + __popcll(bal & lt)] = p.emit(base + (uint64_t)k * kFilterThreads);
        }
    }
}

template <class P>
hipError_t mark_as(const P &pr, uint64_t n, uint16_t *mask, uint64_t *blk, hipStream_t s) {
    const uint64_t g = filter_blocks(n);
    if (g == 0) return hipSuccess;
    hipLaunchKernelGGL(k_filter_mark<P>, dim3((uint32_t)g), dim3(kFilterThreads), 0, s, pr, n, mask, blk);
    return hipGetLastError();
}
template <class P>
hipError_t emit_as(const P &pr, uint64_t n, const uint16_t *mask, const uint64_t *off, row_t *out, hipStream_t s) {
    const uint64_t g = filter_blocks(n);
    if (g == 0) return hipSuccess;
    hipLaunchKernelGGL(k_filter_emit<P>, dim3((uint32_t)g), dim3(kFilterThreads), 0, s, pr, n, mask, off, out);
    return hipGetLastError();
}

// The predicate object of selection id (date bounds of DateFilter as in the reference).
template <class F>
hipError_t with_filter(FilterId id, const FilterCols &c, F &&f) {
    constexpr uint64_t NONE = ~0ull;
    switch (id) {
        case kQ3Customer: return f(Q3Customer{c});
        case kQ3Orders: return f(Q3Orders{{c, 0, TPCH_TIMESTAMP_1995_03_15_SECONDS}});
        case kQ3Lineitem: return f(Q3Lineitem{{c, TPCH_TIMESTAMP_1995_03_16_SECONDS, NONE}});
        case kQ10Orders: return f(Q10Orders{{c, TPCH_TIMESTAMP_1993_10_01_SECONDS, TPCH_TIMESTAMP_1994_01_01_SECONDS}});
        case kQ10Lineitem: return f(Q10Lineitem{c});
        case kQ12Lineitem: return f(Q12Lineitem{c});
        case kQ19Part: return f(Q19Part{c});
        case kQ19Lineitem: return f(Q19Lineitem{c});
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_filter_mark(FilterId id, const FilterCols &c, uint64_t n, uint16_t *mask, uint64_t *blk,
                              hipStream_t s) {
    return with_filter(id, c, [&](const auto &pr) { return mark_as(pr, n, mask, blk, s); });
}

hipError_t launch_filter_emit(FilterId id, const FilterCols &c, uint64_t n, const uint16_t *mask,
                              const uint64_t *off, row_t *out, hipStream_t s) {
    return with_filter(id, c, [&](const auto &pr) { return emit_as(pr, n, mask, off, out, s); });
}

// ------------------------------------------------------------ transforms ---
template <int ID>
__global__ __launch_bounds__(256) void k_transform(const output_triple_t *__restrict__ t, uint64_t n,
                                                   const uint32_t *__restrict__ lookup_key,
                                                   const row_t *__restrict__ lookup_rows, row_t *__restrict__ out) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const output_triple_t x = t[i];
        row_t r;
        if constexpr (ID == kSpSp) r = row_t{x.Spayload, x.Spayload};
        else if constexpr (ID == kRpToKeySp) r = row_t{lookup_key[x.Rpayload], x.Spayload};
        else r = row_t{lookup_rows[x.Spayload].key, 0};
        out[i] = r;
    }
}

static uint32_t stream_grid(uint64_t n) {
    const uint64_t g = (n + 255) / 256;
    return (uint32_t)(g < 1 ? 1 : g > 8192 ? 8192 : g);
}

hipError_t launch_transform(TransformId id, const output_triple_t *t, uint64_t n, const uint32_t *lookup_key,
                            const row_t *lookup_rows, row_t *out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const dim3 g(stream_grid(n)), b(256);
    switch (id) {
        case kSpSp: hipLaunchKernelGGL(k_transform<kSpSp>, g, b, 0, s, t, n, lookup_key, lookup_rows, out); break;
        case kRpToKeySp:
            hipLaunchKernelGGL(k_transform<kRpToKeySp>, g, b, 0, s, t, n, lookup_key, lookup_rows, out);
            break;
        case kSpToTuple:
            hipLaunchKernelGGL(k_transform<kSpToTuple>, g, b, 0, s, t, n, lookup_key, lookup_rows, out);
            break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ------------------------------------------------------------- Q19 final ---
__device__ __forceinline__ bool q19_final(uint8_t brand, uint8_t cont, uint32_t size, float q) {
    const bool p1 = brand == TPCH_P_BRAND_12 && cont >= TPCH_P_CONTAINER_SM_CASE && cont <= TPCH_P_CONTAINER_SM_PKG &&
                    size >= 1 && size <= 5 && q >= 1.f && q <= 11.f;
    const bool p2 = brand == TPCH_P_BRAND_23 && cont >= TPCH_P_CONTAINER_MED_BAG &&
                    cont <= TPCH_P_CONTAINER_MED_PACK && size >= 1 && size <= 10 && q >= 10.f && q <= 20.f;
    const bool p3 = brand == TPCH_P_BRAND_34 && cont >= TPCH_P_CONTAINER_LG_CASE && cont <= TPCH_P_CONTAINER_LG_PKG &&
                    size >= 1 && size <= 15 && q >= 20.f && q <= 30.f;
    return p1 || p2 || p3;
}

__global__ __launch_bounds__(256) void k_q19_final(const output_triple_t *__restrict__ t, uint64_t n,
                                                   const uint8_t *__restrict__ brand,
                                                   const uint8_t *__restrict__ cont,
                                                   const uint32_t *__restrict__ size,
                                                   const float *__restrict__ qty, uint64_t *__restrict__ count) {
    uint64_t c = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const output_triple_t x = t[i];
        c += q19_final(brand[x.Rpayload], cont[x.Rpayload], size[x.Rpayload], qty[x.Spayload]);
    }
    c = wave_sum_u64(c);
    if (__lane_id() == 0 && c) atomicAdd((unsigned long long *)count, (unsigned long long)c);
}

hipError_t launch_q19_final(const output_triple_t *t, uint64_t n, const uint8_t *brand, const uint8_t *cont,
                            const uint32_t *size, const float *qty, uint64_t *count, hipStream_t s) {
    hipError_t e = hipMemsetAsync(count, 0, sizeof(uint64_t), s);
    if (e != hipSuccess || n == 0) return e;
    hipLaunchKernelGGL(k_q19_final, dim3(stream_grid(n)), dim3(256), 0, s, t, n, brand, cont, size, qty, count);
    return hipGetLastError();
}

// ------------------------------------------------------------- generator ---
__global__ __launch_bounds__(256) void k_gen_simple(uint32_t sm, uint64_t seed, CustomerTable c, PartTable p,
                                                    NationTable na, OrdersTable o) {
    const uint64_t nc = n_customer(sm), np = n_part(sm), no = n_orders(sm);
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < no; i += stride) {
        if (i < nc) {
            if (c.c_custkey) c.c_custkey[i] = row_t{(type_key)(i + 1), (type_value)i};
            if (c.c_mktsegment) c.c_mktsegment[i] = c_mktsegment(seed, i);
            if (c.c_nationkey) c.c_nationkey[i] = c_nationkey(seed, i);
        }
        if (i < np) {
            if (p.p_partkey) p.p_partkey[i] = row_t{(type_key)(i + 1), (type_value)i};
            if (p.p_brand) p.p_brand[i] = p_brand(seed, i);
            if (p.p_size) p.p_size[i] = p_size(seed, i);
            if (p.p_container) p.p_container[i] = p_container(seed, i);
        }
        if (i < kNations && na.n_nationkey) na.n_nationkey[i] = row_t{(type_key)i, (type_value)i};
        if (o.o_orderkey) o.o_orderkey[i] = row_t{o_orderkey(i), (type_value)i};
        if (o.o_orderdate) o.o_orderdate[i] = (uint64_t)o_orderday(seed, i) * kDay;
        if (o.o_custkey) o.o_custkey[i] = o_custkey(seed, i, nc);
    }
}

hipError_t launch_gen_simple(uint32_t sm, uint64_t seed, const CustomerTable &c, const PartTable &p,
                             const NationTable &n, const OrdersTable &o, hipStream_t s) {
    hipLaunchKernelGGL(k_gen_simple, dim3(stream_grid(n_orders(sm))), dim3(256), 0, s, sm, seed, c, p, n, o);
    return hipGetLastError();
}

// lineitems of the orders of one generator block
__global__ __launch_bounds__(256) void k_gen_lines_per_block(uint32_t sm, uint64_t seed, uint64_t *blk_lines) {
    const uint64_t no = n_orders(sm);
    const uint64_t a = (uint64_t)blockIdx.x * kGenOrdersPerBlock;
    uint64_t c = 0;
    for (uint64_t i = a + threadIdx.x; i < no && i < a + kGenOrdersPerBlock; i += 256) c += o_lines(seed, i);
    __shared__ uint64_t red[256 / kWave];
    c = wave_sum_u64(c);
    if (__lane_id() == 0) red[threadIdx.x / kWave] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = 0;
        for (int w = 0; w < 256 / kWave; ++w) t += red[w];
        blk_lines[blockIdx.x] = t;
    }
}

hipError_t launch_gen_lines_per_block(uint32_t sm, uint64_t seed, uint64_t *blk_lines, hipStream_t s) {
    const uint64_t g = (n_orders(sm) + kGenOrdersPerBlock - 1) / kGenOrdersPerBlock;
    hipLaunchKernelGGL(k_gen_lines_per_block, dim3((uint32_t)g), dim3(256), 0, s, sm, seed, blk_lines);
    return hipGetLastError();
}

// Each thread owns 32 consecutive orders of its block's 8192 and writes their lineitems.
__global__ __launch_bounds__(256) void k_gen_lineitem(uint32_t sm, uint64_t seed, const uint64_t *blk_off,
                                                      LineItemTable l) {
    constexpr uint64_t per = kGenOrdersPerBlock / 256;
    __shared__ uint64_t scratch[256 / kWave + 1];
    const uint64_t no = n_orders(sm), np = n_part(sm);
    const uint64_t a = (uint64_t)blockIdx.x * kGenOrdersPerBlock + threadIdx.x * per;
    uint64_t mine = 0;
    for (uint64_t i = a; i < a + per && i < no; ++i) mine += o_lines(seed, i);
    uint64_t tot;
    uint64_t r = blk_off[blockIdx.x] + block_excl_scan_u64(mine, scratch, &tot);
    for (uint64_t i = a; i < a + per && i < no; ++i) {
        const uint32_t day = o_orderday(seed, i), key = o_orderkey(i), k = o_lines(seed, i);
        for (uint32_t j = 0; j < k; ++j, ++r) {
            const Line L = make_line(seed, r, day, np);
            if (l.l_orderkey) l.l_orderkey[r] = row_t{key, (type_value)r};
            if (l.l_shipdate) l.l_shipdate[r] = L.shipdate;
            if (l.l_commitdate) l.l_commitdate[r] = L.commitdate;
            if (l.l_receiptdate) l.l_receiptdate[r] = L.receiptdate;
            if (l.l_shipmode) l.l_shipmode[r] = L.shipmode;
            if (l.l_partkey) l.l_partkey[r] = L.partkey;
            if (l.l_quantity) l.l_quantity[r] = L.quantity;
            if (l.l_shipinstruct) l.l_shipinstruct[r] = L.shipinstruct;
            if (l.l_returnflag) l.l_returnflag[r] = L.returnflag;
        }
    }
}

hipError_t launch_gen_lineitem(uint32_t sm, uint64_t seed, const uint64_t *blk_off, const LineItemTable &l,
                               hipStream_t s) {
    const uint64_t g = (n_orders(sm) + kGenOrdersPerBlock - 1) / kGenOrdersPerBlock;
    hipLaunchKernelGGL(k_gen_lineitem, dim3((uint32_t)g), dim3(256), 0, s, sm, seed, blk_off, l);
    return hipGetLastError();
}

}  // namespace tpch
}  // namespace sgxamd
