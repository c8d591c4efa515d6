// Host side of the MI355X predicate scan: the C-ABI of sgxamd/scan.h.
//
// Each entry point is the blocking equivalent of one SIMD512:: call
// (SIMD512.hpp:39-84).  Inputs/outputs may live in host or device memory; host
// buffers are staged through HBM.  Device inputs that are not 16-byte aligned
// are copied to an aligned buffer first (the kernels load 16 bytes per lane).
#include <algorithm>
#include <cstring>
#include <string>

#include "common.hpp"
#include "runtime.hpp"
#include "scan_internal.hpp"
#include "sgxamd/rho.h"
#include "sgxamd/scan.h"

namespace sgxamd {
namespace scan {
namespace {

#define SCAN_HIP(call)                                                                     \
    do {                                                                                   \
        hipError_t _e = (call);                                                            \
        if (_e != hipSuccess) {                                                            \
            set_last_error(std::string(#call) + ": " + hipGetErrorString(_e));             \
            return (_e == hipErrorOutOfMemory) ? MI355_ERR_OOM : MI355_ERR_HIP;            \
        }                                                                                  \
    } while (0)

struct Geometry {
    uint64_t rows_per_chunk;
    uint32_t nchunks;
};

Geometry geometry(uint64_t n) {
    uint64_t rpc = (n + kChunkTarget - 1) / kChunkTarget;
    rpc = std::max<uint64_t>((rpc + kChunkQuantum - 1) / kChunkQuantum * kChunkQuantum, kChunkQuantum);
    return {rpc, (uint32_t)((n + rpc - 1) / rpc)};
}

enum class Op { kCount, kBitvector, kIndex, kValues };

// Device-resident, 16-byte aligned view of the input column.
template <typename T>
int stage_input(Context *ctx, hipStream_t s, const T *in, size_t n, const T **dev) {
    if (is_device_pointer(in)) {
        if ((reinterpret_cast<uintptr_t>(in) & 15u) == 0) {
            *dev = in;
            return MI355_OK;
        }
        SCAN_HIP(ctx->scan_in.ensure(n * sizeof(T)));
        SCAN_HIP(hipMemcpyAsync(ctx->scan_in.ptr, in, n * sizeof(T), hipMemcpyDeviceToDevice, s));
    } else {
        SCAN_HIP(ctx->scan_in.ensure(n * sizeof(T)));
        SCAN_HIP(hipMemcpyAsync(ctx->scan_in.ptr, in, n * sizeof(T), hipMemcpyHostToDevice, s));
    }
    *dev = ctx->scan_in.as<T>();
    return MI355_OK;
}

template <typename T, typename OutT>
int run(Op op, T lo, T hi, const T *in, size_t n, void *out, size_t cap, uint64_t *result) {
    int status = MI355_OK;
    Context *ctx = current_context(&status);
    if (!ctx) return status;
    std::lock_guard<std::mutex> lk(ctx->mu);
    hipStream_t s = thread_stream(ctx, nullptr);
    Timer &tm = thread_timer();
    tm.begin_call(s, thread_timing_enabled());

    const T *din = nullptr;
    int rc = stage_input(ctx, s, in, n, &din);
    if (rc) return rc;
    const Geometry g = geometry(n);
    const uint64_t nwords = (n + 63) / 64;

    Arena &A = ctx->scratch;
    A.reset();
    const size_t o_counts = A.reserve(sizeof(uint64_t) * g.nchunks);
    const size_t o_offs = A.reserve(sizeof(uint64_t) * g.nchunks);
    const size_t o_res = A.reserve(sizeof(uint64_t) * 2);
    SCAN_HIP(A.buf.ensure(A.used));
    uint64_t *counts = A.at<uint64_t>(o_counts);
    uint64_t *offs = A.at<uint64_t>(o_offs);
    uint64_t *res = A.at<uint64_t>(o_res);

    // where the bitvector goes
    uint64_t *bv = nullptr;
    const bool out_dev = out && is_device_pointer(out);
    if (op == Op::kBitvector && out_dev) {
        bv = static_cast<uint64_t *>(out);
    } else if (op != Op::kCount) {
        SCAN_HIP(ctx->scan_aux.ensure(std::max<uint64_t>(nwords, 1) * sizeof(uint64_t)));
        bv = ctx->scan_aux.as<uint64_t>();
    }

    tm.mark(op == Op::kCount ? "scan_count" : "scan_bitvector");
    SCAN_HIP(launch_predicate<T>(din, n, lo, hi, g.rows_per_chunk, g.nchunks, bv, counts, s));
    size_t copy_bytes = 0;
    void *dev_out = nullptr;
    if (op == Op::kCount || op == Op::kBitvector) {
        tm.mark("scan_sum");
        SCAN_HIP(launch_sum(counts, g.nchunks, res, s));
        if (op == Op::kBitvector && !out_dev) {
            dev_out = bv;
            copy_bytes = nwords * sizeof(uint64_t);
        }
    } else {
        tm.mark("scan_chunk_scan");
        SCAN_HIP(launch_chunk_scan(counts, g.nchunks, offs, res, s));
        OutT *o = static_cast<OutT *>(out);
        if (!out_dev) {
            SCAN_HIP(ctx->scan_out.ensure(std::max<size_t>(cap, 1) * sizeof(OutT)));
            o = ctx->scan_out.as<OutT>();
            dev_out = o;
        }
        tm.mark(op == Op::kIndex ? "scan_expand_index" : "scan_expand_values");
        if (op == Op::kIndex)
            SCAN_HIP((launch_expand<T, OutT, 0>(bv, din, n, g.rows_per_chunk, g.nchunks, offs, o, cap, s)));
        else
            SCAN_HIP((launch_expand<T, OutT, 1>(bv, din, n, g.rows_per_chunk, g.nchunks, offs, o, cap, s)));
    }
    tm.end_call();
    SCAN_HIP(hipMemcpyAsync(ctx->host_result, res, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    SCAN_HIP(hipStreamSynchronize(s));
    const uint64_t total = ctx->host_result[0];
    if (result) *result = total;
    if (dev_out && out) {
        if (op == Op::kIndex || op == Op::kValues) copy_bytes = std::min<uint64_t>(total, cap) * sizeof(OutT);
        if (copy_bytes) SCAN_HIP(hipMemcpy(out, dev_out, copy_bytes, hipMemcpyDeviceToHost));
    }
    tm.collect();
    if ((op == Op::kIndex || op == Op::kValues) && total > cap) {
        set_last_error("output capacity " + std::to_string(cap) + " < " + std::to_string(total) + " matches");
        return MI355_ERR_CAPACITY;
    }
    return MI355_OK;
}

inline bool bad(const void *in, size_t n, const void *out, bool need_out) {
    if (!in && n) return true;
    if (need_out && !out && n) return true;
    return false;
}

}  // namespace
}  // namespace scan
}  // namespace sgxamd

using sgxamd::set_last_error;
using sgxamd::scan::Op;
using sgxamd::scan::run;

#define SCAN_ARGCHECK(cond)                     \
    do {                                        \
        if (cond) {                             \
            set_last_error("invalid argument"); \
            return MI355_ERR_INVALID;           \
        }                                       \
    } while (0)

extern "C" {

int mi355_scan_count_u8(uint8_t lo, uint8_t hi, const uint8_t *in, size_t n, uint64_t *count) {
    SCAN_ARGCHECK(sgxamd::scan::bad(in, n, count, true) || !count);
    if (n == 0) { *count = 0; return MI355_OK; }
    return run<uint8_t, uint64_t>(Op::kCount, lo, hi, in, n, nullptr, 0, count);
}

int mi355_scan_count_i32(int32_t lo, int32_t hi, const int32_t *in, size_t n, uint64_t *count) {
    SCAN_ARGCHECK(sgxamd::scan::bad(in, n, count, true) || !count);
    if (n == 0) { *count = 0; return MI355_OK; }
    return run<int32_t, uint64_t>(Op::kCount, lo, hi, in, n, nullptr, 0, count);
}

int mi355_scan_bitvector_u8(uint8_t lo, uint8_t hi, const uint8_t *in, size_t n, uint64_t *out_words) {
    SCAN_ARGCHECK(sgxamd::scan::bad(in, n, out_words, true));
    if (n == 0) return MI355_OK;
    return run<uint8_t, uint64_t>(Op::kBitvector, lo, hi, in, n, out_words, 0, nullptr);
}

int mi355_scan_bitvector_i32(int32_t lo, int32_t hi, const int32_t *in, size_t n, uint64_t *out_words) {
    SCAN_ARGCHECK(sgxamd::scan::bad(in, n, out_words, true));
    if (n == 0) return MI355_OK;
    return run<int32_t, uint64_t>(Op::kBitvector, lo, hi, in, n, out_words, 0, nullptr);
}

int mi355_scan_index_u8(uint8_t lo, uint8_t hi, const uint8_t *in, size_t n, uint64_t *out, size_t cap,
                        uint64_t *n_out) {
    SCAN_ARGCHECK(sgxamd::scan::bad(in, n, out, cap > 0) || !n_out);
    if (n == 0) { *n_out = 0; return MI355_OK; }
    return run<uint8_t, uint64_t>(Op::kIndex, lo, hi, in, n, out, cap, n_out);
}

int mi355_scan_index_i32(int32_t lo, int32_t hi, const int32_t *in, size_t n, uint64_t *out, size_t cap,
                         uint64_t *n_out) {
    SCAN_ARGCHECK(sgxamd::scan::bad(in, n, out, cap > 0) || !n_out);
    if (n == 0) { *n_out = 0; return MI355_OK; }
    return run<int32_t, uint64_t>(Op::kIndex, lo, hi, in, n, out, cap, n_out);
}

int mi355_scan_values_u8(uint8_t lo, uint8_t hi, const uint8_t *in, size_t n, uint32_t *out, size_t cap,
                         uint64_t *n_out) {
    SCAN_ARGCHECK(sgxamd::scan::bad(in, n, out, cap > 0) || !n_out);
    if (n == 0) { *n_out = 0; return MI355_OK; }
    return run<uint8_t, uint32_t>(Op::kValues, lo, hi, in, n, out, cap, n_out);
}

int mi355_scan_values_i32(int32_t lo, int32_t hi, const int32_t *in, size_t n, int32_t *out, size_t cap,
                          uint64_t *n_out) {
    SCAN_ARGCHECK(sgxamd::scan::bad(in, n, out, cap > 0) || !n_out);
    if (n == 0) { *n_out = 0; return MI355_OK; }
    return run<int32_t, int32_t>(Op::kValues, lo, hi, in, n, out, cap, n_out);
}

}  // extern "C"
