// Host side of the MI355X predicate scan: the C-ABI of sgxamd/scan.h.
//
// Each entry point is the blocking equivalent of one SIMD512:: call
// (SIMD512.hpp:39-84).  Inputs/outputs may live in host or device memory; host
// buffers are staged through HBM.  Device inputs that are not 16-byte aligned
// are copied to an aligned buffer first (the kernels load 16 bytes per lane).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <type_traits>

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

enum class Op { kCount, kBitvector, kIndex, kValues, kExplicit };

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

// kExplicit: SIMD512::explicit_index_scan, the outputs are entries of the index array
// `aux` (aux_len u64 entries, host or device) instead of row numbers.
template <typename T, typename OutT>
int run(Op op, T lo, T hi, const T *in, size_t n, void *out, size_t cap, uint64_t *result,
        const uint64_t *aux = nullptr, uint64_t aux_len = 0) {
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
    const int64_t *daux = reinterpret_cast<const int64_t *>(aux);
    if (op == Op::kExplicit && aux_len && !is_device_pointer(aux)) {
        SCAN_HIP(ctx->scan_dict.ensure(aux_len * sizeof(uint64_t)));
        SCAN_HIP(hipMemcpyAsync(ctx->scan_dict.ptr, aux, aux_len * sizeof(uint64_t), hipMemcpyHostToDevice, s));
        daux = ctx->scan_dict.as<int64_t>();
    }
    const bool selects = op == Op::kIndex || op == Op::kValues || op == Op::kExplicit;

    Arena &A = ctx->scratch;
    A.reset();
    const size_t o_counts = A.reserve(sizeof(uint64_t) * g.nchunks);
    const size_t o_res = A.reserve(sizeof(uint64_t) * 2);
    const size_t o_status = A.reserve(sizeof(uint64_t) * (selects ? select_chunks(n) : 0) + 16);
    SCAN_HIP(A.buf.ensure(A.used));
    uint64_t *counts = A.at<uint64_t>(o_counts);
    uint64_t *res = A.at<uint64_t>(o_res);
    uint64_t *sel_status = A.at<uint64_t>(o_status) + 2;
    uint32_t *ticket = A.at<uint32_t>(o_status);

    const bool out_dev = out && is_device_pointer(out);
    if (selects) {  // one pass: k_select with a decoupled look-back
        OutT *o = static_cast<OutT *>(out);
        if (!out_dev) {
            SCAN_HIP(ctx->scan_out.ensure(std::max<size_t>(cap, 1) * sizeof(OutT)));
            o = ctx->scan_out.as<OutT>();
        }
        tm.mark(op == Op::kIndex ? "scan_select_index" : op == Op::kValues ? "scan_select_values"
                                                                              : "scan_select_explicit");
        if (op == Op::kIndex)
            SCAN_HIP((launch_select<T, OutT, 0>(din, n, lo, hi, ticket, sel_status, o, cap, res, s)));
        else if (op == Op::kValues)
            SCAN_HIP((launch_select<T, OutT, 1>(din, n, lo, hi, ticket, sel_status, o, cap, res, s)));
        else if constexpr (std::is_same<T, uint8_t>::value && std::is_same<OutT, uint64_t>::value)
            SCAN_HIP((launch_select<T, OutT, 3>(din, n, lo, hi, ticket, sel_status, o, cap, res, s, daux, aux_len)));
        tm.end_call();
        SCAN_HIP(hipMemcpyAsync(ctx->host_result, res, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
        SCAN_HIP(hipMemcpyAsync(ctx->host_result + 1, ticket, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        SCAN_HIP(hipStreamSynchronize(s));
        const uint64_t total = ctx->host_result[0];
        const uint32_t flags = reinterpret_cast<const uint32_t *>(ctx->host_result + 1)[1];
        if (flags & 1u) {
            set_last_error("one-pass selection: look-back poll gave up");
            return MI355_ERR_HIP;
        }
        if (flags & 2u) {
            set_last_error("explicit_index_scan: a match's index entry lies past the index array");
            return MI355_ERR_INVALID;
        }
        if (result) *result = total;
        if (!out_dev && out && total)
            SCAN_HIP(hipMemcpy(out, o, std::min<uint64_t>(total, cap) * sizeof(OutT), hipMemcpyDeviceToHost));
        tm.collect();
        if (total > cap) {
            set_last_error("output capacity " + std::to_string(cap) + " < " + std::to_string(total) + " matches");
            return MI355_ERR_CAPACITY;
        }
        return MI355_OK;
    }
    // where the bitvector goes
    uint64_t *bv = nullptr;
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
    tm.mark("scan_sum");
    SCAN_HIP(launch_sum(counts, g.nchunks, res, s));
    if (op == Op::kBitvector && !out_dev) {
        dev_out = bv;
        copy_bytes = nwords * sizeof(uint64_t);
    }
    tm.end_call();
    SCAN_HIP(hipMemcpyAsync(ctx->host_result, res, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    SCAN_HIP(hipStreamSynchronize(s));
    if (result) *result = ctx->host_result[0];
    if (dev_out && out && copy_bytes) SCAN_HIP(hipMemcpy(out, dev_out, copy_bytes, hipMemcpyDeviceToHost));
    tm.collect();
    return MI355_OK;
}

// SIMD512::sum (SIMD512.cpp:34-88): sum of the u8 codes in [lo, hi].
int run_sum_u8(uint8_t lo, uint8_t hi, const uint8_t *in, size_t n, uint64_t *sum) {
    int status = MI355_OK;
    Context *ctx = current_context(&status);
    if (!ctx) return status;
    std::lock_guard<std::mutex> lk(ctx->mu);
    hipStream_t s = thread_stream(ctx, nullptr);
    Timer &tm = thread_timer();
    tm.begin_call(s, thread_timing_enabled());
    const uint8_t *din = nullptr;
    int rc = stage_input(ctx, s, in, n, &din);
    if (rc) return rc;
    const Geometry g = geometry(n);
    Arena &A = ctx->scratch;
    A.reset();
    const size_t o_counts = A.reserve(sizeof(uint64_t) * g.nchunks);
    const size_t o_res = A.reserve(sizeof(uint64_t) * 2);
    SCAN_HIP(A.buf.ensure(A.used));
    tm.mark("scan_sum_values");
    SCAN_HIP(launch_sum_u8(din, n, lo, hi, g.rows_per_chunk, g.nchunks, A.at<uint64_t>(o_counts), s));
    tm.mark("scan_sum");
    SCAN_HIP(launch_sum(A.at<uint64_t>(o_counts), g.nchunks, A.at<uint64_t>(o_res), s));
    tm.end_call();
    SCAN_HIP(hipMemcpyAsync(ctx->host_result, A.at<uint64_t>(o_res), sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    SCAN_HIP(hipStreamSynchronize(s));
    tm.collect();
    *sum = ctx->host_result[0];
    return MI355_OK;
}

// dict_scan_{8,16,32}bit_64bit (SIMD512.cpp:289-338, 531-579, 581-629): the value
// predicate [lo, hi] becomes a code range through the dictionary exactly as the
// reference computes it, including its casts: codes [(C)lo_idx, (C)(hi_end - 1)]
// with C = uint8_t / uint16_t / uint16_t (the 32-bit variant casts its indexes to
// uint16_t too, :588-589); then the matching codes are decoded to dict[code] in
// row order.  CodeT is the code width, CastT the reference's index cast.
template <typename CodeT, typename CastT>
int run_dict(int64_t lo, int64_t hi, const int64_t *dict, uint64_t dict_size, const CodeT *in, size_t n,
             int64_t *out, size_t cap, uint64_t *n_out) {
    int status = MI355_OK;
    Context *ctx = current_context(&status);
    if (!ctx) return status;
    std::lock_guard<std::mutex> lk(ctx->mu);
    hipStream_t s = thread_stream(ctx, nullptr);
    Timer &tm = thread_timer();
    tm.begin_call(s, thread_timing_enabled());

    const int64_t *ddict = dict;
    if (!is_device_pointer(dict)) {
        SCAN_HIP(ctx->scan_dict.ensure(dict_size * sizeof(int64_t)));
        SCAN_HIP(hipMemcpyAsync(ctx->scan_dict.ptr, dict, dict_size * sizeof(int64_t), hipMemcpyHostToDevice, s));
        ddict = ctx->scan_dict.as<int64_t>();
    }
    const CodeT *din = nullptr;
    int rc = stage_input(ctx, s, in, n, &din);
    if (rc) return rc;
    Arena &A = ctx->scratch;
    A.reset();
    const size_t o_res = A.reserve(sizeof(uint64_t) * 2);
    const size_t o_range = A.reserve(sizeof(uint64_t) * 2);
    const size_t o_status = A.reserve(sizeof(uint64_t) * select_chunks(n) + 16);
    SCAN_HIP(A.buf.ensure(A.used));
    uint64_t *range = A.at<uint64_t>(o_range);
    tm.mark("dict_range");
    const uint64_t init[2] = {dict_size, dict_size};
    SCAN_HIP(hipMemcpyAsync(range, init, sizeof(init), hipMemcpyHostToDevice, s));
    SCAN_HIP(launch_dict_range(ddict, dict_size, lo, hi, range, s));
    SCAN_HIP(hipMemcpyAsync(ctx->host_result, range, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    SCAN_HIP(hipStreamSynchronize(s));
    const CodeT clo = (CodeT)(CastT)ctx->host_result[0];
    const CodeT chi = (CodeT)(CastT)(int64_t)(ctx->host_result[1] - 1);

    uint64_t *res = A.at<uint64_t>(o_res);
    const bool out_dev = out && is_device_pointer(out);
    int64_t *o = out;
    if (!out_dev) {
        SCAN_HIP(ctx->scan_out.ensure(std::max<size_t>(cap, 1) * sizeof(int64_t)));
        o = ctx->scan_out.as<int64_t>();
    }
    tm.mark("dict_select");
    SCAN_HIP((launch_select<CodeT, int64_t, 2>(din, n, clo, chi, A.at<uint32_t>(o_status),
                                               A.at<uint64_t>(o_status) + 2, o, cap, res, s, ddict)));
    tm.end_call();
    SCAN_HIP(hipMemcpyAsync(ctx->host_result, res, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    SCAN_HIP(hipMemcpyAsync(ctx->host_result + 1, A.at<uint32_t>(o_status), 2 * sizeof(uint32_t),
                            hipMemcpyDeviceToHost, s));
    SCAN_HIP(hipStreamSynchronize(s));
    const uint64_t total = ctx->host_result[0];
    if (reinterpret_cast<const uint32_t *>(ctx->host_result + 1)[1] != 0) {
        set_last_error("one-pass selection: look-back poll gave up");
        return MI355_ERR_HIP;
    }
    *n_out = total;
    if (!out_dev && out && total) SCAN_HIP(hipMemcpy(out, o, std::min<uint64_t>(total, cap) * sizeof(int64_t),
                                                     hipMemcpyDeviceToHost));
    tm.collect();
    if (total > cap) {
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
using sgxamd::scan::run_dict;

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

int mi355_scan_explicit_index_u8(uint8_t lo, uint8_t hi, const uint64_t *index, size_t index_len, const uint8_t *in,
                                 size_t n, uint64_t *out, size_t cap, uint64_t *n_out) {
    SCAN_ARGCHECK(sgxamd::scan::bad(in, n, out, cap > 0) || !n_out || (!index && index_len));
    if (n == 0) { *n_out = 0; return MI355_OK; }
    return run<uint8_t, uint64_t>(Op::kExplicit, lo, hi, in, n, out, cap, n_out, index, index_len);
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

int mi355_scan_sum_u8(uint8_t lo, uint8_t hi, const uint8_t *in, size_t n, uint64_t *sum) {
    SCAN_ARGCHECK(sgxamd::scan::bad(in, n, sum, true) || !sum);
    if (n == 0) { *sum = 0; return MI355_OK; }
    return sgxamd::scan::run_sum_u8(lo, hi, in, n, sum);
}

int mi355_dict_scan_8bit_64bit(int64_t lo, int64_t hi, const int64_t *dict, const uint8_t *in, size_t n,
                               int64_t *out, size_t cap, uint64_t *n_out) {
    SCAN_ARGCHECK(sgxamd::scan::bad(in, n, out, cap > 0) || !n_out || !dict);
    if (n == 0) { *n_out = 0; return MI355_OK; }
    return run_dict<uint8_t, uint8_t>(lo, hi, dict, 256, in, n, out, cap, n_out);
}

int mi355_dict_scan_16bit_64bit(int64_t lo, int64_t hi, const int64_t *dict, const uint16_t *in, size_t n,
                                int64_t *out, size_t cap, uint64_t *n_out) {
    SCAN_ARGCHECK(sgxamd::scan::bad(in, n, out, cap > 0) || !n_out || !dict);
    if (n == 0) { *n_out = 0; return MI355_OK; }
    return run_dict<uint16_t, uint16_t>(lo, hi, dict, 65536, in, n, out, cap, n_out);
}

int mi355_dict_scan_32bit_64bit(int64_t lo, int64_t hi, const int64_t *dict, size_t dict_size, const uint32_t *in,
                                size_t n, int64_t *out, size_t cap, uint64_t *n_out) {
    SCAN_ARGCHECK(sgxamd::scan::bad(in, n, out, cap > 0) || !n_out || !dict || dict_size == 0);
    if (n == 0) { *n_out = 0; return MI355_OK; }
    return run_dict<uint32_t, uint16_t>(lo, hi, dict, dict_size, in, n, out, cap, n_out);
}

}  // extern "C"
