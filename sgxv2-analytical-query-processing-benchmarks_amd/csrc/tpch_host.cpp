// TPC-H Q3/Q10/Q12/Q19 on the GPU: the reference's query pipelines
// (lib/TPCH-Queries/src/tpch.cpp:36-309) with every step device-resident.
//
// Per query: stage the host columns it reads into HBM (timed apart, ms_h2d),
// then run its selections (order-preserving compaction, tpch_kernels.hip), its
// joins (rho::join_device — RHO or RHT build/probe — materialising into a device
// triple buffer where the reference sets MATERIALIZE), and the result transforms
// between them as gathers.  The only host round trips are the sizes the next
// step needs (filtered row counts, join cardinalities).
#include <algorithm>
#include <chrono>
#include <cstring>
#include <string>
#include <vector>

#include "common.hpp"
#include "rho_device.hpp"
#include "rho_internal.hpp"
#include "runtime.hpp"
#include "sgxamd/rho.h"
#include "sgxamd/tpch.h"
#include "tpch_gen.hpp"
#include "tpch_internal.hpp"

namespace sgxamd {
namespace tpch {
namespace {

#define TP_HIP(expr)                                                                          \
    do {                                                                                      \
        hipError_t _e = (expr);                                                               \
        if (_e != hipSuccess) {                                                               \
            set_last_error(std::string("HIP: ") + hipGetErrorString(_e) + " at " #expr);      \
            return (_e == hipErrorOutOfMemory) ? MI355_ERR_OOM : MI355_ERR_HIP;               \
        }                                                                                     \
    } while (0)

#define TP_RC(expr)                \
    do {                           \
        int _rc = (expr);          \
        if (_rc) return _rc;       \
    } while (0)

// One query call: staging, phase events, selection / join / transform steps.
struct Query {
    Context *ctx;
    hipStream_t s;
    int algo;
    int nstaged = 0;
    uint64_t column_bytes = 0;
    std::vector<hipEvent_t> ev;

    ~Query() {
        for (hipEvent_t e : ev) (void)hipEventDestroy(e);
    }

    // Device view of a column: the pointer itself if it is device memory, else a staged copy.
    template <typename T>
    int stage(const T *p, uint64_t n, const T **out, const char *name) {
        if (p == nullptr) {
            if (n == 0) {
                *out = nullptr;
                return MI355_OK;
            }
            set_last_error(std::string("TPC-H column ") + name + " is NULL");
            return MI355_ERR_INVALID;
        }
        column_bytes += n * sizeof(T);
        if (is_device_pointer(p)) {
            *out = p;
            return MI355_OK;
        }
        if (nstaged >= (int)(sizeof(ctx->tp_cols) / sizeof(ctx->tp_cols[0]))) {
            set_last_error("too many staged TPC-H columns");
            return MI355_ERR_INVALID;
        }
        DeviceBuffer &b = ctx->tp_cols[nstaged++];
        TP_HIP(b.ensure(std::max<uint64_t>(n, 1) * sizeof(T)));
        if (n) TP_HIP(hipMemcpyAsync(b.ptr, p, n * sizeof(T), hipMemcpyHostToDevice, s));
        *out = b.as<T>();
        return MI355_OK;
    }

    int mark() {
        hipEvent_t e;
        TP_HIP(hipEventCreate(&e));
        ev.push_back(e);
        TP_HIP(hipEventRecord(e, s));
        return MI355_OK;
    }
    double span(size_t a, size_t b) const {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, ev[a], ev[b]) != hipSuccess) return 0.0;
        return ms;
    }

    // Selection `id` over n rows into dst; *n_out = surviving rows.
    int filter(FilterId id, const FilterCols &c, uint64_t n, DeviceBuffer &dst, uint64_t *n_out) {
        *n_out = 0;
        if (n == 0) return MI355_OK;
        const uint64_t nblk = filter_blocks(n);
        TP_HIP(ctx->tp_mask.ensure(nblk * kFilterThreads * sizeof(uint16_t)));
        TP_HIP(ctx->tp_blk.ensure((2 * nblk + 1) * sizeof(uint64_t)));
        uint64_t *cnt = ctx->tp_blk.as<uint64_t>(), *off = cnt + nblk, *total = off + nblk;
        TP_HIP(launch_filter_mark(id, c, n, ctx->tp_mask.as<uint16_t>(), cnt, s));
        TP_HIP(rho::launch_excl_scan(cnt, nullptr, nblk, off, total, s));
        TP_HIP(hipMemcpyAsync(ctx->host_result, total, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
        TP_HIP(hipStreamSynchronize(s));
        *n_out = ctx->host_result[0];
        TP_HIP(dst.ensure(std::max<uint64_t>(*n_out, 1) * sizeof(row_t)));
        TP_HIP(launch_filter_emit(id, c, n, ctx->tp_mask.as<uint16_t>(), off, dst.as<row_t>(), s));
        return MI355_OK;
    }

    // R ⋈ S; with `mat` the matches land in ctx->tp_trip.
    int join(const row_t *R, uint64_t nR, const row_t *S, uint64_t nS, bool mat, uint64_t *matches) {
        *matches = 0;
        if (nR == 0 || nS == 0) return MI355_OK;
        mi355_rho_opts o{};
        o.algorithm = algo;
        o.materialize = mat ? 1 : 0;
        mi355_rho_stats st{};
        DeviceBuffer &t = ctx->tp_trip;
        TP_RC(rho::join_device(ctx, s, R, nR, S, nS, &o, &st, mat ? t.as<output_triple_t>() : nullptr,
                               mat ? t.bytes / sizeof(output_triple_t) : 0, mat ? &t : nullptr));
        *matches = st.matches;
        return MI355_OK;
    }
};

// Columns of selection `which` (1-based, tpch.cpp order) of `query`, staged.
int selection(Query &q, int query, int which, const CustomerTable *c, const OrdersTable *o, const LineItemTable *l,
              const PartTable *p, FilterId *id, FilterCols *fc, uint64_t *n) {
    *fc = FilterCols{};
    auto need = [](const void *t) {
        if (!t) set_last_error("TPC-H table is NULL");
        return t != nullptr;
    };
    const int key = query * 10 + which;
    switch (key) {
        case 31:  // Q3 customer: c_mktsegment == BUILDING -> c_custkey
            if (!need(c)) return MI355_ERR_INVALID;
            *id = kQ3Customer, *n = c->numTuples;
            TP_RC(q.stage(c->c_custkey, *n, &fc->rows, "c_custkey"));
            return q.stage(c->c_mktsegment, *n, &fc->b0, "c_mktsegment");
        case 32:  // Q3 orders: o_orderdate < 1995-03-15 -> {o_custkey, o_orderkey}
        case 101:  // Q10 orders: 1993-10-01 <= o_orderdate < 1994-01-01 -> {o_custkey, row id}
            if (!need(o)) return MI355_ERR_INVALID;
            *id = key == 32 ? kQ3Orders : kQ10Orders, *n = o->numTuples;
            TP_RC(q.stage(o->o_orderkey, *n, &fc->rows, "o_orderkey"));
            TP_RC(q.stage(o->o_custkey, *n, &fc->keys, "o_custkey"));
            return q.stage(o->o_orderdate, *n, &fc->d0, "o_orderdate");
        case 33:  // Q3 lineitem: l_shipdate >= 1995-03-16 -> l_orderkey
            if (!need(l)) return MI355_ERR_INVALID;
            *id = kQ3Lineitem, *n = l->numTuples;
            TP_RC(q.stage(l->l_orderkey, *n, &fc->rows, "l_orderkey"));
            return q.stage(l->l_shipdate, *n, &fc->d0, "l_shipdate");
        case 102:  // Q10 lineitem: l_returnflag == 'R' -> l_orderkey
            if (!need(l)) return MI355_ERR_INVALID;
            *id = kQ10Lineitem, *n = l->numTuples;
            TP_RC(q.stage(l->l_orderkey, *n, &fc->rows, "l_orderkey"));
            return q.stage(l->l_returnflag, *n, &fc->c0, "l_returnflag");
        case 121:  // Q12 lineitem
            if (!need(l)) return MI355_ERR_INVALID;
            *id = kQ12Lineitem, *n = l->numTuples;
            TP_RC(q.stage(l->l_orderkey, *n, &fc->rows, "l_orderkey"));
            TP_RC(q.stage(l->l_shipmode, *n, &fc->b0, "l_shipmode"));
            TP_RC(q.stage(l->l_shipdate, *n, &fc->d0, "l_shipdate"));
            TP_RC(q.stage(l->l_commitdate, *n, &fc->d1, "l_commitdate"));
            return q.stage(l->l_receiptdate, *n, &fc->d2, "l_receiptdate");
        case 191:  // Q19 part
            if (!need(p)) return MI355_ERR_INVALID;
            *id = kQ19Part, *n = p->numTuples;
            TP_RC(q.stage(p->p_partkey, *n, &fc->rows, "p_partkey"));
            TP_RC(q.stage(p->p_brand, *n, &fc->b0, "p_brand"));
            TP_RC(q.stage(p->p_container, *n, &fc->b1, "p_container"));
            return q.stage(p->p_size, *n, &fc->u0, "p_size");
        case 192:  // Q19 lineitem -> {l_partkey, row id}
            if (!need(l)) return MI355_ERR_INVALID;
            *id = kQ19Lineitem, *n = l->numTuples;
            TP_RC(q.stage(l->l_orderkey, *n, &fc->rows, "l_orderkey"));
            TP_RC(q.stage(l->l_partkey, *n, &fc->keys, "l_partkey"));
            TP_RC(q.stage(l->l_quantity, *n, &fc->f0, "l_quantity"));
            TP_RC(q.stage(l->l_shipmode, *n, &fc->b0, "l_shipmode"));
            return q.stage(l->l_shipinstruct, *n, &fc->b1, "l_shipinstruct");
        default:
            set_last_error("no such TPC-H selection");
            return MI355_ERR_INVALID;
    }
}

// Common prologue: context, lock, stream; staging is timed until begin().
struct Call {
    int status = MI355_OK;
    Context *ctx = nullptr;
    std::unique_lock<std::mutex> lk;
    std::chrono::steady_clock::time_point t0;
    Call() {
        ctx = current_context(&status);
        if (ctx) lk = std::unique_lock<std::mutex>(ctx->mu);
        t0 = std::chrono::steady_clock::now();
    }
};

int finish_staging(Query &q, const Call &call, mi355_tpch_stats *st) {
    TP_HIP(hipStreamSynchronize(q.s));
    st->ms_h2d = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - call.t0).count();
    st->column_bytes = q.column_bytes;
    return q.mark();  // event 0: the query starts
}

int check_algo(int algo) {
    if (algo != MI355_ALGO_RHO && algo != MI355_ALGO_RHT) {
        set_last_error("algorithm must be MI355_ALGO_RHO or MI355_ALGO_RHT");
        return MI355_ERR_INVALID;
    }
    return MI355_OK;
}

}  // namespace
}  // namespace tpch
}  // namespace sgxamd

using namespace sgxamd;
using namespace sgxamd::tpch;

extern "C" {

int mi355_tpch_q3(const CustomerTable *c, const OrdersTable *o, const LineItemTable *l, int algorithm,
                  mi355_tpch_stats *stats) {
    TP_RC(check_algo(algorithm));
    mi355_tpch_stats local{};
    mi355_tpch_stats *st = stats ? stats : &local;
    std::memset(st, 0, sizeof(*st));
    if (!c || !o || !l) {
        set_last_error("Q3 needs customer, orders and lineitem");
        return MI355_ERR_INVALID;
    }
    Call call;
    if (!call.ctx) return call.status;
    Query q{call.ctx, thread_stream(call.ctx, nullptr), algorithm};
    FilterId f1, f2, f3;
    FilterCols c1, c2, c3;
    uint64_t n1, n2, n3;
    TP_RC(selection(q, 3, 1, c, o, l, nullptr, &f1, &c1, &n1));
    TP_RC(selection(q, 3, 2, c, o, l, nullptr, &f2, &c2, &n2));
    TP_RC(selection(q, 3, 3, c, o, l, nullptr, &f3, &c3, &n3));
    st->input_tuples = c->numTuples + o->numTuples + l->numTuples;
    TP_RC(finish_staging(q, call, st));
    Context *ctx = call.ctx;
    // selection 1 + 2, join customers ⋈ orders (materialised), transform, selection 3, join ⋈ lineitem
    TP_RC(q.filter(f1, c1, n1, ctx->tp_rel[0], &st->filtered[0]));
    TP_RC(q.mark());
    TP_RC(q.filter(f2, c2, n2, ctx->tp_rel[1], &st->filtered[1]));
    TP_RC(q.mark());
    TP_RC(q.join(ctx->tp_rel[0].as<row_t>(), st->filtered[0], ctx->tp_rel[1].as<row_t>(), st->filtered[1], true,
                 &st->join_matches[0]));
    TP_RC(q.mark());
    TP_HIP(ctx->tp_rel[2].ensure(std::max<uint64_t>(st->join_matches[0], 1) * sizeof(row_t)));
    TP_HIP(launch_transform(kSpSp, ctx->tp_trip.as<output_triple_t>(), st->join_matches[0], nullptr, nullptr,
                            ctx->tp_rel[2].as<row_t>(), q.s));
    TP_RC(q.mark());
    TP_RC(q.filter(f3, c3, n3, ctx->tp_rel[0], &st->filtered[2]));
    TP_RC(q.mark());
    TP_RC(q.join(ctx->tp_rel[2].as<row_t>(), st->join_matches[0], ctx->tp_rel[0].as<row_t>(), st->filtered[2],
                 false, &st->join_matches[1]));
    TP_RC(q.mark());
    TP_HIP(hipStreamSynchronize(q.s));
    st->ms_selection[0] = q.span(0, 1);
    st->ms_selection[1] = q.span(1, 2);
    st->ms_join[0] = q.span(2, 3);
    st->ms_copy = q.span(3, 4);
    st->ms_selection[2] = q.span(4, 5);
    st->ms_join[1] = q.span(5, 6);
    st->ms_total = q.span(0, 6);
    st->result = st->join_matches[1];
    return MI355_OK;
}

int mi355_tpch_q10(const CustomerTable *c, const OrdersTable *o, const LineItemTable *l, const NationTable *n,
                   int algorithm, mi355_tpch_stats *stats) {
    TP_RC(check_algo(algorithm));
    mi355_tpch_stats local{};
    mi355_tpch_stats *st = stats ? stats : &local;
    std::memset(st, 0, sizeof(*st));
    if (!c || !o || !l || !n) {
        set_last_error("Q10 needs customer, orders, lineitem and nation");
        return MI355_ERR_INVALID;
    }
    Call call;
    if (!call.ctx) return call.status;
    Query q{call.ctx, thread_stream(call.ctx, nullptr), algorithm};
    FilterId f1, f2;
    FilterCols c1, c2;
    uint64_t n1, n2;
    TP_RC(selection(q, 10, 1, c, o, l, nullptr, &f1, &c1, &n1));
    TP_RC(selection(q, 10, 2, c, o, l, nullptr, &f2, &c2, &n2));
    const row_t *cust, *nat, *okey = c1.rows;
    const uint32_t *nationkey;
    TP_RC(q.stage(c->c_custkey, c->numTuples, &cust, "c_custkey"));
    TP_RC(q.stage(c->c_nationkey, c->numTuples, &nationkey, "c_nationkey"));
    TP_RC(q.stage(n->n_nationkey, n->numTuples, &nat, "n_nationkey"));
    st->input_tuples = c->numTuples + o->numTuples + l->numTuples + n->numTuples;
    TP_RC(finish_staging(q, call, st));
    Context *ctx = call.ctx;
    TP_RC(q.filter(f1, c1, n1, ctx->tp_rel[0], &st->filtered[0]));
    TP_RC(q.mark());  // 1
    // customer ⋈ filtered orders, materialised; {c_nationkey[Rp], Sp}
    TP_RC(q.join(cust, c->numTuples, ctx->tp_rel[0].as<row_t>(), st->filtered[0], true, &st->join_matches[0]));
    TP_RC(q.mark());  // 2
    TP_HIP(ctx->tp_rel[1].ensure(std::max<uint64_t>(st->join_matches[0], 1) * sizeof(row_t)));
    TP_HIP(launch_transform(kRpToKeySp, ctx->tp_trip.as<output_triple_t>(), st->join_matches[0], nationkey,
                            nullptr, ctx->tp_rel[1].as<row_t>(), q.s));
    TP_RC(q.mark());  // 3
    // nation ⋈ previous, materialised; {o_orderkey[Sp].key, 0}
    TP_RC(q.join(nat, n->numTuples, ctx->tp_rel[1].as<row_t>(), st->join_matches[0], true, &st->join_matches[1]));
    TP_RC(q.mark());  // 4
    TP_HIP(ctx->tp_rel[2].ensure(std::max<uint64_t>(st->join_matches[1], 1) * sizeof(row_t)));
    TP_HIP(launch_transform(kSpToTuple, ctx->tp_trip.as<output_triple_t>(), st->join_matches[1], nullptr, okey,
                            ctx->tp_rel[2].as<row_t>(), q.s));
    TP_RC(q.mark());  // 5
    TP_RC(q.filter(f2, c2, n2, ctx->tp_rel[0], &st->filtered[1]));
    TP_RC(q.mark());  // 6
    TP_RC(q.join(ctx->tp_rel[2].as<row_t>(), st->join_matches[1], ctx->tp_rel[0].as<row_t>(), st->filtered[1],
                 false, &st->join_matches[2]));
    TP_RC(q.mark());  // 7
    TP_HIP(hipStreamSynchronize(q.s));
    st->ms_selection[0] = q.span(0, 1);
    st->ms_join[0] = q.span(1, 2);
    st->ms_join[1] = q.span(3, 4);
    st->ms_copy = q.span(2, 3) + q.span(4, 5);
    st->ms_selection[1] = q.span(5, 6);
    st->ms_join[2] = q.span(6, 7);
    st->ms_total = q.span(0, 7);
    st->result = st->join_matches[2];
    return MI355_OK;
}

int mi355_tpch_q12(const LineItemTable *l, const OrdersTable *o, int algorithm, mi355_tpch_stats *stats) {
    TP_RC(check_algo(algorithm));
    mi355_tpch_stats local{};
    mi355_tpch_stats *st = stats ? stats : &local;
    std::memset(st, 0, sizeof(*st));
    if (!l || !o) {
        set_last_error("Q12 needs lineitem and orders");
        return MI355_ERR_INVALID;
    }
    Call call;
    if (!call.ctx) return call.status;
    Query q{call.ctx, thread_stream(call.ctx, nullptr), algorithm};
    FilterId f1;
    FilterCols c1;
    uint64_t n1;
    TP_RC(selection(q, 12, 1, nullptr, o, l, nullptr, &f1, &c1, &n1));
    const row_t *ord;
    TP_RC(q.stage(o->o_orderkey, o->numTuples, &ord, "o_orderkey"));
    st->input_tuples = l->numTuples + o->numTuples;
    TP_RC(finish_staging(q, call, st));
    Context *ctx = call.ctx;
    TP_RC(q.filter(f1, c1, n1, ctx->tp_rel[0], &st->filtered[0]));
    TP_RC(q.mark());
    TP_RC(q.join(ord, o->numTuples, ctx->tp_rel[0].as<row_t>(), st->filtered[0], false, &st->join_matches[0]));
    TP_RC(q.mark());
    TP_HIP(hipStreamSynchronize(q.s));
    st->ms_selection[0] = q.span(0, 1);
    st->ms_join[0] = q.span(1, 2);
    st->ms_total = q.span(0, 2);
    st->result = st->join_matches[0];
    return MI355_OK;
}

int mi355_tpch_q19(const LineItemTable *l, const PartTable *p, int algorithm, mi355_tpch_stats *stats,
                   int want_join, chunked_table_t **join_out) {
    TP_RC(check_algo(algorithm));
    mi355_tpch_stats local{};
    mi355_tpch_stats *st = stats ? stats : &local;
    std::memset(st, 0, sizeof(*st));
    if (join_out) *join_out = nullptr;
    if (!l || !p || (want_join && !join_out)) {
        set_last_error("Q19 needs lineitem and part (and join_out when want_join)");
        return MI355_ERR_INVALID;
    }
    Call call;
    if (!call.ctx) return call.status;
    Query q{call.ctx, thread_stream(call.ctx, nullptr), algorithm};
    FilterId f1, f2;
    FilterCols c1, c2;
    uint64_t n1, n2;
    TP_RC(selection(q, 19, 1, nullptr, nullptr, l, p, &f1, &c1, &n1));
    TP_RC(selection(q, 19, 2, nullptr, nullptr, l, p, &f2, &c2, &n2));
    st->input_tuples = l->numTuples + p->numTuples;
    TP_RC(finish_staging(q, call, st));
    Context *ctx = call.ctx;
    TP_RC(q.filter(f1, c1, n1, ctx->tp_rel[0], &st->filtered[0]));
    TP_RC(q.mark());
    TP_RC(q.filter(f2, c2, n2, ctx->tp_rel[1], &st->filtered[1]));
    TP_RC(q.mark());
    TP_RC(q.join(ctx->tp_rel[0].as<row_t>(), st->filtered[0], ctx->tp_rel[1].as<row_t>(), st->filtered[1], true,
                 &st->join_matches[0]));
    TP_RC(q.mark());
    // the final predicate over (part row, lineitem row) of every join match
    TP_HIP(ctx->tp_blk.ensure(sizeof(uint64_t)));
    uint64_t *count = ctx->tp_blk.as<uint64_t>();
    TP_HIP(launch_q19_final(ctx->tp_trip.as<output_triple_t>(), st->join_matches[0], c1.b0, c1.b1, c1.u0, c2.f0,
                            count, q.s));
    TP_RC(q.mark());
    TP_HIP(hipMemcpyAsync(ctx->host_result, count, sizeof(uint64_t), hipMemcpyDeviceToHost, q.s));
    TP_HIP(hipStreamSynchronize(q.s));
    st->result = ctx->host_result[0];
    st->ms_selection[0] = q.span(0, 1);
    st->ms_selection[1] = q.span(1, 2);
    st->ms_join[0] = q.span(2, 3);
    st->ms_selection[2] = q.span(3, 4);
    st->ms_total = q.span(0, 4);
    if (want_join) {  // the reference's result->result: the materialised join 1, as a host chunked table
        std::vector<output_triple_t> host(st->join_matches[0]);
        if (!host.empty())
            TP_HIP(hipMemcpy(host.data(), ctx->tp_trip.ptr, host.size() * sizeof(output_triple_t),
                             hipMemcpyDeviceToHost));
        *join_out = rho::make_chunked_table(host.data(), host.size());
        if (!*join_out) {
            set_last_error("out of host memory for the chunked table");
            return MI355_ERR_OOM;
        }
    }
    return MI355_OK;
}

int mi355_tpch_filter(int query, int which, const CustomerTable *c, const OrdersTable *o, const LineItemTable *l,
                      const PartTable *p, row_t *out, uint64_t capacity, uint64_t *n_out) {
    if (n_out) *n_out = 0;
    if (!n_out || (capacity && !out)) {
        set_last_error("mi355_tpch_filter: n_out (and out) required");
        return MI355_ERR_INVALID;
    }
    Call call;
    if (!call.ctx) return call.status;
    Query q{call.ctx, thread_stream(call.ctx, nullptr), MI355_ALGO_RHO};
    FilterId id;
    FilterCols fc;
    uint64_t n;
    TP_RC(selection(q, query, which, c, o, l, p, &id, &fc, &n));
    DeviceBuffer &dst = call.ctx->tp_rel[0];
    uint64_t k = 0;
    TP_RC(q.filter(id, fc, n, dst, &k));
    *n_out = k;
    if (k > capacity) {
        TP_HIP(hipStreamSynchronize(q.s));
        set_last_error("filter output too small: " + std::to_string(k) + " rows needed");
        return MI355_ERR_CAPACITY;
    }
    if (k) TP_HIP(hipMemcpyAsync(out, dst.ptr, k * sizeof(row_t), hipMemcpyDefault, q.s));
    TP_HIP(hipStreamSynchronize(q.s));
    return MI355_OK;
}

int mi355_tpch_generate_dev(uint32_t sm, uint64_t seed, const LineItemTable *l, const OrdersTable *o,
                            const CustomerTable *c, const PartTable *p, const NationTable *n, void *stream) {
    if (sm == 0) {
        set_last_error("scale_milli must be > 0");
        return MI355_ERR_INVALID;
    }
    Call call;
    if (!call.ctx) return call.status;
    hipStream_t s = thread_stream(call.ctx, stream);
    const CustomerTable c0{};
    const PartTable p0{};
    const NationTable n0{};
    const OrdersTable o0{};
    TP_HIP(launch_gen_simple(sm, seed, c ? *c : c0, p ? *p : p0, n ? *n : n0, o ? *o : o0, s));
    if (l) {
        const uint64_t nblk = (n_orders(sm) + kGenOrdersPerBlock - 1) / kGenOrdersPerBlock;
        TP_HIP(call.ctx->tp_blk.ensure((2 * nblk + 1) * sizeof(uint64_t)));
        uint64_t *cnt = call.ctx->tp_blk.as<uint64_t>(), *off = cnt + nblk, *total = off + nblk;
        TP_HIP(launch_gen_lines_per_block(sm, seed, cnt, s));
        TP_HIP(rho::launch_excl_scan(cnt, nullptr, nblk, off, total, s));
        TP_HIP(launch_gen_lineitem(sm, seed, off, *l, s));
    }
    TP_HIP(hipStreamSynchronize(s));
    return MI355_OK;
}

}  // extern "C"
