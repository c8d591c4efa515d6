// Internal interface between the TPC-H kernels (tpch_kernels.hip) and the query
// pipelines (tpch_host.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "sgxamd/tpch.h"

namespace sgxamd {
namespace tpch {

// The selections of the four queries, in tpch.cpp order.
enum FilterId : int {
    kQ3Customer = 0,  // Q3Predicates.hpp:166-174
    kQ3Orders,        // :176-185
    kQ3Lineitem,      // :187-195
    kQ10Orders,       // Q10Predicates.hpp:26-35
    kQ10Lineitem,     // :37-45
    kQ12Lineitem,     // Q12Predicates.hpp:22-37
    kQ19Part,         // Q19Predicates.hpp:40-55
    kQ19Lineitem,     // :27-38
    kNumFilters
};

// Device column pointers a selection reads (unused ones null).
struct FilterCols {
    const row_t *rows = nullptr;     // the table's key/row-id column (c_custkey, o_orderkey, ...)
    const uint32_t *keys = nullptr;  // o_custkey / l_partkey
    const uint64_t *d0 = nullptr, *d1 = nullptr, *d2 = nullptr;  // date columns
    const uint8_t *b0 = nullptr, *b1 = nullptr;                  // 1-byte codes
    const uint32_t *u0 = nullptr;    // p_size
    const float *f0 = nullptr;       // l_quantity
    const char *c0 = nullptr;        // l_returnflag
};

constexpr int kFilterThreads = 256;
constexpr int kFilterItems = 16;
constexpr uint64_t kFilterSeg = (uint64_t)kFilterThreads * kFilterItems;  // rows per workgroup

inline uint64_t filter_blocks(uint64_t n) { return (n + kFilterSeg - 1) / kFilterSeg; }

// Pass 1: predicate bits (u16 per thread, mask[nblk * kFilterThreads]) and per-block counts.
hipError_t launch_filter_mark(FilterId id, const FilterCols &c, uint64_t n, uint16_t *mask, uint64_t *blk_count,
                              hipStream_t s);
// Pass 2: order-preserving compaction of the marked rows to out[blk_off[b] + ...].
hipError_t launch_filter_emit(FilterId id, const FilterCols &c, uint64_t n, const uint16_t *mask,
                              const uint64_t *blk_off, row_t *out, hipStream_t s);

// Join-result transforms (result_transformers.hpp:50-64), triples -> rows.
enum TransformId : int {
    kSpSp = 0,      // copy_Sp_Sp: {Spayload, Spayload}
    kRpToKeySp,     // copy_RpToKeySp: {lookup_key[Rpayload], Spayload}
    kSpToTuple,     // copy_SpToTupleST: {lookup_rows[Spayload].key, 0}
};
hipError_t launch_transform(TransformId id, const output_triple_t *t, uint64_t n, const uint32_t *lookup_key,
                            const row_t *lookup_rows, row_t *out, hipStream_t s);

// Q19's predicate over the join result (Q19Predicates.hpp:57-78): *count += matches.
hipError_t launch_q19_final(const output_triple_t *t, uint64_t n, const uint8_t *p_brand,
                            const uint8_t *p_container, const uint32_t *p_size, const float *l_quantity,
                            uint64_t *count, hipStream_t s);

// Synthetic tables in HBM (tpch_gen.hpp).  lines_off: n_orders + 1 exclusive prefix of
// lineitems per order, built by launch_gen_order_lines + a scan.
hipError_t launch_gen_simple(uint32_t scale_milli, uint64_t seed, const CustomerTable &c, const PartTable &p,
                             const NationTable &n, const OrdersTable &o, hipStream_t s);
hipError_t launch_gen_lines_per_block(uint32_t scale_milli, uint64_t seed, uint64_t *blk_lines, hipStream_t s);
hipError_t launch_gen_lineitem(uint32_t scale_milli, uint64_t seed, const uint64_t *blk_off,
                               const LineItemTable &l, hipStream_t s);
constexpr uint64_t kGenOrdersPerBlock = 8192;

}  // namespace tpch
}  // namespace sgxamd
