// Device-level RHO entry points shared by the C-ABI (rho_host.cpp) and the
// TPC-H pipelines (tpch_host.cpp).
#pragma once

#include "runtime.hpp"
#include "sgxamd/rho.h"

namespace sgxamd {
namespace rho {

// The whole join on device-resident inputs; caller holds ctx->mu.  With
// opts->materialize the matches go to out (capacity out_cap triples); a non-null
// `grow` replaces a too-small out by grow's (enlarged) buffer instead of failing.
int join_device(Context *ctx, hipStream_t s, const row_t *dR, uint64_t nR, const row_t *dS, uint64_t nS,
                const mi355_rho_opts *opts, mi355_rho_stats *st, output_triple_t *out, uint64_t out_cap,
                DeviceBuffer *grow = nullptr);

// Host chunked table (ChunkedTable.cpp layout) holding a copy of n triples.
chunked_table_t *make_chunked_table(const output_triple_t *src, uint64_t n);

}  // namespace rho
}  // namespace sgxamd
