// TPC-H driver with the reference's CLI (App/TpcH/TpcHNative.cpp:12-102,
// TpcHCommons.cpp:93-139): -a algorithm (RHO|RHT), -q query (3|10|12|19),
// -s scale (tables under $SGXAMD_TPCH_DATA/scale%03d, default ../data),
// -n threads (reported only), -b bits (ignored, as RADIXBITS = -1 in the reference).
// Extra: -g <scale_milli> runs on synthetic tables generated in memory instead
// of loading them (sgxamd/tpch.h generator), -G <root> writes them to disk first.
// The reference's memory hogging (TpcHNative.cpp:45-66) tunes glibc malloc for the
// CPU joins; it has no role for device-resident joins and is omitted.
#include <getopt.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "sgxamd/rho.h"
#include "sgxamd/tpch.h"
#include "sgxamd/tpch.hpp"

int main(int argc, char **argv) {
    char algorithm[128] = "RHO";
    int query = 12, threads = 4, scale = 1;
    long gen_milli = 0;
    const char *gen_root = nullptr;
    int c;
    while ((c = getopt(argc, argv, "a:b:n:q:s:pg:G:")) != -1) {
        switch (c) {
            case 'a': std::snprintf(algorithm, sizeof(algorithm), "%s", optarg); break;
            case 'n': threads = std::atoi(optarg); break;
            case 'q': query = std::atoi(optarg); break;
            case 's': scale = std::atoi(optarg); break;
            case 'g': gen_milli = std::atol(optarg); break;
            case 'G': gen_root = optarg; break;
            default: break;
        }
    }
    joinconfig_t cfg{};
    cfg.NTHREADS = threads;
    cfg.RADIXBITS = -1;
    std::printf("************* TPC-H APP (MI355X) *************\n");
    std::printf("Run Q%d (scale %d) with join algorithm %s (%d threads)\n", query, scale, algorithm, threads);

    LineItemTable l{};
    OrdersTable o{};
    CustomerTable cu{};
    PartTable p{};
    NationTable n{};
    if (gen_milli > 0) {
        if (mi355_tpch_generate((uint32_t)gen_milli, 0, &l, &o, &cu, &p, &n) != 0) {
            std::fprintf(stderr, "table generation failed\n");
            return 1;
        }
        if (gen_root && mi355_tpch_store(gen_root, scale, &l, &o, &cu, &p, &n) != 0) {
            std::fprintf(stderr, "storing tables under %s failed\n", gen_root);
            return 1;
        }
    } else {
        std::printf("Loading tables from storage.\n");
        const uint8_t q = (uint8_t)query, s = (uint8_t)scale;
        if (load_orders_from_binary(&o, q, s) || load_customers_from_binary(&cu, q, s) ||
            load_parts_from_binary(&p, q, s) || load_nations_from_binary(&n, q, s) ||
            load_lineitems_from_binary(&l, q, s)) {
            std::fprintf(stderr, "loading tables from %s failed\n", getPath(scale, "").c_str());
            return 1;
        }
    }
    result_t result{};
    switch (query) {
        case 3: tpch_q3(&result, &cu, &o, &l, algorithm, &cfg); break;
        case 10: tpch_q10(&result, &cu, &o, &l, &n, algorithm, &cfg); break;
        case 12: tpch_q12(&result, &l, &o, algorithm, &cfg); break;
        case 19: tpch_q19(&result, &l, &p, algorithm, &cfg); break;
        default: std::fprintf(stderr, "TPC-H Q%d is not supported\n", query); return 1;
    }
    std::printf("Query result: %ld\n", (long)result.totalresults);
    std::printf("Query completed\n");
    if (result.result_type == 1 && result.result) mi355_free_chunked_table(static_cast<chunked_table_t *>(result.result));
    free_orders(&o);
    free_part(&p);
    free_customer(&cu);
    free_lineitem(&l);
    free_nation(&n);
    return 0;
}
