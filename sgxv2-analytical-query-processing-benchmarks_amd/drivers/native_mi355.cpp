// native_mi355 — the reference's native join driver (Join-Benchmarks/App/TEEBench/native.cpp)
// running RHO or RHT (-a) on an MI355X through run_join() of libsgxamd.so; -m materialises
// the result into the reference's chunked table (CHUNKED_TABLE build).
//
// Same CLI (commons.cpp:10-190 getopt "a:c:d:e:l:n:mr:s:t:u:x:y:z:hv"), the same
// relation generation (seeds 11111 / 22222, pk R, fk / fk_sel / Zipf S: native.cpp:62-101,
// with Zipf seeded by the S seed because the reference's std::random_device seed is
// not reproducible), and the same closing log lines (native.cpp:140-144).
#include <getopt.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "sgxamd/generator.h"
#include "sgxamd/joins.hpp"
#include "sgxamd/rho.h"

int main(int argc, char **argv) {
    uint64_t r_size = 2097152, s_size = 2097152;
    unsigned r_seed = 11111, s_seed = 22222;
    int nthreads = 2, selectivity = 100, materialize = 0;
    double skew = 0;
    char algorithm[128] = "RHO";
    static struct option long_options[] = {{"sort-r", no_argument, nullptr, 1},
                                           {"sort-s", no_argument, nullptr, 2},
                                           {"mitigation", no_argument, nullptr, 3},
                                           {nullptr, 0, nullptr, 0}};
    int c, idx = 0;
    while ((c = getopt_long(argc, argv, "a:c:d:e:l:n:mr:s:t:u:x:y:z:hv", long_options, &idx)) != -1) {
        switch (c) {
            case 'a': std::snprintf(algorithm, sizeof(algorithm), "%s", optarg); break;
            case 'd':
                if (!std::strcmp(optarg, "cache-fit")) { r_size = 10ull * 1024 * 1024 / 8; s_size = 40ull * 1024 * 1024 / 8; }
                else if (!std::strcmp(optarg, "cache-exceed")) { r_size = 100ull * 1024 * 1024 / 8; s_size = 400ull * 1024 * 1024 / 8; }
                else if (!std::strcmp(optarg, "L")) { r_size = 50000000; s_size = 200000000; }
                break;
            case 'l': selectivity = std::atoi(optarg); break;
            case 'm': materialize = 1; break;
            case 'n': nthreads = std::atoi(optarg); break;
            case 'r': r_size = std::strtoull(optarg, nullptr, 10); break;
            case 's': s_size = std::strtoull(optarg, nullptr, 10); break;
            case 'x': r_size = std::strtoull(optarg, nullptr, 10) * 1024 * 1024 / 8; break;
            case 'y': s_size = std::strtoull(optarg, nullptr, 10) * 1024 * 1024 / 8; break;
            case 'z': skew = std::atof(optarg); break;
            case 'h': std::printf("native_mi355 -a RHO|RHT -r N -s N [-l sel] [-z theta] [-n threads] [-m]\n"); return 0;
            default: break;
        }
    }
    std::vector<row_t> R(r_size), S(s_size);
    std::printf("[INFO] Build relation R with size = %.2lf MB (%lu tuples)\n", 8.0 * r_size / 1048576.0,
                (unsigned long)r_size);
    mi355_gen_seed(r_seed);
    mi355_gen_pk(R.data(), r_size);
    std::printf("[INFO] Build relation S with size = %.2lf MB (%lu tuples)\n", 8.0 * s_size / 1048576.0,
                (unsigned long)s_size);
    mi355_gen_seed(s_seed);
    if (skew > 0) {
        mi355_gen_zipf(S.data(), s_size, (uint32_t)r_size, skew, s_seed,
                       (int)std::max(1u, std::thread::hardware_concurrency()));
    } else if (selectivity != 100) {
        const uint32_t maxid = selectivity != 0 ? (uint32_t)(100 * r_size / selectivity) : 0;
        mi355_gen_fk_sel(S.data(), s_size, maxid);
    } else {
        mi355_gen_fk(S.data(), s_size, (int64_t)r_size);
    }
    table_t tR{R.data(), r_size, 0, 0}, tS{S.data(), s_size, 0, 0};
    joinconfig_t cfg{};
    cfg.NTHREADS = nthreads;
    cfg.MATERIALIZE = materialize;
    result_t res{};
    const auto t0 = std::chrono::steady_clock::now();
    run_join(&res, &tR, &tS, algorithm, &cfg);
    const double time_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::printf("[INFO] Total join runtime: %.2fs\n", time_s);
    std::printf("[INFO] throughput = %.2lf [M rec / s]\n", (double)(r_size + s_size) / time_s);
    std::printf("[INFO] Matches = %lu\n", (unsigned long)res.totalresults);
    if (res.materialized && res.result_type == 1) {
        auto *t = static_cast<chunked_table_t *>(res.result);
        std::printf("[INFO] Materialized %lu tuples in %lu chunks\n", (unsigned long)t->num_tuples,
                    (unsigned long)t->num_chunks);
        mi355_free_chunked_table(t);
    }
    return 0;
}
