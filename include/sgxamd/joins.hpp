// sgxamd/joins.hpp — C++-linkage drop-ins for the reference's join entry points.
//
// Same declarations (and therefore the same mangled symbols) as the reference:
//   result_t *RHO(const table_t*, const table_t*, const joinconfig_t*)
//       Join-Benchmarks/lib/Joins/include/radix/radix_join.h:29-30   (_Z3RHOPK7table_tS1_PK12joinconfig_t)
//   result_t *RHT(const table_t*, const table_t*, const joinconfig_t*)
//       radix_join.h (RHT, implemented at radix_join.cpp:1645-1648)    (_Z3RHTPK7table_tS1_PK12joinconfig_t)
//   void run_join(result_t*, const table_t*, const table_t*, const char*, const joinconfig_t*)
//       Join-Benchmarks/lib/Joins/include/joins.hpp / src/joins.cpp:55-78
// so an unmodified run_join-style caller (App/TEEBench/native.cpp:137, the TPC-H
// queries) links against libsgxamd.so instead of the CPU join library.
// With config->MATERIALIZE = 1 the result carries the reference's chunked_table_t
// (result_type 1; release with mi355_free_chunked_table).
// RHO() / RHT() run the join on the current MI355X, prints the reference's timing log
// lines (radix_join.cpp:252-293) and exits on error like the reference
// (ocall_exit(EXIT_FAILURE)); the returned result_t is malloc'd by the callee.
#pragma once

#include "sgxamd/data_types.h"

result_t *RHO(const table_t *relR, const table_t *relS, const joinconfig_t *config);
result_t *RHT(const table_t *relR, const table_t *relS, const joinconfig_t *config);

void run_join(result_t *res, const table_t *relR, const table_t *relS, const char *algorithm_name,
              const joinconfig_t *config);
