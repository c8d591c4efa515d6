/*
 * sgxamd/data_types.h — relation / result / config layouts of the RHO boundary.
 *
 * These structs are layout-compatible with the reference's
 *   Join-Benchmarks/lib/SharedHeaders/include/data-types.h
 * (row_t :44-47, table_t :49-54, algorithm_t :94-97, result_t :107-114,
 *  joinconfig_t :162-176) so that a caller compiled against the reference's
 * header can hand its relations to this library unchanged.  The sizes and
 * offsets are pinned by the static asserts at the bottom (x86-64 / LP64).
 *
 * Plain C: the C-ABI (sgxamd/rho.h) is declared in terms of these types.
 */
#ifndef SGXAMD_DATA_TYPES_H
#define SGXAMD_DATA_TYPES_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef uint32_t type_key;   /* data-types.h:33 */
typedef uint32_t type_value; /* data-types.h:34 */

/* data-types.h:44-47: one 8-byte AoS tuple. */
struct row_t {
    type_key key;
    type_value payload;
};
typedef struct row_t tuple_t;

/* data-types.h:49-54: caller-owned relation handle (24 bytes). */
struct table_t {
    struct row_t *tuples;
    uint64_t num_tuples;
    int ratio_holes;
    int sorted;
};
typedef struct table_t relation_t;

/* data-types.h:72-76: one materialised join result (12 bytes). */
struct output_triple_t {
    type_key key;
    type_value Rpayload;
    type_value Spayload;
};

/* data-types.h:78-92: the reference's CHUNKED_TABLE result (CSKB = 16). */
#define SGXAMD_CHUNK_SIZE (1024 * 16)
#define SGXAMD_TUPLES_PER_CHUNK ((SGXAMD_CHUNK_SIZE - 8) / sizeof(struct output_triple_t))
struct table_chunk_t {
    uint64_t num_tuples;
    struct output_triple_t tuples[SGXAMD_TUPLES_PER_CHUNK];
};
struct chunked_table_t {
    struct table_chunk_t **chunks; /* pointers to the chunks */
    uint64_t current_chunk;        /* the chunk that is currently being filled */
    uint64_t num_chunks;           /* allocated chunks (non-null pointers in chunks) */
    uint64_t chunk_capacity;       /* pointers that fit into chunks */
    uint64_t num_tuples;           /* total tuples over all chunks */
};

/* data-types.h:107-114: join result (48 bytes with padding). */
struct result_t {
    int64_t totalresults;
    int nthreads;
    double throughput;
    int materialized;
    void *result;
    int result_type; /* 0 = threadresult_t*, 1 = chunked_table_t*, 2 = mi355 device triples */
};

/* data-types.h:155 */
enum numa_strategy_t { RANDOM, RING, NEXT };

/* data-types.h:162-176: join configuration (48 bytes). RHO reads NTHREADS,
 * MATERIALIZE and ALLOC_CORE only (radix_join.cpp:1372,1378,1397,1518). */
struct joinconfig_t {
    int NTHREADS;
    int PARTFANOUT;
    int SCALARSORT;
    int SCALARMERGE;
    int MWAYMERGEBUFFERSIZE;
    enum numa_strategy_t NUMASTRATEGY;
    int RADIXBITS;
    int WRITETOFILE;
    int MATERIALIZE;
    int PRINT;
    int CRACKING_THRESHOLD;
    int ALLOC_CORE;
};

/* data-types.h:94-97: name -> join function table entry. */
struct algorithm_t {
    char name[128];
    struct result_t *(*join)(const struct table_t *, const struct table_t *, const struct joinconfig_t *);
};

#ifdef __cplusplus
} /* extern "C" */
#define SGXAMD_STATIC_ASSERT(c, m) static_assert(c, m)
#else
#define SGXAMD_STATIC_ASSERT(c, m) _Static_assert(c, m)
#endif

SGXAMD_STATIC_ASSERT(sizeof(struct row_t) == 8, "row_t must be 8 bytes");
SGXAMD_STATIC_ASSERT(offsetof(struct row_t, payload) == 4, "row_t.payload at 4");
SGXAMD_STATIC_ASSERT(sizeof(struct table_t) == 24, "table_t must be 24 bytes");
SGXAMD_STATIC_ASSERT(offsetof(struct table_t, num_tuples) == 8, "table_t.num_tuples at 8");
SGXAMD_STATIC_ASSERT(sizeof(struct output_triple_t) == 12, "output_triple_t must be 12 bytes");
SGXAMD_STATIC_ASSERT(sizeof(struct table_chunk_t) == 16376, "table_chunk_t: 8 + 1364 * 12 bytes");
SGXAMD_STATIC_ASSERT(sizeof(struct chunked_table_t) == 40, "chunked_table_t must be 40 bytes");
SGXAMD_STATIC_ASSERT(sizeof(struct result_t) == 48, "result_t must be 48 bytes");
SGXAMD_STATIC_ASSERT(offsetof(struct result_t, throughput) == 16, "result_t.throughput at 16");
SGXAMD_STATIC_ASSERT(offsetof(struct result_t, result) == 32, "result_t.result at 32");
SGXAMD_STATIC_ASSERT(offsetof(struct result_t, result_type) == 40, "result_t.result_type at 40");
SGXAMD_STATIC_ASSERT(sizeof(struct joinconfig_t) == 48, "joinconfig_t must be 48 bytes");
SGXAMD_STATIC_ASSERT(offsetof(struct joinconfig_t, MATERIALIZE) == 32, "joinconfig_t.MATERIALIZE at 32");
SGXAMD_STATIC_ASSERT(offsetof(struct joinconfig_t, ALLOC_CORE) == 44, "joinconfig_t.ALLOC_CORE at 44");
SGXAMD_STATIC_ASSERT(sizeof(struct algorithm_t) == 136, "algorithm_t must be 136 bytes");

#endif /* SGXAMD_DATA_TYPES_H */
