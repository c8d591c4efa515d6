/*
 * sgxamd/generator.h — synthetic relations and scan columns.
 *
 * Host generators restate the reference's AppUtilities generators bit for bit
 * (Join-Benchmarks/lib/AppUtilities/src/generator.cpp, genzipf.cpp) so that the
 * GPU join and the CPU oracle see exactly the relations the reference's
 * native driver (App/TEEBench/native.cpp:62-101) would build:
 *   seed_generator        generator.cpp:75-80   -> mi355_gen_seed
 *   RAND_RANGE / rand()   generator.cpp:19      -> mi355_gen_rand (glibc TYPE_3 restated)
 *   knuth_shuffle         generator.cpp:100-109
 *   create_relation_pk    generator.cpp:352-377 -> mi355_gen_pk
 *   create_relation_fk    generator.cpp:474-512 -> mi355_gen_fk
 *   create_relation_fk_sel generator.cpp:515-553 -> mi355_gen_fk_sel
 *   create_relation_zipf  generator.cpp:638-660 / genzipf.cpp:34-144 -> mi355_gen_zipf
 * The reference leaves payloads uninitialised; here payload = row index.
 * The reference seeds Zipf from std::random_device (genzipf.cpp:44,104), which
 * is not reproducible; mi355_gen_zipf takes an explicit mt19937_64 seed.
 *
 * Device generators (mi355_gen_*_dev) build relations of the same shape
 * directly in HBM from a keyed bijection of the row index, so multi-GPU
 * ranks can each generate their own slice of one global relation.
 */
#ifndef SGXAMD_GENERATOR_H
#define SGXAMD_GENERATOR_H

#include "sgxamd/data_types.h"

#ifdef __cplusplus
extern "C" {
#endif

/* srand(seed) of the restated glibc generator (seed 0 behaves as 1, like glibc). */
void mi355_gen_seed(unsigned int seed);
/* Next value of the restated glibc rand() (0 .. 2^31-1). */
int mi355_gen_rand(void);

/* Host relations; `out` is caller-allocated (n tuples).  Return 0 on success. */
int mi355_gen_pk(struct row_t *out, uint64_t n);
int mi355_gen_fk(struct row_t *out, uint64_t n, int64_t maxid);
int mi355_gen_fk_sel(struct row_t *out, uint64_t n, int64_t maxid);
/* Zipf keys over alphabet 1..alphabet_size with exponent theta; mt19937_64(seed)
 * drives the alphabet permutation and the draws.  nthreads parallelises the
 * CDF search (results are independent of nthreads). */
int mi355_gen_zipf(struct row_t *out, uint64_t n, uint32_t alphabet_size, double theta,
                   uint64_t seed, int nthreads);

/* Scan column of the reference's Allocator.hpp:94-117: data[i] = i % 256. */
int mi355_gen_scan_u8(uint8_t *out, size_t n);
int mi355_gen_scan_i32(int32_t *out, size_t n);

/* Device relations (device pointer `out`, `count` rows starting at global row
 * `first`).  pk: keys are perm(row) + 1 for a keyed bijection perm of [0, n).
 * fk: row r gets perm_{seed + r / maxid}(r % maxid) + 1, i.e. consecutive
 * independently shuffled copies of 1..maxid (create_relation_fk's shape). */
int mi355_gen_pk_dev(struct row_t *out, uint64_t count, uint64_t first, uint64_t n,
                     uint64_t seed, void *stream);
int mi355_gen_fk_dev(struct row_t *out, uint64_t count, uint64_t first, uint64_t maxid,
                     uint64_t seed, void *stream);
/* Zipf(theta) keys over the alphabet 1..alphabet_size (genzipf.cpp:87-144 on the
 * device: CDF lookup table, binary search of a uniform draw, random alphabet
 * permutation); rows [first, first + count) of the same global relation for a
 * given seed, so ranks can generate disjoint slices.  payload = row index. */
int mi355_gen_zipf_dev(struct row_t *out, uint64_t count, uint64_t first, uint32_t alphabet_size, double theta,
                       uint64_t seed, void *stream);
/* Device scan columns: mode 0 = i % 256 (reference), mode 1 = keyed uniform random. */
int mi355_gen_scan_u8_dev(uint8_t *out, size_t n, int mode, uint64_t seed, void *stream);
int mi355_gen_scan_i32_dev(int32_t *out, size_t n, int mode, uint64_t seed, void *stream);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* SGXAMD_GENERATOR_H */
