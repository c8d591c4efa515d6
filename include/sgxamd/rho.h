/*
 * sgxamd/rho.h — C-ABI of the MI355X radix hash join (RHO).
 *
 * Drop-in boundary.  The reference exposes RHO as
 *     result_t *RHO(const table_t *relR, const table_t *relS, const joinconfig_t *config);
 * (Join-Benchmarks/lib/Joins/include/radix/radix_join.h:29-30, implemented at
 *  lib/Joins/src/radix/radix_join.cpp:1640-1643) and dispatches it by name through
 *     void run_join(result_t*, const table_t*, const table_t*, const char*, const joinconfig_t*);
 * (lib/Joins/src/joins.cpp:55-78, table entry {"RHO", RHO} at :42).
 *
 * This header declares the plain-C entry points a cgo / ctypes / JNI binding
 * would bind.  The C++-linkage adapters with the reference's exact (mangled)
 * signatures, RHO() and run_join(), live in sgxamd/joins.hpp.
 *
 * Pointers: every tuple pointer may be host memory or device (hipMalloc /
 * torch) memory; the library classifies it with hipPointerGetAttributes and
 * stages host buffers through HBM.  All calls are blocking, like the reference.
 */
#ifndef SGXAMD_RHO_H
#define SGXAMD_RHO_H

#include "sgxamd/data_types.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Status codes returned by every mi355_* entry point (0 = success). */
#define MI355_OK 0
#define MI355_ERR_INVALID (-1)   /* bad argument (null pointer, size, capacity) */
#define MI355_ERR_NO_DEVICE (-2) /* no gfx950 device visible */
#define MI355_ERR_HIP (-3)       /* a HIP runtime call failed; see mi355_last_error() */
#define MI355_ERR_OOM (-4)       /* device allocation failed */
#define MI355_ERR_CAPACITY (-5)  /* output buffer too small; required size reported */

/* Build/probe algorithm over the radix partitions (joins.cpp:42-43 table names). */
#define MI355_ALGO_RHO 0 /* bucket_chaining_join, radix_join.cpp:359-458 */
#define MI355_ALGO_RHT 1 /* histogram_join, radix_join.cpp:463-612 */

/* Options of one join call (NULL = defaults). */
typedef struct mi355_rho_opts {
    int radix_bits;      /* total radix bits; 0 = GPU policy (DESIGN.md "partitioning policy") */
    int passes;          /* 1 or 2; 0 = policy */
    uint32_t key_shift;  /* low key bits already fixed by a shard exchange (multi-GPU); 0 otherwise */
    int materialize;     /* 1 = write every match to out (radix_join.cpp:437-446, MATERIALIZE) */
    int timing;          /* 1 = record per-kernel HIP events (mi355_timing_* below) */
    int algorithm;       /* MI355_ALGO_RHO (bucket chaining) or MI355_ALGO_RHT (histogram join) */
    void *stream;        /* hipStream_t to launch on; NULL = the library's stream */
    struct output_triple_t *out; /* materialize: {key, R payload, S payload} per match, host or
                                    device memory; order unspecified (the reference's is per thread) */
    uint64_t out_capacity;       /* triples that fit in out; if fewer than the matches, the call
                                    returns MI355_ERR_CAPACITY with stats->matches = required */
} mi355_rho_opts;

/* What one join call did. */
typedef struct mi355_rho_stats {
    uint64_t matches;         /* join cardinality (bit-exact vs the reference's totalresults) */
    uint32_t radix_bits;      /* total bits used */
    uint32_t passes;          /* partition passes */
    uint32_t pass1_bits;
    uint32_t pass2_bits;
    uint64_t num_partitions;  /* 2^radix_bits */
    uint64_t num_tasks;       /* build/probe tasks (partition x S-chunk) */
    uint64_t max_part_r;      /* largest R partition (tuples) */
    uint64_t max_part_s;      /* largest S partition (tuples) */
    double ms_h2d;            /* host->device staging (0 when inputs were resident) */
    double ms_partition;      /* partition phase (pass 1 + pass 2), device time */
    double ms_pass1;
    double ms_pass2;
    double ms_join;           /* build + probe ("Build+Join Overall"), device time */
    double ms_total;          /* partition + join, device time */
    /* the reference's finer phase timers (radix_timers_t, radix_join.cpp:94-107) */
    double ms_pass1_r;        /* pass 1 of R ("Partition R") */
    double ms_pass1_s;        /* pass 1 of S ("Partition S") */
    double ms_pass1_hist;     /* pass-1 histograms + prefix sums, R and S ("One Hist") */
    double ms_pass1_copy;     /* pass-1 scatters, R and S ("One Copy") */
    double ms_pass2_hist;     /* "Two Hist" */
    double ms_pass2_copy;     /* "Two Copy" */
    double ms_build;          /* "Build": ms_join split by the build/probe wall-clock ticks the */
    double ms_probe;          /* "Join":   fused build+probe kernel measures per workgroup */
    /* partition layout: 0 = tuples, pass-1 histogram + cursors; 1 = pooled pass 1 (no
     * pass-1 histogram), tuples; 2 = pooled pass 1, 4-byte keys (counting joins, RHO and RHT);
     * 3 = as 2, with the pass-2 digits counted per chain in pass 1 (no digit side stream);
     * 4 = as 2 for a narrow plan: pass 1 writes the keys' 16-bit residuals (and their pass-2
     * digits beside them), repeated as 4-byte keys for a relation whose residuals do not fit */
    uint32_t layout;
    uint32_t elem_bytes;      /* bytes per partitioned element after the input read (8 or 4) */
    /* bit 0 / bit 1: R's / S's final partitions hold 16-bit key residuals (key >> radix
     * bits, when every key's residual fits; counting RHO over key partitions) */
    uint32_t narrow;
    uint32_t reserved0;
} mi355_rho_stats;

/* Number of gfx950 devices visible (0 on a CPU-only host). */
int mi355_device_count(void);

/* Text of the last error on this thread. */
const char *mi355_last_error(void);

/* Library version string. */
const char *mi355_version(void);

/*
 * RHO join with the reference's semantics.  Replaces RHO() at radix_join.cpp:1640 /
 * radix_join.h:29.  Fills out->totalresults, nthreads (= config->NTHREADS),
 * materialized, result, result_type and throughput (M rec/s = (|R|+|S|) / join
 * time, which the reference leaves unset).  With config->MATERIALIZE = 1 the
 * matches come back as a host chunked_table_t (result_type 1, as the reference's
 * CHUNKED_TABLE build, radix_join.cpp:1554-1557); free it with
 * mi355_free_chunked_table.  Otherwise result = NULL, result_type = 0.
 */
int mi355_rho_join(const struct table_t *relR, const struct table_t *relS,
                   const struct joinconfig_t *config, struct result_t *out);

/* Drop-in for RHT() (radix_join.cpp:1645-1648, radix_join.h): the same radix
 * partitioning with the histogram build/probe of histogram_join.  Same result
 * contract as mi355_rho_join. */
int mi355_rht_join(const struct table_t *relR, const struct table_t *relS,
                   const struct joinconfig_t *config, struct result_t *out);

/* Statistics of the last join call made on this thread (any entry point). */
int mi355_last_join_stats(mi355_rho_stats *out);

/* Frees the chunked_table_t that mi355_rho_join / RHO() return in result->result
 * when config->MATERIALIZE = 1 (result_type 1, the reference's CHUNKED_TABLE form,
 * ChunkedTable.cpp:21-171).  NULL is ignored. */
void mi355_free_chunked_table(struct chunked_table_t *table);

/* Same join on raw tuple arrays with explicit options and per-phase statistics. */
int mi355_rho_join_ex(const struct row_t *R, uint64_t nR, const struct row_t *S, uint64_t nS,
                      const mi355_rho_opts *opts, mi355_rho_stats *stats);

/*
 * Multi-GPU shard step: stable radix partition of n device-resident tuples by
 * destination d = (key >> key_shift) & (2^dest_bits - 1) into `out` (device,
 * n tuples), destination-major.  dest_counts (host, 2^dest_bits entries) receives
 * the tuple count per destination, i.e. the send split of the all-to-all.
 */
int mi355_rho_shard_partition(const struct row_t *in, uint64_t n, uint32_t key_shift,
                              uint32_t dest_bits, struct row_t *out, uint64_t *dest_counts,
                              void *stream);

/*
 * Pipelined join in two calls, for callers whose S arrives later in the stream
 * order than R (the multi-GPU exchange: R's local partition passes run while S is
 * still on the wire).  begin plans both relations (|S| = nS), enqueues R's partition
 * passes on opts->stream (or the library stream) and returns without waiting;
 * finish enqueues S's passes and the build/probe on the same stream, waits, and
 * fills stats.  Both relations must be device-resident; S only has to be valid in
 * the stream order when finish is called (e.g. after a hipStreamWaitEvent on the
 * exchange).  opts (key_shift, algorithm, materialize with a device out) must be the
 * same in both calls.  One pending join per device; other join or shard calls on
 * that device fail with MI355_ERR_INVALID until finish.  begin + finish computes
 * exactly what mi355_rho_join_ex computes.
 */
int mi355_rho_join_begin(const struct row_t *R, uint64_t nR, uint64_t nS, const mi355_rho_opts *opts);
int mi355_rho_join_finish(const struct row_t *S, uint64_t nS, const mi355_rho_opts *opts,
                          mi355_rho_stats *stats);

/*
 * Per-kernel timing of the last call on this thread that ran with timing
 * enabled (opts->timing or mi355_timing_enable(1)): names and milliseconds
 * of every recorded kernel, in launch order.  Returns the number of records
 * (up to `cap` are copied).  mi355_timing_enable(2) (sparse): only R's pass-1
 * scatter and the build/probe are timed, the launches between them as one
 * span "other" -- four events per join instead of one per kernel.
 */
void mi355_timing_enable(int on);
int mi355_timing_get(const char **names, double *ms, int cap);

/*
 * Partition-chain overlap of this thread's joins (default 0): 1 runs R's and S's
 * partition passes on two HIP streams, joined before build/probe; 0 runs them back
 * to back on one stream, so each kernel's event time is its own.  Results are
 * identical either way (DESIGN.md §7 has the measurements behind the default).
 */
void mi355_set_partition_overlap(int on);

/*
 * Partition layout of this thread's counting joins (RHO and RHT) (default 1): 1 moves the 4-byte
 * key of every tuple after the input read (the build/probe of a count reads keys only),
 * 0 moves whole 8-byte tuples as the reference does.  Counts are identical; the
 * environment switch SGXAMD_KEYS=0 forces 0 for the whole process.
 */
void mi355_set_key_layout(int on);

/* Stream used by calls that take no explicit stream (NULL = library stream). */
void mi355_set_stream(void *stream);

/* Frees the current device's workspace (partition buffers, scratch, staging, scan and
 * TPC-H buffers) after the work queued on its library stream has finished; the next
 * call allocates again.  The workspace is otherwise grow-only and kept for the
 * process.  MI355_ERR_INVALID while a pipelined join is pending. */
int mi355_release_workspace(void);

/* HBM ceiling probe (measurement: bench.py's roofline ceilings).  One grid-stride
 * streaming kernel of 256-thread workgroups over device buffers, enqueued on `stream`
 * (null: the library stream): kind 0 copies `bytes` from src to dst, 1 reads src (dst:
 * one 16-byte word, written only if an impossible xor appears), 2 writes dst.  nt_load /
 * nt_store: non-temporal accesses; loads_in_flight: 16-byte accesses per thread and
 * step (1, 2, 4 or 8); grid: workgroups (0: 4096).  16-byte aligned buffers, bytes a
 * multiple of 16 (MI355_ERR_INVALID otherwise). */
int mi355_stream_probe(int kind, const void *src, void *dst, uint64_t bytes, int nt_load, int nt_store,
                       int loads_in_flight, uint32_t grid, void *stream);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* SGXAMD_RHO_H */
