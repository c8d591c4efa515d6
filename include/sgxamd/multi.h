/*
 * sgxamd/multi.h — C-ABI of the multi-GPU RHO join (radix-shard exchange).
 *
 * The reference runs RHO with NTHREADS pthreads, each owning a contiguous slice of
 * R and S (radix_join.cpp:1457-1500), sharing the partitioned tmpR/tmpS arrays
 * (:1421-1433) through memory.  Across GPUs the slices stay where they are; the
 * first radix level (the low log2(G) key bits) picks the owning GPU, and one
 * exchange step moves every tuple to its owner:
 *   1. per relation, in pieces: stable shard partition of the local slice by
 *      d = key & (G - 1) (the pass-1 machinery of radix_join.cpp:851-931 with G bins);
 *   2. the G x G piece counts: a host table between the rank threads of one process,
 *      or an RCCL all-gather on a second communicator (never queued behind the
 *      previous piece's tuples on the tuple communicator);
 *   3. the tuples (RCCL send/recv per peer, on a communication stream, while the next
 *      piece is partitioned), into a contiguous receive buffer per relation;
 *   4. the local join of the received relations with key_shift = log2(G) (R's local
 *      passes while S is still on the wire);
 *   5. an all-reduce of the match counts.
 * Every rank issues the same collectives whether or not it failed: a rank whose
 * allocation, shard pass or local join fails flags it in the next count exchange or in
 * the final all-reduce, and every rank returns an error at that step (the first-hand
 * error on the failed rank, MI355_ERR_COMM "another rank failed" on the others).
 * The caller, native.cpp:137 -> run_join -> RHO, is unchanged: RHO() (joins.hpp)
 * takes this path when SGXAMD_GPUS > 1 (joinconfig_t has no spare field for a GPU
 * count).
 *
 * Transports:
 *   MI355_TRANSPORT_RCCL      — RCCL over xGMI, one rank per GPU (librccl.so.1 is
 *                               loaded on first use);
 *   MI355_TRANSPORT_REHEARSAL — G logical ranks on the current GPU, each with its own
 *                               stream and workspace, the exchange done by device-to-
 *                               device copies: the whole C++ path on one GPU, for tests;
 *   MI355_TRANSPORT_AUTO      — RCCL when G devices are visible, else rehearsal.
 *   SGXAMD_MULTI_TRANSPORT=rccl|rehearsal overrides AUTO.
 * G must be a power of two (1..256).
 * Materialising joins (opts->materialize, radix_join.cpp:437-446): whole tuples travel
 * (the payloads), each rank writes its matches as output_triple_t {key, R payload,
 * S payload} into a growable buffer of its own -- its output chunk, as the reference's
 * threads write theirs (ChunkedTable.cpp:98-171) -- and the chunks reach opts->out:
 * mi355_rho_join_multi_ex concatenates every rank's (rank 0 first) into opts->out
 * (host or device memory, out_capacity triples; MI355_ERR_CAPACITY with
 * stats->matches = the triples needed when they do not fit); mi355_rho_join_sharded
 * writes the calling rank's own chunk (stats->local_matches triples) to its opts->out.
 */
#ifndef SGXAMD_MULTI_H
#define SGXAMD_MULTI_H

#include "sgxamd/rho.h"

#ifdef __cplusplus
extern "C" {
#endif

#define MI355_TRANSPORT_AUTO 0
#define MI355_TRANSPORT_RCCL 1
#define MI355_TRANSPORT_REHEARSAL 2

#define MI355_ERR_COMM (-6) /* an RCCL call failed (or librccl.so.1 is missing); see mi355_last_error() */

typedef struct mi355_multi_stats {
    uint64_t matches;          /* global join cardinality (sum over ranks) */
    int world;                 /* ranks (GPUs) */
    int transport;             /* MI355_TRANSPORT_RCCL or MI355_TRANSPORT_REHEARSAL */
    int pieces;                /* pieces per relation in the exchange */
    int rank;                  /* the calling rank (one process per GPU), else 0 */
    uint64_t local_matches;    /* this rank's matches (rank 0 in single-process mode) */
    uint64_t recv_r_max, recv_r_min;  /* received R tuples per rank (load report) */
    uint64_t recv_s_max, recv_s_min;  /* received S tuples per rank */
    uint64_t max_part_s;       /* largest local S partition over the ranks seen */
    uint64_t sent_bytes;       /* bytes sent to other ranks (ranks seen): tuples, keys, or on the
                                  u16 wire residuals and counts rows */
    double ms_total;           /* wall time of the call (max over the ranks seen) */
    double ms_exchange_post;   /* shard partitions + count exchanges + posting the pieces */
    double ms_local;           /* from the last piece posted to the local join's end */
    double ms_allreduce;       /* final match-count all-reduce */
    mi355_rho_stats local;     /* the local join of rank 0 (or of the calling rank) */
    uint32_t elem_bytes;       /* bytes per exchanged element: 8 (tuples), 4 (keys only: a
                                  counting join whose local join reads keys) or 2 (the u16
                                  wire, mi355_multi_set_wire: R's keys travel as 4 bytes, and
                                  for S every sender runs the receiver's two partition passes
                                  and sends 2-byte residuals grouped by partition, plus per
                                  peer one row of P + 1 u64 words: the partition counts and
                                  its largest key) */
    double ms_tail;            /* device time from S's last piece landing to the local join's
                                  end (max over the ranks seen; the part of the join that no
                                  exchange hides); -1 when no rank measured it (a world of
                                  one, a failed or untimed tail) */
} mi355_multi_stats;

/* Single process, `ngpus` ranks driven by one host thread each.  R and S are host or
 * device memory (device memory of the current GPU); rank g joins the slice
 * [g*floor(n/G), ...) of each relation (the last rank takes the remainder), staged to
 * its GPU.  opts: algorithm / radix_bits / passes of the local joins (NULL = defaults),
 * materialize / out / out_capacity (above); key_shift and stream must be 0. */
int mi355_rho_join_multi_ex(const struct row_t *R, uint64_t nR, const struct row_t *S, uint64_t nS, int ngpus,
                            int transport, const mi355_rho_opts *opts, mi355_multi_stats *stats);

/* Drop-in multi-GPU RHO on reference relations (counting join; fills out like
 * mi355_rho_join, throughput = (|R|+|S|) / call time). */
int mi355_rho_join_multi(const struct table_t *relR, const struct table_t *relS, const struct joinconfig_t *config,
                         int ngpus, struct result_t *out);

/* One process per GPU (torchrun / MPI style).  Rank 0 creates a unique id
 * (128 bytes), the caller distributes it, every rank creates its communicator on
 * its current device (collective), then calls mi355_rho_join_sharded with its
 * device-resident slices (collective; the same `pieces` everywhere).  The rank's
 * compute runs on opts->stream (else the mi355_set_stream stream, else the library's);
 * the exchange on a communication stream of its own. */
int mi355_multi_unique_id(void *id128);
int mi355_multi_comm_init(const void *id128, int nranks, int rank, void **comm);
int mi355_multi_comm_destroy(void *comm);
int mi355_rho_join_sharded(void *comm, const struct row_t *R, uint64_t nR, const struct row_t *S, uint64_t nS,
                           const mi355_rho_opts *opts, mi355_multi_stats *stats);

/* Statistics of this thread's last multi-GPU join (either entry point). */
int mi355_last_multi_stats(mi355_multi_stats *out);

/* Pieces each relation is exchanged in (default 4; 1..64); applies to later calls. */
void mi355_multi_set_pieces(int pieces);

/* S's keys on the wire as 2-byte residuals of sender-side partitions (the u16 wire,
 * DESIGN.md §5): 0 never (4-byte keys), 1 (default; SGXAMD_WIRE16 sets the initial mode)
 * when the local join takes the narrow 16,384-key-table plan anyway and every residual
 * fits 16 bits (log2 G + the local radix bits >= 16), 2 whenever the residuals fit
 * (forcing the narrow plan; tests).  Every rank of a join must use the same mode (the
 * ranks agree on the lowest). */
void mi355_multi_set_wire(int mode);

/* Frees the workspaces (exchange and join buffers) of the rehearsal transport's
 * logical ranks, which are otherwise kept for the process: call it between large
 * rehearsal joins that do not reuse them.  The calling thread's device must be the
 * rehearsal's. */
int mi355_multi_release(void);

/* Test hook: rank `rank` fails at `step` of every later multi-GPU join (1: exchange
 * buffer allocation, 2: a shard pass of S, 3: the local join, 4: no device context,
 * 5: the stream synchronisation after the local join, as an asynchronous kernel fault
 * would) as an allocation or kernel error would; step 0 clears it. */
void mi355_multi_inject_failure(int rank, int step);

/* Test hook: the RCCL library later multi-GPU calls load instead of librccl.so.1 (NULL:
 * back to librccl.so.1).  It must export the RCCL entry points the transport uses
 * (ncclGetUniqueId, ncclCommInitRank/InitAll/Split/Destroy/Abort, ncclGroupStart/End,
 * ncclSend/Recv, ncclAllGather/AllReduce, ncclGetErrorString).  A library named here is
 * taken to be a test double that may hold several ranks on one GPU (tests/rccl_double:
 * ranks are threads of one process, data moves by device copies): the single-process
 * RCCL mode then runs every rank on the current GPU with a context of its own, so the
 * RCCL transport itself runs at G > 1 on one MI355X.  Refused (MI355_ERR_INVALID) while
 * communicators of mi355_multi_comm_init exist; the single-process communicators of the
 * previous library are aborted. */
int mi355_multi_set_rccl_library(const char *path);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* SGXAMD_MULTI_H */
