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

// Multi-GPU building blocks (multi_host.cpp), on a context the caller holds:
// the stable shard partition by destination (host counts; synchronises s), and the
// two halves of the pipelined local join (begin enqueues R's passes on s and returns;
// finish runs S's passes and the build/probe on the same stream and waits).
// out_elem 8: out holds the tuples; 4: only their key words (a keys-only exchange).
int shard_partition_device(Context *ctx, hipStream_t s, const row_t *in, uint64_t n, uint32_t key_shift,
                           uint32_t dest_bits, void *out, uint64_t *dest_counts, uint32_t out_elem = 8);
// The same partition in two phases over several pieces, so that one count exchange
// serves a whole join: shard_count_pieces plans pieces (in[j], n[j]), j < npieces, runs
// their histograms and returns every piece's destination counts in counts[j * G + d]
// (G = 2^dest_bits; one synchronisation of s); shard_scatter_piece then enqueues piece
// j's scatter into out (no wait).  The plans stay valid until the next shard or join
// call on ctx, which reuses the scratch in stream order.
int shard_count_pieces(Context *ctx, hipStream_t s, const row_t *const *in, const uint64_t *n, int npieces,
                       uint32_t key_shift, uint32_t dest_bits, uint32_t out_elem, uint64_t *counts);
int shard_scatter_piece(Context *ctx, hipStream_t s, int j, void *out);
// Drops the per-context state of the shard and pipelined-join calls (the pinned count
// block of the shard pieces): called when a context of its own is destroyed.
void forget_context(const Context *ctx);
// in_elem 8: dR / dS are row_t relations; 4: packed keys (needs keys_exchange_plan's plan).
// s_piece_n[0..s_pieces): S arrives in contiguous pieces of these sizes (they add up to
// nS); a pooled S pass 1 then runs per piece, each launch after its event in
// s_landed[i] (finish; null: no waits), so that only the last piece's pass 1, the pool
// layout, pass 2 and the build/probe follow S's last piece.
// wire16: S will come as u16-wire residuals (join_pipelined_finish_wire16).
int join_pipelined_begin(Context *ctx, hipStream_t s, const void *dR, uint64_t nR, uint64_t nS,
                         const mi355_rho_opts *opts, uint32_t in_elem = 8, const uint64_t *s_piece_n = nullptr,
                         int s_pieces = 0, bool wire16 = false);
// mat (materialising joins, opts->materialize at begin): the triples go to this growable
// device buffer (st->matches of them).
int join_pipelined_finish(Context *ctx, const void *dS, uint64_t nS, mi355_rho_stats *st,
                          const hipEvent_t *s_landed = nullptr, DeviceBuffer *mat = nullptr);
// Whether a multi-GPU counting join can exchange keys only: fixes lo's local policy
// (radix bits / passes) from the expected local sizes nR / nS when the caller left it
// open, and checks that this policy takes the pooled keys layout for any local size up
// to cap_r / cap_s (the receive capacities).  SGXAMD_KEYS=0 disables it.
bool keys_exchange_plan(uint64_t nR, uint64_t nS, uint64_t cap_r, uint64_t cap_s, mi355_rho_opts *lo);

// ---- multi-GPU u16 wire (DESIGN.md §5 "Residuals on the wire") ----
// Whether a keys exchange (lo from keys_exchange_plan, lo->key_shift = log2 G) can send
// S as 2-byte residuals instead (R's keys still travel as 4 bytes: R's local passes run
// while S is on the wire, S's sender-side passes while R is): the local plan of nR x nS
// (the mean local sizes) is a two-pass narrow counting RHO plan, and every 32-bit key's
// residual above the shard and partition bits fits 16 bits (key_shift + bits >= 16) --
// or, with need_kmax, may: then *need_kmax is set and the caller must check S's largest
// key over all ranks (2-byte residuals only when (kmax >> (key_shift + bits)) < 2^16).
// mi355_multi_set_wire / SGXAMD_WIRE16 select the mode.  Returns the plan's partition
// count P (0: no).
uint32_t wire16_plan(uint64_t nR, uint64_t nS, int G, const mi355_rho_opts *lo, bool *need_kmax = nullptr);
// mi355_multi_set_wire: 0 off, 1 where the local plan is narrow anyway, 2 whenever the
// residuals fit (tests).
void set_wire_mode(int mode);
int wire_mode();
// Sender (out16: 4 bytes per key -- a destination whose residuals do not fit 16 bits,
// possible only with need_kmax, is written as keys and the caller sends S as keys):
// partitions the keys this rank sends each destination (runs of packed u32
// keys in `keys`: destination q's runs at run_off[q * runs + j], run_n[...]) with the
// plan of wire16_plan(nR, nS, ...): destination q's residuals go to out16 +
// sum_{q' < q} wire_slot(keys of q', P) (a 16-byte boundary: k_place_seg's whole-line
// copies), grouped by partition, every partition on a multiple of 8 residuals;
// counts[q * (2 P + 1) + p] = its partition p's keys, [+ P + p] its start in the run,
// [+ 2 P] its largest key.  Enqueued on s (no wait).
int wire_partition(Context *ctx, hipStream_t s, const uint32_t *keys, int G, int runs, const uint64_t *run_off,
                   const uint64_t *run_n, uint64_t nR, uint64_t nS, const mi355_rho_opts *lo, uint16_t *out16,
                   uint64_t *counts, const char *tag);
// Receiver: after join_pipelined_begin(..., wire16 = true) (R's passes, the plan of
// wire16_plan, R's pass 2 writing residuals), S's residuals as the G senders sent them
// (sender q's run of s_n[q] keys at s_base[q] u16 elements in a slot of s_span[q], its
// counts row as wire_partition wrote it; nS keys in all): after s_landed (an event on the
// communication stream) the build/probe reads S's partitions in place as their G pieces
// (G <= 8; more, or SGXAMD_WIRE_GATHER=1: the pieces are gathered into contiguous
// partitions first).  scratch: wire_scratch_u64(G, P) u64.  Synchronises the stream; st
// as join_pipelined_finish.
int join_pipelined_finish_wire16(Context *ctx, const uint16_t *s16, const uint64_t *s_cnt, const uint64_t *s_base,
                                 const uint64_t *s_n, const uint64_t *s_span, uint64_t nS, int G, uint64_t *scratch,
                                 hipEvent_t s_landed, mi355_rho_stats *st);
// A destination's (sender's) run of u16 residuals on the wire, padded to 8 (16 bytes).
inline uint64_t wire_pad(uint64_t n) { return (n + 7) & ~uint64_t(7); }
// The slot of a run of n keys on the wire: its P partitions each start on a multiple of 8
// (at most 8 P + 8 residuals of padding, rho_internal.hpp wire_pad_slack), so the
// receiver reads them in place.  A multiple of 8; none for an empty run (wire_partition
// writes nothing for it).
inline uint64_t wire_slot(uint64_t n, uint32_t P) { return n ? wire_pad(n) + 8ull * P + 8 : 0; }
// Words of one counts row: P partition counts, P partition starts, the largest key.
inline uint64_t wire_row_words(uint32_t P) { return 2ull * P + 1; }
uint64_t wire_scratch_u64(int G, uint32_t P);
// Tests: enqueue `us` microseconds of waiting on stream s (rho_kernels.hip k_spin).
hipError_t launch_spin(uint32_t us, hipStream_t s);
// What mi355_last_join_stats reports for this thread's last join (multi-GPU calls).
void set_last_join_stats(const mi355_rho_stats &st);

// Host chunked table (ChunkedTable.cpp layout) holding a copy of n triples.
chunked_table_t *make_chunked_table(const output_triple_t *src, uint64_t n);

}  // namespace rho
}  // namespace sgxamd
