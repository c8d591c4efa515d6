// Internal interface between the RHO kernels (rho_kernels.hip) and the host
// orchestration (rho_host.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "sgxamd/data_types.h"

namespace sgxamd {
namespace rho {

constexpr int kBlock = 256;   // threads per workgroup for partition/join kernels
constexpr int kMaxF = 512;    // max fanout of one partition pass (9 radix bits)
constexpr int kScatterThreads = 512;                  // threads per scatter workgroup
constexpr int kScatterItems = 8;                      // tuples per thread per tile
constexpr int kTile = kScatterThreads * kScatterItems;  // tuples per scatter tile

// Which contiguous slice of the input a partition workgroup owns.  Regions are
// the bins of the previous pass (or the whole relation); each region is cut into
// segments of seg_size tuples, one workgroup per segment.
struct SegMap {
    const uint64_t *reg_start;  // nullptr => one region [0, single_n)
    const uint64_t *reg_count;
    const uint32_t *seg_base;   // nreg + 1 prefix of segments per region (device)
    uint32_t nreg;
    uint64_t seg_size;
    uint64_t single_n;
};

// Histogram layout selector: digit-major [d][g] (single region: column scans)
// or segment-major [g][d] (many regions: per-region scans).
enum HistLayout : int { kDigitMajor = 0, kSegMajor = 1 };

hipError_t launch_hist(const row_t *in, const SegMap &m, uint32_t grid, uint32_t shift, uint32_t bits,
                       uint64_t *hist, HistLayout layout, uint32_t nseg_stride, hipStream_t s);

// Single-region scan: hist [F][nseg] -> exclusive per-digit column prefix (in place);
// then digit starts/counts, and (optionally) the segment table of the next pass.
hipError_t launch_scan_single(uint64_t *hist, uint32_t nseg, uint32_t bits, uint64_t *totals,
                              uint64_t *out_start, uint64_t *out_count, uint64_t base,
                              uint32_t *next_seg_base, uint64_t next_seg_size, hipStream_t s);

// Multi-region scan: hist [g][F] -> absolute write cursors (in place) and the
// (region, digit) partition table part_start/part_count [nreg * F].  pad: every
// partition starts on a multiple of 8 elements (the u16 wire's senders), the layout
// then spans at most wire_pad_slack(nreg * F) elements more.
hipError_t launch_scan_regions(uint64_t *hist, const uint32_t *seg_base, const uint64_t *reg_start,
                               uint32_t nreg, uint32_t bits, uint64_t *part_start, uint64_t *part_count,
                               hipStream_t s, bool pad = false);
inline uint64_t wire_pad_slack(uint64_t partitions) { return 8 * partitions + 8; }

// Context::sync (u64 words, zero when allocated): the digit totals of the small join's
// histograms (launch_hist_pair), in two sets that alternate per call (the scatter of a
// call zeroes the other set), and the ticket of the build/probe count reduction (left
// zero by the kernel that takes it).
constexpr uint32_t kSyncTicketJoin = 3;
// sync[kSyncTicketJoin + 1] holds the device address of the context's mapped host
// result block (set once, never written by a kernel): the small join's last
// workgroup stores the six result words there, then the device span of the call
// (word 6, wall-clock ticks since k_hist_pair's first workgroup stored its start in
// sync[kSyncT0]) and last the done flag (word 7), which the host spins on instead of
// synchronising the stream.
constexpr uint32_t kSyncHostResult = kSyncTicketJoin + 1, kSyncT0 = kSyncTicketJoin + 2;
// the small join's count reduction (rho_kernels.hip join_reduce_last): arrivals << 48 |
// the summed counts, and the summed build / probe ticks (two 32-bit halves); zero
// between calls
constexpr uint32_t kSyncJoinSum = kSyncTicketJoin + 3, kSyncJoinTicks = kSyncTicketJoin + 4;
static_assert(kSyncJoinTicks < 8, "sync words below the digit totals");
constexpr uint32_t kHostJoinSpan = 6, kHostJoinDone = 7, kHostJoinWords = 8;
// Hand-offs spread over kSyncSpread groups of workgroups (segment or workgroup index mod
// kSyncSpread), so that no device-scope atomic address takes more than 1/kSyncSpread of
// the grid's updates: the digit totals are kSyncSpread copies [c][kMaxF] (a segment's
// offset is its place inside its copy; its cursor base adds the copies before it), and a
// ticket of n arrivals is kSyncSpread sub-tickets (sync[ticket + kSyncSub + kNumTickets *
// c]) whose last arrivers take the ticket itself.  Default 1 (no spreading): 8 groups
// measured no faster, 56.7 vs 55.7 us per 2^20 join (r04l; the small path is
// latency-bound, not atomic-bound).  SGXAMD_SMALL_SPREAD=8 builds.
#ifndef SGXAMD_SMALL_SPREAD
#define SGXAMD_SMALL_SPREAD 1
#endif
constexpr uint32_t kSyncSpread = SGXAMD_SMALL_SPREAD, kNumTickets = 4;
constexpr uint32_t kSyncTot0 = 8, kSyncTotWords = kSyncSpread * kMaxF;
// totals set `parity` (0 / 1) of relation rel (0 R, 1 S)
constexpr uint32_t sync_tot(uint32_t parity, uint32_t rel) { return kSyncTot0 + (2 * parity + rel) * kSyncTotWords; }
constexpr uint32_t kSyncSub = kSyncTot0 + 4 * kSyncTotWords;  // relative to a ticket's word
// the count reduction's group word pairs (join_reduce_last: kJoinGroups of them)
constexpr uint32_t kJoinGroups = 16;
constexpr uint32_t kSyncJoinGrp = kSyncSub + kNumTickets * (kSyncSpread + 1);
// R's largest key (k_hist_pair; the direct table of k_join), one word per parity set: the
// scatter's layout workgroup zeroes the next call's
constexpr uint32_t kSyncKmax = kSyncJoinGrp + 2 * kJoinGroups;
constexpr uint32_t kSyncWords = kSyncKmax + 2;
// Development: small-join workgroup stamps (rho_kernels.hip dbg_stamp), 3 kernels + the
// build/probe reduction x 3
// stamps x kStampWgs u64; null turns them off.
constexpr uint32_t kStampWgs = 1024;
hipError_t set_debug_stamps(uint64_t *p);

// Small one-pass joins: histograms of R and S in one launch (gridR / gridS workgroups
// each take two segments of mR / mS, 2g and 2g + 1: the scatter's segments).  offs:
// [d][2 grid] segment offsets inside the segment's copy (g mod kSyncSpread) of digit d's
// total in tot (sync_tot of this call's parity, zero at entry).  t0: the call's start
// (sync[kSyncT0]).
// kmaxR (nullable, zero at entry): R's largest key, max-ed in.
hipError_t launch_hist_pair(const row_t *R, const SegMap &mR, uint32_t gridR, const row_t *S, const SegMap &mS,
                            uint32_t gridS, uint32_t shift, uint32_t bits, uint64_t *offsR, uint64_t *offsS,
                            uint64_t *totR, uint64_t *totS, uint64_t *t0, hipStream_t s, uint64_t *kmaxR = nullptr);
// Both relations' one-pass scatters in one launch (cursors: the segment offsets + the
// digit starts of the segment's totals copy, taken by each workgroup from tot), plus one
// workgroup that writes the partition table (start / cnt), the task list (over, meta as
// launch_make_tasks) and zeroes the other totals set (tot_next) for the next call.
hipError_t launch_scatter_pair(const row_t *R, row_t *outR, const SegMap &mR, uint32_t gridR, const uint64_t *offsR,
                               const uint64_t *totR, uint64_t *totR_next, uint64_t *startR, uint64_t *cntR,
                               const row_t *S, row_t *outS, const SegMap &mS, uint32_t gridS, const uint64_t *offsS,
                               const uint64_t *totS, uint64_t *totS_next, uint64_t *startS, uint64_t *cntS,
                               uint32_t shift, uint32_t bits, uint64_t *over, uint32_t over_cap, uint64_t *meta,
                               uint64_t s_chunk, hipStream_t s, uint64_t *kmax_next = nullptr);

// Digit side stream of a two-pass partition: the pass-1 scatter also writes, for the
// tuple it stores at position a of its output, the tuple's pass-2 digit
// (key >> shift2) & (2^bits2 - 1) to side[a].  Pass 2's histogram then reads one byte
// per tuple (launch_hist_side) instead of the 8-byte tuple.
struct DigitSide {
    uint8_t *side;
    uint32_t shift2;
    uint32_t bits2;
};

// Pass-2 histogram from the digit side stream (segment-major [g][F]; segments as m).
hipError_t launch_hist_side(const uint8_t *side, const SegMap &m, uint32_t grid, uint32_t bits, uint64_t *hist,
                            hipStream_t s);

// ---- pooled pass 1 (two-pass plans without a pass-1 histogram) ----
// Every pass-1 workgroup owns a pool of pool_blocks blocks of kBlk tuples in the
// pass-1 output and fills one chain of blocks per digit (one LDS atomic per new block,
// no global atomics).  A block holds tuples of one digit: every block of a chain is
// full except its last.  Pass 2 reads each region (pass-1 digit) through a list of its
// blocks, so the pass-1 scatter needs no cursors and the relation is read once in pass 1
// instead of twice (histogram + scatter).
constexpr uint32_t kBlkShift = 8;
constexpr uint32_t kBlk = 1u << kBlkShift;          // elements per block (2 KiB of tuples, 1 KiB of keys)
// 288 blocks (73,728 keys; k_place_seg's LDS copy of a narrow segment, 144 KiB of u16
// residuals, is the limit): a 2^28-key fk relation's ~8,450 blocks per region make 30
// segments (3,840, 15 per CU) instead of 33 at 256 (4,224: a 17th, half-empty round of
// one-workgroup-per-CU placements) -- 2.413-2.422 vs 2.435-2.450 ms per step, round 6
// (profiles/r06za_pass2_ents288_ab.log); 128 blocks (two placements per CU) measured
// slower (r06s).
#ifndef SGXAMD_PASS2_ENTS
#define SGXAMD_PASS2_ENTS 288
#endif
constexpr uint32_t kPass2Ents = SGXAMD_PASS2_ENTS;  // blocks per pass-2 segment (LDS list copy)
struct PoolOut {
    uint32_t *binfo;       // per pool block: digit | fill << 16
    uint64_t *cnt;         // [d][g] (stride nseg): blocks << 40 | tuples of digit d in segment g
    uint32_t *used;        // per segment: blocks taken from its pool
    uint32_t pool_blocks;  // blocks per segment pool
    uint32_t nseg;
    uint32_t g0 = 0;       // this launch's first segment (a pass 1 launched per input piece)
    uint32_t *kmax = nullptr;  // keys (nullable): per segment, its largest key (narrow residuals)
    // narrow pool (keys): the elements written are the residuals key >> rshift as u16
    // (k_scatter_pool's OB 2), speculatively: kmax tells afterwards whether they fit
    bool narrow16 = false;
    uint32_t rshift = 0;
    // the 4-byte pool repeated after a narrow pool: its launches (scatter, layout, block
    // list) return at once when guard (the relation's largest key) >> guard_shift fits 16
    // bits (nullable: unguarded)
    const uint32_t *guard = nullptr;
    uint32_t guard_shift = 0;
    // (nullable) 8 words the layout's first workgroup zeroes: the join's result block, so
    // that launch_make_tasks needs no fill of its own
    uint64_t *zero8 = nullptr;
};
// Pass 1 of a pooled plan: contiguous input segments (m), pooled output in out, digit
// side stream ds beside every stored element.  Elements: in_size-byte input
// (8: row_t, 4: keys), out_size-byte output (8: row_t; 4: the key words only — counting
// joins, whose build/probe reads nothing but keys).
// chain (chain histograms, keys only, chain_hist_supported): instead of the side stream,
// every chain's (segment g, pass-1 digit d) histogram of pass-2 digits (ds.shift2,
// ds.bits2), counted in LDS while the tile is in registers, u32 [d][g][F2] in chain.
hipError_t launch_scatter_pool(const void *in, uint32_t in_size, void *out, uint32_t out_size, const SegMap &m,
                               uint32_t grid, uint32_t shift, uint32_t bits, const PoolOut &po, const DigitSide &ds,
                               hipStream_t s, uint32_t *chain = nullptr);
// Digit widths (pass 1, pass 2) with a chain-histogram pass 1.
bool chain_hist_supported(uint32_t bits1, uint32_t bits2);
// Whether pass 2 of key partitions is the LDS sort k_sort_blk (SGXAMD_SORT2).
bool sort2_enabled();
// After launch_scan_single-style column scans of po.cnt (k_scan_cols, in place): region
// tuple starts / counts (the pass-2 output layout), region block-list bases / lengths
// and the pass-2 segment table (kPass2Ents blocks per segment).
// kmax (nullable): the segments' largest keys (PoolOut::kmax), folded into kmax[nseg] —
// the relation's largest key, which tells pass 2 and the build/probe whether the key
// residuals above the radix bits fit 16 bits (narrow partitions, launch_scatter_blk).
// guard / gshift (nullable): the launches return at once when *guard >> gshift fits 16
// bits (the 4-byte pool repeated after a narrow pool that stood, PoolOut::guard).
hipError_t launch_pool_layout(uint64_t *cnt, uint32_t nseg, uint32_t bits, uint64_t *totals, uint64_t *start,
                              uint64_t *count, uint64_t *lbase, uint64_t *lcount, uint32_t *seg_base, hipStream_t s,
                              uint32_t *kmax = nullptr, const uint32_t *guard = nullptr,
                              uint32_t gshift = 0);
// The block list: region d's blocks at [lbase[d], lbase[d] + lcount[d]) as
// physical block | fill << 32.
hipError_t launch_block_list(const PoolOut &po, const uint64_t *lbase, uint64_t *list, uint32_t bits, hipStream_t s);
// launch_pool_layout + launch_block_list with the layout folded into the block list's
// launch (pass-1 digits up to 8 bits; wider ones take the two launches).
hipError_t launch_pool_layout_list(const PoolOut &po, uint32_t bits, uint64_t *totals, uint64_t *start,
                                   uint64_t *count, uint64_t *lbase, uint64_t *lcount, uint32_t *seg_base,
                                   uint64_t *list, hipStream_t s);
// Pass-2 histogram / scatter over block-list segments (m: reg_start = lbase,
// reg_count = lcount, seg_size = kPass2Ents).
hipError_t launch_hist_side_blk(const uint8_t *side, const uint64_t *list, const SegMap &m, uint32_t grid,
                                uint32_t bits, uint64_t *hist, hipStream_t s);
// The same histogram from the chain histograms (chain plans: no side stream): cnt / tot
// the column-scanned chain records and their totals (launch_pool_layout), chain the chain
// histograms u32 [d][g][F2] (launch_scatter_pool), keys the pass-1 output; the cut and
// possibly wrapped chains' parts are counted from their keys (digit (key >> shift2) &
// (F2 - 1)).  nseg <= kHistChainMaxSegs pass-1 segments.
constexpr uint32_t kHistChainMaxSegs = 16384;
hipError_t launch_hist_chain(const uint64_t *cnt, const uint64_t *tot, uint32_t nseg, const uint32_t *chain,
                             const uint64_t *list, const uint32_t *keys, const SegMap &m, uint32_t grid,
                             uint32_t shift2, uint32_t bits2, uint64_t *hist, hipStream_t s);
// narrow (nullable; key partitions through k_sort_blk only): the relation's largest key
// (launch_pool_layout).  When every key's residual above the radix bits (key >>
// (shift + bits)) fits 16 bits, the partitions are written as those u16 residuals —
// the build/probe (launch_join with the same word) compares residuals, which within
// one partition are equal exactly when the keys are.
// part_start / part_count (nullable; fixed-size segments, launch_scan_regions' partition
// table [region][digit]): with them a narrow relation's pass 2 is the segment placement
// k_place_seg, each segment's digit counts taken from consecutive cursors.
hipError_t launch_scatter_blk(const void *in, const uint64_t *list, void *out, uint32_t elem_size, const SegMap &m,
                              uint32_t grid, uint32_t shift, uint32_t bits, const uint64_t *cursors, hipStream_t s,
                              const uint32_t *narrow = nullptr, const uint64_t *part_start = nullptr,
                              const uint64_t *part_count = nullptr, const uint8_t *side16 = nullptr);
// side16 (nullable): in is a narrow pool (launch_scatter_pool with PoolOut::narrow16)
// whose digits are in this side stream: k_place_seg reads its u16 residuals, while
// k_sort_blk (guarded by the largest key) reads the 4-byte pool repeated when a residual
// did not fit.
bool place_enabled();
// launch_scatter's one-pass cursor scatter writing only the key word of every tuple
// (the multi-GPU shard partition of a counting join, whose exchange moves keys).
hipError_t launch_scatter_keys(const row_t *in, uint32_t *out, const SegMap &m, uint32_t grid, uint32_t shift,
                               uint32_t bits, const uint64_t *cursors, HistLayout layout, uint32_t nseg_stride,
                               const uint64_t *digit_base, hipStream_t s);

// Stable scatter of every segment into `out` at the cursors of the scan.
// digit_base (nullable) is added to the cursors: base[r * F + d].
// ds (nullable): also write the digit side stream for the next pass.
hipError_t launch_scatter(const row_t *in, row_t *out, const SegMap &m, uint32_t grid, uint32_t shift,
                          uint32_t bits, const uint64_t *cursors, HistLayout layout, uint32_t nseg_stride,
                          const uint64_t *digit_base, const DigitSide *ds, hipStream_t s);

// Build + probe over tasks (partition x S chunk of at most s_chunk tuples: kSChunk, or
// kBigSChunk with the kBigRcap table).
// Tasks 0..P-1 are the partitions' first chunks; over[0 .. *n_over) holds the
// further chunks of large S partitions as p | chunk << 32 (launch_make_tasks).
// rcap (2048 / 4096 / 8192, or kBigRcap for counting) = R tuples per LDS chain table.
// mode 0: counts[blockIdx] = per-workgroup partial count (grid entries);
// mode 1: counts[t] = per-task count (P + *n_over entries);
// mode 2: write every match to out[task_off[t] + ...] as output_triple_t.
// cyc (nullable): per workgroup, the wall-clock ticks spent building and probing
// (cyc[2g], cyc[2g+1]); they split the fused kernel's time into the reference's
// Build / Join phases (radix_join.cpp:1291-1352 build_in_depth / join_in_depth timers).
constexpr uint64_t kSChunk = 8192;
// Counting joins of partitions above 8192 R tuples: a 16,384-tuple chain table per
// 1,024-thread workgroup (160 KiB of LDS) and 32,768-tuple S chunks, so that neither
// side is read twice at the 2^30-tuple sizes.
constexpr uint32_t kBigRcap = 16384;
constexpr uint64_t kBigSChunk = 32768;
// S tuples per partition the planner aims at with the big table; partitions that large
// on average are probed in chunks of this size (one task per partition when uniform)
constexpr uint64_t kBigSPart = 65536;
enum JoinMode : int { kJoinCount = 0, kJoinTaskCount = 1, kJoinWrite = 2 };
// Build/probe algorithm of one task: RHO's bucket chaining or RHT's histogram join.
enum JoinAlgo : int { kAlgoChaining = 0, kAlgoHistogram = 1 };
// meta (zeroed here, with the word before it, unless `zeroed`: an earlier launch of the
// call did, PoolOut::zero8): [0] = largest R partition, [1] = largest S partition,
// [2] = the number of extra tasks (u32 n_over, read by launch_join / launch_excl_scan),
// [3..5] zero as well ([5]: launch_join's task tickets).
// zero / zero2 (nullable): nzero / 2 nzero u64 words zeroed as well (k_join_n's count
// and tick slots).
hipError_t launch_make_tasks(const uint64_t *r_count, const uint64_t *s_count, uint64_t P, uint64_t *over,
                             uint32_t over_cap, uint64_t *meta, uint64_t s_chunk, hipStream_t s,
                             uint64_t *zero = nullptr, uint64_t *zero2 = nullptr, uint32_t nzero = 0, bool zeroed = false);
// reduce (mode 0, nullable): the last workgroup to finish sums the partial counts and
// ticks into reduce->result as launch_reduce does (reduce->ticket: a Context::sync word).
struct JoinReduce {
    uint64_t *result;
    uint64_t *ticket;
};
hipError_t launch_join(const row_t *R, const row_t *S, const uint64_t *r_start, const uint64_t *r_count,
                       const uint64_t *s_start, const uint64_t *s_count, uint64_t P, const uint64_t *over,
                       const uint32_t *n_over, uint32_t hash_shift, uint32_t rcap, uint64_t s_chunk, uint32_t grid,
                       int mode, int algo, uint64_t *counts, const uint64_t *task_off, output_triple_t *out,
                       uint64_t *cyc, hipStream_t s, const JoinReduce *reduce = nullptr, int key_stride = 2,
                       uint32_t *tickets = nullptr, const uint32_t *narrow_r = nullptr,
                       const uint32_t *narrow_s = nullptr, uint32_t tasks_max = 0,
                       const uint64_t *small_kmax = nullptr, uint64_t *fold = nullptr,
                       uint64_t *fold_host = nullptr);
// fold (nullable; counting joins on the 16,384-key table, k_join_x): the join's 8-word
// result block -- k_join_x's last workgroup sums the count and tick slots into
// fold[0] / [4] / [5] (k_reduce's job; fold[7], zeroed by launch_make_tasks, is the
// fold_host (nullable, with fold): mapped host memory that also receives the result
// block's words 0..6 (the caller reads them after the stream synchronisation: no copy).
// arrival ticket), whether k_join_x joined or k_join_n did.  Returns
// hipErrorNotSupported (nothing launched) when the plan takes another kernel.
// small_kmax (nullable; tuples, counting, the small joins' 1,024-thread chaining table):
// R's largest key -- chunks whose residuals fit count in a direct table.
// key_stride 2: R / S are row_t partitions; 1: packed u32 keys (counting RHO only —
// the partitions of a counting join carry keys only after the input read).
// tickets (nullable; a u32 that is zero at the launch, e.g. meta[5] of launch_make_tasks):
// the 16,384-key counting table takes its tasks by ticket (k_join_x, SGXAMD_JOIN_TICKETS
// builds) instead of by grid stride.
// narrow_r / narrow_s (nullable; the 16,384-key counting table, key_stride 1): the
// largest keys given to launch_scatter_blk for R / S — a relation whose residuals fit 16
// bits was written as u16 residuals.  Then the join runs in k_join_n (SGXAMD_JOIN_N),
// one workgroup per task: tasks_max (>= P + *n_over) workgroups, their counts and
// ticks added into counts[0 .. grid) / cyc[0 .. 2 grid), which must be zero (the zero
// words of launch_make_tasks).
bool narrow_join_enabled();
// One-block exclusive scan of n_base + *n_extra values; *total = their sum.
hipError_t launch_excl_scan(const uint64_t *in, const uint32_t *n_extra, uint64_t n_base, uint64_t *out,
                            uint64_t *total, hipStream_t s);

// result[0] = sum of the n partials (skipped when partials is null); cyc (nullable, two
// u64 per join workgroup: build / probe wall-clock ticks) -> result[4] / result[5].
hipError_t launch_reduce(const uint64_t *partials, uint32_t n, uint64_t *result, const uint64_t *cyc, uint32_t ncyc,
                         hipStream_t s);

// Multi-GPU u16 wire (wire_kernels.hip): the G senders' runs of u16 residuals, run q at
// bases.b[q] residuals of the receive buffer (a multiple of 8) with bases.n[q] keys in a
// slot of bases.span[q] residuals, each grouped by partition, every partition starting
// on a multiple of 8; rows = G rows of 2 P + 1 words: P partition counts, P partition
// starts (relative to the run) and the sender's largest key.  A row whose counts do not
// add up to n[q], or whose pieces pass its slot, is left out; *narrow = the largest key
// of the rows kept.  scratch: wire_scratch_words(G, P) u64; P <= 2^20.
constexpr uint32_t kWireMaxG = 64;
struct WireBases {
    uint64_t b[kWireMaxG];     // where sender q's run starts (a multiple of 8 residuals)
    uint64_t n[kWireMaxG];     // its keys (the count exchange's announcement)
    uint64_t span[kWireMaxG];  // its slot (residuals)
};
// The piece table in the scratch: ub / nk [p][q] (u32: piece (p, q)'s first unit of 8
// residuals in the receive buffer, its keys), units8[p] = 8 x partition p's units.
struct WirePieces {
    uint32_t *ub, *nk;
    uint64_t *units8;
    uint32_t G, P;
};
uint64_t wire_scratch_words(uint32_t G, uint32_t P);
WirePieces wire_pieces_of(uint64_t *scratch, uint32_t G, uint32_t P);
// The piece table (k_join_np reads S in place) and pc[p] = partition p's keys.
hipError_t launch_wire_pieces(const uint64_t *rows, uint32_t G, uint32_t P, const WireBases &bases, uint64_t *scratch,
                              uint64_t *pc, uint32_t *narrow, hipStream_t s);
// The piece table, then every partition's pieces gathered into out (contiguous
// partitions ps / pc): the path for G > kPieceMax.
hipError_t launch_wire_merge(const uint16_t *in, const uint64_t *rows, uint32_t G, uint32_t P,
                             const WireBases &bases, uint64_t *scratch, uint64_t *ps, uint64_t *pc, uint32_t *narrow,
                             uint16_t *out, hipStream_t s);
// k_join_np (the build/probe over R's contiguous narrow partitions and S's pieces,
// kPieceMax = 8 senders at most), then k_join_x with the count reduction folded in
// (fold: the join's result block).
constexpr uint32_t kPieceMaxG = 8;
hipError_t launch_join_pieces(const void *R, const uint64_t *r_start, const uint64_t *r_count, const uint16_t *s16,
                              uint64_t s_bytes, const WirePieces &w, uint64_t P, const uint64_t *over,
                              const uint32_t *n_over, uint32_t hash_shift, uint64_t s_chunk, uint32_t grid,
                              uint32_t tasks_max, uint64_t *counts, uint64_t *cyc, uint32_t *tickets,
                              const uint32_t *narrow_r, const uint32_t *narrow_s, uint64_t *fold, hipStream_t s);

}  // namespace rho
}  // namespace sgxamd
