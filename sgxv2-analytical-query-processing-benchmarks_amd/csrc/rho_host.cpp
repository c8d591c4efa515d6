// Host orchestration of the MI355X RHO join: partitioning policy, workspace,
// kernel sequence and the C-ABI entry points of sgxamd/rho.h.
//
// Mirrors the phase structure of join_init_run / prj_thread
// (radix_join.cpp:1369-1638 / :1067-1356): pass-1 partition of R then S, optional
// pass 2, then build+probe of every partition pair; but each phase is a sequence
// of device-wide kernels instead of T pthreads with barriers, and partitions are
// sized for the LDS of a CU rather than for L2 (calc_num_radix_bits :295-317).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>
#include <cstdio>

#include "common.hpp"
#include "rho_device.hpp"
#include "rho_internal.hpp"
#include "runtime.hpp"
#include "sgxamd/rho.h"

namespace sgxamd {
namespace rho {

namespace {

constexpr uint64_t kTargetPartition = 4096;  // R tuples per partition (= RCAP of an 8192-slot table)
constexpr uint32_t kMaxBits = 18;
constexpr uint64_t kMaxRChunk = 8192;         // largest LDS chain table (k_join RCAP)
constexpr uint32_t kSegTarget = 2048;        // workgroups per partition pass and relation

inline uint32_t ceil_log2(uint64_t x) {
    uint32_t b = 0;
    while ((1ull << b) < x) ++b;
    return b;
}

struct Policy {
    uint32_t bits, passes, b1, b2, rcap;
};
// Development A/B switch for the 16,384-tuple counting table (SGXAMD_BIG_JOIN=0: R
// partitions above 8192 tuples are built in 8192-tuple chunks, each S chunk probed once
// per chunk).  Read once per process.
inline bool big_join_enabled() {
    static const bool on = [] {
        const char *e = std::getenv("SGXAMD_BIG_JOIN");
        return !(e && std::atoi(e) == 0);
    }();
    return on;
}

// Counting joins (no materialisation; RHO's chain table k_join_x, RHT's bucket table
// k_join_hist<kBigRcap>) build partitions above 8192 R tuples in kBigRcap-tuple LDS
// tables; materialising joins in 8192-tuple chunks.
inline bool uses_big_table(const mi355_rho_opts *o) { return !(o && o->materialize) && big_join_enabled(); }
// The caller left the radix bits to the planner (an explicit plan keeps its tables).
inline bool opts_free_bits(const mi355_rho_opts *o) { return !(o && o->radix_bits > 0); }

Policy choose_policy(uint64_t nR, uint64_t nS, const mi355_rho_opts *o) {
    Policy p{};
    if (o && o->radix_bits > 0) {
        p.bits = std::min<uint32_t>((uint32_t)o->radix_bits, kMaxBits);
    } else {
        // R partitions fit one LDS chain table; and when S is much larger than R, enough
        // partitions that an average S partition is one build/probe task (kSChunk):
        // every further S chunk of a partition rebuilds its R table.
        // The S-driven bits stop at 16 (two passes of <= 8 bits: a 9-bit pass-1 scatter
        // holds 512 digits in LDS and runs at half speed).
        // Past 2^28 R tuples the partition target asks for 17-18 bits, i.e. a 9-bit pass;
        // that costs more than giving the join two LDS tables per partition (each S
        // chunk probed twice), so the R-driven bits stay at 16 until an average
        // partition would exceed two tables.
        // Counting joins with the 16,384-tuple table size partitions for that table
        // once there are enough of them to fill the chip (>= 2^13 tasks): fewer digits
        // per partition pass; S-driven bits aim at 65,536 S keys per partition
        // (BASELINE config 4, 2^27 x 2^30: 14 bits = 7 + 7, 7.71-7.94 ms per join even
        // with R's table built twice per partition, vs 8.04-8.28 at 15 bits = 8 + 7 with
        // 32,768 per partition: an 8-bit pass over 2^30 keys costs more than that build;
        // 13 bits = 7 + 6, 131,072 per partition: 7.77-7.79).
        // scripts/size_sweep.py, DESIGN.md §3 (|R| = |S|, ms): 2^28: 14 / 15 / 16 bits
        // 5.53 / 5.58 / 5.71; 2^30: 16 / 17 / 18 bits 23.2 / 30.4 / 41.3; 2^31: 16 / 17
        // / 18 bits 47.2 / 60.7 / 83.5.
        const bool big = uses_big_table(o);
        const uint64_t table = big ? kBigRcap : kMaxRChunk;
        const auto clog2 = [](uint64_t num, uint64_t den) {
            return ceil_log2(std::max<uint64_t>((num + den - 1) / den, 1));
        };
        const uint32_t cap_r = std::max<uint32_t>(16, clog2(nR, 2 * table));
        uint32_t bits_r = std::min(clog2(nR, kTargetPartition), cap_r);
        uint32_t bits_s = std::min<uint32_t>(clog2(nS, kSChunk), 16);
        if (big && clog2(nR, kBigRcap) >= 13) {
            bits_r = std::min(clog2(nR, kBigRcap), cap_r);
            bits_s = std::min<uint32_t>(clog2(nS, kBigSPart), 16);
        }
        p.bits = std::min(std::max(bits_r, bits_s), kMaxBits);
    }
    p.passes = (o && o->passes > 0) ? (uint32_t)o->passes : (p.bits <= 8 ? 1u : 2u);
    if (p.passes > 2) p.passes = 2;
    if (p.bits > 9 && p.passes == 1) p.passes = 2;  // one pass is limited to kMaxF = 2^9 bins
    if (p.passes == 2 && p.bits < 2) p.passes = 1;
    if (p.passes == 1) {
        p.b1 = p.bits;
        p.b2 = 0;
    } else {
        // odd bit counts: the larger digit in pass 1
        p.b1 = (p.bits + 1) / 2;
        static const int forced_b1 = [] {  // SGXAMD_PASS1_BITS: development A/B of the split
            const char *e = std::getenv("SGXAMD_PASS1_BITS");
            return e ? std::atoi(e) : 0;
        }();
        // (single-GPU joins only: it is a per-process setting, and the ranks of a multi-GPU
        // join -- key_shift > 0 -- must agree on the split, which numbers the u16 wire's
        // partitions; a pass-1 digit is at most kMaxF = 2^9 bins)
        if (forced_b1 > 0 && forced_b1 <= 9 && (uint32_t)forced_b1 < p.bits && p.bits - (uint32_t)forced_b1 <= 8 &&
            !(o && o->key_shift > 0))
            p.b1 = (uint32_t)forced_b1;
        p.b2 = p.bits - p.b1;
    }
    // chain table large enough that the average partition needs one R chunk
    const uint64_t avg = (nR + (1ull << p.bits) - 1) >> p.bits;
    p.rcap = avg <= 2048 ? 2048 : (avg <= 4096 ? 4096 : 8192);
    return p;
}

// Two-pass plans carry the pass-2 digit of every pass-1 output tuple in a byte side
// stream (launch_hist_side); a 9-bit pass-2 digit does not fit and takes the tuple
// histogram instead.
// SGXAMD_DIGIT_SIDE=0 turns it off (development A/B switch; results are identical).
inline bool digit_side_enabled() {
    static const bool on = [] {
        const char *e = std::getenv("SGXAMD_DIGIT_SIDE");
        return !(e && std::atoi(e) == 0);
    }();
    return on;
}
inline bool uses_digit_side(const Policy &p) { return p.passes == 2 && p.b2 <= 8 && digit_side_enabled(); }

// Two-pass plans with the digit side stream take the pooled pass 1 (no pass-1
// histogram: rho_internal.hpp PoolOut).  SGXAMD_POOL=0 keeps the histogram
// + cursor pass 1 (development A/B switch; results are identical).  SGXAMD_POOL_SEGS:
// pass-1 workgroups per relation (development; default kPoolSegs).
inline bool pool_enabled() {
    static const bool on = [] {
        const char *e = std::getenv("SGXAMD_POOL");
        return !(e && std::atoi(e) == 0);
    }();
    return on;
}
// Counting RHO joins (no materialisation, bucket chaining) move keys only after the
// input read: the build/probe of a count reads nothing else (radix_join.cpp:429-436
// compares keys; the payloads are never read), so the pooled pass 1 writes the key
// word of every tuple and pass 2 and the build/probe run on 4-byte keys.
// SGXAMD_KEYS=0 keeps whole tuples (development A/B switch; results are identical).
inline bool keys_enabled() {
    static const bool on = [] {
        const char *e = std::getenv("SGXAMD_KEYS");
        return !(e && std::atoi(e) == 0);
    }();
    return on && thread_key_layout();
}
// Pooled key plans with a 7-bit pass 1 and a 6- or 7-bit pass 2 count every chain's
// pass-2 digits in the pass-1 scatter (chain histograms, rho_internal.hpp
// launch_scatter_pool): no digit side stream is written, and the pass-2 histogram sums
// the chain histograms of a segment's whole chains and counts only its cut chains' keys
// (launch_hist_chain).  Round 6: 2.50-2.51 ms per step vs 2.60-2.62 with the side stream
// (pass 1 0.72 vs 0.745 ms, the pass-2 histogram 0.035 vs 0.071 ms per relation;
// profiles/r06n_chain_hist_ab.log).  SGXAMD_CHAIN_HIST=0 keeps the side stream
// (development A/B switch; results identical); the narrow pool (SGXAMD_NARROW_POOL=1)
// writes the side stream and takes no chain histograms.
// Narrow key partitions (counting RHO with the 16,384-key table over key partitions):
// pass 1 takes the largest key, and when the residuals above the radix bits fit 16 bits, pass 2
// writes them as u16 and the build/probe reads 2 instead of 4 bytes per key
// (launch_scatter_blk).  SGXAMD_NARROW=0 keeps 4-byte keys (development A/B switch).
inline bool narrow_enabled() {
    static const bool on = [] {
        const char *e = std::getenv("SGXAMD_NARROW");
        return !(e && std::atoi(e) == 0);
    }();
    return on;
}
// SGXAMD_NARROW_POOL=1 (development A/B switch, read once): narrow plans' pass 1 writes
// the narrow pool (u16 residuals + the digit side stream, 11 B per tuple instead of 13;
// repeated as 4-byte keys when a residual does not fit) instead of 4-byte keys.  Measured
// and not the default (r05j): pass 1 takes the same 0.74 ms either way -- it is bound by
// its tile sort in LDS, not by the bytes it writes -- and pass 2 gains 0.02 ms.
inline bool narrow_pool_enabled() {
    static const bool on = [] {
        const char *e = std::getenv("SGXAMD_NARROW_POOL");
        return e && std::atoi(e) == 1;
    }();
    return on;
}
inline bool chain_enabled() {
    static const bool on = [] {
        const char *e = std::getenv("SGXAMD_CHAIN_HIST");
        return !(e && std::atoi(e) == 0);
    }();
    return on && !narrow_pool_enabled();
}
constexpr uint32_t kPoolSegs = 512;  // two 512-thread workgroups per CU: one wave of workgroups
inline uint32_t pool_segs() {
    static const uint32_t v = [] {
        const char *e = std::getenv("SGXAMD_POOL_SEGS");
        const long x = e ? std::atol(e) : 0;
        return x > 0 ? (uint32_t)x : kPoolSegs;
    }();
    return v;
}


inline uint64_t seg_size_for(uint64_t n) {
    uint64_t s = (n + kSegTarget - 1) / kSegTarget;
    s = (s + kTile - 1) / kTile * kTile;
    return std::max<uint64_t>(s, kTile);
}

struct RelPlan {
    uint64_t n;
    uint64_t seg1;
    uint32_t nseg1;
    uint64_t seg2;
    uint32_t grid2;
    bool pooled;           // pooled pass 1 + block-list pass 2
    bool keys;             // the partitions hold 4-byte keys (counting joins; pooled, or a shard pass)
    bool chain;            // chain histograms instead of the digit side stream (pooled keys)
    uint32_t in_size;      // bytes per input element: 8 (row_t) or 4 (keys, a keys-only exchange)
    uint32_t pool_blocks;  // blocks per pass-1 segment pool
    uint64_t t1_tuples;    // capacity of the pass-1 output (and side stream) in tuples
    // scratch offsets (pooled: hist1 holds the chain records, tot1 their column totals)
    size_t hist1, tot1, start1, cnt1, segbase2, hist2, pstart, pcnt;
    size_t binfo, used, lbase, lcount, list;
    size_t chist;  // chain histograms [F1][nseg1][F2]
    size_t kmax;   // pooled keys: the segments' largest keys, then the relation's ([nseg1])
    bool narrow;   // pass 2 writes u16 residuals when the largest key allows (plan_join)
    bool narrow16; // pass 1 writes a narrow pool first (u16 residuals, the 4-byte pool repeated if a residual does not fit)
    bool pad_parts = false;  // pass 2's partitions start on multiples of 8 elements (the u16 wire's senders)
    // pooled pass 1 per input piece (the multi-GPU exchange's received pieces): piece i is
    // elements [piece_off[i], + piece_n[i]), its segments start at piece_g0[i]; its launch
    // waits for piece_ev[i] (null: no wait)
    std::vector<uint64_t> piece_off, piece_n;
    std::vector<uint32_t> piece_g0;
    std::vector<hipEvent_t> piece_ev;
    uint64_t *zero8 = nullptr;  // pooled pass 1: its layout zeroes these 8 words (the join's result block)
};

#define RHO_HIP(call)                                                                      \
    do {                                                                                   \
        hipError_t _e = (call);                                                            \
        if (_e != hipSuccess) {                                                            \
            set_last_error(std::string(#call) + ": " + hipGetErrorString(_e));             \
            return (_e == hipErrorOutOfMemory) ? MI355_ERR_OOM : MI355_ERR_HIP;            \
        }                                                                                  \
    } while (0)

// Pooled two-pass partition of one relation (pass 1 when !pass2_now, else pass 2).
// arena: where rp's scratch lives (null: the context's join scratch)
int partition_relation_pooled(Context *ctx, hipStream_t s, Timer &tm, const std::string &t, const row_t *in,
                              row_t *t1, row_t *t2, uint8_t *side, RelPlan &rp, const Policy &pol, uint32_t key_shift,
                              const row_t **final_rel, const uint64_t **pstart, const uint64_t **pcnt,
                              bool pass2_now, Arena *arena = nullptr) {
    Arena &A = arena ? *arena : ctx->scratch;
    uint64_t *start1 = A.at<uint64_t>(rp.start1);
    uint64_t *cnt1 = A.at<uint64_t>(rp.cnt1);
    uint32_t *segbase2 = A.at<uint32_t>(rp.segbase2);
    uint64_t *lbase = A.at<uint64_t>(rp.lbase), *lcount = A.at<uint64_t>(rp.lcount);
    uint64_t *list = A.at<uint64_t>(rp.list);
    const uint32_t F1 = 1u << pol.b1;
    if (!pass2_now) {
        PoolOut po{A.at<uint32_t>(rp.binfo), A.at<uint64_t>(rp.hist1), A.at<uint32_t>(rp.used), rp.pool_blocks,
                   rp.nseg1};
        po.kmax = rp.narrow ? A.at<uint32_t>(rp.kmax) : nullptr;
        po.zero8 = rp.zero8;
        const DigitSide ds{rp.chain ? nullptr : side, key_shift + pol.b1, pol.b2};
        uint32_t *chist = rp.chain ? A.at<uint32_t>(rp.chist) : nullptr;
        // pass 1 over the relation (one launch, or one per piece as it lands, its segments
        // numbered after the earlier pieces' -- one pool layout over all of them)
        const auto scatter = [&](PoolOut &p) -> int {
            if (rp.piece_n.empty()) {
                const SegMap m1{nullptr, nullptr, nullptr, 1, rp.seg1, rp.n};
                RHO_HIP(launch_scatter_pool(in, rp.in_size, t1, rp.keys ? 4u : 8u, m1, rp.nseg1, key_shift, pol.b1, p,
                                            ds, s, chist));
                return MI355_OK;
            }
            const char *ib = reinterpret_cast<const char *>(in);
            for (size_t i = 0; i < rp.piece_n.size(); ++i) {
                if (i < rp.piece_ev.size() && rp.piece_ev[i]) RHO_HIP(hipStreamWaitEvent(s, rp.piece_ev[i], 0));
                const uint64_t n = rp.piece_n[i];
                if (!n) continue;
                const SegMap mi{nullptr, nullptr, nullptr, 1, rp.seg1, n};
                p.g0 = rp.piece_g0[i];
                RHO_HIP(launch_scatter_pool(ib + rp.piece_off[i] * rp.in_size, rp.in_size, t1, rp.keys ? 4u : 8u, mi,
                                            (uint32_t)((n + rp.seg1 - 1) / rp.seg1), key_shift, pol.b1, p, ds, s,
                                            chist));
            }
            return MI355_OK;
        };
        const auto layout = [&](const PoolOut &p) -> int {
            RHO_HIP(launch_pool_layout_list(p, pol.b1, A.at<uint64_t>(rp.tot1), start1, cnt1, lbase, lcount, segbase2,
                                            list, s));
            return MI355_OK;
        };
        int rc;
        if (rp.narrow16) {
            // the narrow pool (u16 residuals + the side stream), then the 4-byte pool's
            // launches guarded by the relation's largest key: they return at once when
            // every residual fit (the guards read the word the narrow pool's layout wrote)
            PoolOut pn = po;
            pn.narrow16 = true;
            pn.rshift = key_shift + pol.b1 + pol.b2;
            tm.mark((t + "pass1_scatter").c_str());
            if ((rc = scatter(pn))) return rc;
            tm.mark((t + "pass1_scan").c_str());
            if ((rc = layout(pn))) return rc;
            PoolOut pw = po;
            pw.guard = po.kmax + rp.nseg1;
            pw.guard_shift = pn.rshift;
            tm.mark((t + "pass1_wide").c_str());
            if ((rc = scatter(pw))) return rc;
            if ((rc = layout(pw))) return rc;
        } else {
            tm.mark((t + "pass1_scatter").c_str());
            if ((rc = scatter(po))) return rc;
            tm.mark((t + "pass1_scan").c_str());
            if ((rc = layout(po))) return rc;
        }
        *final_rel = t1;
        *pstart = start1;
        *pcnt = cnt1;
        return MI355_OK;
    }
    uint64_t *hist2 = A.at<uint64_t>(rp.hist2);
    uint64_t *ps = A.at<uint64_t>(rp.pstart);
    uint64_t *pc = A.at<uint64_t>(rp.pcnt);
    const SegMap m2{lbase, lcount, segbase2, F1, kPass2Ents, rp.n};
    const uint32_t *narrow = rp.narrow ? A.at<uint32_t>(rp.kmax) + rp.nseg1 : nullptr;
    tm.mark((t + "pass2_hist").c_str());
    if (rp.chain)  // from the chain histograms pass 1 stored (and the cut chains' keys)
        RHO_HIP(launch_hist_chain(A.at<uint64_t>(rp.hist1), A.at<uint64_t>(rp.tot1), rp.nseg1,
                                  A.at<uint32_t>(rp.chist), list, reinterpret_cast<const uint32_t *>(t1), m2,
                                  rp.grid2, key_shift + pol.b1, pol.b2, hist2, s));
    else
        RHO_HIP(launch_hist_side_blk(side, list, m2, rp.grid2, pol.b2, hist2, s));
    tm.mark((t + "pass2_scan").c_str());
    RHO_HIP(launch_scan_regions(hist2, segbase2, start1, F1, pol.b2, ps, pc, s, rp.pad_parts));
    tm.mark((t + "pass2_scatter").c_str());
    RHO_HIP(launch_scatter_blk(t1, list, t2, rp.keys ? 4u : 8u, m2, rp.grid2, key_shift + pol.b1, pol.b2, hist2, s,
                               narrow, ps, pc, rp.narrow16 ? side : nullptr));
    *final_rel = t2;
    *pstart = ps;
    *pcnt = pc;
    return MI355_OK;
}

// Pass 1 of an unpooled plan in its two halves: the histogram and its scan (digit
// starts / counts in start1 / cnt1), then the scatter (side: the pass-2 digit stream, or
// null).  The shard exchange runs every piece's first half before any second half.
int pass1_counts(Context *ctx, hipStream_t s, Timer &tm, const std::string &t, const row_t *in, const RelPlan &rp,
                 const Policy &pol, uint32_t key_shift) {
    Arena &A = ctx->scratch;
    const SegMap m1{nullptr, nullptr, nullptr, 1, rp.seg1, rp.n};
    uint64_t *hist1 = A.at<uint64_t>(rp.hist1);
    tm.mark((t + "pass1_hist").c_str());
    RHO_HIP(launch_hist(in, m1, rp.nseg1, key_shift, pol.b1, hist1, kDigitMajor, rp.nseg1, s));
    tm.mark((t + "pass1_scan").c_str());
    RHO_HIP(launch_scan_single(hist1, rp.nseg1, pol.b1, A.at<uint64_t>(rp.tot1), A.at<uint64_t>(rp.start1),
                               A.at<uint64_t>(rp.cnt1), 0, pol.passes == 2 ? A.at<uint32_t>(rp.segbase2) : nullptr,
                               rp.seg2, s));
    return MI355_OK;
}

int pass1_scatter(Context *ctx, hipStream_t s, Timer &tm, const std::string &t, const row_t *in, row_t *t1,
                  uint8_t *side, const RelPlan &rp, const Policy &pol, uint32_t key_shift) {
    Arena &A = ctx->scratch;
    const SegMap m1{nullptr, nullptr, nullptr, 1, rp.seg1, rp.n};
    uint64_t *hist1 = A.at<uint64_t>(rp.hist1), *start1 = A.at<uint64_t>(rp.start1);
    tm.mark((t + "pass1_scatter").c_str());
    const DigitSide ds{side, key_shift + pol.b1, pol.b2};
    if (rp.keys)  // one pass writing key words (the keys-only shard partition)
        RHO_HIP(launch_scatter_keys(in, reinterpret_cast<uint32_t *>(t1), m1, rp.nseg1, key_shift, pol.b1, hist1,
                                    kDigitMajor, rp.nseg1, start1, s));
    else
        RHO_HIP(launch_scatter(in, t1, m1, rp.nseg1, key_shift, pol.b1, hist1, kDigitMajor, rp.nseg1, start1,
                               side ? &ds : nullptr, s));
    return MI355_OK;
}

// One relation through pass 1 (and pass 2).  Returns the final buffer and
// partition table pointers through *final / *pstart / *pcnt.  side (n bytes, two-pass
// plans whose pass-2 digit fits a byte): the pass-1 scatter writes every tuple's pass-2
// digit there, and pass 2's histogram reads those bytes instead of the tuples.
int partition_relation(Context *ctx, hipStream_t s, Timer &tm, const char *tag, const row_t *in, row_t *t1,
                       row_t *t2, uint8_t *side, RelPlan &rp, const Policy &pol, uint32_t key_shift,
                       const row_t **final_rel, const uint64_t **pstart, const uint64_t **pcnt, bool pass2_now) {
    Arena &A = ctx->scratch;
    uint64_t *start1 = A.at<uint64_t>(rp.start1);
    uint64_t *cnt1 = A.at<uint64_t>(rp.cnt1);
    uint32_t *segbase2 = A.at<uint32_t>(rp.segbase2);
    std::string t(tag);
    const bool use_side = side != nullptr && uses_digit_side(pol);
    if (rp.pooled) return partition_relation_pooled(ctx, s, tm, t, in, t1, t2, side, rp, pol, key_shift, final_rel,
                                                    pstart, pcnt, pass2_now);
    if (!pass2_now)  // pieces (multi-GPU exchange): an unpooled pass reads the whole input at once
        for (hipEvent_t e : rp.piece_ev)
            if (e) RHO_HIP(hipStreamWaitEvent(s, e, 0));
    if (!pass2_now) {
        int rc = pass1_counts(ctx, s, tm, t, in, rp, pol, key_shift);
        if (!rc) rc = pass1_scatter(ctx, s, tm, t, in, t1, use_side ? side : nullptr, rp, pol, key_shift);
        if (rc) return rc;
        *final_rel = t1;
        *pstart = start1;
        *pcnt = cnt1;
        return MI355_OK;
    }
    uint64_t *hist2 = A.at<uint64_t>(rp.hist2);
    uint64_t *ps = A.at<uint64_t>(rp.pstart);
    uint64_t *pc = A.at<uint64_t>(rp.pcnt);
    const uint32_t F1 = 1u << pol.b1;
    SegMap m2{start1, cnt1, segbase2, F1, rp.seg2, rp.n};
    const uint32_t shift2 = key_shift + pol.b1;
    tm.mark((t + "pass2_hist").c_str());
    if (use_side)
        RHO_HIP(launch_hist_side(side, m2, rp.grid2, pol.b2, hist2, s));
    else
        RHO_HIP(launch_hist(t1, m2, rp.grid2, shift2, pol.b2, hist2, kSegMajor, 0, s));
    tm.mark((t + "pass2_scan").c_str());
    RHO_HIP(launch_scan_regions(hist2, segbase2, start1, F1, pol.b2, ps, pc, s));
    tm.mark((t + "pass2_scatter").c_str());
    RHO_HIP(launch_scatter(t1, t2, m2, rp.grid2, shift2, pol.b2, hist2, kSegMajor, 0, nullptr, nullptr, s));
    *final_rel = t2;
    *pstart = ps;
    *pcnt = pc;
    return MI355_OK;
}

// Pass-1 segment size of a pooled plan: whole tiles, about pool_segs() segments.
inline uint64_t pool_seg_size(uint64_t n) {
    const uint64_t seg = (n + pool_segs() - 1) / pool_segs();
    return std::max<uint64_t>((seg + kTile - 1) / kTile * kTile, kTile);
}
// Whether a relation of n tuples can take the pooled plan: a two-pass plan with the
// digit side stream, and block counts that fit the 24-bit chain records.
inline bool pool_fits(uint64_t n, const Policy &pol, uint64_t extra_segs = 0) {
    if (!(pol.passes == 2 && uses_digit_side(pol) && pool_enabled())) return false;
    const uint64_t seg = pool_seg_size(n), nseg = (n + seg - 1) / seg + extra_segs;
    const uint64_t pb = (seg + kBlk - 1) / kBlk + (1u << pol.b1);
    return n / kBlk + nseg * (1u << pol.b1) < (1ull << 24) && nseg * pb < (1ull << 27);
}
enum PoolMode : int { kNoPool = 0, kPoolTuples = 1, kPoolKeys = 2 };

void plan_relation(Arena &A, RelPlan &rp, uint64_t n, const Policy &pol, int pool = kNoPool,
                   const std::vector<uint64_t> *pieces = nullptr) {
    rp.n = n;
    rp.seg1 = seg_size_for(n);
    rp.nseg1 = (uint32_t)((n + rp.seg1 - 1) / rp.seg1);
    const uint32_t F1 = 1u << pol.b1, F2 = 1u << pol.b2;
    rp.seg2 = seg_size_for(n);
    rp.grid2 = (uint32_t)((n + rp.seg2 - 1) / rp.seg2) + F1;
    rp.t1_tuples = n;
    rp.pooled = false;
    rp.keys = false;
    rp.chain = false;
    rp.narrow = false;
    rp.narrow16 = false;
    rp.pad_parts = false;
    rp.kmax = 0;
    rp.in_size = sizeof(row_t);
    rp.piece_off.clear();
    rp.piece_n.clear();
    rp.piece_g0.clear();
    rp.piece_ev.clear();
    rp.zero8 = nullptr;
    if (pieces && !pieces->empty()) {  // the input arrives in pieces (every plan waits for them)
        uint64_t off = 0;
        for (uint64_t pn : *pieces) {
            rp.piece_off.push_back(off);
            rp.piece_n.push_back(pn);
            rp.piece_g0.push_back(0);
            off += pn;
        }
    }
    if (pool != kNoPool) {
        // pass-1 segments of whole tiles, about pool_segs() of them; every digit of a
        // segment fills ceil(elements / kBlk) blocks, so a pool of ceil(seg1 / kBlk) + F1
        // blocks always suffices.  Chain records pack blocks << 40 | elements.
        const uint64_t seg = pool_seg_size(n);
        uint32_t nseg = (uint32_t)((n + seg - 1) / seg);
        if (!rp.piece_n.empty()) {  // segments never straddle two pieces
            nseg = 0;
            for (size_t i = 0; i < rp.piece_n.size(); ++i) {
                rp.piece_g0[i] = nseg;
                nseg += (uint32_t)((rp.piece_n[i] + seg - 1) / seg);
            }
        }
        const uint64_t pb = (seg + kBlk - 1) / kBlk + F1;
        const uint64_t max_blocks = n / kBlk + (uint64_t)nseg * F1;
        rp.pooled = true;
        rp.keys = pool == kPoolKeys;
        // chain histograms: 32-bit list positions and a u32 segment slot table
        rp.chain = rp.keys && chain_enabled() && sort2_enabled() && chain_hist_supported(pol.b1, pol.b2) &&
                   nseg <= kHistChainMaxSegs;
        rp.seg1 = seg;
        rp.nseg1 = nseg;
        rp.pool_blocks = (uint32_t)pb;
        rp.t1_tuples = (uint64_t)nseg * pb * kBlk;
        // pass-2 segments: kPass2Ents blocks, at most one partial segment per region
        rp.grid2 = (uint32_t)(max_blocks / kPass2Ents) + F1 + 1;
    }
    // (+ 1: a small join's histogram workgroups write two offsets per 2-tile segment)
    rp.hist1 = A.reserve(sizeof(uint64_t) * (size_t)F1 * (std::max<uint32_t>(rp.nseg1, 1) + 1));
    rp.tot1 = A.reserve(sizeof(uint64_t) * F1);
    rp.start1 = A.reserve(sizeof(uint64_t) * F1);
    rp.cnt1 = A.reserve(sizeof(uint64_t) * F1);
    rp.segbase2 = A.reserve(sizeof(uint32_t) * (F1 + 1));
    if (pol.passes == 2) {
        rp.hist2 = A.reserve(sizeof(uint64_t) * (size_t)rp.grid2 * F2);
        rp.pstart = A.reserve(sizeof(uint64_t) * (size_t)F1 * F2);
        rp.pcnt = A.reserve(sizeof(uint64_t) * (size_t)F1 * F2);
    }
    if (rp.pooled) {
        rp.binfo = A.reserve(sizeof(uint32_t) * (size_t)rp.nseg1 * rp.pool_blocks);
        rp.used = A.reserve(sizeof(uint32_t) * rp.nseg1);
        rp.lbase = A.reserve(sizeof(uint64_t) * F1);
        rp.lcount = A.reserve(sizeof(uint64_t) * F1);
        rp.list = A.reserve(sizeof(uint64_t) * (size_t)(rp.n / kBlk + (uint64_t)rp.nseg1 * F1));
        if (rp.keys) rp.kmax = A.reserve(sizeof(uint32_t) * ((size_t)rp.nseg1 + 1));
    }
    if (rp.chain) {
        rp.chist = A.reserve(sizeof(uint32_t) * (size_t)F1 * rp.nseg1 * F2);
    }
}

}  // namespace

// One join between its two halves (join_begin / join_finish): the policy and plans of
// both relations, R's partitioned result and the scratch offsets of the join.
struct PendingJoin {
    bool active = false;
    hipStream_t s = nullptr;
    Policy pol{};
    RelPlan pr{}, ps{};
    uint64_t nR = 0, nS = 0;
    uint32_t key_shift = 0;
    bool materialize = false;
    int algo = kAlgoChaining;
    hipStream_t s2 = nullptr;
    const row_t *fR = nullptr;
    const uint64_t *psR = nullptr, *pcR = nullptr;
    size_t off_over = 0, off_counts = 0, off_toff = 0, off_result = 0, off_cyc = 0;
    uint32_t over_cap = 0, join_grid = 0;
    uint64_t s_chunk = kSChunk;  // S tuples per build/probe task
};

namespace {
std::mutex g_pending_mu;
std::unordered_map<const Context *, PendingJoin> g_pending;

PendingJoin &pending_of(const Context *ctx) {
    std::lock_guard<std::mutex> lk(g_pending_mu);
    return g_pending[ctx];
}
}  // namespace

// First half: plans both relations (|S| = nS, its tuples are not read yet), then
// enqueues R's partition passes on s and returns without waiting.  The second half
// may start after S has been produced later in the stream order of s (multi-GPU:
// R's local passes run while S is still being exchanged).  Caller holds ctx->mu.
// Policy, workspace and scratch layout of a join of nR x nS tuples (no launches).
// The 16,384-key counting table with 32,768-key S chunks: partitions above 8192 R keys,
// and plans sized for those S chunks (plan_join).
bool takes_big_table(const Policy &pol, uint64_t nR, uint64_t nS, const mi355_rho_opts *opts) {
    const uint64_t P = 1ull << pol.bits;
    const uint64_t avgR = (nR + P - 1) / P, avgS = (nS + P - 1) / P;
    return uses_big_table(opts) && ((pol.rcap == 8192 && avgR > 8192) ||
                                    (P >= 8192 && avgS > kSChunk && avgR <= kBigRcap && opts_free_bits(opts)));
}

// wire16: S's partitions arrive as narrow residuals (the multi-GPU u16 wire,
// join_pipelined_finish_wire16): the 16,384-key table and the narrow join (R's pass 2
// writes residuals too), whatever the received sizes.
int plan_join(Context *ctx, hipStream_t s, uint64_t nR, uint64_t nS, const mi355_rho_opts *opts, PendingJoin &pj,
              const std::vector<uint64_t> *s_pieces = nullptr, bool wire16 = false) {
    pj = PendingJoin{};
    pj.s = s;
    pj.nR = nR;
    pj.nS = nS;
    pj.key_shift = opts ? opts->key_shift : 0;
    pj.materialize = opts && opts->materialize;
    pj.algo = (opts && opts->algorithm == MI355_ALGO_RHT) ? kAlgoHistogram : kAlgoChaining;
    pj.pol = choose_policy(nR, nS, opts);
    const Policy &pol = pj.pol;
    if (pj.key_shift + pol.bits > 31) {
        set_last_error("key_shift + radix bits must stay below 32");
        return MI355_ERR_INVALID;
    }
    Arena &A = ctx->scratch;
    A.reset();
    // both relations take the same layout (the build/probe reads both alike)
    // counting joins (RHO and RHT) move 4-byte keys after the input read
    const bool counting = !pj.materialize;
    const uint64_t ks = s_pieces ? s_pieces->size() : 0;
    const int pool = !(pool_fits(nR, pol) && pool_fits(nS, pol, ks)) ? kNoPool
                     : (counting && keys_enabled())                  ? kPoolKeys
                                                                      : kPoolTuples;
    plan_relation(A, pj.pr, nR, pol, pool);
    plan_relation(A, pj.ps, nS, pol, pool, s_pieces);
    const uint64_t c1R = pj.pr.t1_tuples, c1S = pj.ps.t1_tuples;  // pooled pass 1 needs room for its pools
    RHO_HIP(ctx->t1R.ensure(std::max<uint64_t>(c1R, 1) * sizeof(row_t)));
    RHO_HIP(ctx->t1S.ensure(std::max<uint64_t>(c1S, 1) * sizeof(row_t)));
    if (pol.passes == 2) {
        RHO_HIP(ctx->t2R.ensure(std::max<uint64_t>(nR, 1) * sizeof(row_t)));
        RHO_HIP(ctx->t2S.ensure(std::max<uint64_t>(nS, 1) * sizeof(row_t)));
    }
    if (uses_digit_side(pol) && !(pj.pr.chain && pj.ps.chain)) {  // chain histograms need no side stream
        RHO_HIP(ctx->sideR.ensure(std::max<uint64_t>(c1R, 16)));
        RHO_HIP(ctx->sideS.ensure(std::max<uint64_t>(c1S, 16)));
    }
    const uint64_t P = 1ull << pol.bits;
    // the 16,384-key counting table with 32,768-key S chunks: partitions above 8192 R
    // keys, and plans sized for those S chunks (S much larger than R, e.g. BASELINE config
    // 4: 4096 R and 32,768 S keys per partition read R once per partition instead of once
    // per 8192-key S chunk); enough partitions that one task each fills the chip
    const uint64_t avgS = (nS + P - 1) / P;
    if (wire16 || takes_big_table(pol, nR, nS, opts)) {
        pj.pol.rcap = kBigRcap;
        // S-heavy plans (BASELINE config 4: 65,536 S keys per partition) probe a
        // partition in one task: 7.24-7.35 vs 7.46-7.52 ms per join with two 32,768-key
        // tasks that build the R table twice; at 16,384 S keys per partition (configs 2
        // and 5) the 32,768-key chunks split hot partitions finer (Zipf: 0.544 vs 0.56 ms)
        pj.s_chunk = avgS >= kBigSPart ? kBigSPart : kBigSChunk;
    }
    // narrow key partitions: the counting chaining join over key partitions with the
    // 16,384-key table (k_sort_blk writes them, k_join_x reads them)
    const bool narrow = pool == kPoolKeys && counting && pj.algo == kAlgoChaining && pj.pol.rcap == kBigRcap &&
                        pol.passes == 2 && sort2_enabled() && narrow_enabled();
    if (wire16 && !narrow) {
        set_last_error("u16 wire: the received partitions need the narrow counting plan");
        return MI355_ERR_INVALID;
    }
    pj.pr.narrow = pj.ps.narrow = narrow;
    // ... and pass 1 writes them first as a narrow pool (u16 residuals, read by
    // k_place_seg with their digit side stream); the chain-histogram layout keeps keys,
    // and so do pass-1 digits above 7 bits (the narrow pool's 64-residual granules keep
    // up to 63 carried keys per digit in LDS: 64 KiB at 8 bits, one workgroup per CU)
    const bool n16 = narrow && !wire16 && pol.b1 <= 7 && uses_digit_side(pol) && place_enabled() &&
                     narrow_pool_enabled();
    pj.pr.narrow16 = n16 && !pj.pr.chain;
    pj.ps.narrow16 = n16 && !pj.ps.chain;
    // (wire16: S may come as pieces, each partition's task list over 8 x its units: up to
    // 7 more per piece, kPieceMaxG pieces)
    pj.over_cap = (uint32_t)((nS + (wire16 ? 7ull * kPieceMaxG * P : 0ull)) / pj.s_chunk + 1);
    // one workgroup per task up to 2048 (few partitions with a large S — a tiny build
    // side — still spread their S chunks over the chip)
    pj.join_grid = (uint32_t)std::min<uint64_t>(P + pj.over_cap - 1, 2048);
    pj.off_over = A.reserve(sizeof(uint64_t) * pj.over_cap);
    pj.off_counts = A.reserve(sizeof(uint64_t) * (pj.materialize ? P + pj.over_cap : pj.join_grid));
    pj.off_toff = A.reserve(sizeof(uint64_t) * (pj.materialize ? P + pj.over_cap : 1));
    // result[0] = matches, [1] / [2] = largest R / S partition, [3] = extra S-chunk tasks
    // (u32), [4] / [5] = build / probe ticks: one read-back for all six; [6] = the
    // build/probe's task tickets (zeroed by launch_make_tasks with [1..5])
    pj.off_result = A.reserve(sizeof(uint64_t) * 8);  // (launch_make_tasks zeroes all 8 words, [7] the reduction ticket)
    pj.off_cyc = A.reserve(sizeof(uint64_t) * 2 * pj.join_grid);
    RHO_HIP(A.buf.ensure(A.used));
    return MI355_OK;
}

// First half: plans both relations (|S| = nS, its tuples are not read yet), then
// enqueues R's partition passes on s and returns without waiting.  The second half
// may start after S has been produced later in the stream order of s (multi-GPU:
// R's local passes run while S is still being exchanged).  Caller holds ctx->mu.
int join_begin(Context *ctx, hipStream_t s, const row_t *dR, uint64_t nR, uint64_t nS, const mi355_rho_opts *opts,
               PendingJoin &pj, uint32_t in_elem = sizeof(row_t), const std::vector<uint64_t> *s_pieces = nullptr,
               bool wire16 = false) {
    int prc = plan_join(ctx, s, nR, nS, opts, pj, s_pieces, wire16);
    if (prc) return prc;
    if (in_elem != sizeof(row_t)) {  // key input: only the pooled keys layout reads it
        if (!(pj.pr.keys && pj.ps.keys)) {
            set_last_error("key-only input needs a counting two-pass plan with the pooled layout");
            return MI355_ERR_INVALID;
        }
        pj.pr.in_size = pj.ps.in_size = in_elem;
    }
    const Policy &pol = pj.pol;
    Timer &tm = thread_timer();
    // the call's device time is always recorded (throughput in result_t); per kernel
    // only with timing on (mi355_timing_enable / opts->timing): each event record is a
    // few microseconds of GPU time, a large part of a small join
    const bool per_kernel = thread_timing_enabled() || (opts && opts->timing);
    tm.begin_call(s, true, !per_kernel);

    // R's and S's partition chains are independent: with overlap on, S's runs on the
    // side stream so that one relation's scatter shares the chip with the other's
    // kernels (fork/join events around it).
    pj.s2 = thread_partition_overlap() ? side_stream(ctx) : nullptr;
    if (pj.s2) {
        RHO_HIP(hipEventRecord(ctx->ev_t0, s));
        RHO_HIP(hipEventRecord(ctx->ev_fork, s));
    }
    // R's pooled pass-1 layout zeroes the join's result block (launch_make_tasks then
    // needs no fill)
    if (pj.pr.pooled) pj.pr.zero8 = ctx->scratch.at<uint64_t>(pj.off_result);
    int rc;
    for (int pass = 0; pass < (int)pol.passes; ++pass)
        if ((rc = partition_relation(ctx, s, tm, "R_", dR, ctx->t1R.as<row_t>(), ctx->t2R.as<row_t>(),
                                     ctx->sideR.as<uint8_t>(), pj.pr, pol, pj.key_shift, &pj.fR, &pj.psR, &pj.pcR,
                                     pass == 1)))
            return rc;
    pj.active = true;
    return MI355_OK;
}

// Statistics of a finished join from the read-back result words and the call's events.
void fill_join_stats(const Context *ctx, const PendingJoin &pj, const Timer &tm, float wall, mi355_rho_stats *st) {
    const Policy &pol = pj.pol;
    const uint64_t P = 1ull << pol.bits;
    if (st) {
        st->matches = ctx->host_result[0];
        st->radix_bits = pol.bits;
        st->passes = pol.passes;
        st->pass1_bits = pol.b1;
        st->pass2_bits = pol.b2;
        st->layout = pj.pr.chain ? 3u : pj.pr.narrow16 ? 4u : (pj.pr.keys ? 2u : (pj.pr.pooled ? 1u : 0u));
        st->elem_bytes = pj.pr.keys ? 4u : 8u;
        // (k_join_x: the high word of result[6] = 1 | narrow R << 1 | narrow S << 2)
        st->narrow = (uint32_t)(ctx->host_result[6] >> 33) & 3u;
        st->num_partitions = P;
        st->num_tasks = P + (uint32_t)ctx->host_result[3];
        st->max_part_r = ctx->host_result[1];
        st->max_part_s = ctx->host_result[2];
        // (RS_: both relations in one launch, the small-join path)
        st->ms_pass1 = tm.ms_of_prefix("R_pass1") + tm.ms_of_prefix("S_pass1") + tm.ms_of_prefix("RS_pass1");
        st->ms_pass2 = tm.ms_of_prefix("R_pass2") + tm.ms_of_prefix("S_pass2");
        st->ms_partition = st->ms_pass1 + st->ms_pass2;
        st->ms_join = tm.ms_of_prefix("join_");
        // with two streams the phase spans overlap: the total is the wall span
        st->ms_total = wall >= 0.f ? (double)wall
                                   : (tm.coarse() ? tm.ms_of_prefix("total") : st->ms_partition + st->ms_join);
        st->ms_pass1_r = tm.ms_of_prefix("R_pass1");
        st->ms_pass1_s = tm.ms_of_prefix("S_pass1");
        st->ms_pass1_hist = tm.ms_of_prefix("R_pass1_hist") + tm.ms_of_prefix("R_pass1_scan") +
                            tm.ms_of_prefix("S_pass1_hist") + tm.ms_of_prefix("S_pass1_scan") +
                            tm.ms_of_prefix("RS_pass1_hist");
        st->ms_pass1_copy = tm.ms_of_prefix("R_pass1_scatter") + tm.ms_of_prefix("S_pass1_scatter") +
                            tm.ms_of_prefix("RS_pass1_scatter");
        st->ms_pass2_hist = tm.ms_of_prefix("R_pass2_hist") + tm.ms_of_prefix("R_pass2_scan") +
                            tm.ms_of_prefix("S_pass2_hist") + tm.ms_of_prefix("S_pass2_scan");
        st->ms_pass2_copy = tm.ms_of_prefix("R_pass2_scatter") + tm.ms_of_prefix("S_pass2_scatter");
        // the build/probe kernel is one launch: its time is split by the ticks its
        // workgroups spent building and probing
        const double b = (double)ctx->host_result[4], pr = (double)ctx->host_result[5];
        const double bp = tm.ms_of_prefix("join_build_probe") + tm.ms_of_prefix("join_materialize");
        st->ms_build = b + pr > 0 ? bp * b / (b + pr) : 0.0;
        st->ms_probe = bp - st->ms_build;
    }
}

// Second half: S's partition passes, build/probe (and materialisation), then the
// result read-back.  fork_now: the side stream (overlap on) forks from s here instead
// of at join_begin, because S only became valid in between.
// given_s (nullable): S's partitions are already there (fS, part starts, part counts;
// the u16 wire's gathered residuals): no S passes.
struct GivenParts {
    const row_t *f;
    const uint64_t *ps, *pc;
    // the u16 wire's S read in place (join_pipelined_finish_wire16): f = the receive
    // buffer of residuals (bytes), its pieces; ps unused
    bool pieces = false;
    uint64_t bytes = 0;
    WirePieces w{};
};
int join_finish(Context *ctx, PendingJoin &pj, const row_t *dS, uint64_t nS, mi355_rho_stats *st,
                output_triple_t *out, uint64_t out_cap, DeviceBuffer *grow, bool fork_now,
                const GivenParts *given_s = nullptr) {
    if (!pj.active) {
        set_last_error("join_finish without join_begin");
        return MI355_ERR_INVALID;
    }
    pj.active = false;
    if (nS != pj.nS) {
        set_last_error("join_finish: |S| differs from the one given to join_begin");
        return MI355_ERR_INVALID;
    }
    hipStream_t s = pj.s;
    const Policy &pol = pj.pol;
    Arena &A = ctx->scratch;
    Timer &tm = thread_timer();
    Timer &tm2 = thread_side_timer();
    hipStream_t s2 = pj.s2;
    if (s2) {
        if (fork_now) RHO_HIP(hipEventRecord(ctx->ev_fork, s));
        RHO_HIP(hipStreamWaitEvent(s2, ctx->ev_fork, 0));
        tm2.begin_call(s2, true, tm.coarse());
    }
    hipStream_t sS = s2 ? s2 : s;
    Timer &tmS = s2 ? tm2 : tm;
    const row_t *fS = nullptr;
    const uint64_t *psS = nullptr, *pcS = nullptr;
    int rc;
    if (given_s) {
        fS = given_s->f;
        psS = given_s->ps;
        pcS = given_s->pc;
    } else {
        for (int pass = 0; pass < (int)pol.passes; ++pass)
            if ((rc = partition_relation(ctx, sS, tmS, "S_", dS, ctx->t1S.as<row_t>(), ctx->t2S.as<row_t>(),
                                         ctx->sideS.as<uint8_t>(), pj.ps, pol, pj.key_shift, &fS, &psS, &pcS,
                                         pass == 1)))
                return rc;
    }
    if (s2) {
        tm2.end_call();
        RHO_HIP(hipEventRecord(ctx->ev_join, s2));
        RHO_HIP(hipStreamWaitEvent(s, ctx->ev_join, 0));
    }
    const row_t *fR = pj.fR;
    const uint64_t *psR = pj.psR, *pcR = pj.pcR;
    const uint64_t P = 1ull << pol.bits;
    const uint32_t join_grid = pj.join_grid;
    const int algo = pj.algo;
    uint64_t *over = A.at<uint64_t>(pj.off_over);
    uint64_t *counts = A.at<uint64_t>(pj.off_counts);
    uint64_t *task_off = A.at<uint64_t>(pj.off_toff);
    uint64_t *result = A.at<uint64_t>(pj.off_result);
    uint64_t *cyc = A.at<uint64_t>(pj.off_cyc);
    uint32_t *n_over = reinterpret_cast<uint32_t *>(result + 3);
    const uint32_t hash_shift = pj.key_shift + pol.bits;
    uint64_t *fold_host = nullptr;  // (the count reduction's mapped result words)
    tm.mark("join_tasks");
    // narrow plans: k_join_n adds into the count and tick slots, zeroed here
    const bool nar = !pj.materialize && (pj.pr.narrow || pj.ps.narrow) && narrow_join_enabled();
    const bool pieces = given_s && given_s->pieces;
    // (S in pieces: the task list splits each partition's units, 8 per unit)
    RHO_HIP(launch_make_tasks(pcR, pieces ? given_s->w.units8 : pcS, P, over, pj.over_cap, result + 1, pj.s_chunk, s,
                              nar || pieces ? counts : nullptr, cyc, join_grid, pj.pr.zero8 != nullptr));
    if (pieces) {
        if (pj.materialize || pj.algo != kAlgoChaining || pol.rcap != kBigRcap || !pj.pr.narrow || !pj.ps.narrow) {
            set_last_error("u16 wire pieces: the plan is not the narrow counting table");
            return MI355_ERR_INVALID;
        }
        tm.mark("join_build_probe");
        RHO_HIP(launch_join_pieces(fR, psR, pcR, reinterpret_cast<const uint16_t *>(fS), given_s->bytes, given_s->w,
                                   P, over, n_over, hash_shift, pj.s_chunk, join_grid,
                                   (uint32_t)std::min<uint64_t>(P + pj.over_cap - 1, 0xFFFFFFFFull), counts, cyc,
                                   reinterpret_cast<uint32_t *>(result + 6), A.at<uint32_t>(pj.pr.kmax) + pj.pr.nseg1,
                                   A.at<uint32_t>(pj.ps.kmax) + pj.ps.nseg1, result, s));
    } else if (!pj.materialize) {
        tm.mark("join_build_probe");
        // the 16,384-key table's k_join_x sums the count slots itself (k_reduce folded in),
        // and writes the result words into mapped host memory too (no copy after it)
        const bool fold = algo == kAlgoChaining && pol.rcap == kBigRcap;
        if (fold && !ctx->host_fold) {
            void *dp = nullptr;
            if (hipHostMalloc(reinterpret_cast<void **>(&ctx->host_fold), 8 * sizeof(uint64_t),
                              hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess &&
                hipHostGetDevicePointer(&dp, ctx->host_fold, 0) == hipSuccess)
                ctx->host_fold_dev = static_cast<uint64_t *>(dp);
            else
                (void)hipGetLastError();
        }
        fold_host = fold ? ctx->host_fold_dev : nullptr;
        RHO_HIP(launch_join(fR, fS, psR, pcR, psS, pcS, P, over, n_over, hash_shift, pol.rcap, pj.s_chunk, join_grid,
                            kJoinCount, algo, counts, nullptr, nullptr, cyc, s, nullptr, pj.pr.keys ? 1 : 2,
                            reinterpret_cast<uint32_t *>(result + 6),
                            pj.pr.narrow ? A.at<uint32_t>(pj.pr.kmax) + pj.pr.nseg1 : nullptr,
                            pj.ps.narrow ? A.at<uint32_t>(pj.ps.kmax) + pj.ps.nseg1 : nullptr,
                            (uint32_t)std::min<uint64_t>(P + pj.over_cap - 1, 0xFFFFFFFFull), nullptr,
                            fold ? result : nullptr, fold_host));
        if (!fold) {
            tm.mark("join_reduce");
            RHO_HIP(launch_reduce(counts, join_grid, result, cyc, join_grid, s));
        }
    } else {
        tm.mark("join_build_probe");
        RHO_HIP(launch_join(fR, fS, psR, pcR, psS, pcS, P, over, n_over, hash_shift, pol.rcap, pj.s_chunk, join_grid,
                            kJoinTaskCount, algo, counts, nullptr, nullptr, cyc, s));
        tm.mark("join_offsets");
        RHO_HIP(launch_excl_scan(counts, n_over, P, task_off, result, s));
        RHO_HIP(hipMemcpyAsync(ctx->host_result, result, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
        RHO_HIP(hipStreamSynchronize(s));
        const uint64_t total = ctx->host_result[0];
        if (grow && total > out_cap) {  // caller-owned growable output (device pipelines)
            RHO_HIP(grow->ensure(std::max<uint64_t>(total, 1) * sizeof(output_triple_t)));
            out = grow->as<output_triple_t>();
            out_cap = total;
        }
        if (total > out_cap || (total > 0 && out == nullptr)) {
            tm.end_call();
            tm.collect();
            if (st) st->matches = total;
            set_last_error("materialisation output too small: " + std::to_string(total) + " triples needed");
            return MI355_ERR_CAPACITY;
        }
        tm.mark("join_materialize");
        RHO_HIP(launch_join(fR, fS, psR, pcR, psS, pcS, P, over, n_over, hash_shift, pol.rcap, pj.s_chunk, join_grid,
                            kJoinWrite, algo, counts, task_off, out, nullptr, s));
        tm.mark("join_reduce");
        RHO_HIP(launch_reduce(nullptr, 0, result, cyc, join_grid, s));  // ticks of the count pass
    }
    tm.end_call();
    if (s2) RHO_HIP(hipEventRecord(ctx->ev_t1, s));
    if (!fold_host) RHO_HIP(hipMemcpyAsync(ctx->host_result, result, 7 * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    RHO_HIP(hipStreamSynchronize(s));
    if (fold_host) std::memcpy(ctx->host_result, ctx->host_fold, 7 * sizeof(uint64_t));
    if (std::getenv("SGXAMD_DEBUG_WG_TICKS") && !pj.materialize) {
        // development: the build/probe workgroups' wall-clock ticks (load balance)
        const uint32_t ng = std::min<uint32_t>(join_grid, 4096);
        std::vector<uint64_t> c(2 * (size_t)ng);
        if (hipMemcpy(c.data(), cyc, c.size() * sizeof(uint64_t), hipMemcpyDeviceToHost) == hipSuccess) {
            uint64_t mx = 0, sum = 0, n = 0, mb = 0, mp = 0;
            for (uint32_t i = 0; i < ng; ++i) {
                const uint64_t t = c[2 * i] + c[2 * i + 1];
                if (!t) continue;
                ++n;
                sum += t;
                if (t > mx) {
                    mx = t;
                    mb = c[2 * i];
                    mp = c[2 * i + 1];
                }
            }
            std::fprintf(stderr, "[wg ticks] wgs %llu mean %.0f max %llu (build %llu probe %llu) max/mean %.3f\n",
                         (unsigned long long)n, n ? (double)sum / n : 0.0, (unsigned long long)mx,
                         (unsigned long long)mb, (unsigned long long)mp, n && sum ? (double)mx * n / sum : 0.0);
        }
    }
    tm.collect();
    float wall = -1.f;
    if (s2) {
        tm2.collect();
        tm.append(tm2);
        if (hipEventElapsedTime(&wall, ctx->ev_t0, ctx->ev_t1) != hipSuccess) wall = -1.f;
    }

    fill_join_stats(ctx, pj, tm, wall, st);
    return MI355_OK;
}

// Small one-pass counting joins in three launches (DESIGN.md §3 "Small joins"): a join
// of 2^20 x 2^20 tuples is a dozen ~5 us launches on the regular path (histogram, two
// scans and scatter per relation, a memset and the task list, build/probe, reduce).
// Here: k_hist_pair (both histograms, digit layout and task list, with in-launch
// hand-offs), k_scatter_pair (both scatters) and the build/probe with its own
// last-workgroup reduction.  SGXAMD_SMALL_JOIN=0 turns it off (A/B; results identical).
constexpr uint64_t kSmallJoinMax = 1ull << 23;  // |R| + |S| up to which the path is taken

// Waits for the small join's done flag in mapped host memory: a spin of at most 2 ms
// (a 2^23-tuple small join takes ~0.2 ms), then the stream synchronisation, which
// also reports a kernel fault; the flag must be set after it.
int wait_host_flag(volatile uint64_t *flag, hipStream_t s) {
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 1;; ++i) {
        if (*flag) {
            std::atomic_thread_fence(std::memory_order_acquire);
            return MI355_OK;
        }
        if ((i & 1023) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) break;
        __builtin_ia32_pause();
    }
    RHO_HIP(hipStreamSynchronize(s));
    if (!*flag) {
        set_last_error("small join: the build/probe finished without its done flag");
        return MI355_ERR_HIP;
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    return MI355_OK;
}

// The device's constant wall clock (wall_clock64()) in kHz, queried once.
double wall_clock_khz() {
    static const double khz = [] {
        int dev = 0, v = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeWallClockRate, dev) !=
                                                     hipSuccess || v <= 0)
            return 100000.0;  // 100 MHz on CDNA3/4
        return (double)v;
    }();
    return khz;
}

bool small_join_enabled() {
    static const bool on = [] {
        const char *e = std::getenv("SGXAMD_SMALL_JOIN");
        return !(e && std::atoi(e) == 0);
    }();
    return on;
}

// SGXAMD_SMALL_DIRECT=0 (development A/B, read once): the small joins' build/probe keeps
// the chain table where the direct count table would fit.
bool small_direct_enabled() {
    static const bool on = [] {
        const char *e = std::getenv("SGXAMD_SMALL_DIRECT");
        return !(e && std::atoi(e) == 0);
    }();
    return on;
}

int join_small(Context *ctx, hipStream_t s, const row_t *dR, uint64_t nR, const row_t *dS, uint64_t nS,
               const mi355_rho_opts *opts, mi355_rho_stats *st) {
    PendingJoin &pj = pending_of(ctx);
    int rc = plan_join(ctx, s, nR, nS, opts, pj);
    if (rc) return rc;
    const Policy &pol = pj.pol;
    // hand-off words: zero once, every kernel leaves them zero -- and zeroed again after a
    // call that failed between the parity flip and its result (a launch error, a flag
    // timeout): its totals, kmax words or tickets may be left behind
    if (!ctx->sync.ptr || ctx->sync_dirty) {
        RHO_HIP(ctx->sync.ensure(kSyncWords * sizeof(uint64_t)));
        RHO_HIP(hipMemsetAsync(ctx->sync.ptr, 0, kSyncWords * sizeof(uint64_t), s));
        // the mapped host result block and its device address in sync[kSyncHostResult]
        if (!ctx->host_join)
            RHO_HIP(hipHostMalloc(reinterpret_cast<void **>(&ctx->host_join), kHostJoinWords * sizeof(uint64_t),
                                  hipHostMallocMapped | hipHostMallocCoherent));
        void *dp = nullptr;
        RHO_HIP(hipHostGetDevicePointer(&dp, ctx->host_join, 0));
        ctx->host_result[8] = reinterpret_cast<uint64_t>(dp);
        RHO_HIP(hipMemcpyAsync(ctx->sync.as<uint64_t>() + kSyncHostResult, ctx->host_result + 8, sizeof(uint64_t),
                               hipMemcpyHostToDevice, s));
        RHO_HIP(hipStreamSynchronize(s));
        ctx->small_parity = 0;
        ctx->sync_dirty = false;
    }
    Timer &tm = thread_timer();
    const bool per_kernel = thread_timing_enabled() || (opts && opts->timing);
    // development: per-workgroup stamps of the three kernels (SGXAMD_DEBUG_STAMPS)
    static DeviceBuffer stamps;
    static const bool want_stamps = std::getenv("SGXAMD_DEBUG_STAMPS") != nullptr;
    if (want_stamps) {
        RHO_HIP(stamps.ensure(12 * kStampWgs * sizeof(uint64_t)));
        RHO_HIP(hipMemsetAsync(stamps.ptr, 0, 12 * kStampWgs * sizeof(uint64_t), s));
        RHO_HIP(set_debug_stamps(stamps.as<uint64_t>()));
    }
    tm.begin_call(s, per_kernel);  // without per-kernel events the kernels time the call
    volatile uint64_t *hj = ctx->host_join;
    hj[kHostJoinDone] = 0;
    // segments of at least 8192 tuples: fewer digit-total atomics per address (2^20 x 2^20:
    // 4096 / 8192 / 16384 / 32768-tuple segments 67.9 / 58.5 / 64.6 / 85.3 us per join;
    // SGXAMD_SMALL_SEG overrides, development)
    // a histogram workgroup takes two scatter segments (whole tiles each), so a segment
    // is an even number of tiles
    static const uint64_t small_seg = [] {
        const char *e = std::getenv("SGXAMD_SMALL_SEG");
        const uint64_t v = e ? std::strtoull(e, nullptr, 10) : 8192;
        return std::max<uint64_t>(2 * kTile, (v + 2 * kTile - 1) / (2 * kTile) * (2 * kTile));
    }();
    for (RelPlan *rp : {&pj.pr, &pj.ps}) {
        const uint32_t cap = rp->nseg1 + 1;  // the plan's offset table holds F1 x (nseg1 + 1)
        rp->seg1 = std::max<uint64_t>(rp->seg1, small_seg);
        rp->nseg1 = (uint32_t)((rp->n + rp->seg1 - 1) / rp->seg1);
        if (2 * rp->nseg1 > cap) {
            set_last_error("small join: segment offsets do not fit the plan's table");
            return MI355_ERR_INVALID;
        }
    }
    Arena &A = ctx->scratch;
    uint64_t *sync = ctx->sync.as<uint64_t>();
    uint64_t *result = A.at<uint64_t>(pj.off_result);
    uint64_t *over = A.at<uint64_t>(pj.off_over);
    // the scatter's segments: halves of the histogram workgroups' segments
    const SegMap mR{nullptr, nullptr, nullptr, 1, pj.pr.seg1 / 2, nR}, mS{nullptr, nullptr, nullptr, 1, pj.ps.seg1 / 2, nS};
    uint64_t *offsR = A.at<uint64_t>(pj.pr.hist1), *offsS = A.at<uint64_t>(pj.ps.hist1);
    uint64_t *startR = A.at<uint64_t>(pj.pr.start1), *cntR = A.at<uint64_t>(pj.pr.cnt1);
    uint64_t *startS = A.at<uint64_t>(pj.ps.start1), *cntS = A.at<uint64_t>(pj.ps.cnt1);
    row_t *oR = ctx->t1R.as<row_t>(), *oS = ctx->t1S.as<row_t>();
    // the digit totals alternate between two sets per call (each call's scatter zeroes
    // the set the next call's histograms add into)
    const uint32_t par = ctx->small_parity;
    ctx->small_parity ^= 1u;
    ctx->sync_dirty = true;  // until the result is in (every error return below leaves it set)
    tm.mark("RS_pass1_hist");
    // R's largest key (the direct count table of the build/probe), per parity set
    uint64_t *kmax = small_direct_enabled() ? sync + kSyncKmax : nullptr;
    RHO_HIP(launch_hist_pair(dR, mR, pj.pr.nseg1, dS, mS, pj.ps.nseg1, pj.key_shift, pol.b1, offsR, offsS,
                             sync + sync_tot(par, 0), sync + sync_tot(par, 1), sync + kSyncT0, s,
                             kmax ? kmax + par : nullptr));
    tm.mark("RS_pass1_scatter");
    // cursors: each segment's offset inside its copy of the digit totals + that copy's
    // digit start (each scatter workgroup scans the totals itself)
    RHO_HIP(launch_scatter_pair(dR, oR, mR, 2 * pj.pr.nseg1, offsR, sync + sync_tot(par, 0), sync + sync_tot(par ^ 1, 0),
                                startR, cntR, dS, oS, mS, 2 * pj.ps.nseg1, offsS, sync + sync_tot(par, 1),
                                sync + sync_tot(par ^ 1, 1), startS, cntS, pj.key_shift, pol.b1, over, pj.over_cap,
                                result + 1, pj.s_chunk, s, kmax ? kmax + (par ^ 1) : nullptr));
    tm.mark("join_build_probe");
    const uint64_t P = 1ull << pol.bits;
    const JoinReduce red{result, sync + kSyncTicketJoin};
    RHO_HIP(launch_join(oR, oS, startR, cntR, startS, cntS, P, over, reinterpret_cast<uint32_t *>(result + 3),
                        pj.key_shift + pol.bits, pol.rcap, pj.s_chunk, pj.join_grid, kJoinCount, pj.algo,
                        A.at<uint64_t>(pj.off_counts), nullptr, nullptr, A.at<uint64_t>(pj.off_cyc), s, &red, 2,
                        nullptr, nullptr, nullptr, 0, kmax ? kmax + par : nullptr));
    tm.end_call();
    // the join's last workgroup wrote the result words into host_join: no copy back, and
    // without per-kernel events no stream synchronisation either (a launch + synchronise
    // round trip costs ~9 us, launch + a spin on a mapped flag ~6 us)
    float span = -1.f;
    if (per_kernel) {
        RHO_HIP(hipStreamSynchronize(s));
    } else {
        const int rc2 = wait_host_flag(hj + kHostJoinDone, s);
        if (rc2) return rc2;
        span = (float)((double)hj[kHostJoinSpan] / wall_clock_khz());
    }
    for (int i = 0; i < 6; ++i) ctx->host_result[i] = hj[i];
    ctx->host_result[6] = 0;  // (no narrow partitions in a small join)
    ctx->sync_dirty = false;
    tm.collect();
    fill_join_stats(ctx, pj, tm, span, st);
    if (want_stamps) {
        RHO_HIP(hipStreamSynchronize(s));
        RHO_HIP(set_debug_stamps(nullptr));
        std::vector<uint64_t> h(12 * (size_t)kStampWgs);
        RHO_HIP(hipMemcpy(h.data(), stamps.ptr, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
        uint64_t t0 = UINT64_MAX;
        for (uint64_t v : h)
            if (v) t0 = std::min(t0, v);
        const double us = 1000.0 / wall_clock_khz();
        std::fprintf(stderr, "[stamps]");
        for (int k = 0; k < 4; ++k) {
            uint64_t e_min = UINT64_MAX, e_max = 0, x_max = 0, h_max = 0;
            std::vector<double> body;
            for (uint32_t w = 0; w < kStampWgs; ++w) {
                const uint64_t e = h[(k * 3 + 0) * kStampWgs + w], m = h[(k * 3 + 1) * kStampWgs + w],
                               x = h[(k * 3 + 2) * kStampWgs + w];
                if (!e) continue;
                e_min = std::min(e_min, e);
                e_max = std::max(e_max, e);
                x_max = std::max(x_max, x);
                if (m) h_max = std::max(h_max, m);
                if (m) body.push_back((double)(m - e) * us);
            }
            std::sort(body.begin(), body.end());
            std::fprintf(stderr, " k%d: first entry %.1f last entry %.1f body med %.1f max %.1f last pre-handoff %.1f exit %.1f |",
                         k, (double)(e_min - t0) * us, (double)(e_max - t0) * us,
                         body.empty() ? 0.0 : body[body.size() / 2], body.empty() ? 0.0 : body.back(),
                         h_max ? (double)(h_max - t0) * us : 0.0, (double)(x_max - t0) * us);
        }
        std::fprintf(stderr, "\n");
    }
    return MI355_OK;
}

// The whole join on device-resident inputs.  Caller holds ctx->mu.
// Materialisation (opts->materialize): a per-task count pass, an exclusive scan of
// the task counts into output offsets, then a write pass; `out` must be device
// memory with room for out_cap triples (MI355_ERR_CAPACITY otherwise).
int join_device(Context *ctx, hipStream_t s, const row_t *dR, uint64_t nR, const row_t *dS, uint64_t nS,
                const mi355_rho_opts *opts, mi355_rho_stats *st, output_triple_t *out, uint64_t out_cap,
                DeviceBuffer *grow) {
    PendingJoin &pj = pending_of(ctx);
    if (pj.active) {
        set_last_error("a pipelined join (mi355_rho_join_begin) is pending on this device");
        return MI355_ERR_INVALID;
    }
    if (small_join_enabled() && nR > 0 && nS > 0 && nR + nS <= kSmallJoinMax && !(opts && opts->materialize) &&
        !thread_partition_overlap() && choose_policy(nR, nS, opts).passes == 1) {
        const int rc = join_small(ctx, s, dR, nR, dS, nS, opts, st);
        pj.active = false;
        return rc;
    }
    int rc = join_begin(ctx, s, dR, nR, nS, opts, pj);
    if (rc) {
        pj.active = false;
        return rc;
    }
    return join_finish(ctx, pj, dS, nS, st, out, out_cap, grow, false);
}

int join_pipelined_begin(Context *ctx, hipStream_t s, const void *dR, uint64_t nR, uint64_t nS,
                         const mi355_rho_opts *opts, uint32_t in_elem, const uint64_t *s_piece_n, int s_pieces,
                         bool wire16) {
    PendingJoin &pj = pending_of(ctx);
    if (pj.active) {
        set_last_error("a pipelined join is already pending on this context");
        return MI355_ERR_INVALID;
    }
    std::vector<uint64_t> pieces;
    if (s_piece_n && s_pieces > 0) {
        pieces.assign(s_piece_n, s_piece_n + s_pieces);
        uint64_t sum = 0;
        for (uint64_t x : pieces) sum += x;
        if (sum != nS) {
            set_last_error("join_pipelined_begin: the S pieces do not add up to |S|");
            return MI355_ERR_INVALID;
        }
    }
    const int rc = join_begin(ctx, s, static_cast<const row_t *>(dR), nR, nS, opts, pj, in_elem,
                              pieces.empty() ? nullptr : &pieces, wire16);
    if (rc) pj.active = false;
    return rc;
}

int join_pipelined_finish(Context *ctx, const void *dS, uint64_t nS, mi355_rho_stats *st, const hipEvent_t *s_landed,
                          DeviceBuffer *mat) {
    PendingJoin &pj = pending_of(ctx);
    pj.ps.piece_ev.clear();
    if (s_landed) pj.ps.piece_ev.assign(s_landed, s_landed + pj.ps.piece_n.size());
    if (pj.materialize && !mat) {
        pj.active = false;
        set_last_error("join_pipelined_finish: a materialising join needs an output buffer");
        return MI355_ERR_INVALID;
    }
    return join_finish(ctx, pj, static_cast<const row_t *>(dS), nS, st, nullptr, 0, mat, true);
}

bool keys_exchange_plan(uint64_t nR, uint64_t nS, uint64_t cap_r, uint64_t cap_s, mi355_rho_opts *lo) {
    if (!keys_enabled() || lo->materialize) return false;
    if (lo->radix_bits <= 0) {  // fix the local policy now: the received sizes are not known yet
        const Policy p = choose_policy(nR, nS, lo);
        lo->radix_bits = (int)p.bits;
        lo->passes = (int)p.passes;
    }
    const Policy p = choose_policy(nR, nS, lo);
    return pool_fits(cap_r, p) && pool_fits(cap_s, p) && lo->key_shift + p.bits <= 31;
}

// ---------------------------------------------------------------- multi-GPU u16 wire
// The exchange's sender runs the receiver's two partition passes (the same plan: both
// derive it from the global sizes) on the keys it sends each destination, so that the
// destination's shard bits and partition bits are implied by where a key lands and only
// its residual above them travels: 2 bytes instead of 4.  The receiver gathers each
// partition's pieces (one per sender, wire_kernels.hip) and runs the build/probe.
namespace {
std::atomic<int> g_wire_mode{-1};  // -1: not set (SGXAMD_WIRE16, default 1)
}
void set_wire_mode(int mode) { g_wire_mode = mode < 0 ? 0 : (mode > 2 ? 2 : mode); }
int wire_mode() {
    const int m = g_wire_mode.load();
    if (m >= 0) return m;
    const char *e = std::getenv("SGXAMD_WIRE16");
    return e ? std::max(0, std::min(2, std::atoi(e))) : 1;
}

uint32_t wire16_plan(uint64_t nR, uint64_t nS, int G, const mi355_rho_opts *lo, bool *need_kmax) {
    if (need_kmax) *need_kmax = false;
    const int mode = wire_mode();
    if (!mode || !lo || lo->materialize || lo->algorithm == MI355_ALGO_RHT || G < 2 || (uint32_t)G > kWireMaxG)
        return 0;
    if (!(keys_enabled() && narrow_enabled() && sort2_enabled())) return 0;
    const Policy p = choose_policy(nR, nS, lo);
    // mode 1: only where the local join takes the narrow plan anyway (the 16,384-key
    // table): elsewhere (BASELINE config 4 at G = 8: 1,024 R keys per partition) forcing
    // it costs more compute than the halved S bytes save (r05x5)
    if (mode == 1 && !takes_big_table(p, nR, nS, lo)) return 0;
    if (p.passes != 2 || !uses_digit_side(p) || lo->key_shift + p.bits > 31 || p.bits > 20) return 0;
    // every 32-bit key's residual fits 16 bits, or (need_kmax) the caller checks S's
    // largest key over all ranks before the residuals are posted
    if (lo->key_shift + p.bits < 16) {
        if (!need_kmax) return 0;
        *need_kmax = true;
    }
    return 1u << p.bits;
}

int wire_partition(Context *ctx, hipStream_t s, const uint32_t *keys, int G, int runs, const uint64_t *run_off,
                   const uint64_t *run_n, uint64_t nR, uint64_t nS, const mi355_rho_opts *lo, uint16_t *out16,
                   uint64_t *counts, const char *tag) {
    if (pending_of(ctx).active) {
        set_last_error("wire_partition while a pipelined join is pending on this device");
        return MI355_ERR_INVALID;
    }
    const Policy pol = choose_policy(nR, nS, lo);
    const uint32_t P = 1u << pol.bits;
    // a scratch of its own: the shard pieces' plans in ctx->scratch stay valid for the
    // other relation's scatters, which follow this relation's passes in the stream
    Arena &A = ctx->wscratch;
    // every destination's plan first: the arena and the pools sized for the largest, so
    // that no buffer grows while the loop's launches are queued
    std::vector<std::vector<uint64_t>> pn((size_t)G);
    std::vector<uint64_t> nq((size_t)G, 0);
    size_t arena = 0;
    uint64_t t1max = 0;
    RelPlan rp{};
    for (int q = 0; q < G; ++q) {
        pn[q].assign(run_n + (size_t)q * runs, run_n + (size_t)(q + 1) * runs);
        for (uint64_t x : pn[q]) nq[q] += x;
        if (!nq[q]) continue;
        if (!pool_fits(nq[q], pol, (uint64_t)runs)) {
            set_last_error("u16 wire: a destination's keys do not fit the pooled plan");
            return MI355_ERR_INVALID;
        }
        A.reset();
        plan_relation(A, rp, nq[q], pol, kPoolKeys, &pn[q]);
        arena = std::max(arena, A.used);
        t1max = std::max(t1max, rp.t1_tuples);
    }
    RHO_HIP(A.buf.ensure(std::max<size_t>(arena, 256)));
    RHO_HIP(ctx->t1R.ensure(std::max<uint64_t>(t1max, 1) * sizeof(row_t)));
    RHO_HIP(ctx->sideR.ensure(std::max<uint64_t>(t1max, 16)));
    Timer &tm = thread_timer();
    tm.begin_call(s, false);
    const std::string t = tag;
    uint64_t doff = 0;
    const uint64_t RW = 2ull * P + 1;  // a row: counts, starts, the largest key
    for (int q = 0; q < G; ++q) {
        uint64_t *cq = counts + (size_t)q * RW;
        if (!nq[q]) {
            RHO_HIP(hipMemsetAsync(cq, 0, sizeof(uint64_t) * RW, s));
            continue;
        }
        A.reset();
        plan_relation(A, rp, nq[q], pol, kPoolKeys, &pn[q]);
        for (int j = 0; j < runs; ++j) rp.piece_off[j] = run_off[(size_t)q * runs + j];
        rp.narrow = true;  // wire16_plan: every residual fits 16 bits
        rp.narrow16 = false;
        rp.pad_parts = true;  // every partition on 16 bytes: the receiver reads them in place
        rp.in_size = sizeof(uint32_t);
        const row_t *f = nullptr;
        const uint64_t *pst = nullptr, *pcn = nullptr;
        for (int pass = 0; pass < 2; ++pass) {
            const int rc = partition_relation_pooled(
                ctx, s, tm, t, reinterpret_cast<const row_t *>(keys), ctx->t1R.as<row_t>(),
                reinterpret_cast<row_t *>(out16 + doff), ctx->sideR.as<uint8_t>(), rp, pol, lo->key_shift, &f, &pst,
                &pcn, pass == 1, &A);
            if (rc) return rc;
        }
        RHO_HIP(hipMemcpyAsync(cq, pcn, sizeof(uint64_t) * P, hipMemcpyDeviceToDevice, s));
        RHO_HIP(hipMemcpyAsync(cq + P, pst, sizeof(uint64_t) * P, hipMemcpyDeviceToDevice, s));
        RHO_HIP(hipMemsetAsync(cq + 2 * P, 0, sizeof(uint64_t), s));
        RHO_HIP(hipMemcpyAsync(cq + 2 * P, A.at<uint32_t>(rp.kmax) + rp.nseg1, sizeof(uint32_t),
                               hipMemcpyDeviceToDevice, s));
        // every destination's run starts on 16 bytes (k_place_seg's copies) and spans its
        // padded partitions
        doff += wire_slot(nq[q], P);
    }
    tm.end_call();
    return MI355_OK;
}

uint64_t wire_scratch_u64(int G, uint32_t P) { return wire_scratch_words((uint32_t)G, P); }

// SGXAMD_WIRE_GATHER=1 (development A/B switch, read once): the u16 wire's receiver
// gathers S's pieces into contiguous partitions before the build/probe (round 5's path)
// instead of reading them in place.
inline bool wire_gather_forced() {
    static const bool on = [] {
        const char *e = std::getenv("SGXAMD_WIRE_GATHER");
        return e && std::atoi(e) == 1;
    }();
    return on;
}

int join_pipelined_finish_wire16(Context *ctx, const uint16_t *s16, const uint64_t *s_cnt, const uint64_t *s_base,
                                 const uint64_t *s_n, const uint64_t *s_span, uint64_t nS, int G, uint64_t *scratch,
                                 hipEvent_t s_landed, mi355_rho_stats *st) {
    PendingJoin &pj = pending_of(ctx);
    if (!pj.active || !pj.ps.narrow) {
        pj.active = false;
        set_last_error("join_pipelined_finish_wire16 without a u16-wire join_pipelined_begin");
        return MI355_ERR_INVALID;
    }
    if (G < 1 || (uint32_t)G > kWireMaxG) {
        pj.active = false;
        set_last_error("u16 wire: unsupported world size");
        return MI355_ERR_INVALID;
    }
    const uint32_t P = 1u << pj.pol.bits;
    Arena &A = ctx->scratch;
    Timer &tm = thread_timer();
    WireBases bs{};
    uint64_t end = 0;
    for (int q = 0; q < G; ++q) {
        bs.b[q] = s_base[q];
        bs.n[q] = s_n[q];
        bs.span[q] = s_span[q];
        end = std::max(end, s_base[q] + s_span[q]);
    }
    uint64_t *psS = A.at<uint64_t>(pj.ps.pstart), *pcS = A.at<uint64_t>(pj.ps.pcnt);
    uint32_t *narrowS = A.at<uint32_t>(pj.ps.kmax) + pj.ps.nseg1;
    RHO_HIP(hipStreamWaitEvent(pj.s, s_landed, 0));
    if ((uint32_t)G <= kPieceMaxG && !wire_gather_forced() && end * 2 <= 0xFFFFFFF0ull) {
        // S's partitions read in place: only the piece table is built
        tm.mark("S_wire_pieces");
        RHO_HIP(launch_wire_pieces(s_cnt, (uint32_t)G, P, bs, scratch, pcS, narrowS, pj.s));
        const GivenParts gs{reinterpret_cast<const row_t *>(s16), psS, pcS, true, end * 2,
                            wire_pieces_of(scratch, (uint32_t)G, P)};
        return join_finish(ctx, pj, nullptr, nS, st, nullptr, 0, nullptr, false, &gs);
    }
    uint16_t *mS = ctx->t2S.as<uint16_t>();
    tm.mark("S_wire_merge");
    RHO_HIP(launch_wire_merge(s16, s_cnt, (uint32_t)G, P, bs, scratch, psS, pcS, narrowS, mS, pj.s));
    const GivenParts gs{reinterpret_cast<const row_t *>(mS), psS, pcS};
    return join_finish(ctx, pj, nullptr, nS, st, nullptr, 0, nullptr, false, &gs);
}

// Stable partition by destination shard (multi-GPU exchange step).
int shard_partition_device(Context *ctx, hipStream_t s, const row_t *in, uint64_t n, uint32_t key_shift,
                           uint32_t dest_bits, void *out, uint64_t *dest_counts, uint32_t out_elem) {
    if (pending_of(ctx).active) {  // the arena holds the pending join's R partitions
        set_last_error("shard_partition while a pipelined join is pending on this device");
        return MI355_ERR_INVALID;
    }
    Policy pol{};
    pol.bits = pol.b1 = dest_bits;
    pol.passes = 1;
    Arena &A = ctx->scratch;
    A.reset();
    RelPlan rp{};
    plan_relation(A, rp, n, pol);
    rp.keys = out_elem == 4;
    RHO_HIP(A.buf.ensure(A.used));
    Timer &tm = thread_timer();
    tm.begin_call(s, thread_timing_enabled());
    const row_t *f;
    const uint64_t *pst, *pcn;
    int rc = partition_relation(ctx, s, tm, "shard_", in, static_cast<row_t *>(out), nullptr, nullptr, rp, pol,
                                key_shift, &f, &pst, &pcn, false);
    if (rc) return rc;
    tm.end_call();
    const uint32_t F = 1u << dest_bits;
    RHO_HIP(hipMemcpyAsync(dest_counts, pcn, F * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    RHO_HIP(hipStreamSynchronize(s));
    tm.collect();
    return MI355_OK;
}

// The pieces of a two-phase shard partition (shard_count_pieces / shard_scatter_piece).
struct ShardPieces {
    Policy pol{};
    uint32_t key_shift = 0;
    std::vector<RelPlan> rp;
    std::vector<const row_t *> in;
    uint64_t *host = nullptr;  // pinned: every piece's destination counts
    size_t host_words = 0;
};
namespace {
std::mutex g_shard_mu;
std::unordered_map<const Context *, ShardPieces> g_shard;
ShardPieces &shard_of(const Context *ctx) {
    std::lock_guard<std::mutex> lk(g_shard_mu);
    return g_shard[ctx];
}
}  // namespace

void forget_context(const Context *ctx) {
    {
        std::lock_guard<std::mutex> lk(g_shard_mu);
        auto it = g_shard.find(ctx);
        if (it != g_shard.end()) {
            if (it->second.host) (void)hipHostFree(it->second.host);
            g_shard.erase(it);
        }
    }
    std::lock_guard<std::mutex> lk(g_pending_mu);
    g_pending.erase(ctx);
}

int shard_count_pieces(Context *ctx, hipStream_t s, const row_t *const *in, const uint64_t *n, int npieces,
                       uint32_t key_shift, uint32_t dest_bits, uint32_t out_elem, uint64_t *counts) {
    if (pending_of(ctx).active) {
        set_last_error("shard_count_pieces while a pipelined join is pending on this device");
        return MI355_ERR_INVALID;
    }
    ShardPieces &sp = shard_of(ctx);
    sp.pol = Policy{};
    sp.pol.bits = sp.pol.b1 = dest_bits;
    sp.pol.passes = 1;
    sp.key_shift = key_shift;
    Arena &A = ctx->scratch;
    A.reset();
    sp.rp.assign(npieces, RelPlan{});
    sp.in.assign(in, in + npieces);
    for (int j = 0; j < npieces; ++j) {
        plan_relation(A, sp.rp[j], n[j], sp.pol);
        sp.rp[j].keys = out_elem == 4;
    }
    RHO_HIP(A.buf.ensure(A.used));
    const size_t F = 1u << dest_bits, words = F * (size_t)npieces;
    if (sp.host_words < words) {
        if (sp.host) (void)hipHostFree(sp.host);
        sp.host = nullptr;
        sp.host_words = 0;
        RHO_HIP(hipHostMalloc(reinterpret_cast<void **>(&sp.host), words * sizeof(uint64_t)));
        sp.host_words = words;
    }
    Timer &tm = thread_timer();
    tm.begin_call(s, thread_timing_enabled());
    for (int j = 0; j < npieces; ++j) {
        if (!n[j]) continue;
        const int rc = pass1_counts(ctx, s, tm, "shard_", in[j], sp.rp[j], sp.pol, key_shift);
        if (rc) return rc;
        RHO_HIP(hipMemcpyAsync(sp.host + (size_t)j * F, A.at<uint64_t>(sp.rp[j].cnt1), F * sizeof(uint64_t),
                               hipMemcpyDeviceToHost, s));
    }
    tm.end_call();
    RHO_HIP(hipStreamSynchronize(s));
    tm.collect();
    for (int j = 0; j < npieces; ++j)
        for (size_t d = 0; d < F; ++d) counts[(size_t)j * F + d] = n[j] ? sp.host[(size_t)j * F + d] : 0;
    return MI355_OK;
}

int shard_scatter_piece(Context *ctx, hipStream_t s, int j, void *out) {
    ShardPieces &sp = shard_of(ctx);
    if (j < 0 || j >= (int)sp.rp.size()) {
        set_last_error("shard_scatter_piece: no such piece");
        return MI355_ERR_INVALID;
    }
    if (!sp.rp[j].n) return MI355_OK;
    Timer &tm = thread_timer();
    tm.begin_call(s, false);
    const int rc = pass1_scatter(ctx, s, tm, "shard_", sp.in[j], static_cast<row_t *>(out), nullptr, sp.rp[j], sp.pol,
                                 sp.key_shift);
    tm.end_call();
    return rc;
}

}  // namespace rho
}  // namespace sgxamd

using namespace sgxamd;

namespace {
thread_local mi355_rho_stats g_last_stats{};
}

void rho::set_last_join_stats(const mi355_rho_stats &st) { g_last_stats = st; }

extern "C" {

int mi355_release_workspace(void) {
    int status = MI355_OK;
    Context *ctx = current_context(&status);
    if (!ctx) return status;
    std::lock_guard<std::mutex> lk(ctx->mu);
    if (rho::pending_of(ctx).active) {
        set_last_error("mi355_release_workspace: a pipelined join is pending");
        return MI355_ERR_INVALID;
    }
    RHO_HIP(hipStreamSynchronize(ctx->stream));
    release_workspace(ctx);
    return MI355_OK;
}

int mi355_last_join_stats(mi355_rho_stats *out) {
    if (!out) return MI355_ERR_INVALID;
    *out = g_last_stats;
    return MI355_OK;
}

int mi355_rho_join_ex(const row_t *R, uint64_t nR, const row_t *S, uint64_t nS, const mi355_rho_opts *opts,
                      mi355_rho_stats *stats) {
    if ((!R && nR) || (!S && nS)) {
        set_last_error("null relation");
        return MI355_ERR_INVALID;
    }
    const bool materialize = opts && opts->materialize;
    if (materialize && opts->out_capacity > 0 && opts->out == nullptr) {
        set_last_error("materialize: out is NULL");
        return MI355_ERR_INVALID;
    }
    int status = MI355_OK;
    Context *ctx = current_context(&status);
    if (!ctx) return status;
    std::lock_guard<std::mutex> lk(ctx->mu);
    hipStream_t s = thread_stream(ctx, opts ? opts->stream : nullptr);
    mi355_rho_stats local{};
    mi355_rho_stats *st = stats ? stats : &local;
    std::memset(st, 0, sizeof(*st));
    if (nR == 0 || nS == 0) {
        g_last_stats = *st;
        return MI355_OK;
    }
    struct Remember {  // publish the stats of this call on every return path
        mi355_rho_stats *st;
        ~Remember() { g_last_stats = *st; }
    } remember{st};

    const row_t *dR = R, *dS = S;
    const auto t0 = std::chrono::steady_clock::now();
    bool staged = false;
    if (!is_device_pointer(R)) {
        RHO_HIP(ctx->inR.ensure(nR * sizeof(row_t)));
        RHO_HIP(hipMemcpyAsync(ctx->inR.ptr, R, nR * sizeof(row_t), hipMemcpyHostToDevice, s));
        dR = ctx->inR.as<row_t>();
        staged = true;
    }
    if (!is_device_pointer(S)) {
        RHO_HIP(ctx->inS.ensure(nS * sizeof(row_t)));
        RHO_HIP(hipMemcpyAsync(ctx->inS.ptr, S, nS * sizeof(row_t), hipMemcpyHostToDevice, s));
        dS = ctx->inS.as<row_t>();
        staged = true;
    }
    if (staged) {
        RHO_HIP(hipStreamSynchronize(s));
        st->ms_h2d = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    if (!materialize) return rho::join_device(ctx, s, dR, nR, dS, nS, opts, st, nullptr, 0);
    // materialise: straight into a device buffer, or through the context's buffer into host memory
    const uint64_t cap = opts->out_capacity;
    if (opts->out == nullptr || is_device_pointer(opts->out))
        return rho::join_device(ctx, s, dR, nR, dS, nS, opts, st, opts->out, cap);
    RHO_HIP(ctx->mat.ensure(std::max<uint64_t>(cap, 1) * sizeof(output_triple_t)));
    int rc = rho::join_device(ctx, s, dR, nR, dS, nS, opts, st, ctx->mat.as<output_triple_t>(), cap);
    if (rc) return rc;
    RHO_HIP(hipMemcpyAsync(opts->out, ctx->mat.ptr, st->matches * sizeof(output_triple_t), hipMemcpyDeviceToHost, s));
    RHO_HIP(hipStreamSynchronize(s));
    return MI355_OK;
}

}  // extern "C"

// Host chunked table of n triples (ChunkedTable.cpp layout: TUPLES_PER_CHUNK per chunk).
chunked_table_t *rho::make_chunked_table(const output_triple_t *src, uint64_t n) {
    auto *t = static_cast<chunked_table_t *>(std::calloc(1, sizeof(chunked_table_t)));
    if (!t) return nullptr;
    const uint64_t per = SGXAMD_TUPLES_PER_CHUNK;
    const uint64_t nchunks = std::max<uint64_t>((n + per - 1) / per, 1);
    t->chunks = static_cast<table_chunk_t **>(std::calloc(nchunks, sizeof(table_chunk_t *)));
    if (!t->chunks) {
        std::free(t);
        return nullptr;
    }
    t->chunk_capacity = nchunks;
    for (uint64_t c = 0; c < nchunks; ++c) {
        auto *ch = static_cast<table_chunk_t *>(std::malloc(sizeof(table_chunk_t)));
        if (!ch) {
            t->num_chunks = c;
            mi355_free_chunked_table(t);
            return nullptr;
        }
        const uint64_t k = std::min<uint64_t>(per, n - std::min<uint64_t>(n, c * per));
        ch->num_tuples = k;
        if (k) std::memcpy(ch->tuples, src + c * per, k * sizeof(output_triple_t));
        t->chunks[c] = ch;
    }
    t->num_chunks = nchunks;
    t->current_chunk = nchunks - 1;
    t->num_tuples = n;
    return t;
}

extern "C" {

void mi355_free_chunked_table(chunked_table_t *table) {
    if (!table) return;
    for (uint64_t c = 0; c < table->num_chunks; ++c) std::free(table->chunks[c]);
    std::free(table->chunks);
    std::free(table);
}

// Drop-ins for RHO() / RHT() (radix_join.cpp:1640-1648): join_init_run with
// bucket_chaining_join or histogram_join.
static int table_join(const table_t *relR, const table_t *relS, const joinconfig_t *config, result_t *out,
                      int algorithm) {
    if (!relR || !relS || !out) {
        set_last_error("null argument");
        return MI355_ERR_INVALID;
    }
    const bool materialize = config && config->MATERIALIZE;
    mi355_rho_stats st{};
    int rc;
    output_triple_t *host = nullptr;
    mi355_rho_opts o{};
    o.algorithm = algorithm;
    o.timing = 1;  // the drop-in logs the reference's phase lines (print_timing)
    if (!materialize) {
        rc = mi355_rho_join_ex(relR->tuples, relR->num_tuples, relS->tuples, relS->num_tuples, &o, &st);
    } else {
        // count first (capacity 0 -> MI355_ERR_CAPACITY with the size), then materialise
        o.materialize = 1;
        rc = mi355_rho_join_ex(relR->tuples, relR->num_tuples, relS->tuples, relS->num_tuples, &o, &st);
        if (rc == MI355_ERR_CAPACITY || (rc == MI355_OK && st.matches > 0)) {
            const uint64_t need = st.matches;
            host = static_cast<output_triple_t *>(std::malloc(std::max<uint64_t>(need, 1) * sizeof(output_triple_t)));
            if (!host) {
                set_last_error("host allocation of the materialised result failed");
                return MI355_ERR_OOM;
            }
            o.out = host;
            o.out_capacity = need;
            rc = mi355_rho_join_ex(relR->tuples, relR->num_tuples, relS->tuples, relS->num_tuples, &o, &st);
        }
    }
    if (rc) {
        std::free(host);
        return rc;
    }
    out->totalresults = (int64_t)st.matches;
    out->nthreads = config ? config->NTHREADS : 1;
    const double us = st.ms_total * 1000.0;
    out->throughput = us > 0 ? (double)(relR->num_tuples + relS->num_tuples) / us : 0.0;  // M rec/s
    out->materialized = materialize ? 1 : 0;
    out->result = nullptr;
    out->result_type = 0;
    if (materialize) {
        chunked_table_t *t = rho::make_chunked_table(host, st.matches);
        std::free(host);
        if (!t) {
            set_last_error("host allocation of the chunked table failed");
            return MI355_ERR_OOM;
        }
        out->result = t;
        out->result_type = 1;
    }
    return MI355_OK;
}

int mi355_rho_join(const table_t *relR, const table_t *relS, const joinconfig_t *config, result_t *out) {
    return table_join(relR, relS, config, out, MI355_ALGO_RHO);
}

int mi355_rht_join(const table_t *relR, const table_t *relS, const joinconfig_t *config, result_t *out) {
    return table_join(relR, relS, config, out, MI355_ALGO_RHT);
}

// Pipelined join (multi-GPU exchange): begin enqueues R's partition passes and returns;
// finish runs S's passes and build/probe once S is valid in the stream order.
int mi355_rho_join_begin(const row_t *R, uint64_t nR, uint64_t nS, const mi355_rho_opts *opts) {
    if ((!R && nR) || nR == 0 || nS == 0) {
        set_last_error("join_begin needs non-empty relations");
        return MI355_ERR_INVALID;
    }
    if (!is_device_pointer(R)) {
        set_last_error("join_begin needs a device-resident R");
        return MI355_ERR_INVALID;
    }
    if (opts && opts->materialize && opts->out && !is_device_pointer(opts->out)) {
        set_last_error("join_begin: materialisation output must be device memory");
        return MI355_ERR_INVALID;
    }
    int status = MI355_OK;
    Context *ctx = current_context(&status);
    if (!ctx) return status;
    std::lock_guard<std::mutex> lk(ctx->mu);
    rho::PendingJoin &pj = rho::pending_of(ctx);
    if (pj.active) {
        set_last_error("a pipelined join is already pending on this device");
        return MI355_ERR_INVALID;
    }
    const int rc = rho::join_begin(ctx, thread_stream(ctx, opts ? opts->stream : nullptr), R, nR, nS, opts, pj);
    if (rc) pj.active = false;
    return rc;
}

int mi355_rho_join_finish(const row_t *S, uint64_t nS, const mi355_rho_opts *opts, mi355_rho_stats *stats) {
    int status = MI355_OK;
    Context *ctx = current_context(&status);
    if (!ctx) return status;
    std::lock_guard<std::mutex> lk(ctx->mu);
    rho::PendingJoin &pj = rho::pending_of(ctx);
    mi355_rho_stats local{};
    mi355_rho_stats *st = stats ? stats : &local;
    std::memset(st, 0, sizeof(*st));
    if (!pj.active) {
        set_last_error("mi355_rho_join_finish without mi355_rho_join_begin");
        return MI355_ERR_INVALID;
    }
    if ((!S && nS) || !is_device_pointer(S)) {
        pj.active = false;
        set_last_error("join_finish needs a device-resident S");
        return MI355_ERR_INVALID;
    }
    struct Remember {
        mi355_rho_stats *st;
        ~Remember() { g_last_stats = *st; }
    } remember{st};
    const bool materialize = opts && opts->materialize;
    return rho::join_finish(ctx, pj, S, nS, st, materialize ? opts->out : nullptr,
                            materialize ? opts->out_capacity : 0, nullptr, true);
}

int mi355_rho_shard_partition(const row_t *in, uint64_t n, uint32_t key_shift, uint32_t dest_bits, row_t *out,
                              uint64_t *dest_counts, void *stream) {
    if ((!in && n) || !out || !dest_counts || dest_bits > 9 || key_shift + dest_bits > 32) {
        set_last_error("invalid shard_partition arguments");
        return MI355_ERR_INVALID;
    }
    if (!is_device_pointer(in) || !is_device_pointer(out)) {
        set_last_error("shard_partition needs device-resident in/out");
        return MI355_ERR_INVALID;
    }
    int status = MI355_OK;
    Context *ctx = current_context(&status);
    if (!ctx) return status;
    std::lock_guard<std::mutex> lk(ctx->mu);
    hipStream_t s = thread_stream(ctx, stream);
    if (n == 0) {
        std::memset(dest_counts, 0, sizeof(uint64_t) << dest_bits);
        return MI355_OK;
    }
    return rho::shard_partition_device(ctx, s, in, n, key_shift, dest_bits, out, dest_counts);
}

}  // extern "C"
