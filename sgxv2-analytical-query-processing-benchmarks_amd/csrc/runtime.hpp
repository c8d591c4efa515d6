// Per-device runtime: library stream, grow-only device buffers, per-kernel
// event timing and pointer classification.  Native replacement for the
// reference's per-call aligned_alloc/memset workspace (radix_join.cpp:1419-1450)
// and its rdtscp phase timers (rdtscpWrapper.h:6-35).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace sgxamd {

// Grow-only device allocation (HBM).  Never shrinks; freed with the context.
struct DeviceBuffer {
    void *ptr = nullptr;
    size_t bytes = 0;
    hipError_t ensure(size_t n);
    void release();
    template <typename T>
    T *as() const { return static_cast<T *>(ptr); }
};

// Bump allocator over one DeviceBuffer (256-B aligned slices).
struct Arena {
    DeviceBuffer buf;
    size_t used = 0;
    std::vector<std::pair<size_t, size_t>> plan;
    void reset() { used = 0; }
    size_t reserve(size_t bytes) {
        size_t off = (used + 255) & ~size_t(255);
        used = off + bytes;
        return off;
    }
    template <typename T>
    T *at(size_t off) const { return reinterpret_cast<T *>(static_cast<char *>(buf.ptr) + off); }
};

// Per-kernel HIP event timing, enabled per thread.
class Timer {
   public:
    // coarse: one span "total" from the first mark to end_call (two events per call
    // instead of one per kernel: what a join records when per-kernel timing is off)
    void begin_call(hipStream_t s, bool enabled, bool coarse = false);
    void mark(const char *name);  // closes the previous span, opens `name`
    void end_call();              // closes the last span (before the final sync)
    // after the stream synchronised: fold event pairs into (name, ms)
    void collect();
    const std::vector<std::pair<std::string, double>> &records() const { return records_; }
    double ms_of_prefix(const std::string &prefix) const;
    // after collect(): take over another timer's records (a second stream of the same call)
    void append(const Timer &other) {
        records_.insert(records_.end(), other.records_.begin(), other.records_.end());
    }
    bool enabled() const { return enabled_; }
    bool coarse() const { return coarse_; }

   private:
    bool coarse_ = false;
    bool sparse_ = false;  // mi355_timing_enable(2): Timer::mark
    hipEvent_t get_event();
    bool enabled_ = false;
    hipStream_t stream_ = nullptr;
    std::vector<hipEvent_t> pool_;
    size_t used_ = 0;
    std::vector<std::pair<std::string, std::pair<hipEvent_t, hipEvent_t>>> spans_;
    std::vector<std::pair<std::string, double>> records_;
    std::string open_name_;
    hipEvent_t open_ev_ = nullptr;
};

struct Context {
    int device = -1;
    hipStream_t stream = nullptr;  // library stream (non-blocking)
    hipStream_t side = nullptr;    // second stream: the S partition chain runs beside R's
    hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_t0 = nullptr, ev_t1 = nullptr;
    std::mutex mu;                 // one call at a time per device context
    // join workspace
    DeviceBuffer inR, inS;         // staging of host relations
    DeviceBuffer t1R, t1S, t2R, t2S;
    DeviceBuffer sideR, sideS;     // pass-2 digit per pass-1 output tuple (two-pass plans)
    Arena scratch;
    DeviceBuffer mat;              // materialised output_triple_t (when the caller's buffer is host memory)
    // TPC-H workspace: staged host columns, selection bits/offsets, intermediate
    // relations and join-result triples
    DeviceBuffer tp_cols[12], tp_mask, tp_blk, tp_rel[3], tp_trip;
    // scan workspace
    DeviceBuffer scan_in, scan_out, scan_aux, scan_dict;
    uint64_t *host_result = nullptr;  // pinned 64 x u64
    uint64_t *host_join = nullptr;    // coherent, mapped 8 x u64: written by the small join's kernel
    // coherent, mapped 8 x u64 (and its device address): the result words the large join's
    // count reduction writes (k_join_x's fold), read after the stream synchronisation
    uint64_t *host_fold = nullptr, *host_fold_dev = nullptr;
    // multi-GPU exchange workspace (multi_host.cpp): shard-partitioned send buffers and
    // the receive buffers the peers' pieces land in
    DeviceBuffer xsendR, xsendS, xrecvR, xrecvS;
    // the u16 wire: residuals grouped by destination and partition, then the partition
    // counts rows (send); the senders' runs, their counts rows and the gather's scratch (receive)
    DeviceBuffer wsendR, wsendS, wrecvR, wrecvS;
    Arena wscratch;  // the u16 wire's sender-side passes (rho::wire_partition)
    // in-launch hand-off words (tickets, digit totals) of the small-join path: zeroed
    // once when allocated (rho_internal.hpp kSync*)
    DeviceBuffer sync;
    uint32_t small_parity = 0;  // the small join's digit-totals set for the next call
    bool sync_dirty = false;    // a small join failed after its parity flip: re-zero sync first
};

// Context of the calling thread's current HIP device (created on first use).
// Returns nullptr (and sets the last error) when no device is available.
Context *current_context(int *status);
// A context of its own on `device` (its own stream and workspace), for callers that run
// several independent joins on one device: the multi-GPU rehearsal's logical ranks.
// The caller keeps it for the process lifetime.  nullptr (last error set) on failure.
std::unique_ptr<Context> make_context(int device, int *status);

// Frees every workspace buffer of ctx (the caller holds ctx->mu and no work is pending
// on its streams); later calls allocate again.
void release_workspace(Context *ctx);

Timer &thread_timer();
Timer &thread_side_timer();
// Lazily created side stream and fork/join/total events of ctx (nullptr on failure).
hipStream_t side_stream(Context *ctx);
bool thread_timing_enabled();
bool thread_partition_overlap();
// Counting joins move keys only after the input read (mi355_set_key_layout, default on).
bool thread_key_layout();
hipStream_t thread_stream(Context *ctx, void *explicit_stream);

bool is_device_pointer(const void *p);

}  // namespace sgxamd
