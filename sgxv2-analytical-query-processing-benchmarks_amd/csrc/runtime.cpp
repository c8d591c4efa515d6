// Per-device runtime (see runtime.hpp) and the error / timing C-ABI.
#include "runtime.hpp"

#include <cstdlib>

#include <map>
#include <memory>

#include "common.hpp"
#include "sgxamd/rho.h"

namespace sgxamd {

namespace {
thread_local std::string t_last_error;
thread_local int t_timing = 0;  // 0 off, 1 every kernel, 2 sparse (Timer::mark)
thread_local void *t_stream = nullptr;
thread_local Timer t_timer;
thread_local bool t_overlap = false;
thread_local bool t_keys = true;
std::mutex g_ctx_mu;
std::map<int, std::unique_ptr<Context>> g_ctx;
}  // namespace

void set_last_error(const std::string &msg) { t_last_error = msg; }
const char *last_error() { return t_last_error.c_str(); }

hipError_t DeviceBuffer::ensure(size_t n) {
    if (n <= bytes && ptr) return hipSuccess;
    release();
    size_t want = n < 256 ? 256 : n;
    hipError_t e = hipMalloc(&ptr, want);
    if (e != hipSuccess) {
        ptr = nullptr;
        bytes = 0;
        return e;
    }
    bytes = want;
    return hipSuccess;
}

void DeviceBuffer::release() {
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    bytes = 0;
}

// The per-kernel timing events skip the system-scope release fence an event performs by
// default (hipEventDisableSystemFence): they only time kernels of one stream, whose
// results the next kernel sees through the kernel boundary's own device-scope release.
// With the fence, every event between two kernels wrote the L2's dirty lines back to
// memory first: 5.5-6.3 us between the kernels of a join step at each of its 12 events
// (r06l kernel trace), about 70 us of a 2.6-ms step.  SGXAMD_TIMER_FENCE=1 keeps the
// fence (development A/B switch, read once).
static unsigned timer_event_flags() {
    static const unsigned f = [] {
        const char *e = std::getenv("SGXAMD_TIMER_FENCE");
        return (e && std::atoi(e) == 1) ? (unsigned)hipEventDefault : (unsigned)hipEventDisableSystemFence;
    }();
    return f;
}

hipEvent_t Timer::get_event() {
    if (used_ == pool_.size()) {
        hipEvent_t ev = nullptr;
        if (hipEventCreateWithFlags(&ev, timer_event_flags()) != hipSuccess) return nullptr;
        pool_.push_back(ev);
    }
    return pool_[used_++];
}

void Timer::begin_call(hipStream_t s, bool enabled, bool coarse) {
    enabled_ = enabled;
    coarse_ = coarse;
    sparse_ = enabled && !coarse && t_timing == 2;
    stream_ = s;
    used_ = 0;
    spans_.clear();
    records_.clear();
    open_name_.clear();
    open_ev_ = nullptr;
}

// Sparse timing (mi355_timing_enable(2)): events only around the spans a roofline reads
// -- R's pass-1 scatter and the build/probe -- and one "other" span between them, so a
// timed step carries 4 events instead of one per kernel (each event between two kernels
// costs 4.5-4.8 us of GPU time even without the system fence: r06q kernel trace).
static bool sparse_kept(const std::string &n) { return n == "R_pass1_scatter" || n == "join_build_probe"; }

void Timer::mark(const char *name) {
    if (!enabled_ || (coarse_ && open_ev_)) return;
    if (sparse_ && !sparse_kept(name) && !(open_ev_ && sparse_kept(open_name_))) return;
    hipEvent_t ev = get_event();
    if (!ev) return;
    (void)hipEventRecord(ev, stream_);
    if (open_ev_) spans_.push_back({open_name_, {open_ev_, ev}});
    open_name_ = coarse_ ? "total" : (sparse_ && !sparse_kept(name)) ? "other" : name;
    open_ev_ = ev;
}

void Timer::end_call() {
    if (!enabled_ || !open_ev_) return;
    hipEvent_t ev = get_event();
    if (!ev) return;
    (void)hipEventRecord(ev, stream_);
    spans_.push_back({open_name_, {open_ev_, ev}});
    open_ev_ = nullptr;
}

void Timer::collect() {
    records_.clear();
    for (auto &s : spans_) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, s.second.first, s.second.second) != hipSuccess) ms = 0.f;
        records_.push_back({s.first, (double)ms});
    }
}

double Timer::ms_of_prefix(const std::string &prefix) const {
    double t = 0;
    for (auto &r : records_)
        if (r.first.compare(0, prefix.size(), prefix) == 0) t += r.second;
    return t;
}

Timer &thread_timer() { return t_timer; }
Timer &thread_side_timer() {
    static thread_local Timer t;
    return t;
}

hipStream_t side_stream(Context *ctx) {
    if (!ctx->side) {
        if (hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking) != hipSuccess) return nullptr;
        for (hipEvent_t *e : {&ctx->ev_fork, &ctx->ev_join})
            if (hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess) return nullptr;
        for (hipEvent_t *e : {&ctx->ev_t0, &ctx->ev_t1})
            if (hipEventCreate(e) != hipSuccess) return nullptr;
    }
    return ctx->side;
}
bool thread_timing_enabled() { return t_timing != 0; }
bool thread_partition_overlap() { return t_overlap; }
bool thread_key_layout() { return t_keys; }


Context *current_context(int *status) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        (void)hipGetLastError();
        set_last_error("no HIP device visible (mi355_* needs a gfx950 GPU)");
        if (status) *status = MI355_ERR_NO_DEVICE;
        return nullptr;
    }
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) {
        set_last_error("hipGetDevice failed");
        if (status) *status = MI355_ERR_HIP;
        return nullptr;
    }
    std::lock_guard<std::mutex> lk(g_ctx_mu);
    auto it = g_ctx.find(dev);
    if (it != g_ctx.end()) return it->second.get();
    auto ctx = make_context(dev, status);
    if (!ctx) return nullptr;
    Context *raw = ctx.get();
    g_ctx[dev] = std::move(ctx);
    return raw;
}

std::unique_ptr<Context> make_context(int device, int *status) {
    int prev = 0;
    if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(device) != hipSuccess) {
        set_last_error("hipSetDevice failed");
        if (status) *status = MI355_ERR_HIP;
        return nullptr;
    }
    auto ctx = std::make_unique<Context>();
    ctx->device = device;
    const bool ok = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) == hipSuccess &&
                    hipHostMalloc(reinterpret_cast<void **>(&ctx->host_result), 64 * sizeof(uint64_t)) == hipSuccess;
    (void)hipSetDevice(prev);
    if (!ok) {
        set_last_error("stream / pinned allocation failed");
        if (status) *status = MI355_ERR_HIP;
        return nullptr;
    }
    return ctx;
}

void release_workspace(Context *ctx) {
    for (DeviceBuffer *b : {&ctx->inR, &ctx->inS, &ctx->t1R, &ctx->t1S, &ctx->t2R, &ctx->t2S, &ctx->sideR, &ctx->sideS,
                            &ctx->scratch.buf, &ctx->mat, &ctx->tp_mask, &ctx->tp_blk, &ctx->tp_trip, &ctx->scan_in,
                            &ctx->scan_out, &ctx->scan_aux, &ctx->scan_dict, &ctx->xsendR, &ctx->xsendS, &ctx->xrecvR,
                            &ctx->xrecvS, &ctx->wsendR, &ctx->wsendS, &ctx->wrecvR, &ctx->wrecvS, &ctx->wscratch.buf})
        b->release();
    for (DeviceBuffer &b : ctx->tp_cols) b.release();
    for (DeviceBuffer &b : ctx->tp_rel) b.release();
    ctx->scratch.reset();
    ctx->wscratch.reset();
}

hipStream_t thread_stream(Context *ctx, void *explicit_stream) {
    if (explicit_stream) return static_cast<hipStream_t>(explicit_stream);
    if (t_stream) return static_cast<hipStream_t>(t_stream);
    return ctx->stream;
}

bool is_device_pointer(const void *p) {
    if (!p) return false;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
}

}  // namespace sgxamd

extern "C" {

const char *mi355_last_error(void) { return sgxamd::last_error(); }

const char *mi355_version(void) { return "sgxamd-mi355 0.1 (gfx950)"; }

int mi355_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}

void mi355_timing_enable(int on) { sgxamd::t_timing = on == 2 ? 2 : on != 0 ? 1 : 0; }

void mi355_set_partition_overlap(int on) { sgxamd::t_overlap = on != 0; }

void mi355_set_key_layout(int on) { sgxamd::t_keys = on != 0; }

int mi355_timing_get(const char **names, double *ms, int cap) {
    const auto &rec = sgxamd::t_timer.records();
    const int n = (int)rec.size();
    for (int i = 0; i < n && i < cap; ++i) {
        if (names) names[i] = rec[i].first.c_str();
        if (ms) ms[i] = rec[i].second;
    }
    return n;
}

void mi355_set_stream(void *stream) { sgxamd::t_stream = stream; }

}  // extern "C"
