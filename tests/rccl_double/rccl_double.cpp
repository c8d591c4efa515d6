// Test double of RCCL for the multi-GPU join's RcclTransport (csrc/multi_host.cpp).
//
// RCCL refuses two ranks on one GPU, so on a one-GPU box the transport's grouped
// Send/Recv, its count all-gather on the split communicator and its all-reduces could
// otherwise first run at G > 1 on the driver's 8-GPU node.  This library exports the
// RCCL entry points the transport binds (loaded through mi355_multi_set_rccl_library)
// and implements them for ranks that are threads of ONE process, each with its own
// stream, all on one GPU:
//   - communicators: ncclCommInitRank (a registry keyed by the unique id; blocks until
//     every rank joined, like RCCL), ncclCommInitAll, ncclCommSplit (a collective over
//     the parent), ncclCommDestroy, ncclCommAbort (releases every waiter of the world
//     with an error);
//   - ncclSend/ncclRecv inside ncclGroupStart/End: at GroupEnd a rank publishes its
//     sends (source, size, an event recorded on its stream), then for every receive
//     takes the peer's next send on that channel, makes its stream wait for the
//     sender's event and copies device to device on its own stream with a copy kernel
//     (k_copy: RCCL's own p2p transfers are kernels on the communication stream, a
//     workgroup per channel, so they compete with the join's kernels for CUs; a
//     hipMemcpyAsync would use the DMA engines and hide that); the sender's stream
//     then waits for the receiver's copy (the sender must not overwrite its buffer
//     before the copy ran: RCCL's stream semantics).  Sizes must match (else
//     ncclInvalidUsage), as RCCL's would;
//   - ncclAllGather: every rank copies every rank's block into its receive buffer on its
//     own stream (k_copy) after the owner's ready event; every stream then waits for every
//     copy;
//   - ncclAllReduce: staged through the host (sum / max / min of integer and double
//     types), synchronous with respect to the caller's stream.
// Fault injection for the failure protocol tests: rccl_double_fail(rank, n) makes rank's
// n-th later call (counting Send, Recv, AllGather, AllReduce and CommSplit) return
// ncclSystemError.  Unlike RCCL, GroupEnd and the collectives block the calling host
// thread until the peers' matching calls arrived; every such wait is bounded
// (rccl_double_set_timeout_ms, default 20 s) and then fails with ncclSystemError, so a
// rank that never posts its part cannot hang a test.  ncclCommAbort releases every
// waiter of the communicator's world at once.
//
// Ranks as PROCESSES (RCCL_DOUBLE_XPROC=1; round 6): the one-process-per-GPU path of a
// torchrun job -- mi355_multi_comm_init with rank 0's unique id broadcast by the caller,
// the split count communicator, mi355_rho_join_sharded -- run by rank processes that
// share this box's one GPU.  A communicator is a POSIX shared-memory block named after
// the unique id (created by the first rank to arrive, unlinked once every rank mapped
// it): a barrier, per (src, dst) channel a ring of posted sends and their acks, and a
// host slot per rank for the collectives.  ncclSend publishes the IPC handle of its
// buffer's allocation (hipIpcGetMemHandle) and offset once the send's data is ready on
// its stream (the host waits for it); the receiver maps the allocation
// (hipIpcOpenMemHandle, cached), copies with k_copy on its stream, waits for the copy and
// acks; the sender returns from ncclGroupEnd once every send is acked.  All-gather and
// all-reduce go through the host slots.  Every wait is bounded (rccl_double_set_timeout_ms).
//
// Test infrastructure only: the product loads librccl.so.1; nothing here is on the path.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace {

// The transfer kernel: kCopyWgs workgroups (RCCL_DOUBLE_COPY_WGS; RCCL's p2p runs a
// workgroup per channel, of the order of 16 per peer set) copying 16-byte words when
// source, destination and size allow, 4-byte words, or bytes.
int copy_wgs() {
    static const int n = [] {
        const char *e = std::getenv("RCCL_DOUBLE_COPY_WGS");
        const int v = e ? std::atoi(e) : 16;
        return v > 0 && v <= 1024 ? v : 16;
    }();
    return n;
}

__global__ __launch_bounds__(512) void k_copy(const char *__restrict__ src, char *__restrict__ dst, size_t bytes) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (size_t)gridDim.x * blockDim.x;
    const uintptr_t al = reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst) | bytes;
    if ((al & 15) == 0) {
        const uint4 *s4 = reinterpret_cast<const uint4 *>(src);
        uint4 *d4 = reinterpret_cast<uint4 *>(dst);
        for (size_t i = t; i < bytes / 16; i += stride) d4[i] = s4[i];
    } else if ((al & 3) == 0) {
        const uint32_t *s1 = reinterpret_cast<const uint32_t *>(src);
        uint32_t *d1 = reinterpret_cast<uint32_t *>(dst);
        for (size_t i = t; i < bytes / 4; i += stride) d1[i] = s1[i];
    } else {
        for (size_t i = t; i < bytes; i += stride) dst[i] = src[i];
    }
}

hipError_t copy_d2d(void *dst, const void *src, size_t bytes, hipStream_t s) {
    if (!bytes) return hipSuccess;
    hipLaunchKernelGGL(k_copy, dim3(copy_wgs()), dim3(512), 0, s, static_cast<const char *>(src),
                       static_cast<char *>(dst), bytes);
    return hipGetLastError();
}

struct SendPost {
    const void *src = nullptr;
    size_t bytes = 0;
    hipEvent_t ready = nullptr;  // on the sender's stream, after everything before the send
    hipEvent_t done = nullptr;   // on the receiver's stream, after the copy (set by the receiver)
    bool failed = false;         // the receiver rejected it (size mismatch)
};

struct Slot {  // one rank's part of a collective
    const void *ptr = nullptr;
    hipEvent_t ev = nullptr;
    std::vector<uint64_t> host;  // all-reduce operands (as raw 8-byte words)
    int color = 0, key = 0;
};

struct World {
    explicit World(int n) : n(n), slots(n), done(n) {}
    const int n;
    std::mutex mu;
    std::condition_variable cv;
    bool aborted = false;
    uint64_t gen = 0;
    int waiting = 0;
    std::map<std::pair<int, int>, std::deque<std::shared_ptr<SendPost>>> chan;  // (src, dst)
    std::vector<Slot> slots;
    std::vector<hipEvent_t> done;
    std::map<int, std::shared_ptr<World>> split;  // color -> new world (one split at a time)

    // all n ranks meet; false when the world was aborted or the wait timed out (lk held)
    bool barrier(std::unique_lock<std::mutex> &lk);
    template <typename Pred>
    bool wait(std::unique_lock<std::mutex> &lk, Pred p);
};

std::atomic<int> g_timeout_ms{20000};

template <typename Pred>
bool World::wait(std::unique_lock<std::mutex> &lk, Pred p) {
    const bool ok = cv.wait_for(lk, std::chrono::milliseconds(g_timeout_ms.load()), [&] { return p() || aborted; });
    if (!ok) {  // a peer never came: the world is unusable for every rank
        aborted = true;
        cv.notify_all();
    }
    return ok && !aborted;
}

bool World::barrier(std::unique_lock<std::mutex> &lk) {
    if (aborted) return false;
    const uint64_t g = gen;
    if (++waiting == n) {
        waiting = 0;
        ++gen;
        cv.notify_all();
        return true;
    }
    if (wait(lk, [&] { return gen != g; })) return true;
    if (gen == g) --waiting;  // timed out or aborted: leave the barrier
    return gen != g;
}

}  // namespace

// ---------------------------------------------------------------- ranks as processes
namespace {

constexpr int kXMax = 16;          // ranks
constexpr int kXRing = 64;         // posted sends in flight per channel
constexpr size_t kXSlot = 1 << 16; // host bytes per rank for a collective

struct XPost {
    std::atomic<uint64_t> seq;  // the post's sequence number once published (0: empty)
    std::atomic<uint64_t> ack;  // the receiver's ack of that sequence number
    hipIpcMemHandle_t mem;
    uint64_t off, bytes;
    int failed;
};

struct XShm {
    std::atomic<int> joined, n, aborted;
    std::atomic<uint64_t> bar_count, bar_gen;
    XPost chan[kXMax][kXMax][kXRing];  // [src][dst]
    int color[kXMax], key[kXMax];
    uint64_t slot_bytes[kXMax];
    uint8_t slot[kXMax][kXSlot];
};

bool xproc() {
    static const bool on = [] {
        const char *e = std::getenv("RCCL_DOUBLE_XPROC");
        return e && std::atoi(e) == 1;
    }();
    return on;
}

}  // namespace

struct ncclComm {
    std::shared_ptr<World> w;
    int rank = 0, dev = 0;
    // ranks as processes
    XShm *x = nullptr;
    int n = 0;
    std::string name;
    uint64_t sseq[kXMax] = {}, rseq[kXMax] = {};  // last send / receive sequence per peer
    int splits = 0;
};

namespace {

std::mutex g_reg_mu;
std::condition_variable g_reg_cv;
struct Pending {
    std::shared_ptr<World> w;
    int joined = 0;
};
std::map<std::string, Pending> g_reg;  // unique id -> world being formed

// fault injection: per rank, calls left before the failing one (0 = none)
std::mutex g_fail_mu;
std::map<int, int> g_fail;

bool fail_now(int rank) {
    std::lock_guard<std::mutex> lk(g_fail_mu);
    auto it = g_fail.find(rank);
    if (it == g_fail.end()) return false;
    if (--it->second > 0) return false;
    g_fail.erase(it);
    return true;
}

thread_local int t_group = 0;
struct Op {
    bool send;
    ncclComm_t comm;
    int peer;
    void *buf;
    size_t bytes;
    hipStream_t stream;
};
thread_local std::vector<Op> t_ops;

size_t type_size(ncclDataType_t t) {
    switch (t) {
        case ncclInt8: case ncclUint8: return 1;
        case ncclFloat16: case ncclBfloat16: return 2;
        case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
        case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
        default: return 0;
    }
}

ncclResult_t xrun_group(std::vector<Op> &ops);

ncclResult_t run_group(std::vector<Op> &ops) {
    if (!ops.empty() && ops[0].comm->x) return xrun_group(ops);
    // phase 1: publish every send
    std::vector<std::shared_ptr<SendPost>> mine;
    for (const Op &o : ops) {
        if (!o.send) continue;
        auto p = std::make_shared<SendPost>();
        p->src = o.buf;
        p->bytes = o.bytes;
        if (hipEventCreateWithFlags(&p->ready, hipEventDisableTiming) != hipSuccess ||
            hipEventRecord(p->ready, o.stream) != hipSuccess)
            return ncclUnhandledCudaError;
        World &w = *o.comm->w;
        std::lock_guard<std::mutex> lk(w.mu);
        w.chan[{o.comm->rank, o.peer}].push_back(p);
        w.cv.notify_all();
        mine.push_back(p);
    }
    // phase 2: every receive takes the peer's next send on the channel
    ncclResult_t rc = ncclSuccess;
    for (const Op &o : ops) {
        if (o.send) continue;
        World &w = *o.comm->w;
        std::shared_ptr<SendPost> p;
        {
            std::unique_lock<std::mutex> lk(w.mu);
            auto &q = w.chan[{o.peer, o.comm->rank}];
            if (!w.wait(lk, [&] { return !q.empty(); })) return ncclSystemError;
            p = q.front();
            q.pop_front();
        }
        hipEvent_t done = nullptr;
        bool ok = p->bytes == o.bytes;
        if (!ok) rc = ncclInvalidUsage;
        if (ok && (hipStreamWaitEvent(o.stream, p->ready, 0) != hipSuccess ||
                   copy_d2d(o.buf, p->src, o.bytes, o.stream) != hipSuccess))
            return ncclUnhandledCudaError;
        if (hipEventCreateWithFlags(&done, hipEventDisableTiming) != hipSuccess ||
            hipEventRecord(done, o.stream) != hipSuccess)
            return ncclUnhandledCudaError;
        std::lock_guard<std::mutex> lk(w.mu);
        p->failed = !ok;
        p->done = done;
        w.cv.notify_all();
    }
    // phase 3: the sender's stream waits for the receiver's copy
    size_t k = 0;
    for (const Op &o : ops) {
        if (!o.send) continue;
        auto &p = mine[k++];
        World &w = *o.comm->w;
        {
            std::unique_lock<std::mutex> lk(w.mu);
            if (!w.wait(lk, [&] { return p->done != nullptr; })) return ncclSystemError;
        }
        if (p->failed) rc = ncclInvalidUsage;
        if (hipStreamWaitEvent(o.stream, p->done, 0) != hipSuccess) return ncclUnhandledCudaError;
        (void)hipEventDestroy(p->ready);
        (void)hipEventDestroy(p->done);
    }
    return rc;
}

ncclResult_t enqueue(bool send, void *buf, size_t count, ncclDataType_t t, int peer, ncclComm_t comm,
                     hipStream_t s) {
    if (!comm || peer < 0 || peer >= (comm->x ? comm->n : comm->w->n) || !type_size(t)) return ncclInvalidArgument;
    if (fail_now(comm->rank)) return ncclSystemError;
    t_ops.push_back(Op{send, comm, peer, buf, count * type_size(t), s});
    if (t_group > 0) return ncclSuccess;
    std::vector<Op> ops;
    ops.swap(t_ops);
    return run_group(ops);
}

template <typename T>
void reduce_into(std::vector<uint64_t> &acc, const std::vector<uint64_t> &x, size_t count, ncclRedOp_t op) {
    T *a = reinterpret_cast<T *>(acc.data());
    const T *b = reinterpret_cast<const T *>(x.data());
    for (size_t i = 0; i < count; ++i) {
        if (op == ncclSum) a[i] = a[i] + b[i];
        else if (op == ncclMax) a[i] = std::max(a[i], b[i]);
        else a[i] = std::min(a[i], b[i]);
    }
}

// ---- ranks as processes (XShm communicators)

template <typename Pred>
bool xwait(XShm *x, Pred p) {
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0;; ++i) {
        if (p()) return true;
        if (x->aborted.load()) return false;
        if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(g_timeout_ms.load())) {
            x->aborted.store(1);  // a peer never came: the communicator is unusable
            return false;
        }
        if (i > 64) std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
}

bool xbarrier(ncclComm *c) {
    XShm *x = c->x;
    const uint64_t g = x->bar_gen.load();
    if (x->bar_count.fetch_add(1) + 1 == (uint64_t)c->n) {
        x->bar_count.store(0);
        x->bar_gen.fetch_add(1);
        return true;
    }
    return xwait(x, [&] { return x->bar_gen.load() != g; });
}

// map (creating if first) the block `name`, join it as `rank` of n, wait for every rank;
// rank 0 unlinks the name once all have mapped it
ncclResult_t xjoin(const std::string &name, int n, int rank, ncclComm *c) {
    if (n > kXMax) return ncclInvalidArgument;
    const int fd = shm_open(name.c_str(), O_CREAT | O_RDWR, 0600);
    if (fd < 0) return ncclSystemError;
    if (ftruncate(fd, sizeof(XShm)) != 0) {
        close(fd);
        return ncclSystemError;
    }
    void *m = mmap(nullptr, sizeof(XShm), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (m == MAP_FAILED) return ncclSystemError;
    XShm *x = static_cast<XShm *>(m);
    int expect = 0;
    if (!x->n.compare_exchange_strong(expect, n) && expect != n) {
        munmap(m, sizeof(XShm));
        return ncclInvalidArgument;
    }
    c->x = x;
    c->n = n;
    c->rank = rank;
    c->name = name;
    x->joined.fetch_add(1);
    const bool ok = xwait(x, [&] { return x->joined.load() >= n; }) && xbarrier(c);
    if (rank == 0) shm_unlink(name.c_str());
    if (!ok) {
        munmap(m, sizeof(XShm));
        c->x = nullptr;
        return ncclSystemError;
    }
    return ncclSuccess;
}

std::string xname(const ncclUniqueId &id) {
    static const char *hex = "0123456789abcdef";
    std::string s = "/rccld_";
    for (int i = 0; i < 24; ++i) {
        const uint8_t b = static_cast<uint8_t>(id.internal[i]);
        s += hex[b >> 4];
        s += hex[b & 15];
    }
    return s;
}

// a peer's allocation mapped into this process (never unmapped: test double)
std::mutex g_ipc_mu;
std::map<std::string, char *> g_ipc;
char *xopen(const hipIpcMemHandle_t &h) {
    const std::string k(reinterpret_cast<const char *>(&h), sizeof(h));
    std::lock_guard<std::mutex> lk(g_ipc_mu);
    auto it = g_ipc.find(k);
    if (it != g_ipc.end()) return it->second;
    void *p = nullptr;
    if (hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) return nullptr;
    g_ipc[k] = static_cast<char *>(p);
    return static_cast<char *>(p);
}

ncclResult_t xrun_group(std::vector<Op> &ops) {
    ncclResult_t rc = ncclSuccess;
    struct Mine {
        XShm *x;
        XPost *p;
        uint64_t seq;
    };
    std::vector<Mine> mine;
    // phase 1: every send published once its data is ready on its stream
    for (const Op &o : ops) {
        if (!o.send) continue;
        ncclComm *c = o.comm;
        XShm *x = c->x;
        hipIpcMemHandle_t h{};
        uint64_t off = 0;
        if (o.bytes) {
            hipEvent_t e = nullptr;
            if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess || hipEventRecord(e, o.stream) != hipSuccess ||
                hipEventSynchronize(e) != hipSuccess)
                return ncclUnhandledCudaError;
            (void)hipEventDestroy(e);
            void *base = nullptr;
            size_t sz = 0;
            if (hipMemGetAddressRange(&base, &sz, o.buf) != hipSuccess || hipIpcGetMemHandle(&h, base) != hipSuccess)
                return ncclUnhandledCudaError;
            off = static_cast<uint64_t>(static_cast<char *>(o.buf) - static_cast<char *>(base));
        }
        const uint64_t seq = ++c->sseq[o.peer];
        XPost &p = x->chan[c->rank][o.peer][seq % kXRing];
        if (seq > (uint64_t)kXRing && !xwait(x, [&] { return p.ack.load() >= seq - kXRing; })) return ncclSystemError;
        p.mem = h;
        p.off = off;
        p.bytes = o.bytes;
        p.failed = 0;
        p.seq.store(seq, std::memory_order_release);
        mine.push_back({x, &p, seq});
    }
    // phase 2: every receive takes the peer's next post on the channel, copies, acks
    for (const Op &o : ops) {
        if (o.send) continue;
        ncclComm *c = o.comm;
        XShm *x = c->x;
        const uint64_t seq = ++c->rseq[o.peer];
        XPost &p = x->chan[o.peer][c->rank][seq % kXRing];
        if (!xwait(x, [&] { return p.seq.load(std::memory_order_acquire) == seq; })) return ncclSystemError;
        const bool ok = p.bytes == o.bytes;
        if (!ok) rc = ncclInvalidUsage;
        if (ok && o.bytes) {
            char *src = xopen(p.mem);
            if (!src || copy_d2d(o.buf, src + p.off, o.bytes, o.stream) != hipSuccess ||
                hipStreamSynchronize(o.stream) != hipSuccess)
                return ncclUnhandledCudaError;
        }
        p.failed = ok ? 0 : 1;
        p.ack.store(seq, std::memory_order_release);
    }
    // phase 3: the sender returns once every send was copied (its buffer is free again)
    for (const Mine &m : mine) {
        if (!xwait(m.x, [&] { return m.p->ack.load(std::memory_order_acquire) >= m.seq; })) return ncclSystemError;
        if (m.p->failed) rc = ncclInvalidUsage;
    }
    return rc;
}

// one rank's bytes into its host slot, a barrier, then f(slots), a barrier
template <typename F>
ncclResult_t xcollective(ncclComm *c, const void *send, size_t bytes, hipStream_t s, F f) {
    XShm *x = c->x;
    if (bytes > kXSlot) return ncclInvalidArgument;
    if (hipMemcpyAsync(x->slot[c->rank], send, bytes, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return ncclUnhandledCudaError;
    x->slot_bytes[c->rank] = bytes;
    if (!xbarrier(c)) return ncclSystemError;
    const ncclResult_t r = f();
    if (!xbarrier(c)) return ncclSystemError;
    return r;
}

}  // namespace

extern "C" {

void rccl_double_set_timeout_ms(int ms) { g_timeout_ms = ms > 0 ? ms : 20000; }

void rccl_double_fail(int rank, int nth_call) {
    std::lock_guard<std::mutex> lk(g_fail_mu);
    if (nth_call > 0) g_fail[rank] = nth_call;
    else g_fail.erase(rank);
}

const char *ncclGetErrorString(ncclResult_t r) {
    switch (r) {
        case ncclSuccess: return "no error (rccl double)";
        case ncclUnhandledCudaError: return "unhandled HIP error (rccl double)";
        case ncclSystemError: return "system error: injected, or the communicator was aborted (rccl double)";
        case ncclInvalidArgument: return "invalid argument (rccl double)";
        case ncclInvalidUsage: return "invalid usage: send/recv sizes differ (rccl double)";
        default: return "error (rccl double)";
    }
}

ncclResult_t ncclGetUniqueId(ncclUniqueId *id) {
    static std::atomic<uint64_t> seq{1};
    std::memset(id, 0, sizeof(*id));
    const uint64_t v[3] = {0x52434344424cULL, (uint64_t)getpid(),
                           seq++ ^ (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count()};
    std::memcpy(id->internal, v, sizeof(v));
    return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t *comm, int nranks, ncclUniqueId id, int rank) {
    if (!comm || nranks < 1 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
    if (xproc()) {
        auto *c = new ncclComm;
        const ncclResult_t r = xjoin(xname(id), nranks, rank, c);
        if (r != ncclSuccess) {
            delete c;
            return r;
        }
        (void)hipGetDevice(&c->dev);
        *comm = c;
        return ncclSuccess;
    }
    const std::string key(id.internal, sizeof(id.internal));
    std::shared_ptr<World> w;
    {
        std::unique_lock<std::mutex> lk(g_reg_mu);
        Pending &p = g_reg[key];
        if (!p.w) p.w = std::make_shared<World>(nranks);
        if (p.w->n != nranks) return ncclInvalidArgument;
        w = p.w;
        if (++p.joined == nranks) {
            g_reg.erase(key);
            g_reg_cv.notify_all();
        } else if (!g_reg_cv.wait_for(lk, std::chrono::milliseconds(g_timeout_ms.load()),
                                      [&] { return !g_reg.count(key) || g_reg[key].w != w; })) {
            g_reg.erase(key);  // not every rank came
            return ncclSystemError;
        }
    }
    auto *c = new ncclComm;
    c->w = w;
    c->rank = rank;
    (void)hipGetDevice(&c->dev);
    *comm = c;
    return ncclSuccess;
}

ncclResult_t ncclCommInitAll(ncclComm_t *comms, int ndev, const int *devlist) {
    if (!comms || ndev < 1) return ncclInvalidArgument;
    auto w = std::make_shared<World>(ndev);
    for (int i = 0; i < ndev; ++i) {
        comms[i] = new ncclComm;
        comms[i]->w = w;
        comms[i]->rank = i;
        comms[i]->dev = devlist ? devlist[i] : i;
    }
    return ncclSuccess;
}

ncclResult_t ncclCommSplit(ncclComm_t comm, int color, int key, ncclComm_t *newcomm, ncclConfig_t *) {
    if (!comm || !newcomm) return ncclInvalidArgument;
    if (fail_now(comm->rank)) return ncclSystemError;
    if (comm->x) {
        XShm *x = comm->x;
        x->color[comm->rank] = color;
        x->key[comm->rank] = key;
        if (!xbarrier(comm)) return ncclSystemError;
        std::vector<std::pair<int, int>> members;
        for (int r = 0; r < comm->n; ++r)
            if (x->color[r] == color) members.push_back({x->key[r], r});
        std::sort(members.begin(), members.end());
        int newrank = 0;
        while (members[newrank].second != comm->rank) ++newrank;
        const std::string name = comm->name + "_s" + std::to_string(comm->splits++) + "c" + std::to_string(color);
        if (!xbarrier(comm)) return ncclSystemError;  // (colors read before any rank's next split)
        if (color == NCCL_SPLIT_NOCOLOR) {
            *newcomm = nullptr;
            return ncclSuccess;
        }
        auto *c = new ncclComm;
        const ncclResult_t r = xjoin(name, (int)members.size(), newrank, c);
        if (r != ncclSuccess) {
            delete c;
            return r;
        }
        c->dev = comm->dev;
        *newcomm = c;
        return ncclSuccess;
    }
    World &w = *comm->w;
    std::unique_lock<std::mutex> lk(w.mu);
    w.slots[comm->rank].color = color;
    w.slots[comm->rank].key = key;
    if (!w.barrier(lk)) return ncclSystemError;
    // members of this color, ordered by (key, parent rank)
    std::vector<std::pair<int, int>> members;
    for (int r = 0; r < w.n; ++r)
        if (w.slots[r].color == color) members.push_back({w.slots[r].key, r});
    std::sort(members.begin(), members.end());
    int newrank = 0;
    while (members[newrank].second != comm->rank) ++newrank;
    if (color != NCCL_SPLIT_NOCOLOR && !w.split.count(color)) w.split[color] = std::make_shared<World>((int)members.size());
    if (!w.barrier(lk)) return ncclSystemError;
    if (color == NCCL_SPLIT_NOCOLOR) {
        *newcomm = nullptr;
    } else {
        auto *c = new ncclComm;
        c->w = w.split[color];
        c->rank = newrank;
        c->dev = comm->dev;
        *newcomm = c;
    }
    if (!w.barrier(lk)) return ncclSystemError;
    if (comm->rank == 0) w.split.clear();
    return w.barrier(lk) ? ncclSuccess : ncclSystemError;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
    if (comm && comm->x) munmap(comm->x, sizeof(XShm));
    delete comm;
    return ncclSuccess;
}

// The comm object is not freed: another thread may still be inside a call on it (the
// waiters this abort releases); a few bytes per aborted communicator are leaked.
ncclResult_t ncclCommAbort(ncclComm_t comm) {
    if (!comm) return ncclSuccess;
    if (comm->x) {
        comm->x->aborted.store(1);
        return ncclSuccess;
    }
    std::lock_guard<std::mutex> lk(comm->w->mu);
    comm->w->aborted = true;
    comm->w->cv.notify_all();
    return ncclSuccess;
}

ncclResult_t ncclGroupStart() {
    ++t_group;
    return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
    if (t_group <= 0) return ncclInvalidUsage;
    if (--t_group > 0) return ncclSuccess;
    std::vector<Op> ops;
    ops.swap(t_ops);
    return run_group(ops);
}

ncclResult_t ncclSend(const void *buf, size_t count, ncclDataType_t t, int peer, ncclComm_t comm, hipStream_t s) {
    return enqueue(true, const_cast<void *>(buf), count, t, peer, comm, s);
}

ncclResult_t ncclRecv(void *buf, size_t count, ncclDataType_t t, int peer, ncclComm_t comm, hipStream_t s) {
    return enqueue(false, buf, count, t, peer, comm, s);
}

ncclResult_t ncclAllGather(const void *send, void *recv, size_t count, ncclDataType_t t, ncclComm_t comm,
                           hipStream_t s) {
    const size_t bytes = count * type_size(t);
    if (!comm || !bytes) return ncclInvalidArgument;
    if (fail_now(comm->rank)) return ncclSystemError;
    if (comm->x) {
        return xcollective(comm, send, bytes, s, [&]() -> ncclResult_t {
            for (int q = 0; q < comm->n; ++q)
                if (hipMemcpyAsync(static_cast<char *>(recv) + q * bytes, comm->x->slot[q], bytes,
                                   hipMemcpyHostToDevice, s) != hipSuccess)
                    return ncclUnhandledCudaError;
            return hipStreamSynchronize(s) == hipSuccess ? ncclSuccess : ncclUnhandledCudaError;
        });
    }
    World &w = *comm->w;
    const int r = comm->rank;
    hipEvent_t ready = nullptr, done = nullptr;
    if (hipEventCreateWithFlags(&ready, hipEventDisableTiming) != hipSuccess || hipEventRecord(ready, s) != hipSuccess)
        return ncclUnhandledCudaError;
    std::unique_lock<std::mutex> lk(w.mu);
    w.slots[r].ptr = send;
    w.slots[r].ev = ready;
    if (!w.barrier(lk)) return ncclSystemError;
    for (int q = 0; q < w.n; ++q)
        if (hipStreamWaitEvent(s, w.slots[q].ev, 0) != hipSuccess ||
            copy_d2d(static_cast<char *>(recv) + q * bytes, w.slots[q].ptr, bytes, s) != hipSuccess)
            return ncclUnhandledCudaError;
    if (hipEventCreateWithFlags(&done, hipEventDisableTiming) != hipSuccess || hipEventRecord(done, s) != hipSuccess)
        return ncclUnhandledCudaError;
    w.done[r] = done;
    if (!w.barrier(lk)) return ncclSystemError;
    for (int q = 0; q < w.n; ++q)  // no rank reuses its send buffer before every copy of it ran
        if (hipStreamWaitEvent(s, w.done[q], 0) != hipSuccess) return ncclUnhandledCudaError;
    if (!w.barrier(lk)) return ncclSystemError;
    (void)hipEventDestroy(ready);
    (void)hipEventDestroy(done);
    return ncclSuccess;
}

ncclResult_t ncclAllReduce(const void *send, void *recv, size_t count, ncclDataType_t t, ncclRedOp_t op,
                           ncclComm_t comm, hipStream_t s) {
    const size_t es = type_size(t);
    if (!comm || !count || (es != 4 && es != 8) || t == ncclFloat32 ||
        (op != ncclSum && op != ncclMax && op != ncclMin))
        return ncclInvalidArgument;
    if (fail_now(comm->rank)) return ncclSystemError;
    if (comm->x) {
        return xcollective(comm, send, count * es, s, [&]() -> ncclResult_t {
            const size_t words = (count * es + 7) / 8;
            std::vector<uint64_t> acc(words), x(words);
            std::memcpy(acc.data(), comm->x->slot[0], count * es);
            for (int q = 1; q < comm->n; ++q) {
                std::memcpy(x.data(), comm->x->slot[q], count * es);
                switch (t) {
                    case ncclInt32: reduce_into<int32_t>(acc, x, count, op); break;
                    case ncclUint32: reduce_into<uint32_t>(acc, x, count, op); break;
                    case ncclInt64: reduce_into<int64_t>(acc, x, count, op); break;
                    case ncclUint64: reduce_into<uint64_t>(acc, x, count, op); break;
                    default: reduce_into<double>(acc, x, count, op); break;
                }
            }
            if (hipMemcpyAsync(recv, acc.data(), count * es, hipMemcpyHostToDevice, s) != hipSuccess ||
                hipStreamSynchronize(s) != hipSuccess)
                return ncclUnhandledCudaError;
            return ncclSuccess;
        });
    }
    World &w = *comm->w;
    const int r = comm->rank;
    std::vector<uint64_t> mine((count * es + 7) / 8);
    if (hipMemcpyAsync(mine.data(), send, count * es, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return ncclUnhandledCudaError;
    std::unique_lock<std::mutex> lk(w.mu);
    w.slots[r].host = mine;
    if (!w.barrier(lk)) return ncclSystemError;
    std::vector<uint64_t> acc = w.slots[0].host;
    for (int q = 1; q < w.n; ++q) {
        switch (t) {
            case ncclInt32: reduce_into<int32_t>(acc, w.slots[q].host, count, op); break;
            case ncclUint32: reduce_into<uint32_t>(acc, w.slots[q].host, count, op); break;
            case ncclInt64: reduce_into<int64_t>(acc, w.slots[q].host, count, op); break;
            case ncclUint64: reduce_into<uint64_t>(acc, w.slots[q].host, count, op); break;
            default: reduce_into<double>(acc, w.slots[q].host, count, op); break;
        }
    }
    if (!w.barrier(lk)) return ncclSystemError;
    lk.unlock();
    if (hipMemcpyAsync(recv, acc.data(), count * es, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return ncclUnhandledCudaError;
    return ncclSuccess;
}

}  // extern "C"
