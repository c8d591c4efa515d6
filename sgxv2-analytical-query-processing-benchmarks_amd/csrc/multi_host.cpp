// Multi-GPU RHO join (sgxamd/multi.h): radix-shard exchange over RCCL (xGMI), or over
// device-to-device copies between logical ranks of one GPU (the rehearsal transport).
//
// The reference splits R and S into per-thread slices (radix_join.cpp:1457-1500) that
// all partition into shared tmpR/tmpS arrays (:1421-1433, parallel_radix_partition
// :851-931) before the join threads pop partition pairs (:1319-1334).  Here a rank (a
// GPU) owns a slice; the low log2(G) key bits name the rank that joins a tuple, so one
// exchange step replaces the shared arrays:
//
//   compute stream:  shard R0 | R1 | R2 | R3 | S0 | S1 | S2 | S3 | ...R' local passes | S' passes, build/probe
//   comm stream:          | R0 exchange ... R3 | S0 exchange ... S3 |
//
// Every piece's counts are exchanged (an all-gather of the G per-destination counts)
// and its tuples posted on the communication stream as soon as the piece is
// partitioned; R's local passes (join_pipelined_begin, key_shift = log2 G) start when
// R's last piece has landed, S's passes and the build/probe when S's has.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <unordered_map>
#include <vector>

#include "common.hpp"
#include "rho_device.hpp"
#include "runtime.hpp"
#include "sgxamd/multi.h"

namespace sgxamd {
namespace multi {
namespace {

using Clock = std::chrono::steady_clock;
double ms_since(Clock::time_point t) { return std::chrono::duration<double, std::milli>(Clock::now() - t).count(); }

#define MH_HIP(call)                                                                       \
    do {                                                                                   \
        hipError_t _e = (call);                                                            \
        if (_e != hipSuccess) {                                                            \
            set_last_error(std::string(#call) + ": " + hipGetErrorString(_e));             \
            return (_e == hipErrorOutOfMemory) ? MI355_ERR_OOM : MI355_ERR_HIP;            \
        }                                                                                  \
    } while (0)

// A HIP call inside a transport: the transport is broken, not just this rank's compute
// (the rank leaves the collective sequence; its peers are released by abort()).
#define MH_HIPC(call)                                                                      \
    do {                                                                                   \
        hipError_t _e = (call);                                                            \
        if (_e != hipSuccess) {                                                            \
            set_last_error(std::string(#call) + ": " + hipGetErrorString(_e));             \
            return MI355_ERR_COMM;                                                         \
        }                                                                                  \
    } while (0)

#define MH_RC(call)                  \
    do {                             \
        const int _rc = (call);      \
        if (_rc != MI355_OK) return _rc; \
    } while (0)

// ---------------------------------------------------------------- RCCL, loaded on first use
// libsgxamd.so keeps no link-time dependency on RCCL: the single-GPU library loads on
// hosts without it, and a process that already holds librccl.so.1 (PyTorch's) shares it.
// mi355_multi_set_rccl_library names another library with the same entry points (the
// in-tree test double of tests/rccl_double, which moves data between ranks of one
// process with device copies, so that RcclTransport runs at G > 1 on one GPU).
struct Rccl {
    decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
    decltype(&ncclCommInitRank) CommInitRank = nullptr;
    decltype(&ncclCommInitAll) CommInitAll = nullptr;
    decltype(&ncclCommDestroy) CommDestroy = nullptr;
    decltype(&ncclCommAbort) CommAbort = nullptr;
    decltype(&ncclCommSplit) CommSplit = nullptr;
    decltype(&ncclGroupStart) GroupStart = nullptr;
    decltype(&ncclGroupEnd) GroupEnd = nullptr;
    decltype(&ncclSend) Send = nullptr;
    decltype(&ncclRecv) Recv = nullptr;
    decltype(&ncclAllGather) AllGather = nullptr;
    decltype(&ncclAllReduce) AllReduce = nullptr;
    decltype(&ncclGetErrorString) ErrorString = nullptr;
    std::string error;
    std::string name;      // the library loaded
    bool double_ = false;  // a test double (mi355_multi_set_rccl_library): ranks may share a GPU
    // ncclCommAbort where the library has it, else ncclCommDestroy
    void abort_comm(ncclComm_t c) const {
        if (!c) return;
        if (CommAbort) (void)CommAbort(c);
        else if (CommDestroy) (void)CommDestroy(c);
    }
};

Rccl load_rccl(const std::string &path) {
    Rccl r;
    r.name = path.empty() ? "librccl.so.1" : path;
    r.double_ = !path.empty();
    void *h = dlopen(r.name.c_str(), RTLD_NOW | RTLD_LOCAL);
    if (!h && path.empty()) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
        const char *e = dlerror();
        r.error = "cannot load " + r.name + ": " + (e ? e : "?");
        return r;
    }
    auto sym = [&](auto &fn, const char *name, bool required) {
        fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
        if (!fn && required && r.error.empty()) r.error = r.name + " lacks " + name;
    };
    sym(r.GetUniqueId, "ncclGetUniqueId", true);
    sym(r.CommInitRank, "ncclCommInitRank", true);
    sym(r.CommInitAll, "ncclCommInitAll", true);
    sym(r.CommDestroy, "ncclCommDestroy", true);
    // optional: ncclCommSplit is needed only by the one-process-per-GPU communicator
    // (mi355_multi_comm_init checks it); without ncclCommAbort a broken communicator is
    // destroyed instead
    sym(r.CommAbort, "ncclCommAbort", false);
    sym(r.CommSplit, "ncclCommSplit", false);
    sym(r.GroupStart, "ncclGroupStart", true);
    sym(r.GroupEnd, "ncclGroupEnd", true);
    sym(r.Send, "ncclSend", true);
    sym(r.Recv, "ncclRecv", true);
    sym(r.AllGather, "ncclAllGather", true);
    sym(r.AllReduce, "ncclAllReduce", true);
    sym(r.ErrorString, "ncclGetErrorString", true);
    return r;
}

// The current function table.  Tables are never freed (a library is never unloaded), so
// a reference stays valid after mi355_multi_set_rccl_library switched libraries; the
// switch is refused while communicators exist.
std::mutex g_rccl_mu;
std::string g_rccl_path;                    // "" = the system librccl.so.1
const Rccl *g_rccl = nullptr;
std::vector<std::unique_ptr<Rccl>> g_rccl_tables;
std::atomic<int> g_live_handles{0};         // communicators of mi355_multi_comm_init alive

const Rccl &rccl() {
    std::lock_guard<std::mutex> lk(g_rccl_mu);
    if (!g_rccl) {
        g_rccl_tables.push_back(std::make_unique<Rccl>(load_rccl(g_rccl_path)));
        g_rccl = g_rccl_tables.back().get();
    }
    return *g_rccl;
}

#define MH_NCCL(call)                                                                              \
    do {                                                                                           \
        ncclResult_t _r = (call);                                                                  \
        if (_r != ncclSuccess) {                                                                   \
            set_last_error(std::string(#call) + ": " + ::sgxamd::multi::rccl().ErrorString(_r));     \
            return MI355_ERR_COMM;                                                                 \
        }                                                                                          \
    } while (0)

int require_rccl() {
    if (!rccl().error.empty()) {
        set_last_error(rccl().error);
        return MI355_ERR_COMM;
    }
    return MI355_OK;
}

// ---------------------------------------------------------------- host barrier
// The rank threads of one process meet here (the reference's Barrier.hpp:6-42 between
// its phases); abort() releases every waiter when a rank fails.
class Barrier {
   public:
    explicit Barrier(int n) : n_(n) {}
    bool wait() {
        std::unique_lock<std::mutex> lk(m_);
        if (aborted_) return false;
        const uint64_t gen = gen_;
        if (++waiting_ == n_) {
            waiting_ = 0;
            ++gen_;
            cv_.notify_all();
            return true;
        }
        cv_.wait(lk, [&] { return gen_ != gen || aborted_; });
        return gen_ != gen;
    }
    void abort() {
        std::lock_guard<std::mutex> lk(m_);
        aborted_ = true;
        cv_.notify_all();
    }
    bool aborted() {
        std::lock_guard<std::mutex> lk(m_);
        return aborted_;
    }

   private:
    std::mutex m_;
    std::condition_variable cv_;
    int n_, waiting_ = 0;
    uint64_t gen_ = 0;
    bool aborted_ = false;
};

// ---------------------------------------------------------------- transports
enum ReduceOp { kSum, kMax };
constexpr int kMaxReduce = 4;  // values per all-reduce

// Every collective a rank issues is reached by every rank, failed or not: a rank that
// failed (an allocation, a kernel) says so in the next collective instead of leaving
// it, so all ranks see the failure at the same step and return together (no peer is
// left waiting in a collective the failed rank never posts).
class Transport {
   public:
    virtual ~Transport() = default;
    virtual int world() const = 0;
    virtual int kind() const = 0;
    // collective: send[j * G + d] = tuples this rank sends to rank d in piece j (j < m),
    // fail = this rank has failed; recv[j * G + q] = tuples rank q sends to this rank in
    // piece j, *any_fail = some rank has failed (then nothing is posted, by any rank)
    virtual int exchange_counts(int rank, hipStream_t s, const uint64_t *send, int m, bool fail, uint64_t *recv,
                                bool *any_fail) = 0;
    // collective: after `ready` (the piece's partition on the compute stream), move the
    // piece: the run for destination d starts at send + sum_{d'<d} send_counts[d'];
    // rank q's run lands at recv + sum_{q'<q} recv_counts[q'].  Enqueued on c.
    // elem: bytes per element (8: row_t tuples or counts rows; 4: keys of a keys-only
    // exchange; 2: residuals of the u16 wire).
    virtual int post_exchange(int rank, hipStream_t c, hipEvent_t ready, const void *send,
                              const uint64_t *send_counts, void *recv, const uint64_t *recv_counts, size_t elem) = 0;
    // collective: v[0..n) = element-wise sum / max over the ranks (n <= kMaxReduce)
    virtual int allreduce(int rank, hipStream_t s, uint64_t *v, int n, ReduceOp op) = 0;
    // a rank left the collective sequence (a transport call or a HIP call around one
    // failed): release the host-side waiters; communicators are torn down by the owner
    // afterwards
    virtual void abort() {}
    // abort() was called: a collective that failed now failed because of another rank
    virtual bool aborted() { return false; }
};

std::vector<uint64_t> prefix(const uint64_t *c, int n) {
    std::vector<uint64_t> p(n + 1, 0);
    for (int i = 0; i < n; ++i) p[i + 1] = p[i] + c[i];
    return p;
}

// Counts, flags and reductions of the ranks of ONE process (threads): shared host
// tables between barriers.  No device round trip, and nothing queued behind the tuple
// traffic of a communicator.
class HostCollectives {
   public:
    explicit HostCollectives(int world)
        : world_(world), bar_(world), counts_(world, std::vector<uint64_t>(world + 1)), red_(world) {}
    int world() const { return world_; }
    bool wait() { return bar_.wait(); }
    void abort() { bar_.abort(); }
    bool aborted() { return bar_.aborted(); }

    int exchange_counts(int rank, const uint64_t *send, int m, bool fail, uint64_t *recv, bool *any_fail) {
        const size_t w = (size_t)m * world_;  // the fail flag follows the m rows
        std::vector<uint64_t> &mine = counts_[rank];
        if (mine.size() < w + 1) mine.resize(w + 1);
        std::copy(send, send + w, mine.begin());
        mine[w] = fail ? 1 : 0;
        if (!bar_.wait()) return aborted_rc();
        bool f = false;
        for (int q = 0; q < world_; ++q) {
            for (int j = 0; j < m; ++j) recv[(size_t)j * world_ + q] = counts_[q][(size_t)j * world_ + rank];
            f = f || counts_[q][w];
        }
        *any_fail = f;
        if (!bar_.wait()) return aborted_rc();  // the table is reused by the next piece
        return MI355_OK;
    }

    int allreduce(int rank, uint64_t *v, int n, ReduceOp op) {
        std::copy(v, v + n, red_[rank].begin());
        if (!bar_.wait()) return aborted_rc();
        for (int j = 0; j < n; ++j) {
            uint64_t r = op == kSum ? 0 : red_[0][j];
            for (int q = 0; q < world_; ++q) r = op == kSum ? r + red_[q][j] : std::max(r, red_[q][j]);
            v[j] = r;
        }
        if (!bar_.wait()) return aborted_rc();
        return MI355_OK;
    }

   private:
    int aborted_rc() {
        set_last_error("another rank's transport failed");
        return MI355_ERR_COMM;
    }
    int world_;
    Barrier bar_;
    std::vector<std::vector<uint64_t>> counts_;  // [rank][m rows of G counts + fail flag]
    std::vector<std::array<uint64_t, kMaxReduce>> red_;
};

// RCCL over xGMI.  Tuples (keys) go through `comms` with grouped send/recv on each
// rank's communication stream.  Counts, flags and reductions never share a
// communicator with the tuples: RCCL orders every operation of one communicator, so a
// piece's count all-gather on the tuple communicator would wait for the previous
// piece's transfer (and the host, which needs the counts to post the next piece, with
// it).  They go through a host table between the threads of one process
// (ncclCommInitAll mode), or through a second communicator per rank (ncclCommSplit of
// the tuple communicator, one process per GPU).
class RcclTransport final : public Transport {
   public:
    RcclTransport(int world, int first_rank, std::vector<ncclComm_t> comms, std::vector<ncclComm_t> ccomms,
                  std::shared_ptr<HostCollectives> host)
        : world_(world), first_(first_rank), comms_(std::move(comms)), ccomms_(std::move(ccomms)),
          host_(std::move(host)), buf_(comms_.size()), pinned_(comms_.size(), nullptr),
          pinned_bytes_(comms_.size(), 0) {}
    ~RcclTransport() override {
        for (auto &b : buf_) b.release();
        for (auto *h : pinned_)
            if (h) (void)hipHostFree(h);
    }
    int world() const override { return world_; }
    int kind() const override { return MI355_TRANSPORT_RCCL; }

    int exchange_counts(int rank, hipStream_t s, const uint64_t *send, int m, bool fail, uint64_t *recv,
                        bool *any_fail) override {
        if (host_) return host_->exchange_counts(rank, send, m, fail, recv, any_fail);
        const int i = rank - first_;
        const size_t w = (size_t)m * world_, w1 = w + 1;  // m rows of G counts + the fail flag
        uint64_t *d = nullptr, *h = nullptr;
        MH_RC(scratch(i, w1 * (world_ + 1), &d, &h));
        std::memcpy(h, send, sizeof(uint64_t) * w);
        h[w] = fail ? 1 : 0;
        MH_HIPC(hipMemcpyAsync(d, h, sizeof(uint64_t) * w1, hipMemcpyHostToDevice, s));
        MH_NCCL(rccl().AllGather(d, d + w1, w1, ncclUint64, ccomms_[i], s));
        MH_HIPC(hipMemcpyAsync(h + w1, d + w1, sizeof(uint64_t) * w1 * world_, hipMemcpyDeviceToHost, s));
        MH_HIPC(hipStreamSynchronize(s));
        bool f = false;
        for (int q = 0; q < world_; ++q) {
            const uint64_t *row = h + w1 + (size_t)q * w1;
            for (int j = 0; j < m; ++j) recv[(size_t)j * world_ + q] = row[(size_t)j * world_ + rank];
            f = f || row[w];
        }
        *any_fail = f;
        return MI355_OK;
    }

    int post_exchange(int rank, hipStream_t c, hipEvent_t ready, const void *send_v, const uint64_t *send_counts,
                      void *recv_v, const uint64_t *recv_counts, size_t elem) override {
        const int i = rank - first_;
        const auto so = prefix(send_counts, world_), ro = prefix(recv_counts, world_);
        const char *send = static_cast<const char *>(send_v);
        char *recv = static_cast<char *>(recv_v);
        // (2-byte residuals of the u16 wire travel as bytes)
        const ncclDataType_t type = elem == 8 ? ncclUint64 : elem == 4 ? ncclUint32 : ncclUint8;
        const size_t per = elem == 8 || elem == 4 ? 1 : elem;
        MH_HIPC(hipStreamWaitEvent(c, ready, 0));
        if (send_counts[rank])  // this rank's own run: a local copy
            MH_HIPC(hipMemcpyAsync(recv + ro[rank] * elem, send + so[rank] * elem, send_counts[rank] * elem,
                                  hipMemcpyDeviceToDevice, c));
        const Rccl &L = rccl();
        MH_NCCL(L.GroupStart());
        ncclResult_t r = ncclSuccess;
        const char *what = "";
        for (int p = 0; p < world_ && r == ncclSuccess; ++p) {
            if (p == rank) continue;
            if (send_counts[p] &&
                (r = L.Send(send + so[p] * elem, send_counts[p] * per, type, p, comms_[i], c)) != ncclSuccess)
                what = "ncclSend";
            else if (recv_counts[p] &&
                     (r = L.Recv(recv + ro[p] * elem, recv_counts[p] * per, type, p, comms_[i], c)) != ncclSuccess)
                what = "ncclRecv";
        }
        // the group is closed even after a failed call (the thread's group state stays
        // balanced); the communicators are aborted by the caller then
        const ncclResult_t re = L.GroupEnd();
        if (r == ncclSuccess && re != ncclSuccess) {
            r = re;
            what = "ncclGroupEnd";
        }
        if (r != ncclSuccess) {
            set_last_error(std::string(what) + " (piece exchange): " + L.ErrorString(r));
            return MI355_ERR_COMM;
        }
        return MI355_OK;
    }

    int allreduce(int rank, hipStream_t s, uint64_t *v, int n, ReduceOp op) override {
        if (host_) return host_->allreduce(rank, v, n, op);
        const int i = rank - first_;
        uint64_t *d = nullptr, *h = nullptr;
        MH_RC(scratch(i, kMaxReduce, &d, &h));
        std::memcpy(h, v, sizeof(uint64_t) * n);
        MH_HIPC(hipMemcpyAsync(d, h, sizeof(uint64_t) * n, hipMemcpyHostToDevice, s));
        MH_NCCL(rccl().AllReduce(d, d, n, ncclUint64, op == kSum ? ncclSum : ncclMax, ccomms_[i], s));
        MH_HIPC(hipMemcpyAsync(h, d, sizeof(uint64_t) * n, hipMemcpyDeviceToHost, s));
        MH_HIPC(hipStreamSynchronize(s));
        std::memcpy(v, h, sizeof(uint64_t) * n);
        return MI355_OK;
    }

    void abort() override {
        aborted_ = true;
        if (host_) host_->abort();
    }
    bool aborted() override { return aborted_ || (host_ && host_->aborted()); }

   private:
    // per local rank: at least `words` u64 of device memory and a pinned host mirror
    // (a count exchange: (G + 1) rows of m * G + 1 words)
    int scratch(int i, size_t words, uint64_t **d, uint64_t **h) {
        const size_t bytes = sizeof(uint64_t) * std::max<size_t>(words, kMaxReduce);
        MH_HIPC(buf_[i].ensure(bytes));
        if (pinned_bytes_[i] < bytes) {
            if (pinned_[i]) (void)hipHostFree(pinned_[i]);
            pinned_[i] = nullptr;
            pinned_bytes_[i] = 0;
            MH_HIPC(hipHostMalloc(reinterpret_cast<void **>(&pinned_[i]), bytes));
            pinned_bytes_[i] = bytes;
        }
        *d = buf_[i].as<uint64_t>();
        *h = pinned_[i];
        return MI355_OK;
    }
    int world_, first_;
    std::atomic<bool> aborted_{false};
    std::vector<ncclComm_t> comms_, ccomms_;
    std::shared_ptr<HostCollectives> host_;
    std::vector<DeviceBuffer> buf_;
    std::vector<uint64_t *> pinned_;
    std::vector<size_t> pinned_bytes_;
};

// G logical ranks on one GPU, one host thread each: counts and reductions through the
// host tables, tuples by device-to-device copies that the receiver enqueues on its
// communication stream after the sender's partition event.  Same collective sequence
// and receive layout as the RCCL transport.
class RehearsalTransport final : public Transport {
   public:
    explicit RehearsalTransport(int world) : host_(world), posts_(world) {}
    int world() const override { return host_.world(); }
    int kind() const override { return MI355_TRANSPORT_REHEARSAL; }

    int exchange_counts(int rank, hipStream_t, const uint64_t *send, int m, bool fail, uint64_t *recv,
                        bool *any_fail) override {
        return host_.exchange_counts(rank, send, m, fail, recv, any_fail);
    }

    int post_exchange(int rank, hipStream_t c, hipEvent_t ready, const void *send, const uint64_t *send_counts,
                      void *recv_v, const uint64_t *recv_counts, size_t elem) override {
        const int G = host_.world();
        char *recv = static_cast<char *>(recv_v);
        posts_[rank] = Post{static_cast<const char *>(send), prefix(send_counts, G), ready};
        if (!host_.wait()) return aborted_rc();
        uint64_t off = 0;
        int rc = MI355_OK;
        for (int q = 0; q < G && rc == MI355_OK; ++q) {
            if (!recv_counts[q]) continue;
            const Post &p = posts_[q];
            if (hipStreamWaitEvent(c, p.ready, 0) != hipSuccess ||
                hipMemcpyAsync(recv + off * elem, p.send + p.off[rank] * elem, recv_counts[q] * elem,
                               hipMemcpyDeviceToDevice, c) != hipSuccess) {
                set_last_error("rehearsal exchange copy failed");
                rc = MI355_ERR_COMM;
            }
            off += recv_counts[q];
        }
        if (!host_.wait()) return aborted_rc();  // the posts table is reused by the next piece
        return rc;
    }

    int allreduce(int rank, hipStream_t, uint64_t *v, int n, ReduceOp op) override {
        return host_.allreduce(rank, v, n, op);
    }

    void abort() override { host_.abort(); }
    bool aborted() override { return host_.aborted(); }

   private:
    int aborted_rc() {
        set_last_error("another rank's transport failed");
        return MI355_ERR_COMM;
    }
    struct Post {
        const char *send = nullptr;
        std::vector<uint64_t> off;
        hipEvent_t ready = nullptr;
    };
    HostCollectives host_;
    std::vector<Post> posts_;
};

// ---------------------------------------------------------------- one rank's join
std::atomic<int> g_pieces{4};

// Tests (SGXAMD_DEBUG_EXCHANGE_DELAY_US, read once): the communication stream waits this
// long before every piece, so that a local pass that does not wait for its piece's event
// reads a receive buffer that has not landed (test_multi_gpu.py::test_late_pieces).
uint32_t exchange_delay_us() {
    static const uint32_t us = [] {
        const char *e = std::getenv("SGXAMD_DEBUG_EXCHANGE_DELAY_US");
        const long v = e ? std::atol(e) : 0;
        return (uint32_t)(v > 0 && v < 1000000 ? v : 0);
    }();
    return us;
}

// Communication stream and piece events of a context (created on first use).
struct RankStreams {
    hipStream_t comm = nullptr;
    std::vector<hipEvent_t> ev;
    hipEvent_t t_land = nullptr, t_done = nullptr;  // timed: S landed, local join done
};
std::mutex g_streams_mu;
std::unordered_map<const Context *, RankStreams> g_streams;

int rank_streams(Context *ctx, int nev, RankStreams **out) {
    std::lock_guard<std::mutex> lk(g_streams_mu);
    RankStreams &rs = g_streams[ctx];
    if (!rs.comm) MH_HIP(hipStreamCreateWithFlags(&rs.comm, hipStreamNonBlocking));
    if (!rs.t_land) MH_HIP(hipEventCreate(&rs.t_land));
    if (!rs.t_done) MH_HIP(hipEventCreate(&rs.t_done));
    while ((int)rs.ev.size() < nev) {
        hipEvent_t e = nullptr;
        MH_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        rs.ev.push_back(e);
    }
    *out = &rs;
    return MI355_OK;
}

struct RankOut {
    uint64_t global = 0, local = 0, recv_r = 0, recv_s = 0, sent = 0;
    bool keys = false;       // the exchange moved keys only
    bool wire16 = false;     // S's keys as 2-byte residuals of sender-side partitions (the u16 wire)
    bool peer_fail = false;  // the call failed because another rank did
    bool together = false;   // the call failed at a collective every rank left at (the
                             // sequence is intact; nothing to abort)
    double ms_post = 0, ms_local = 0, ms_allreduce = 0, ms_total = 0;
    double ms_tail = -1;  // device time from S's last piece landing to the local join's end
    mi355_rho_stats st{};
    Context *ctx = nullptr;  // materialising joins: the rank's triples are in ctx->mat (local of them)
};

uint32_t log2_exact(int g) {
    uint32_t b = 0;
    while ((1 << b) < g) ++b;
    return b;
}

// Test hook (mi355_multi_inject_failure): rank `g_fail_rank` fails at step
// `g_fail_step` of its next multi-GPU join, as an allocation or kernel error would.
std::atomic<int> g_fail_rank{-1}, g_fail_step{0};
enum FailStep { kFailBuffers = 1, kFailPiece = 2, kFailLocal = 3, kFailContext = 4, kFailLocalSync = 5 };
bool injected(int rank, int step) {
    if (g_fail_rank.load() != rank || g_fail_step.load() != step) return false;
    set_last_error("injected failure (mi355_multi_inject_failure)");
    return true;
}

// The pipeline of the file comment for rank `rank` on its context (device current,
// ctx->mu held).  R / S: this rank's device-resident slices.
//
// Collectives, identical on every rank whatever fails: two all-reduces (sizes, element
// format), then per piece a count exchange and its post, then one final all-reduce
// (matches, failures).  A rank whose buffers, shard pass or local join fail keeps
// issuing them with its fail flag set; the first count exchange or the final
// all-reduce that carries a flag ends the call on every rank with an error.  Only a
// failing transport call itself (MI355_ERR_COMM) leaves the sequence.
//
// pre_fail != MI355_OK: the rank failed before its join (no context, staging); it
// takes part in the collectives with its flag set (ctx may be null then).
int rank_join(Transport &T, int rank, Context *ctx, hipStream_t s, const row_t *R, uint64_t nR, const row_t *S,
              uint64_t nS, const mi355_rho_opts *opts, RankOut &o, int pre_fail = MI355_OK) {
    const auto t0 = Clock::now();
    const int G = T.world();
    const uint32_t dest_bits = log2_exact(G);
    const int K = std::max(1, std::min(64, g_pieces.load()));
    mi355_rho_opts lo{};
    if (opts) lo = *opts;
    lo.key_shift = dest_bits;
    // materialising joins (MATERIALIZE, radix_join.cpp:437-446): whole tuples travel (the
    // payloads; keys_exchange_plan refuses keys), and each rank's triples stay in its
    // context's growable buffer (ctx->mat), its output chunk (the reference's per-thread
    // chunks of a ChunkedTable, ChunkedTable.cpp:98-171); the caller copies them out
    lo.materialize = opts && opts->materialize ? 1 : 0;
    lo.stream = nullptr;
    lo.out = nullptr;
    lo.out_capacity = 0;
    o.ctx = ctx;
    DeviceBuffer *mat = lo.materialize && ctx ? &ctx->mat : nullptr;
    if (G == 1) {  // nothing to exchange: no collective to leave, so a failure is local
        o.together = true;
        if (pre_fail != MI355_OK) return pre_fail;
        if (injected(rank, kFailLocal)) return MI355_ERR_OOM;
        if (nR && nS) {
            MH_RC(rho::join_pipelined_begin(ctx, s, R, nR, nS, &lo));
            MH_RC(rho::join_pipelined_finish(ctx, S, nS, &o.st, nullptr, mat));
        }
        o.global = o.local = o.st.matches;
        o.recv_r = nR;
        o.recv_s = nS;
        o.ms_local = o.ms_total = ms_since(t0);
        return MI355_OK;
    }
    RankStreams *rs = nullptr;
    // this rank's first error, kept until the next collective reports it
    int fail_rc = pre_fail != MI355_OK ? pre_fail : rank_streams(ctx, 3 * K + 2, &rs);
    std::string fail_msg = fail_rc ? last_error() : "";
    auto fail = [&](int rc) {
        if (rc != MI355_OK && fail_rc == MI355_OK) {
            fail_rc = rc;
            fail_msg = last_error();
        }
    };
    // a HIP call of this rank's own compute or ordering: a failure is flagged at the next
    // collective like any other local failure (the rank stays in the sequence)
    auto hip_ok = [&](hipError_t e, const char *what) {
        if (e == hipSuccess) return true;
        set_last_error(std::string(what) + ": " + hipGetErrorString(e));
        fail(e == hipErrorOutOfMemory ? MI355_ERR_OOM : MI355_ERR_HIP);
        return false;
    };
    // a transport call failed: when the transport was aborted by another rank that left
    // the sequence, this rank failed because of it
    auto transport_rc = [&](int rc) {
        if (rc != MI355_OK && T.aborted()) o.peer_fail = true;
        return rc;
    };
    auto peer_failed = [&]() {
        o.together = true;
        if (fail_rc != MI355_OK) {
            set_last_error(fail_msg);
            return fail_rc;
        }
        o.peer_fail = true;
        set_last_error("another rank failed; every rank left the multi-GPU join at the same step");
        return MI355_ERR_COMM;
    };

    // global sizes: the mean local sizes plan the local join, the largest slices size
    // the receive buffers for the worst case (every rank's piece i comes to this rank)
    uint64_t sum[2] = {nR, nS}, mx[2] = {nR, nS};
    MH_RC(transport_rc(T.allreduce(rank, s, sum, 2, kSum)));
    MH_RC(transport_rc(T.allreduce(rank, s, mx, 2, kMax)));
    const uint64_t cR = (uint64_t)G * K * ((mx[0] + K - 1) / K), cS = (uint64_t)G * K * ((mx[1] + K - 1) / K);
    // the element format must be the same on every rank (the SGXAMD_KEYS switch and the
    // calling thread's key layout are per process / per thread): keys only when every
    // rank's plan, from the same global sizes, takes the pooled keys layout
    // and the u16 wire (keys plans whose every residual fits 16 bits): agreed the same way
    mi355_rho_opts kl = lo;
    uint64_t agree[2] = {rho::keys_exchange_plan(sum[0] / G, sum[1] / G, cR, cS, &kl) ? 0u : 1u, 1u};
    bool need_kmax = false;
    if (agree[0] == 0 && rho::wire16_plan(sum[0] / G, sum[1] / G, G, &kl, &need_kmax)) agree[1] = 0;
    MH_RC(transport_rc(T.allreduce(rank, s, agree, 2, kMax)));
    o.keys = agree[0] == 0;
    o.wire16 = o.keys && agree[1] == 0;
    if (o.keys) lo = kl;  // the local policy fixed from the global sizes
    const uint32_t P16 = o.wire16 ? rho::wire16_plan(sum[0] / G, sum[1] / G, G, &lo, &need_kmax) : 0;
    const size_t elem = o.keys ? sizeof(uint32_t) : sizeof(row_t);
    // u16 wire buffers (S): [residuals (256-B aligned)][G counts rows of P16 + 1 words];
    // the receive side also holds the gather's scratch (rho::wire_scratch_u64)
    // (every sender's run in a slot of rho::wire_slot residuals: its partitions padded to 8)
    const uint64_t slack = (uint64_t)G * (8ull * P16 + 16);  // (rho::wire_slot's padding, per run)
    const auto res_bytes = [slack](uint64_t n) { return ((std::max<uint64_t>(n, 1) + slack) * 2 + 255) & ~uint64_t(255); };
    // (the send side: 4 bytes per key, rho::wire_partition writes a wide destination as keys
    // -- at most 2 n u16 slots past the last destination's start)
    const auto snd_bytes = [slack](uint64_t n) {
        return (std::max<uint64_t>(n, 1) * 4 + slack * 2 + 255) & ~uint64_t(255);
    };
    const uint64_t RW = rho::wire_row_words(P16);
    const uint64_t rows = (uint64_t)G * RW * sizeof(uint64_t);
    if (fail_rc == MI355_OK) {
        hipError_t e = ctx->xsendR.ensure(std::max<uint64_t>(nR, 1) * elem);
        if (e == hipSuccess) e = ctx->xsendS.ensure(std::max<uint64_t>(nS, 1) * elem);
        if (e == hipSuccess) e = ctx->xrecvR.ensure(std::max<uint64_t>(cR, 1) * elem);
        if (!o.wire16) {
            if (e == hipSuccess) e = ctx->xrecvS.ensure(std::max<uint64_t>(cS, 1) * elem);
        } else {
            if (e == hipSuccess) e = ctx->wsendS.ensure(snd_bytes(nS) + rows);
            if (e == hipSuccess && need_kmax) e = ctx->xrecvS.ensure(std::max<uint64_t>(cS, 1) * elem);  // fallback
            if (e == hipSuccess)
                e = ctx->wrecvS.ensure(res_bytes(cS) + rows + rho::wire_scratch_u64(G, P16) * sizeof(uint64_t));
        }
        if (e != hipSuccess) {
            set_last_error(std::string("exchange buffers (") + std::to_string((2 * (nR + nS) + cR + cS) * elem) +
                           " bytes): " + hipGetErrorString(e));
            fail(e == hipErrorOutOfMemory ? MI355_ERR_OOM : MI355_ERR_HIP);
        }
        if (injected(rank, kFailBuffers)) fail(MI355_ERR_OOM);
    }

    // every piece's destination counts first (both relations), then ONE count exchange,
    // then every piece's scatter and post enqueued without a host wait: piece i+1's
    // scatter runs while piece i moves on the communication stream
    const int M = 2 * K;
    std::vector<uint64_t> sc((size_t)M * G, 0), rc((size_t)M * G, 0);
    std::array<uint64_t, 2> nrel{nR, nS};
    std::vector<uint64_t> pa(M), pn(M);  // piece j = rel * K + i: first tuple, tuples
    std::vector<const row_t *> pin(M);
    for (int rel = 0; rel < 2; ++rel) {
        const uint64_t n = nrel[rel], per = (n + K - 1) / K;
        for (int i = 0; i < K; ++i) {
            const int j = rel * K + i;
            pa[j] = std::min(n, i * per);
            pn[j] = std::min(n, (i + 1) * per) - pa[j];
            pin[j] = (rel ? S : R) + pa[j];
        }
    }
    if (fail_rc == MI355_OK) {
        fail(rho::shard_count_pieces(ctx, s, pin.data(), pn.data(), M, 0, dest_bits, (uint32_t)elem, sc.data()));
        if (injected(rank, kFailPiece)) fail(MI355_ERR_HIP);
    }
    if (fail_rc != MI355_OK) std::fill(sc.begin(), sc.end(), 0);
    bool any_fail = false;
    MH_RC(transport_rc(T.exchange_counts(rank, s, sc.data(), M, fail_rc != MI355_OK, rc.data(), &any_fail)));
    if (any_fail) return peer_failed();  // every rank sees the same flags: none posts anything
    // the counts went out unflagged, so every piece is posted whatever happens now; a
    // failure from here on is flagged at the final all-reduce
    uint64_t total[2] = {0, 0};
    std::vector<uint64_t> s_piece(K, 0);  // S tuples landing per piece (S's local pass 1 runs per piece)
    std::vector<uint64_t> wbase, wcount, wspan;  // u16 wire: sender q's run of S residuals: start, keys, slot
    // (u16 wire: R's pieces only; S follows below)
    bool s_scattered = false;
    const auto post_pieces = [&](int j0, int j1) -> int {
        for (int j = j0; j < j1; ++j) {
            const int rel = j / K;
            char *snd = (rel ? ctx->xsendS : ctx->xsendR).as<char>() + pa[j] * elem;
            char *rcv = (rel ? ctx->xrecvS : ctx->xrecvR).as<char>() + total[rel] * elem;
            if (fail_rc == MI355_OK && !(rel && s_scattered)) fail(rho::shard_scatter_piece(ctx, s, j, snd));
            hipEvent_t ready = rs->ev[j];
            hip_ok(hipEventRecord(ready, s), "hipEventRecord (piece ready)");
            if (const uint32_t us = exchange_delay_us())  // tests: every piece lands late
                hip_ok(rho::launch_spin(us, rs->comm), "launch_spin (exchange delay)");
            const uint64_t *scj = sc.data() + (size_t)j * G, *rcj = rc.data() + (size_t)j * G;
            MH_RC(transport_rc(T.post_exchange(rank, rs->comm, ready, snd, scj, rcv, rcj, elem)));
            for (int q = 0; q < G; ++q) {
                total[rel] += rcj[q];
                if (rel) s_piece[j - K] += rcj[q];
                if (q != rank) o.sent += scj[q] * elem;
            }
            if (rel) hip_ok(hipEventRecord(rs->ev[2 * K + 2 + (j - K)], rs->comm), "hipEventRecord (S piece landed)");
            if ((j + 1) % K == 0)
                hip_ok(hipEventRecord(rs->ev[2 * K + rel], rs->comm), "hipEventRecord (relation landed)");
        }
        return MI355_OK;
    };
    MH_RC(post_pieces(0, o.wire16 ? K : M));
    // S on the u16 wire: its pieces' shard scatters, then the receiver's two passes over
    // the keys for each destination (its runs: one per piece), the counts rows and the
    // residuals posted -- all while R's keys are on the wire; R's local passes then run
    // while S's residuals are (DESIGN.md §5 "Residuals on the wire")
    uint16_t *snd16 = o.wire16 ? ctx->wsendS.as<uint16_t>() : nullptr;
    uint64_t *scnt = o.wire16 ? reinterpret_cast<uint64_t *>(ctx->wsendS.as<char>() + snd_bytes(nS)) : nullptr;
    uint64_t *rcnt = o.wire16 ? reinterpret_cast<uint64_t *>(ctx->wrecvS.as<char>() + res_bytes(cS)) : nullptr;
    std::vector<uint64_t> s16(G, 0), r16(G, 0);
    if (o.wire16) {
        for (int i = 0; i < K && fail_rc == MI355_OK; ++i)
            fail(rho::shard_scatter_piece(ctx, s, K + i, ctx->xsendS.as<char>() + pa[K + i] * elem));
        std::vector<uint64_t> roff((size_t)G * K), rn((size_t)G * K);
        for (int q = 0; q < G; ++q)
            for (int i = 0; i < K; ++i) {
                const int j = K + i;
                uint64_t off = pa[j];
                for (int d = 0; d < q; ++d) off += sc[(size_t)j * G + d];
                roff[(size_t)q * K + i] = off;
                rn[(size_t)q * K + i] = sc[(size_t)j * G + q];
                s16[q] += sc[(size_t)j * G + q];
                r16[q] += rc[(size_t)j * G + q];
            }
        s_scattered = true;
        if (fail_rc == MI355_OK)
            fail(rho::wire_partition(ctx, s, ctx->xsendS.as<uint32_t>(), G, K, roff.data(), rn.data(), sum[0] / G,
                                     sum[1] / G, &lo, snd16, scnt, "wireS_"));
        if (need_kmax) {
            // the plan does not guarantee 16-bit residuals (log2 G + bits < 16): S's
            // largest key over all ranks decides; otherwise S goes as keys (its shard
            // scatter is in xsendS already) and the local join takes the 4-byte plan
            std::vector<uint64_t> km(G, 0);
            if (fail_rc == MI355_OK) {
                for (int q = 0; q < G; ++q)
                    hip_ok(hipMemcpyAsync(&km[q], scnt + (size_t)q * RW + 2 * P16, sizeof(uint64_t),
                                          hipMemcpyDeviceToHost, s),
                           "hipMemcpyAsync (largest key)");
                hip_ok(hipStreamSynchronize(s), "hipStreamSynchronize (largest key)");
            }
            uint64_t kmax = fail_rc == MI355_OK ? *std::max_element(km.begin(), km.end()) : 0;
            MH_RC(transport_rc(T.allreduce(rank, s, &kmax, 1, kMax)));
            if (((kmax >> (dest_bits + (uint32_t)__builtin_ctz(P16))) >> 16) != 0) o.wire16 = false;
        }
    }
    if (!o.wire16 && s_scattered) {  // the residuals do not fit: S's pieces as keys
        MH_RC(post_pieces(K, M));
    } else if (o.wire16) {
        // a failed rank still sends (the sizes are agreed): zero counts rows, which no
        // receiver takes (they do not add up to the announced runs)
        if (fail_rc != MI355_OK && ctx->wsendS.ptr) (void)hipMemsetAsync(scnt, 0, rows, s);
        hipEvent_t ready = rs->ev[K];
        hip_ok(hipEventRecord(ready, s), "hipEventRecord (residuals ready)");
        const std::vector<uint64_t> crow(G, RW);
        MH_RC(transport_rc(
            T.post_exchange(rank, rs->comm, ready, scnt, crow.data(), rcnt, crow.data(), sizeof(uint64_t))));
        // every run in a slot of rho::wire_slot residuals on both sides: each sender's run
        // starts on 16 bytes in the send and the receive buffer, its partitions padded to 8
        // residuals (the build/probe reads them in place); the padding is never read
        std::vector<uint64_t> s16p(G), r16p(G);
        for (int q = 0; q < G; ++q) {
            s16p[q] = rho::wire_slot(s16[q], P16);
            r16p[q] = rho::wire_slot(r16[q], P16);
        }
        MH_RC(transport_rc(
            T.post_exchange(rank, rs->comm, ready, snd16, s16p.data(), ctx->wrecvS.ptr, r16p.data(), sizeof(uint16_t))));
        wbase.assign(G, 0);
        uint64_t at = 0;
        for (int q = 0; q < G; ++q) {
            wbase[q] = at;
            at += r16p[q];
            total[1] += r16[q];
            // (the residuals; the slot's padding, at most (8 P + 15) x 2 bytes per peer, is not
            // counted)
            if (q != rank) o.sent += s16[q] * sizeof(uint16_t) + crow[q] * sizeof(uint64_t);
        }
        wcount = r16;
        wspan = r16p;
        hip_ok(hipEventRecord(rs->ev[2 * K + 1], rs->comm), "hipEventRecord (S landed)");
    }
    const bool timed = hipEventRecord(rs->t_land, rs->comm) == hipSuccess;
    o.recv_r = total[0];
    o.recv_s = total[1];
    const auto t1 = Clock::now();
    o.ms_post = std::chrono::duration<double, std::milli>(t1 - t0).count();

    // local join: R's passes once R has landed, S's passes and build/probe once S has.
    // Every failure from here on is this rank's own and is flagged in the final all-reduce.
    if (fail_rc == MI355_OK && o.wire16) {
        const bool waited = hip_ok(hipStreamWaitEvent(s, rs->ev[2 * K], 0), "hipStreamWaitEvent (R landed)");
        if (waited && total[0] && total[1]) {
            // R's passes (narrow residuals, the plan the senders used for S), then S's
            // pieces gathered once they have landed, and the build/probe
            uint64_t *rcS = reinterpret_cast<uint64_t *>(ctx->wrecvS.as<char>() + res_bytes(cS));
            int lrc = injected(rank, kFailLocal)
                          ? MI355_ERR_OOM
                          : rho::join_pipelined_begin(ctx, s, ctx->xrecvR.ptr, total[0], total[1], &lo,
                                                      (uint32_t)elem, nullptr, 0, true);
            if (lrc == MI355_OK)
                lrc = rho::join_pipelined_finish_wire16(ctx, ctx->wrecvS.as<uint16_t>(), rcS, wbase.data(),
                                                        wcount.data(), wspan.data(), total[1], G, rcS + (size_t)G * RW,
                                                        rs->ev[2 * K + 1], &o.st);
            fail(lrc);
            o.local = lrc == MI355_OK ? o.st.matches : 0;
        } else if (waited) {
            hip_ok(hipStreamWaitEvent(s, rs->ev[2 * K + 1], 0), "hipStreamWaitEvent (S landed)");
        }
    } else if (fail_rc == MI355_OK) {
        const bool waited = hip_ok(hipStreamWaitEvent(s, rs->ev[2 * K], 0), "hipStreamWaitEvent (R landed)");
        if (waited && total[0] && total[1]) {
            // S's pass 1 runs per piece as it lands (each launch waits for its piece's
            // event); pass 2 and the build/probe follow the last one
            int lrc = injected(rank, kFailLocal) ? MI355_ERR_OOM
                                                 : rho::join_pipelined_begin(ctx, s, ctx->xrecvR.ptr, total[0],
                                                                             total[1], &lo, (uint32_t)elem,
                                                                             s_piece.data(), K);
            if (lrc == MI355_OK)
                lrc = rho::join_pipelined_finish(ctx, ctx->xrecvS.ptr, total[1], &o.st, &rs->ev[2 * K + 2], mat);
            fail(lrc);
            o.local = lrc == MI355_OK ? o.st.matches : 0;
        } else if (waited) {
            hip_ok(hipStreamWaitEvent(s, rs->ev[2 * K + 1], 0), "hipStreamWaitEvent (S landed)");
        }
    }
    const bool timed_end = timed && fail_rc == MI355_OK && hipEventRecord(rs->t_done, s) == hipSuccess;
    // an asynchronous error of the local join's kernels surfaces here
    hipError_t se = hipStreamSynchronize(s);
    if (injected(rank, kFailLocalSync)) se = hipErrorLaunchFailure;
    hip_ok(se, "hipStreamSynchronize (local join)");
    hip_ok(hipStreamSynchronize(rs->comm), "hipStreamSynchronize (exchange)");
    const auto t2 = Clock::now();
    o.ms_local = std::chrono::duration<double, std::milli>(t2 - t1).count();
    float tail = -1.f;
    if (timed_end && fail_rc == MI355_OK && hipEventElapsedTime(&tail, rs->t_land, rs->t_done) == hipSuccess)
        o.ms_tail = tail;
    uint64_t m[2] = {fail_rc == MI355_OK ? o.local : 0, fail_rc != MI355_OK ? 1u : 0u};
    MH_RC(transport_rc(T.allreduce(rank, s, m, 2, kSum)));
    if (m[1]) return peer_failed();
    o.global = m[0];
    o.ms_allreduce = ms_since(t2);
    o.ms_total = ms_since(t0);
    return MI355_OK;
}

// ---------------------------------------------------------------- single process
int resolve_transport(int transport, int G) {
    if (const char *e = std::getenv("SGXAMD_MULTI_TRANSPORT")) {
        if (!std::strcmp(e, "rccl")) return MI355_TRANSPORT_RCCL;
        if (!std::strcmp(e, "rehearsal")) return MI355_TRANSPORT_REHEARSAL;
    }
    if (transport != MI355_TRANSPORT_AUTO) return transport;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0;
    return (G > 1 && ndev >= G) ? MI355_TRANSPORT_RCCL : MI355_TRANSPORT_REHEARSAL;
}

// Contexts of the rehearsal's logical ranks, per (device, rank), kept for the process.
std::mutex g_reh_mu;
std::unordered_map<uint64_t, std::unique_ptr<Context>> g_reh;

Context *rehearsal_context(int device, int rank, int *status) {
    std::lock_guard<std::mutex> lk(g_reh_mu);
    auto &slot = g_reh[((uint64_t)device << 32) | (uint32_t)rank];
    if (!slot) slot = make_context(device, status);
    return slot.get();
}

// RCCL communicators over devices 0..G-1 for one process (ncclCommInitAll), per G.
std::mutex g_all_mu;
std::unordered_map<int, std::vector<ncclComm_t>> g_all;

// same_dev >= 0: every rank on that device (an RCCL test double only).
int comms_all(int G, int same_dev, std::vector<ncclComm_t> *out) {
    MH_RC(require_rccl());
    std::lock_guard<std::mutex> lk(g_all_mu);
    auto it = g_all.find(G);
    if (it == g_all.end()) {
        std::vector<ncclComm_t> comms(G);
        std::vector<int> devs(G);
        for (int g = 0; g < G; ++g) devs[g] = same_dev >= 0 ? same_dev : g;
        MH_NCCL(rccl().CommInitAll(comms.data(), G, devs.data()));
        it = g_all.emplace(G, std::move(comms)).first;
    }
    *out = it->second;
    return MI355_OK;
}

// A transport call failed on some rank (every rank thread has returned): the
// communicators may hold unmatched operations, so they are aborted and dropped from the
// cache; the next call creates new ones.
void drop_comms_all(int G) {
    std::lock_guard<std::mutex> lk(g_all_mu);
    auto it = g_all.find(G);
    if (it == g_all.end()) return;
    for (ncclComm_t c : it->second) rccl().abort_comm(c);
    g_all.erase(it);
}

void fill_stats(mi355_multi_stats *st, const std::vector<RankOut> &outs, int G, int kind, int rank) {
    if (!st) return;
    std::memset(st, 0, sizeof(*st));
    st->world = G;
    st->transport = kind;
    st->pieces = std::max(1, std::min(64, g_pieces.load()));
    st->rank = rank;
    st->recv_r_min = st->recv_s_min = UINT64_MAX;
    st->ms_tail = -1;  // not measured (a failed or untimed tail), unless a rank measured it
    for (const RankOut &o : outs) {
        st->matches = o.global;
        st->recv_r_max = std::max(st->recv_r_max, o.recv_r);
        st->recv_r_min = std::min(st->recv_r_min, o.recv_r);
        st->recv_s_max = std::max(st->recv_s_max, o.recv_s);
        st->recv_s_min = std::min(st->recv_s_min, o.recv_s);
        st->max_part_s = std::max(st->max_part_s, o.st.max_part_s);
        st->sent_bytes += o.sent;
        st->ms_total = std::max(st->ms_total, o.ms_total);
        st->ms_exchange_post = std::max(st->ms_exchange_post, o.ms_post);
        st->ms_local = std::max(st->ms_local, o.ms_local);
        st->ms_allreduce = std::max(st->ms_allreduce, o.ms_allreduce);
        st->ms_tail = std::max(st->ms_tail, o.ms_tail);
    }
    if (!outs.empty()) {
        st->local_matches = outs[0].local;
        st->local = outs[0].st;
        st->elem_bytes = outs[0].wire16 ? 2u : outs[0].keys ? 4u : 8u;
    }
}

}  // namespace

int join_multi(const row_t *R, uint64_t nR, const row_t *S, uint64_t nS, int G, int transport,
               const mi355_rho_opts *opts, mi355_multi_stats *st) {
    if (G < 1 || G > 256 || (G & (G - 1)) || (!R && nR) || (!S && nS)) {
        set_last_error("mi355_rho_join_multi: ngpus must be a power of two in 1..256, relations non-null");
        return MI355_ERR_INVALID;
    }
    if (opts && (opts->key_shift || opts->stream)) {
        set_last_error("mi355_rho_join_multi: key_shift and stream must be 0");
        return MI355_ERR_INVALID;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        (void)hipGetLastError();
        set_last_error("no HIP device visible (mi355_* needs a gfx950 GPU)");
        return MI355_ERR_NO_DEVICE;
    }
    int cur = 0;
    MH_HIP(hipGetDevice(&cur));
    const int kind = resolve_transport(transport, G);
    // a test double of RCCL (mi355_multi_set_rccl_library) runs every rank on the
    // current GPU, each with a context of its own, like the rehearsal
    const bool one_gpu = kind == MI355_TRANSPORT_RCCL && rccl().double_;
    if (kind == MI355_TRANSPORT_RCCL && ndev < G && !one_gpu) {
        set_last_error("RCCL transport needs " + std::to_string(G) + " visible GPUs");
        return MI355_ERR_INVALID;
    }
    std::unique_ptr<Transport> T;
    if (kind == MI355_TRANSPORT_RCCL) {
        std::vector<ncclComm_t> comms;
        MH_RC(comms_all(G, one_gpu ? cur : -1, &comms));
        T = std::make_unique<RcclTransport>(G, 0, comms, std::vector<ncclComm_t>{},
                                            std::make_shared<HostCollectives>(G));
    } else {
        T = std::make_unique<RehearsalTransport>(G);
    }
    // the rank threads run with the caller's per-thread settings (key layout, timing)
    const bool keys = thread_key_layout(), timing = thread_timing_enabled();
    const bool dR = is_device_pointer(R), dS = is_device_pointer(S);
    std::vector<RankOut> outs(G);
    std::vector<int> rcs(G, MI355_OK);
    std::vector<std::string> errs(G);
    auto body = [&](int g) -> int {
        mi355_set_key_layout(keys ? 1 : 0);
        mi355_timing_enable(timing ? 1 : 0);
        const int dev = kind == MI355_TRANSPORT_RCCL && !one_gpu ? g : cur;
        int status = MI355_OK;
        Context *ctx = nullptr;
        if (hipSetDevice(dev) != hipSuccess) {
            set_last_error("hipSetDevice(" + std::to_string(dev) + ") failed");
            status = MI355_ERR_HIP;
        } else if (injected(g, kFailContext)) {
            status = MI355_ERR_HIP;
        } else {
            ctx = kind == MI355_TRANSPORT_RCCL && !one_gpu ? current_context(&status)
                                                           : rehearsal_context(dev, g, &status);
        }
        // this rank's slices (radix_join.cpp:1488-1499: floor(n/T) each, the last the rest)
        const uint64_t pr = nR / G, ps = nS / G;
        const uint64_t r0 = pr * g, s0 = ps * g;
        const uint64_t rn = g == G - 1 ? nR - r0 : pr, sn = g == G - 1 ? nS - s0 : ps;
        const row_t *lR = R + r0, *lS = S + s0;
        // without a context the rank still takes part in the collectives, flagged as failed
        if (!ctx) return rank_join(*T, g, nullptr, nullptr, nullptr, 0, nullptr, 0, opts, outs[g], status);
        std::lock_guard<std::mutex> lk(ctx->mu);
        int src = MI355_OK;
        auto stage = [&](DeviceBuffer &buf, const row_t *&p, uint64_t n) {
            if (src != MI355_OK) return;
            const hipError_t e1 = buf.ensure(std::max<uint64_t>(n, 1) * sizeof(row_t));
            const hipError_t e2 =
                e1 == hipSuccess ? hipMemcpyAsync(buf.ptr, p, n * sizeof(row_t), hipMemcpyDefault, ctx->stream) : e1;
            if (e2 != hipSuccess) {
                set_last_error(std::string("staging a slice: ") + hipGetErrorString(e2));
                src = e2 == hipErrorOutOfMemory ? MI355_ERR_OOM : MI355_ERR_HIP;
                return;
            }
            p = buf.as<row_t>();
        };
        if (!(dR && dev == cur)) stage(ctx->inR, lR, rn);  // H2D, or peer D2D
        if (!(dS && dev == cur)) stage(ctx->inS, lS, sn);
        if (src == MI355_OK && hipStreamSynchronize(ctx->stream) != hipSuccess) {
            set_last_error("staging the slices failed");
            src = MI355_ERR_HIP;
        }
        if (src != MI355_OK) return rank_join(*T, g, ctx, ctx->stream, nullptr, 0, nullptr, 0, opts, outs[g], src);
        return rank_join(*T, g, ctx, ctx->stream, lR, rn, lS, sn, opts, outs[g]);
    };
    std::vector<std::thread> th;
    for (int g = 0; g < G; ++g)
        th.emplace_back([&, g] {
            rcs[g] = body(g);
            if (rcs[g] != MI355_OK) {
                errs[g] = last_error();
                // a rank that left the sequence of collectives alone (a transport call
                // failed) releases the other ranks' host waits; flagged failures end
                // every rank at the same collective and need nothing
                if (!outs[g].together) T->abort();
            }
        });
    for (auto &t : th) t.join();
    (void)hipSetDevice(cur);
    bool comm_broken = false;
    for (int g = 0; g < G; ++g) comm_broken = comm_broken || (rcs[g] != MI355_OK && !outs[g].together);
    if (comm_broken && kind == MI355_TRANSPORT_RCCL) {
        T.reset();
        drop_comms_all(G);
    }
    // report the rank that failed first-hand, not the peers that followed it
    int first = -1;
    for (int g = 0; g < G; ++g)
        if (rcs[g] != MI355_OK && (first < 0 || (outs[first].peer_fail && !outs[g].peer_fail))) first = g;
    if (first >= 0) {
        set_last_error("rank " + std::to_string(first) + ": " + errs[first]);
        return rcs[first];
    }
    fill_stats(st, outs, G, kind, 0);
    if (opts && opts->materialize) {
        // the ranks' output chunks, rank 0's first, into the caller's buffer
        uint64_t total = 0;
        for (const RankOut &o : outs) total += o.local;
        if (total > opts->out_capacity || (total && !opts->out)) {
            set_last_error("materialisation output too small: " + std::to_string(total) + " triples needed");
            return MI355_ERR_CAPACITY;
        }
        uint64_t off = 0;
        for (int g = 0; g < G; ++g) {
            const RankOut &o = outs[g];
            if (!o.local) continue;
            MH_HIP(hipSetDevice(o.ctx->device));
            const hipError_t e = hipMemcpy(opts->out + off, o.ctx->mat.ptr, o.local * sizeof(output_triple_t),
                                           hipMemcpyDefault);
            (void)hipSetDevice(cur);
            MH_HIP(e);
            off += o.local;
        }
    }
    return MI355_OK;
}

thread_local mi355_multi_stats t_last_multi{};

// ---------------------------------------------------------------- one process per GPU
// comm carries the tuples, ccomm (ncclCommSplit of comm, same ranks) the counts, flags
// and reductions.  broken: a transport call failed; both were aborted.
// ctx: the device's shared context, or -- when another rank of this process already
// holds a communicator on the same device (only an RCCL test double allows that) -- a
// context of its own, so that the ranks' joins do not serialise on one context's lock.
struct CommHandle {
    int world = 0, rank = 0, device = 0;
    ncclComm_t comm = nullptr, ccomm = nullptr;
    bool broken = false;
    std::unique_ptr<RcclTransport> T;
    Context *ctx = nullptr;
    std::unique_ptr<Context> own;
    void abort_comms() {
        T.reset();
        for (ncclComm_t *c : {&comm, &ccomm}) {
            rccl().abort_comm(*c);
            *c = nullptr;
        }
        broken = true;
    }
};

std::mutex g_dev_handles_mu;
std::unordered_map<int, int> g_dev_handles;  // live communicators per device

// Frees a context of its own (its stream, pinned block and workspace) once idle.
void destroy_own_context(std::unique_ptr<Context> &c) {
    if (!c) return;
    {
        std::lock_guard<std::mutex> lk(c->mu);
        (void)hipStreamSynchronize(c->stream);
        release_workspace(c.get());
    }
    {
        std::lock_guard<std::mutex> lk(g_streams_mu);
        auto it = g_streams.find(c.get());
        if (it != g_streams.end()) {
            if (it->second.comm) (void)hipStreamSynchronize(it->second.comm), (void)hipStreamDestroy(it->second.comm);
            for (hipEvent_t e : it->second.ev) (void)hipEventDestroy(e);
            for (hipEvent_t e : {it->second.t_land, it->second.t_done})
                if (e) (void)hipEventDestroy(e);
            g_streams.erase(it);
        }
    }
    rho::forget_context(c.get());
    (void)hipStreamDestroy(c->stream);
    if (c->host_result) (void)hipHostFree(c->host_result);
    c.reset();
}

}  // namespace multi
}  // namespace sgxamd

using namespace sgxamd;

extern "C" {

int mi355_rho_join_multi_ex(const row_t *R, uint64_t nR, const row_t *S, uint64_t nS, int ngpus, int transport,
                            const mi355_rho_opts *opts, mi355_multi_stats *stats) {
    const auto t0 = multi::Clock::now();
    mi355_multi_stats local{};
    mi355_multi_stats *st = stats ? stats : &local;
    const int rc = multi::join_multi(R, nR, S, nS, ngpus, transport, opts, st);
    if (rc == MI355_OK) {
        // what mi355_last_join_stats / print_timing report for this call: the local join
        // of rank 0 with the global cardinality and the whole call's time
        mi355_rho_stats ls = st->local;
        ls.matches = st->matches;
        ls.ms_total = multi::ms_since(t0);
        rho::set_last_join_stats(ls);
        multi::t_last_multi = *st;
    }
    return rc;
}

int mi355_last_multi_stats(mi355_multi_stats *out) {
    if (!out) return MI355_ERR_INVALID;
    *out = multi::t_last_multi;
    return MI355_OK;
}

int mi355_rho_join_multi(const table_t *relR, const table_t *relS, const joinconfig_t *config, int ngpus,
                         result_t *out) {
    if (!relR || !relS || !out) {
        set_last_error("null argument");
        return MI355_ERR_INVALID;
    }
    if (config && config->MATERIALIZE) {
        set_last_error("mi355_rho_join_multi: counting joins only (MATERIALIZE runs on one GPU)");
        return MI355_ERR_INVALID;
    }
    const auto t0 = multi::Clock::now();
    mi355_multi_stats st{};
    const int rc = mi355_rho_join_multi_ex(relR->tuples, relR->num_tuples, relS->tuples, relS->num_tuples, ngpus,
                                           MI355_TRANSPORT_AUTO, nullptr, &st);
    if (rc) return rc;
    const double us = multi::ms_since(t0) * 1000.0;
    out->totalresults = (int64_t)st.matches;
    out->nthreads = config ? config->NTHREADS : 1;
    out->throughput = us > 0 ? (double)(relR->num_tuples + relS->num_tuples) / us : 0.0;  // M rec/s
    out->materialized = 0;
    out->result = nullptr;
    out->result_type = 0;
    return MI355_OK;
}

void mi355_multi_set_pieces(int pieces) { multi::g_pieces = std::max(1, std::min(64, pieces)); }

void mi355_multi_set_wire(int mode) { rho::set_wire_mode(mode); }

int mi355_multi_release(void) {
    std::lock_guard<std::mutex> lk(multi::g_reh_mu);
    int cur = 0;
    MH_HIP(hipGetDevice(&cur));
    int rc = MI355_OK;
    for (auto &kv : multi::g_reh) {
        Context *ctx = kv.second.get();
        std::lock_guard<std::mutex> ck(ctx->mu);
        if (hipSetDevice(ctx->device) != hipSuccess || hipStreamSynchronize(ctx->stream) != hipSuccess) {
            set_last_error("mi355_multi_release: device synchronisation failed");
            rc = MI355_ERR_HIP;
            break;
        }
        release_workspace(ctx);
    }
    (void)hipSetDevice(cur);
    return rc;
}

void mi355_multi_inject_failure(int rank, int step) {
    multi::g_fail_step = step;
    multi::g_fail_rank = step > 0 ? rank : -1;
}

int mi355_multi_unique_id(void *id128) {
    if (!id128) return MI355_ERR_INVALID;
    MH_RC(multi::require_rccl());
    ncclUniqueId id;
    MH_NCCL(multi::rccl().GetUniqueId(&id));
    std::memcpy(id128, &id, sizeof(id));
    return MI355_OK;
}

int mi355_multi_comm_init(const void *id128, int nranks, int rank, void **comm) {
    if (!id128 || !comm || nranks < 1 || nranks > 256 || (nranks & (nranks - 1)) || rank < 0 || rank >= nranks) {
        set_last_error("mi355_multi_comm_init: bad arguments (nranks a power of two)");
        return MI355_ERR_INVALID;
    }
    // counted before the library is even looked up (under g_all_mu, the lock
    // mi355_multi_set_rccl_library checks it under), so it cannot be swapped between here
    // and the communicator's end; rolled back on every early return
    {
        std::lock_guard<std::mutex> lk(multi::g_all_mu);
        ++multi::g_live_handles;
    }
    struct Counted {
        bool keep = false;
        ~Counted() {
            if (!keep) --multi::g_live_handles;
        }
    } counted;
    MH_RC(multi::require_rccl());
    const multi::Rccl &lib = multi::rccl();
    if (!lib.CommSplit) {
        set_last_error(lib.name + " lacks ncclCommSplit (the count communicator of mi355_multi_comm_init)");
        return MI355_ERR_COMM;
    }
    auto h = std::make_unique<multi::CommHandle>();
    h->world = nranks;
    h->rank = rank;
    MH_HIP(hipGetDevice(&h->device));
    ncclUniqueId id;
    std::memcpy(&id, id128, sizeof(id));
    const ncclResult_t ir = lib.CommInitRank(&h->comm, nranks, id, rank);
    if (ir != ncclSuccess) {
        set_last_error(std::string("ncclCommInitRank: ") + lib.ErrorString(ir));
        return MI355_ERR_COMM;
    }
    const ncclResult_t sr = lib.CommSplit(h->comm, 0, rank, &h->ccomm, nullptr);
    if (sr != ncclSuccess) {
        set_last_error(std::string("ncclCommSplit (count communicator): ") + lib.ErrorString(sr));
        h->abort_comms();
        return MI355_ERR_COMM;
    }
    h->T = std::make_unique<multi::RcclTransport>(nranks, rank, std::vector<ncclComm_t>{h->comm},
                                                  std::vector<ncclComm_t>{h->ccomm}, nullptr);
    bool shared_dev;
    {
        std::lock_guard<std::mutex> lk(multi::g_dev_handles_mu);
        shared_dev = multi::g_dev_handles[h->device]++ > 0;
    }
    int status = MI355_OK;
    if (shared_dev) {
        h->own = make_context(h->device, &status);
        h->ctx = h->own.get();
    } else {
        h->ctx = current_context(&status);
    }
    // without a context the rank still takes part in the joins' collectives, flagged as
    // failed (mi355_rho_join_sharded), so the communicator is kept
    *comm = h.release();
    counted.keep = true;  // released by mi355_multi_comm_destroy
    return MI355_OK;
}

int mi355_multi_comm_destroy(void *comm) {
    auto *h = static_cast<multi::CommHandle *>(comm);
    if (!h) return MI355_OK;
    h->T.reset();
    for (ncclComm_t c : {h->ccomm, h->comm})
        if (c && multi::rccl().CommDestroy) (void)multi::rccl().CommDestroy(c);
    multi::destroy_own_context(h->own);
    {
        std::lock_guard<std::mutex> lk(multi::g_dev_handles_mu);
        --multi::g_dev_handles[h->device];
    }
    --multi::g_live_handles;
    delete h;
    return MI355_OK;
}

int mi355_multi_set_rccl_library(const char *path) {
    std::string p = path ? path : "";
    {
        std::lock_guard<std::mutex> lk(multi::g_all_mu);
        if (multi::g_live_handles.load() > 0) {
            set_last_error("mi355_multi_set_rccl_library: communicators of mi355_multi_comm_init are alive");
            return MI355_ERR_INVALID;
        }
    }
    // the single-process communicators of the old library go first
    std::vector<int> sizes;
    {
        std::lock_guard<std::mutex> lk(multi::g_all_mu);
        for (auto &kv : multi::g_all) sizes.push_back(kv.first);
    }
    for (int G : sizes) multi::drop_comms_all(G);
    std::lock_guard<std::mutex> lk(multi::g_rccl_mu);
    multi::g_rccl_path = p;
    multi::g_rccl = nullptr;  // loaded on next use
    return MI355_OK;
}

int mi355_rho_join_sharded(void *comm, const row_t *R, uint64_t nR, const row_t *S, uint64_t nS,
                           const mi355_rho_opts *opts, mi355_multi_stats *stats) {
    auto *h = static_cast<multi::CommHandle *>(comm);
    if (!h || (!R && nR) || (!S && nS)) {
        set_last_error("mi355_rho_join_sharded: null argument");
        return MI355_ERR_INVALID;
    }
    if ((nR && !is_device_pointer(R)) || (nS && !is_device_pointer(S))) {
        set_last_error("mi355_rho_join_sharded needs device-resident slices");
        return MI355_ERR_INVALID;
    }
    if (opts && opts->key_shift) {
        set_last_error("mi355_rho_join_sharded: key_shift must be 0");
        return MI355_ERR_INVALID;
    }
    if (h->broken) {
        set_last_error("mi355_rho_join_sharded: the communicator was aborted after a failed RCCL call");
        return MI355_ERR_COMM;
    }
    MH_HIP(hipSetDevice(h->device));
    int status = MI355_OK;
    Context *ctx = h->ctx ? h->ctx : current_context(&status);
    if (ctx && multi::injected(h->rank, multi::kFailContext)) {
        ctx = nullptr;
        status = MI355_ERR_HIP;
    }
    std::vector<multi::RankOut> outs(1);
    int rc;
    if (!ctx) {  // take part in the collectives, flagged as failed
        if (status == MI355_OK) status = MI355_ERR_HIP;
        rc = multi::rank_join(*h->T, h->rank, nullptr, nullptr, nullptr, 0, nullptr, 0, opts, outs[0], status);
    } else {
        std::lock_guard<std::mutex> lk(ctx->mu);
        // the caller's stream (opts->stream or mi355_set_stream): R and S were produced there
        hipStream_t s = thread_stream(ctx, opts ? opts->stream : nullptr);
        rc = multi::rank_join(*h->T, h->rank, ctx, s, R, nR, S, nS, opts, outs[0]);
    }
    if (rc != MI355_OK) {
        // a rank that left the sequence of collectives (a failed RCCL call, or a HIP call
        // inside the transport) leaves unmatched operations behind: abort this rank's
        // communicators (the peers' calls fail or are torn down with the job)
        if (!outs[0].together) {
            const std::string e = last_error();
            h->abort_comms();
            set_last_error(e);
        }
        return rc;
    }
    mi355_multi_stats local{};
    mi355_multi_stats *st = stats ? stats : &local;
    multi::fill_stats(st, outs, h->world, MI355_TRANSPORT_RCCL, h->rank);
    multi::t_last_multi = *st;
    mi355_rho_stats ls = outs[0].st;
    ls.matches = outs[0].global;
    rho::set_last_join_stats(ls);
    if (opts && opts->materialize) {
        // this rank's output chunk (its local_matches triples) into the caller's buffer
        const uint64_t n = outs[0].local;
        if (n > opts->out_capacity || (n && !opts->out)) {
            set_last_error("materialisation output too small: " + std::to_string(n) + " triples needed (this rank)");
            return MI355_ERR_CAPACITY;
        }
        if (n) MH_HIP(hipMemcpy(opts->out, outs[0].ctx->mat.ptr, n * sizeof(output_triple_t), hipMemcpyDefault));
    }
    return MI355_OK;
}

}  // extern "C"
