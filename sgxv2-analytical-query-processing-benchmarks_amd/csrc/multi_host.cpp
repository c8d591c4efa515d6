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

#define MH_RC(call)                  \
    do {                             \
        const int _rc = (call);      \
        if (_rc != MI355_OK) return _rc; \
    } while (0)

// ---------------------------------------------------------------- RCCL, loaded on first use
// libsgxamd.so keeps no link-time dependency on RCCL: the single-GPU library loads on
// hosts without it, and a process that already holds librccl.so.1 (PyTorch's) shares it.
struct Rccl {
    decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
    decltype(&ncclCommInitRank) CommInitRank = nullptr;
    decltype(&ncclCommInitAll) CommInitAll = nullptr;
    decltype(&ncclCommDestroy) CommDestroy = nullptr;
    decltype(&ncclGroupStart) GroupStart = nullptr;
    decltype(&ncclGroupEnd) GroupEnd = nullptr;
    decltype(&ncclSend) Send = nullptr;
    decltype(&ncclRecv) Recv = nullptr;
    decltype(&ncclAllGather) AllGather = nullptr;
    decltype(&ncclAllReduce) AllReduce = nullptr;
    decltype(&ncclGetErrorString) ErrorString = nullptr;
    std::string error;
};

const Rccl &rccl() {
    static const Rccl lib = [] {
        Rccl r;
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            const char *e = dlerror();
            r.error = std::string("cannot load librccl.so.1: ") + (e ? e : "?");
            return r;
        }
        auto sym = [&](auto &fn, const char *name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
            if (!fn && r.error.empty()) r.error = std::string("librccl.so.1 lacks ") + name;
        };
        sym(r.GetUniqueId, "ncclGetUniqueId");
        sym(r.CommInitRank, "ncclCommInitRank");
        sym(r.CommInitAll, "ncclCommInitAll");
        sym(r.CommDestroy, "ncclCommDestroy");
        sym(r.GroupStart, "ncclGroupStart");
        sym(r.GroupEnd, "ncclGroupEnd");
        sym(r.Send, "ncclSend");
        sym(r.Recv, "ncclRecv");
        sym(r.AllGather, "ncclAllGather");
        sym(r.AllReduce, "ncclAllReduce");
        sym(r.ErrorString, "ncclGetErrorString");
        return r;
    }();
    return lib;
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

   private:
    std::mutex m_;
    std::condition_variable cv_;
    int n_, waiting_ = 0;
    uint64_t gen_ = 0;
    bool aborted_ = false;
};

// ---------------------------------------------------------------- transports
enum ReduceOp { kSum, kMax };

class Transport {
   public:
    virtual ~Transport() = default;
    virtual int world() const = 0;
    virtual int kind() const = 0;
    // collective: send[d] = tuples this rank sends to rank d in this piece;
    // recv[q] = tuples rank q sends to this rank (host arrays of world() entries)
    virtual int exchange_counts(int rank, hipStream_t s, const uint64_t *send, uint64_t *recv) = 0;
    // collective: after `ready` (the piece's partition on the compute stream), move the
    // piece: the run for destination d starts at send + sum_{d'<d} send_counts[d'];
    // rank q's run lands at recv + sum_{q'<q} recv_counts[q'].  Enqueued on c.
    // elem: bytes per element (8: row_t tuples; 4: keys of a keys-only exchange).
    virtual int post_exchange(int rank, hipStream_t c, hipEvent_t ready, const void *send,
                              const uint64_t *send_counts, void *recv, const uint64_t *recv_counts, size_t elem) = 0;
    // collective: *v = sum / max of every rank's *v
    virtual int allreduce(int rank, hipStream_t s, uint64_t *v, ReduceOp op) = 0;
    virtual void abort() {}
};

std::vector<uint64_t> prefix(const uint64_t *c, int n) {
    std::vector<uint64_t> p(n + 1, 0);
    for (int i = 0; i < n; ++i) p[i + 1] = p[i] + c[i];
    return p;
}

// RCCL over xGMI.  One communicator per local rank: all G of them (one process, one
// thread per GPU, ncclCommInitAll) or this process's one (ncclCommInitRank).
class RcclTransport final : public Transport {
   public:
    RcclTransport(int world, int first_rank, std::vector<ncclComm_t> comms, std::vector<int> devices)
        : world_(world), first_(first_rank), comms_(std::move(comms)), devices_(std::move(devices)),
          buf_(comms_.size()), host_(comms_.size(), nullptr) {}
    ~RcclTransport() override {
        for (auto &b : buf_) b.release();
        for (auto *h : host_)
            if (h) (void)hipHostFree(h);
    }
    int world() const override { return world_; }
    int kind() const override { return MI355_TRANSPORT_RCCL; }

    int exchange_counts(int rank, hipStream_t s, const uint64_t *send, uint64_t *recv) override {
        const int i = rank - first_;
        uint64_t *d = nullptr, *h = nullptr;
        MH_RC(scratch(i, &d, &h));
        std::memcpy(h, send, sizeof(uint64_t) * world_);
        MH_HIP(hipMemcpyAsync(d, h, sizeof(uint64_t) * world_, hipMemcpyHostToDevice, s));
        MH_NCCL(rccl().AllGather(d, d + world_, world_, ncclUint64, comms_[i], s));
        MH_HIP(hipMemcpyAsync(h + world_, d + world_, sizeof(uint64_t) * world_ * world_, hipMemcpyDeviceToHost, s));
        MH_HIP(hipStreamSynchronize(s));
        for (int q = 0; q < world_; ++q) recv[q] = h[world_ + (size_t)q * world_ + rank];
        return MI355_OK;
    }

    int post_exchange(int rank, hipStream_t c, hipEvent_t ready, const void *send_v, const uint64_t *send_counts,
                      void *recv_v, const uint64_t *recv_counts, size_t elem) override {
        const int i = rank - first_;
        const auto so = prefix(send_counts, world_), ro = prefix(recv_counts, world_);
        const char *send = static_cast<const char *>(send_v);
        char *recv = static_cast<char *>(recv_v);
        const ncclDataType_t type = elem == 8 ? ncclUint64 : ncclUint32;
        MH_HIP(hipStreamWaitEvent(c, ready, 0));
        if (send_counts[rank])  // this rank's own run: a local copy
            MH_HIP(hipMemcpyAsync(recv + ro[rank] * elem, send + so[rank] * elem, send_counts[rank] * elem,
                                  hipMemcpyDeviceToDevice, c));
        MH_NCCL(rccl().GroupStart());
        for (int p = 0; p < world_; ++p) {
            if (p == rank) continue;
            if (send_counts[p]) MH_NCCL(rccl().Send(send + so[p] * elem, send_counts[p], type, p, comms_[i], c));
            if (recv_counts[p]) MH_NCCL(rccl().Recv(recv + ro[p] * elem, recv_counts[p], type, p, comms_[i], c));
        }
        MH_NCCL(rccl().GroupEnd());
        return MI355_OK;
    }

    int allreduce(int rank, hipStream_t s, uint64_t *v, ReduceOp op) override {
        const int i = rank - first_;
        uint64_t *d = nullptr, *h = nullptr;
        MH_RC(scratch(i, &d, &h));
        h[0] = *v;
        MH_HIP(hipMemcpyAsync(d, h, sizeof(uint64_t), hipMemcpyHostToDevice, s));
        MH_NCCL(rccl().AllReduce(d, d, 1, ncclUint64, op == kSum ? ncclSum : ncclMax, comms_[i], s));
        MH_HIP(hipMemcpyAsync(h, d, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
        MH_HIP(hipStreamSynchronize(s));
        *v = h[0];
        return MI355_OK;
    }

   private:
    // per local rank: device [world + world^2] u64 and its pinned host mirror
    int scratch(int i, uint64_t **d, uint64_t **h) {
        const size_t bytes = sizeof(uint64_t) * (world_ + (size_t)world_ * world_);
        MH_HIP(buf_[i].ensure(bytes));
        if (!host_[i]) MH_HIP(hipHostMalloc(reinterpret_cast<void **>(&host_[i]), bytes));
        *d = buf_[i].as<uint64_t>();
        *h = host_[i];
        return MI355_OK;
    }
    int world_, first_;
    std::vector<ncclComm_t> comms_;
    std::vector<int> devices_;
    std::vector<DeviceBuffer> buf_;
    std::vector<uint64_t *> host_;
};

// G logical ranks on one GPU, one host thread each: counts and reductions through
// shared host tables, tuples by device-to-device copies that the receiver enqueues on
// its communication stream after the sender's partition event.  Same collective
// sequence and receive layout as the RCCL transport.
class RehearsalTransport final : public Transport {
   public:
    explicit RehearsalTransport(int world)
        : world_(world), bar_(world), counts_(world, std::vector<uint64_t>(world)), posts_(world), red_(world) {}
    int world() const override { return world_; }
    int kind() const override { return MI355_TRANSPORT_REHEARSAL; }

    int exchange_counts(int rank, hipStream_t, const uint64_t *send, uint64_t *recv) override {
        std::copy(send, send + world_, counts_[rank].begin());
        if (!bar_.wait()) return aborted();
        for (int q = 0; q < world_; ++q) recv[q] = counts_[q][rank];
        if (!bar_.wait()) return aborted();
        return MI355_OK;
    }

    int post_exchange(int rank, hipStream_t c, hipEvent_t ready, const void *send, const uint64_t *send_counts,
                      void *recv_v, const uint64_t *recv_counts, size_t elem) override {
        char *recv = static_cast<char *>(recv_v);
        posts_[rank] = Post{static_cast<const char *>(send), prefix(send_counts, world_), ready};
        if (!bar_.wait()) return aborted();
        uint64_t off = 0;
        int rc = MI355_OK;
        for (int q = 0; q < world_ && rc == MI355_OK; ++q) {
            if (!recv_counts[q]) continue;
            const Post &p = posts_[q];
            if (hipStreamWaitEvent(c, p.ready, 0) != hipSuccess ||
                hipMemcpyAsync(recv + off * elem, p.send + p.off[rank] * elem, recv_counts[q] * elem,
                               hipMemcpyDeviceToDevice, c) != hipSuccess) {
                set_last_error("rehearsal exchange copy failed");
                rc = MI355_ERR_HIP;
            }
            off += recv_counts[q];
        }
        if (!bar_.wait()) return aborted();  // the posts table is reused by the next piece
        return rc;
    }

    int allreduce(int rank, hipStream_t, uint64_t *v, ReduceOp op) override {
        red_[rank] = *v;
        if (!bar_.wait()) return aborted();
        uint64_t r = op == kSum ? 0 : red_[0];
        for (uint64_t x : red_) r = op == kSum ? r + x : std::max(r, x);
        if (!bar_.wait()) return aborted();
        *v = r;
        return MI355_OK;
    }

    void abort() override { bar_.abort(); }

   private:
    int aborted() {
        set_last_error("another rank of the rehearsal failed");
        return MI355_ERR_INVALID;
    }
    struct Post {
        const char *send = nullptr;
        std::vector<uint64_t> off;
        hipEvent_t ready = nullptr;
    };
    int world_;
    Barrier bar_;
    std::vector<std::vector<uint64_t>> counts_;
    std::vector<Post> posts_;
    std::vector<uint64_t> red_;
};

// ---------------------------------------------------------------- one rank's join
std::atomic<int> g_pieces{4};

// Communication stream and piece events of a context (created on first use).
struct RankStreams {
    hipStream_t comm = nullptr;
    std::vector<hipEvent_t> ev;
};
std::mutex g_streams_mu;
std::unordered_map<const Context *, RankStreams> g_streams;

int rank_streams(Context *ctx, int nev, RankStreams **out) {
    std::lock_guard<std::mutex> lk(g_streams_mu);
    RankStreams &rs = g_streams[ctx];
    if (!rs.comm) MH_HIP(hipStreamCreateWithFlags(&rs.comm, hipStreamNonBlocking));
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
    bool keys = false;  // the exchange moved keys only
    double ms_post = 0, ms_local = 0, ms_allreduce = 0, ms_total = 0;
    mi355_rho_stats st{};
};

uint32_t log2_exact(int g) {
    uint32_t b = 0;
    while ((1 << b) < g) ++b;
    return b;
}

// The pipeline of the file comment for rank `rank` on its context (device current,
// ctx->mu held).  R / S: this rank's device-resident slices.
int rank_join(Transport &T, int rank, Context *ctx, hipStream_t s, const row_t *R, uint64_t nR, const row_t *S,
              uint64_t nS, const mi355_rho_opts *opts, RankOut &o) {
    const auto t0 = Clock::now();
    const int G = T.world();
    const uint32_t dest_bits = log2_exact(G);
    const int K = std::max(1, std::min(64, g_pieces.load()));
    mi355_rho_opts lo{};
    if (opts) lo = *opts;
    lo.key_shift = dest_bits;
    lo.materialize = 0;
    lo.stream = nullptr;
    lo.out = nullptr;
    lo.out_capacity = 0;
    if (G == 1) {  // nothing to exchange
        if (nR && nS) {
            MH_RC(rho::join_pipelined_begin(ctx, s, R, nR, nS, &lo));
            MH_RC(rho::join_pipelined_finish(ctx, S, nS, &o.st));
        }
        o.global = o.local = o.st.matches;
        o.recv_r = nR;
        o.recv_s = nS;
        o.ms_local = o.ms_total = ms_since(t0);
        return MI355_OK;
    }
    RankStreams *rs = nullptr;
    MH_RC(rank_streams(ctx, 2 * K + 2, &rs));
    hipStream_t c = rs->comm;

    // receive buffers for the worst case: every rank's piece i comes to this rank
    uint64_t mR = nR, mS = nS, sumR = nR, sumS = nS;
    MH_RC(T.allreduce(rank, s, &mR, kMax));
    MH_RC(T.allreduce(rank, s, &mS, kMax));
    MH_RC(T.allreduce(rank, s, &sumR, kSum));
    MH_RC(T.allreduce(rank, s, &sumS, kSum));
    const uint64_t capR = (uint64_t)G * K * ((mR + K - 1) / K), capS = (uint64_t)G * K * ((mS + K - 1) / K);
    // a counting join exchanges keys only (4 of the 8 bytes per tuple on xGMI) when its
    // local join, planned from the mean local sizes on every rank alike, reads keys
    o.keys = rho::keys_exchange_plan(sumR / G, sumS / G, capR, capS, &lo);
    const size_t elem = o.keys ? sizeof(uint32_t) : sizeof(row_t);
    MH_HIP(ctx->xsendR.ensure(std::max<uint64_t>(nR, 1) * elem));
    MH_HIP(ctx->xsendS.ensure(std::max<uint64_t>(nS, 1) * elem));
    MH_HIP(ctx->xrecvR.ensure(std::max<uint64_t>(capR, 1) * elem));
    MH_HIP(ctx->xrecvS.ensure(std::max<uint64_t>(capS, 1) * elem));

    std::vector<uint64_t> sc(G), rc(G);
    uint64_t total[2] = {0, 0};
    for (int rel = 0; rel < 2; ++rel) {
        const row_t *in = rel ? S : R;
        const uint64_t n = rel ? nS : nR;
        char *snd = (rel ? ctx->xsendS : ctx->xsendR).as<char>();
        char *rcv = (rel ? ctx->xrecvS : ctx->xrecvR).as<char>();
        const uint64_t per = (n + K - 1) / K;
        for (int i = 0; i < K; ++i) {
            const uint64_t a = std::min(n, i * per), b = std::min(n, (i + 1) * per);
            if (b > a)
                MH_RC(rho::shard_partition_device(ctx, s, in + a, b - a, 0, dest_bits, snd + a * elem, sc.data(),
                                                  (uint32_t)elem));
            else
                std::fill(sc.begin(), sc.end(), 0);
            MH_RC(T.exchange_counts(rank, s, sc.data(), rc.data()));
            hipEvent_t ready = rs->ev[rel * K + i];
            MH_HIP(hipEventRecord(ready, s));
            MH_RC(T.post_exchange(rank, c, ready, snd + a * elem, sc.data(), rcv + total[rel] * elem, rc.data(),
                                  elem));
            for (int q = 0; q < G; ++q) {
                total[rel] += rc[q];
                if (q != rank) o.sent += sc[q] * elem;
            }
        }
        MH_HIP(hipEventRecord(rs->ev[2 * K + rel], c));
    }
    o.recv_r = total[0];
    o.recv_s = total[1];
    const auto t1 = Clock::now();
    o.ms_post = std::chrono::duration<double, std::milli>(t1 - t0).count();

    // local join: R's passes once R has landed, S's passes and build/probe once S has
    MH_HIP(hipStreamWaitEvent(s, rs->ev[2 * K], 0));
    if (total[0] && total[1]) {
        MH_RC(rho::join_pipelined_begin(ctx, s, ctx->xrecvR.ptr, total[0], total[1], &lo, (uint32_t)elem));
        MH_HIP(hipStreamWaitEvent(s, rs->ev[2 * K + 1], 0));
        MH_RC(rho::join_pipelined_finish(ctx, ctx->xrecvS.ptr, total[1], &o.st));
        o.local = o.st.matches;
    } else {
        MH_HIP(hipStreamWaitEvent(s, rs->ev[2 * K + 1], 0));
        MH_HIP(hipStreamSynchronize(s));
    }
    MH_HIP(hipStreamSynchronize(c));
    const auto t2 = Clock::now();
    o.ms_local = std::chrono::duration<double, std::milli>(t2 - t1).count();
    uint64_t m = o.local;
    MH_RC(T.allreduce(rank, s, &m, kSum));
    o.global = m;
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

int comms_all(int G, std::vector<ncclComm_t> *out) {
    MH_RC(require_rccl());
    std::lock_guard<std::mutex> lk(g_all_mu);
    auto it = g_all.find(G);
    if (it == g_all.end()) {
        std::vector<ncclComm_t> comms(G);
        std::vector<int> devs(G);
        for (int g = 0; g < G; ++g) devs[g] = g;
        MH_NCCL(rccl().CommInitAll(comms.data(), G, devs.data()));
        it = g_all.emplace(G, std::move(comms)).first;
    }
    *out = it->second;
    return MI355_OK;
}

void fill_stats(mi355_multi_stats *st, const std::vector<RankOut> &outs, int G, int kind, int rank) {
    if (!st) return;
    std::memset(st, 0, sizeof(*st));
    st->world = G;
    st->transport = kind;
    st->pieces = std::max(1, std::min(64, g_pieces.load()));
    st->rank = rank;
    st->recv_r_min = st->recv_s_min = UINT64_MAX;
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
    }
    if (!outs.empty()) {
        st->local_matches = outs[0].local;
        st->local = outs[0].st;
        st->elem_bytes = outs[0].keys ? 4u : 8u;
    }
}

}  // namespace

int join_multi(const row_t *R, uint64_t nR, const row_t *S, uint64_t nS, int G, int transport,
               const mi355_rho_opts *opts, mi355_multi_stats *st) {
    if (G < 1 || G > 256 || (G & (G - 1)) || (!R && nR) || (!S && nS)) {
        set_last_error("mi355_rho_join_multi: ngpus must be a power of two in 1..256, relations non-null");
        return MI355_ERR_INVALID;
    }
    if (opts && (opts->key_shift || opts->materialize || opts->stream)) {
        set_last_error("mi355_rho_join_multi: key_shift, materialize and stream must be 0");
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
    if (kind == MI355_TRANSPORT_RCCL && ndev < G) {
        set_last_error("RCCL transport needs " + std::to_string(G) + " visible GPUs");
        return MI355_ERR_INVALID;
    }
    std::unique_ptr<Transport> T;
    if (kind == MI355_TRANSPORT_RCCL) {
        std::vector<ncclComm_t> comms;
        MH_RC(comms_all(G, &comms));
        std::vector<int> devs(G);
        for (int g = 0; g < G; ++g) devs[g] = g;
        T = std::make_unique<RcclTransport>(G, 0, comms, devs);
    } else {
        T = std::make_unique<RehearsalTransport>(G);
    }
    const bool dR = is_device_pointer(R), dS = is_device_pointer(S);
    std::vector<RankOut> outs(G);
    std::vector<int> rcs(G, MI355_OK);
    std::vector<std::string> errs(G);
    auto body = [&](int g) -> int {
        const int dev = kind == MI355_TRANSPORT_RCCL ? g : cur;
        MH_HIP(hipSetDevice(dev));
        int status = MI355_OK;
        Context *ctx = kind == MI355_TRANSPORT_RCCL ? current_context(&status) : rehearsal_context(dev, g, &status);
        if (!ctx) return status;
        std::lock_guard<std::mutex> lk(ctx->mu);
        // this rank's slices (radix_join.cpp:1488-1499: floor(n/T) each, the last the rest)
        const uint64_t pr = nR / G, ps = nS / G;
        const uint64_t r0 = pr * g, s0 = ps * g;
        const uint64_t rn = g == G - 1 ? nR - r0 : pr, sn = g == G - 1 ? nS - s0 : ps;
        const row_t *lR = R + r0, *lS = S + s0;
        if (!(dR && dev == cur)) {  // stage into this rank's device (H2D, or peer D2D)
            MH_HIP(ctx->inR.ensure(std::max<uint64_t>(rn, 1) * sizeof(row_t)));
            MH_HIP(hipMemcpyAsync(ctx->inR.ptr, lR, rn * sizeof(row_t), hipMemcpyDefault, ctx->stream));
            lR = ctx->inR.as<row_t>();
        }
        if (!(dS && dev == cur)) {
            MH_HIP(ctx->inS.ensure(std::max<uint64_t>(sn, 1) * sizeof(row_t)));
            MH_HIP(hipMemcpyAsync(ctx->inS.ptr, lS, sn * sizeof(row_t), hipMemcpyDefault, ctx->stream));
            lS = ctx->inS.as<row_t>();
        }
        MH_HIP(hipStreamSynchronize(ctx->stream));
        return rank_join(*T, g, ctx, ctx->stream, lR, rn, lS, sn, opts, outs[g]);
    };
    std::vector<std::thread> th;
    for (int g = 0; g < G; ++g)
        th.emplace_back([&, g] {
            rcs[g] = body(g);
            if (rcs[g] != MI355_OK) {
                errs[g] = last_error();
                T->abort();
            }
        });
    for (auto &t : th) t.join();
    (void)hipSetDevice(cur);
    for (int g = 0; g < G; ++g) {
        if (rcs[g] != MI355_OK) {
            set_last_error("rank " + std::to_string(g) + ": " + errs[g]);
            return rcs[g];
        }
    }
    fill_stats(st, outs, G, kind, 0);
    return MI355_OK;
}

thread_local mi355_multi_stats t_last_multi{};

// ---------------------------------------------------------------- one process per GPU
struct CommHandle {
    int world = 0, rank = 0, device = 0;
    ncclComm_t comm = nullptr;
    std::unique_ptr<RcclTransport> T;
};

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
    MH_RC(multi::require_rccl());
    auto h = std::make_unique<multi::CommHandle>();
    h->world = nranks;
    h->rank = rank;
    MH_HIP(hipGetDevice(&h->device));
    ncclUniqueId id;
    std::memcpy(&id, id128, sizeof(id));
    MH_NCCL(multi::rccl().CommInitRank(&h->comm, nranks, id, rank));
    h->T = std::make_unique<multi::RcclTransport>(nranks, rank, std::vector<ncclComm_t>{h->comm},
                                                  std::vector<int>{h->device});
    *comm = h.release();
    return MI355_OK;
}

int mi355_multi_comm_destroy(void *comm) {
    auto *h = static_cast<multi::CommHandle *>(comm);
    if (!h) return MI355_OK;
    h->T.reset();
    if (h->comm && multi::rccl().CommDestroy) (void)multi::rccl().CommDestroy(h->comm);
    delete h;
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
    if (opts && (opts->key_shift || opts->materialize)) {
        set_last_error("mi355_rho_join_sharded: key_shift and materialize must be 0");
        return MI355_ERR_INVALID;
    }
    MH_HIP(hipSetDevice(h->device));
    int status = MI355_OK;
    Context *ctx = current_context(&status);
    if (!ctx) return status;
    std::lock_guard<std::mutex> lk(ctx->mu);
    std::vector<multi::RankOut> outs(1);
    // the caller's stream (opts->stream or mi355_set_stream): R and S were produced there
    hipStream_t s = thread_stream(ctx, opts ? opts->stream : nullptr);
    MH_RC(multi::rank_join(*h->T, h->rank, ctx, s, R, nR, S, nS, opts, outs[0]));
    mi355_multi_stats local{};
    mi355_multi_stats *st = stats ? stats : &local;
    multi::fill_stats(st, outs, h->world, MI355_TRANSPORT_RCCL, h->rank);
    multi::t_last_multi = *st;
    mi355_rho_stats ls = outs[0].st;
    ls.matches = outs[0].global;
    rho::set_last_join_stats(ls);
    return MI355_OK;
}

}  // extern "C"
