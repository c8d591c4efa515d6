"""Multi-GPU RHO: radix-partition sharding with a pieced all-to-all exchange per relation.

One process per GPU (torch.distributed; backend "nccl" is RCCL over xGMI on
ROCm, "gloo" runs the same code on CPU tensors in tests).  Every rank holds a
contiguous slice of R and of S, like the reference's per-thread slices
(radix_join.cpp:1457-1500).  The exchange step replaces the reference's shared
tmpR/tmpS arrays (:1421-1433) across sockets:

  1. shard partition: stable radix partition of the local slice by destination
     d = key & (G - 1) (the low log2(G) key bits, i.e. pass-1 radix bits of
     radix_join.cpp:1118-1119 taken by the shard level);
  2. split exchange: all_to_all of the G per-destination counts (host integers, on
     a gloo side group so they never queue behind a tuple exchange on the RCCL
     stream);
  3. tuple exchange: all_to_all_single of the 8-byte tuples (viewed as int64);
  4. local join of the received R' and S' with key_shift = log2(G) (all their keys
     agree on the low bits, so the local radix bits start above them);
  5. all_reduce(sum) of the match counts (exact: integer sum).

Pipelining (one timeline per rank; RCCL runs on its own stream):

    compute:  R0 | R1 R2 R3 S0 S1 S2 S3 | ..... R' local passes | S' local passes, build/probe
    xGMI:        | R exchange (4 chunks) ........| S exchange (4 chunks) ..|

Each relation is shard-partitioned in `chunks` contiguous pieces; a piece's tuple
all-to-all is posted as soon as its counts are known, so R is on the wire after the
first piece instead of after the whole shard pass, and the other pieces (and all of S)
are partitioned meanwhile.  R's local partition passes (mi355_rho_join_begin) run
while S is on the wire; S's passes and the build/probe (mi355_rho_join_finish) follow
S's arrival in stream order.  The pieces of one relation land back to back in one
receive buffer (sized for the worst case, every sender's piece coming to this rank:
world x the local slice), so R' and S' are contiguous for the local join.

G must be a power of two.  The local compute (steps 1 and 4) defaults to the
HIP library; tests inject CPU restatements to run the exchange logic on gloo.

With the "nccl" backend (RCCL) and device tensors the whole pipeline runs in C++
(sgxamd/multi.h, mi355_rho_join_sharded): this module only hands rank 0's RCCL unique
id to the other ranks and calls the library, whose rank pipeline is the one above
(pieced shard partition, all-gather of the piece counts on a second communicator,
send/recv of the tuples on a communication stream, pipelined local join, all-reduce).
If it fails, every rank raises (there is no silent fallback).  SGXAMD_DIST_IMPL=python
selects the torch.distributed implementation below explicitly; the gloo tests
exercise it.
"""
from __future__ import annotations

import contextlib
import os
import sys
import time
from dataclasses import dataclass, field

import torch
import torch.distributed as dist

from . import (Mi355Error, multi_comm_init, multi_unique_id, rho_join, rho_join_begin, rho_join_finish,
               rho_join_sharded, shard_partition)

MI355_ERR_COMM = -6  # sgxamd/multi.h


def _log2_exact(g: int) -> int:
    b = g.bit_length() - 1
    if (1 << b) != g:
        raise ValueError(f"world size {g} is not a power of two")
    return b


@dataclass
class ShardedJoinResult:
    matches: int
    local_matches: int
    recv_r: int
    recv_s: int
    ms: dict = field(default_factory=dict)
    local_stats: dict = field(default_factory=dict)
    # this rank's exchange record: world, transport, sent_bytes, elem_bytes and the
    # ms_exchange_post / ms_local / ms_allreduce phases (mi355_multi_stats in C++)
    multi: dict = field(default_factory=dict)


class _Done:
    """Completed exchange (gloo staging is synchronous)."""

    def wait(self):
        return None


def _stream_of(t: torch.Tensor):
    return torch.cuda.current_stream(t.device).cuda_stream if t.is_cuda else None


def _default_partition(t: torch.Tensor, n: int, dest_bits: int):
    out = torch.empty_like(t)
    counts = shard_partition(t, n, 0, dest_bits, out, _stream_of(t))
    return out, counts


class _LibraryLocalJoin:
    """Local join through the pipelined C-ABI: begin (R's passes, asynchronous) and
    finish (S's passes + build/probe, blocking)."""

    def __init__(self, algorithm: str):
        self.algorithm = algorithm
        self.shift = 0

    def begin(self, R, nR, nS, shift):
        self.shift = shift
        if R.is_cuda:
            rho_join_begin(R, nR, nS, key_shift=shift, stream=_stream_of(R), algorithm=self.algorithm)
        else:  # host tensors: one blocking call in finish
            self.R, self.nR = R, nR

    def finish(self, S, nS):
        if S.is_cuda:
            res = rho_join_finish(S, nS, key_shift=self.shift, stream=_stream_of(S), algorithm=self.algorithm)
        else:
            res = rho_join(self.R, self.nR, S, nS, key_shift=self.shift, algorithm=self.algorithm)
        return res.matches, res.stats

    def join(self, R, S):
        """One rank: the whole join in one library call (no exchange to overlap R's passes
        with; 2.396 vs 2.402 ms per config-2 step for begin + finish, and bench.py's step
        was 2.413 through them, scripts/dev/host_gap.py)."""
        res = rho_join(R, R.numel(), S, S.numel(), stream=_stream_of(R) if R.is_cuda else None,
                       algorithm=self.algorithm)
        return res.matches, res.stats


class _InjectedLocalJoin:
    """A caller-supplied local_join_fn(R, nR, S, nS, shift) seen through begin/finish."""

    def __init__(self, fn):
        self.fn = fn

    def begin(self, R, nR, nS, shift):
        self.args = (R, nR, shift)

    def finish(self, S, nS):
        R, nR, shift = self.args
        return self.fn(R, nR, S, nS, shift)


@contextlib.contextmanager
def stdout_to_stderr():
    """Route file descriptor 1 to 2 for the duration (gloo's connection banner is
    printed to stdout by native code; bench.py's stdout carries exactly one JSON line)."""
    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


_count_groups: dict = {}


def _count_group(group):
    """A gloo group over the same ranks for the host-side count exchanges (created
    collectively on first use, cached)."""
    backend = dist.get_backend(group)
    if backend == "gloo":
        return group
    key = id(group)
    if key not in _count_groups:
        ranks = None if group is None else dist.get_process_group_ranks(group)
        with stdout_to_stderr():
            _count_groups[key] = dist.new_group(ranks=ranks, backend="gloo")
    return _count_groups[key]


def _exchange_counts(send_counts: list[int], cgroup) -> list[int]:
    world = dist.get_world_size(cgroup)
    sc = torch.tensor(send_counts, dtype=torch.int64)
    rc = torch.empty(world, dtype=torch.int64)
    dist.all_to_all_single(rc, sc, group=cgroup)
    return [int(x) for x in rc.tolist()]


class _Exchange:
    """One relation's chunked shard partition + tuple all-to-all (see the module doc)."""

    def __init__(self, t: torch.Tensor, dest_bits: int, partition_fn, cgroup, group, chunks: int):
        world = 1 << dest_bits
        n = t.numel()
        chunks = max(1, chunks)
        # every rank makes exactly `chunks` pieces (some may be empty), so all ranks issue
        # the same sequence of collectives whatever their slice sizes
        per = -(-n // chunks)
        self.bounds = [(min(n, i * per), min(n, (i + 1) * per)) for i in range(chunks)]
        # worst case for the receive buffer: every rank's piece i comes to this rank, and
        # no rank's piece is larger than the largest slice's
        nmax = torch.tensor([n], dtype=torch.int64)
        dist.all_reduce(nmax, op=dist.ReduceOp.MAX, group=cgroup)
        cap = world * chunks * -(-int(nmax.item()) // chunks)
        self.out = torch.empty(max(cap, 1), dtype=torch.int64, device=t.device)
        self.world = world
        self.rank = dist.get_rank(group)
        self.sent = 0  # elements sent to other ranks
        self.total = 0
        self.works = []
        self.keep = []  # send buffers stay alive until their exchange completed
        self.t, self.dest_bits, self.partition_fn = t, dest_bits, partition_fn
        self.cgroup, self.group = cgroup, group

    def piece(self, i: int) -> None:
        a, b = self.bounds[i]
        if b > a:
            p, c = self.partition_fn(self.t[a:b], b - a, self.dest_bits)
        else:
            p, c = self.t[:0], [0] * self.world
        rc = _exchange_counts(c, self.cgroup)
        self.sent += sum(c) - c[self.rank]
        got = sum(rc)
        dst = self.out[self.total:self.total + got]
        self.total += got
        self.works.append(_post_exchange(dst, p, c, rc, self.group))
        self.keep.append(p)

    def wait(self) -> None:
        for w in self.works:
            w.wait()


def _post_exchange(dst: torch.Tensor, src: torch.Tensor, send_counts: list[int], recv_counts: list[int], group):
    """all_to_all_single of one piece into dst, left in flight; a gloo group with device
    tensors (single-GPU rehearsal) stages through host memory synchronously."""
    ns, nr = sum(send_counts), sum(recv_counts)
    if src.is_cuda and dist.get_backend(group) == "gloo":
        host = torch.empty(max(nr, 1), dtype=torch.int64)
        dist.all_to_all_single(host[:nr], src[:ns].cpu(), recv_counts, send_counts, group=group)
        dst[:nr].copy_(host[:nr])
        return _Done()
    return dist.all_to_all_single(dst[:nr], src[:ns], recv_counts, send_counts, group=group, async_op=True)


_comms: dict = {}


def _agree_ok(ok: bool, group) -> bool:
    """True on every rank iff `ok` on every rank (a MAX all-reduce of the failure flag on
    the host-side count group)."""
    flag = torch.tensor([0 if ok else 1], dtype=torch.int64)
    dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=_count_group(group))
    return int(flag.item()) == 0


def _cxx_comm(group) -> int:
    """This rank's RCCL communicator of the C++ path for `group` (collective on first use).

    Rank 0's unique id travels with its error, if any, so a failure there ends the call
    on every rank; after the communicator init every rank agrees on the outcome before
    any rank returns a handle (a rank that raised alone would leave its peers waiting in
    the join's first collective)."""
    key = id(group)
    if key not in _comms:
        if os.environ.get("SGXAMD_RCCL_LIBRARY"):  # tests: the RCCL test double (tests/rccl_double)
            from . import multi_set_rccl_library

            multi_set_rccl_library(os.environ["SGXAMD_RCCL_LIBRARY"])
        rank = dist.get_rank(group)
        obj = [None]
        if rank == 0:
            try:
                obj[0] = ("ok", multi_unique_id())
            except Mi355Error as e:
                obj[0] = ("error", str(e))
        src = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast_object_list(obj, src=src, group=group)
        status, payload = obj[0]
        if status != "ok":
            raise Mi355Error(MI355_ERR_COMM, f"sgxamd.dist: rank 0 could not create the RCCL unique id: {payload}")
        handle, err = None, None
        try:
            handle = multi_comm_init(payload, dist.get_world_size(group), rank)
        except Mi355Error as e:
            err = e
        if not _agree_ok(err is None, group):
            raise Mi355Error(err.code if err else MI355_ERR_COMM,
                             "sgxamd.dist: RCCL communicator init failed on some rank"
                             + (f" (this rank: {err})" if err else ""))
        _comms[key] = handle
    return _comms[key]


def _use_cxx(R: torch.Tensor, group, partition_fn, local_join_fn) -> bool:
    """The C++ RCCL path: a torch nccl (RCCL) group, or any torch backend with
    SGXAMD_DIST_IMPL=cxx-any -- the test rehearsal of rank processes sharing one GPU on
    the RCCL test double (gloo carries only the unique id's broadcast there)."""
    impl = os.environ.get("SGXAMD_DIST_IMPL", "cxx")
    return (R.is_cuda and partition_fn is None and local_join_fn is None
            and ((impl == "cxx" and dist.get_backend(group) == "nccl") or impl == "cxx-any"))


def _sharded_cxx(R: torch.Tensor, S: torch.Tensor, group, algorithm: str, chunks: int) -> ShardedJoinResult:
    from . import multi_set_pieces

    h = _cxx_comm(group)
    multi_set_pieces(chunks)
    t0 = time.perf_counter()
    res = rho_join_sharded(h, R, R.numel(), S, S.numel(), algorithm=algorithm)
    st = res.stats
    ms = {"total": (time.perf_counter() - t0) * 1e3, "shard_partition_and_post_exchange": st["ms_exchange_post"],
          "exchange_wait_and_local_join": st["ms_local"], "all_reduce": st["ms_allreduce"],
          "impl": "cxx-rccl (mi355_rho_join_sharded), "
                  + ("keys only: 4 B per tuple on xGMI (counting join)" if st.get("elem_bytes") == 4
                     else "8-byte tuples on xGMI"),
          "sent_bytes": st["sent_bytes"]}
    multi = {k: v for k, v in st.items() if k != "local"}
    return ShardedJoinResult(res.matches, int(st["local_matches"]), int(st["recv_r_max"]), int(st["recv_s_max"]), ms,
                             st["local"], multi)


def sharded_rho_join(R: torch.Tensor, S: torch.Tensor, *, group=None, partition_fn=None,
                     local_join_fn=None, algorithm: str = "RHO", chunks: int = 4) -> ShardedJoinResult:
    """Global RHO join of the row slices R and S (int64 tensors, one tuple each).

    Collective: every rank of `group` must call it (with the same `chunks`).  Returns
    the global match count on every rank.
    """
    # (decided before partition_fn takes its default: an injected partition or local join
    # selects the torch.distributed path; round 6 found this test after the default, so the
    # C++ RCCL path was never taken -- tests/test_rccl_double_gpu.py::
    # test_bench_rank_processes_on_double runs bench.py's ranks through it now)
    cxx = _use_cxx(R, group, partition_fn, local_join_fn) if dist.is_initialized() else False
    partition_fn = partition_fn or _default_partition
    local = _InjectedLocalJoin(local_join_fn) if local_join_fn is not None else _LibraryLocalJoin(algorithm)
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    dest_bits = _log2_exact(world)
    ms = {}
    sync = (lambda: torch.cuda.synchronize()) if R.is_cuda else (lambda: None)
    t0 = time.perf_counter()
    if world == 1:
        if isinstance(local, _LibraryLocalJoin):  # (blocking: no device synchronisation after it)
            m, st = local.join(R, S)
        else:
            local.begin(R, R.numel(), S.numel(), 0)
            m, st = local.finish(S, S.numel())
            sync()
        ms["local_join"] = (time.perf_counter() - t0) * 1e3
        return ShardedJoinResult(int(m), int(m), R.numel(), S.numel(), ms, st)

    if cxx:
        # RCCL through the C++ library; torch's stream is synchronised first (the library
        # runs on its own streams unless mi355_set_stream named torch's).  A failure
        # raises: the library fails every rank at the same collective step, so no rank
        # is left inside a collective, and a failing product path never yields a number
        # from a different implementation.
        torch.cuda.current_stream(R.device).synchronize()
        return _sharded_cxx(R, S, group, algorithm, chunks)
    cgroup = _count_group(group)
    # R piece by piece: each piece's exchange is in flight on the RCCL stream while the
    # next pieces (and then S) are shard-partitioned on the compute stream
    xR = _Exchange(R, dest_bits, partition_fn, cgroup, group, chunks)
    xS = _Exchange(S, dest_bits, partition_fn, cgroup, group, chunks)
    for i in range(len(xR.bounds)):
        xR.piece(i)
    for i in range(len(xS.bounds)):
        xS.piece(i)
    t1 = time.perf_counter()
    ms["shard_partition_and_post_exchange"] = (t1 - t0) * 1e3  # host time; pieces are on the wire
    rR, nR, rS, nS = xR.out, xR.total, xS.out, xS.total
    # R's local passes once R has arrived (stream order), while S is on the wire
    xR.wait()
    if nR and nS:
        local.begin(rR, nR, nS, dest_bits)
        xS.wait()
        m, st = local.finish(rS, nS)
    else:
        xS.wait()
        m, st = 0, {}
    sync()
    t2 = time.perf_counter()
    ms["exchange_wait_and_local_join"] = (t2 - t1) * 1e3
    tot = torch.tensor([int(m)], dtype=torch.int64)
    dist.all_reduce(tot, op=dist.ReduceOp.SUM, group=cgroup)
    ms["all_reduce"] = (time.perf_counter() - t2) * 1e3
    multi = {"world": world, "transport": f"torch.distributed {dist.get_backend(group)} (sgxamd.dist python)",
             "rank": dist.get_rank(group), "pieces": len(xR.bounds), "elem_bytes": 8,
             "sent_bytes": 8 * (xR.sent + xS.sent), "recv_r": nR, "recv_s": nS,
             "ms_exchange_post": ms["shard_partition_and_post_exchange"],
             "ms_local": ms["exchange_wait_and_local_join"], "ms_allreduce": ms["all_reduce"]}
    # keep the send buffers alive until both exchanges completed
    del xR, xS
    return ShardedJoinResult(int(tot.item()), int(m), nR, nS, ms, st, multi)
