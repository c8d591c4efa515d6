"""Multi-GPU RHO: radix-partition sharding with one all-to-all exchange.

One process per GPU (torch.distributed; backend "nccl" is RCCL over xGMI on
ROCm, "gloo" runs the same code on CPU tensors in tests).  Every rank holds a
contiguous slice of R and of S, like the reference's per-thread slices
(radix_join.cpp:1457-1500).  The exchange step replaces the reference's shared
tmpR/tmpS arrays (:1421-1433) across sockets:

  1. shard partition: stable radix partition of the local slice by destination
     d = key & (G - 1) (the low log2(G) key bits, i.e. pass-1 radix bits of
     radix_join.cpp:1118-1119 taken by the shard level);
  2. split exchange: all_to_all of the G per-destination counts;
  3. tuple exchange: all_to_all_single of the 8-byte tuples (viewed as int64); R's
     exchange is left in flight while S is shard-partitioned;
  4. local join of the received R' and S' with key_shift = log2(G) (all their keys
     agree on the low bits, so the local radix bits start above them);
  5. all_reduce(sum) of the match counts (exact: integer sum).

G must be a power of two.  The local compute (steps 1 and 4) defaults to the
HIP library; tests inject CPU restatements to run the exchange logic on gloo.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field

import torch
import torch.distributed as dist

from . import rho_join, shard_partition


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


def _default_partition(t: torch.Tensor, n: int, dest_bits: int):
    out = torch.empty_like(t)
    stream = torch.cuda.current_stream().cuda_stream if t.is_cuda else None
    counts = shard_partition(t, n, 0, dest_bits, out, stream)
    return out, counts


def _default_local_join(R: torch.Tensor, nR: int, S: torch.Tensor, nS: int, key_shift: int,
                        algorithm: str = "RHO"):
    stream = torch.cuda.current_stream().cuda_stream if R.is_cuda else None
    res = rho_join(R, nR, S, nS, key_shift=key_shift, stream=stream, algorithm=algorithm)
    return res.matches, res.stats


def _exchange(t: torch.Tensor, send_counts: list[int], group, async_op: bool = False):
    """all_to_all of the per-destination counts (blocking, tiny), then of the tuples.
    With async_op the tuple exchange is left in flight: (out, total, work)."""
    world = dist.get_world_size(group)
    dev = t.device
    sc = torch.tensor(send_counts, dtype=torch.int64, device=dev)
    rc = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_to_all_single(rc, sc, group=group)
    recv_counts = [int(x) for x in rc.tolist()]
    total = sum(recv_counts)
    out = torch.empty(max(total, 1), dtype=torch.int64, device=dev)
    work = dist.all_to_all_single(out[:total], t, recv_counts, send_counts, group=group, async_op=async_op)
    if async_op:
        return out, total, work
    return out, total


def sharded_rho_join(R: torch.Tensor, S: torch.Tensor, *, group=None, partition_fn=None,
                     local_join_fn=None, algorithm: str = "RHO") -> ShardedJoinResult:
    """Global RHO join of the row slices R and S (int64 tensors, one tuple each).

    Collective: every rank of `group` must call it.  Returns the global match count
    on every rank.
    """
    partition_fn = partition_fn or _default_partition
    if local_join_fn is None:
        def local_join_fn(R_, nR_, S_, nS_, shift_):
            return _default_local_join(R_, nR_, S_, nS_, shift_, algorithm)
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    dest_bits = _log2_exact(world)
    ms = {}
    sync = (lambda: torch.cuda.synchronize()) if R.is_cuda else (lambda: None)
    t0 = time.perf_counter()
    if world == 1:
        local, st = local_join_fn(R, R.numel(), S, S.numel(), 0)
        sync()
        ms["local_join"] = (time.perf_counter() - t0) * 1e3
        return ShardedJoinResult(int(local), int(local), R.numel(), S.numel(), ms, st)

    # R's tuple exchange (xGMI) runs while S is shard-partitioned (HBM): RCCL works on
    # its own stream, the partition kernels on the current one.
    pR, cR = partition_fn(R, R.numel(), dest_bits)
    rR, nR, wR = _exchange(pR, cR, group, async_op=True)
    pS, cS = partition_fn(S, S.numel(), dest_bits)
    t1 = time.perf_counter()
    ms["shard_partition"] = (t1 - t0) * 1e3
    rS, nS, wS = _exchange(pS, cS, group, async_op=True)
    wR.wait()
    wS.wait()
    sync()
    t2 = time.perf_counter()
    ms["exchange"] = (t2 - t1) * 1e3
    local, st = local_join_fn(rR, nR, rS, nS, dest_bits)
    sync()
    t3 = time.perf_counter()
    ms["local_join"] = (t3 - t2) * 1e3
    tot = torch.tensor([int(local)], dtype=torch.int64, device=R.device)
    dist.all_reduce(tot, op=dist.ReduceOp.SUM, group=group)
    ms["all_reduce"] = (time.perf_counter() - t3) * 1e3
    return ShardedJoinResult(int(tot.item()), int(local), nR, nS, ms, st)
