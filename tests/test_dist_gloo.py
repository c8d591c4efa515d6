"""Multi-GPU sharded RHO (sgxamd.dist) exchange logic on CPU with gloo, world_size 2 and 4.

The local compute steps (shard partition, local join) are injected CPU
restatements from the oracle (test infrastructure); the split exchange, tuple
all-to-all and count all-reduce are the product code paths that run over RCCL
on the GPUs."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

DT = np.dtype([("key", "<u4"), ("payload", "<u4")])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, nR, nS, kind, q, chunks=4):
    import sys

    from conftest import PKG, ROOT

    sys.path.insert(0, os.path.join(PKG, "python"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    import sgxamd
    from sgxamd.dist import sharded_rho_join

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    if kind == "ref":
        R, S = sgxamd.reference_relations(nR, nS)
    else:
        rng = np.random.default_rng(11)
        R = np.empty(nR, dtype=DT)
        S = np.empty(nS, dtype=DT)
        R["key"] = rng.integers(0, 2**32, nR, dtype=np.uint64).astype(np.uint32) % 5000
        S["key"] = rng.integers(0, 2**32, nS, dtype=np.uint64).astype(np.uint32) % 5000
        R["payload"] = np.arange(nR)
        S["payload"] = np.arange(nS)
    expected = oracle.count_join_sort(R, S)

    def sl(x):  # contiguous rank slice, last rank takes the remainder (radix_join.cpp:1498)
        per = len(x) // world
        return x[rank * per: len(x) if rank == world - 1 else (rank + 1) * per].copy()

    Rl, Sl = sl(R), sl(S)
    seen = {}

    def partition_fn(t, n, dest_bits):
        arr = t.numpy().view(DT)
        out, starts = oracle.radix_partition(arr, 1, 0, dest_bits)
        return torch.from_numpy(out.view(np.int64).copy()), np.diff(starts).astype(np.int64).tolist()

    def local_join_fn(Rt, nr, St, ns, key_shift):
        r = Rt[:nr].numpy().view(DT)
        s = St[:ns].numpy().view(DT)
        mask = (1 << key_shift) - 1
        seen["low_bits_ok"] = bool(np.all((r["key"] & mask) == rank) and np.all((s["key"] & mask) == rank))
        return oracle.rho_join(r, s, 1)[0] if nr and ns else 0, {}

    res = sharded_rho_join(torch.from_numpy(Rl.view(np.int64)), torch.from_numpy(Sl.view(np.int64)),
                           partition_fn=partition_fn, local_join_fn=local_join_fn, chunks=chunks)
    # no local join runs on a rank that received no R or no S tuple
    seen.setdefault("low_bits_ok", res.recv_r == 0 or res.recv_s == 0)
    tot = torch.tensor([res.recv_r, res.recv_s], dtype=torch.int64)
    dist.all_reduce(tot)
    q.put((rank, res.matches, expected, seen.get("low_bits_ok"), tot.tolist()))
    dist.destroy_process_group()


# chunks: the shard partition + exchange in pieces (4), in one piece (1), and with
# slices too small for every rank to fill its pieces (empty pieces, uneven slices)
@pytest.mark.parametrize("world,nR,nS,kind,chunks", [(2, 1 << 14, 1 << 15, "ref", 4), (2, 9999, 7777, "dup", 4),
                                                     (4, 1 << 13, 1 << 13, "ref", 4), (2, 9999, 7777, "dup", 1),
                                                     (4, 7, 13, "dup", 4)])
def test_sharded_join_gloo(world, nR, nS, kind, chunks):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, nR, nS, kind, q, chunks)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, matches, expected, low_ok, tot in out:
        assert matches == expected, (rank, matches, expected)
        assert low_ok, rank  # each rank received exactly the keys of its shard
        assert tot == [nR, nS]  # every tuple was delivered exactly once


def _comm_init_worker(rank, world, port, fail, q):
    """_cxx_comm (the RCCL communicator set-up of sgxamd.dist) with the library calls
    replaced: rank 0's unique id fails ("uid"), or rank 1's communicator init ("init").
    Every rank must raise Mi355Error with a code (no TypeError, no rank left waiting)."""
    import sys

    from conftest import PKG

    sys.path.insert(0, os.path.join(PKG, "python"))
    import sgxamd
    import sgxamd.dist as D

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def uid():
        if fail == "uid":
            raise sgxamd.Mi355Error(-6, "cannot load librccl.so.1 (test)")
        return bytes(128)

    def init(u, n, r):
        if fail == "init" and r == 1:
            raise sgxamd.Mi355Error(-6, "ncclCommInitRank: unhandled system error (test)")
        return 1000 + r

    D.multi_unique_id, D.multi_comm_init = uid, init
    try:
        h = D._cxx_comm(None)
        out = ("ok", h)
    except sgxamd.Mi355Error as e:
        out = ("Mi355Error", e.code, str(e))
    except Exception as e:  # noqa: BLE001 - the test checks the type
        out = (type(e).__name__, str(e))
    q.put((rank, out))
    dist.destroy_process_group()


@pytest.mark.parametrize("fail", ["uid", "init", "none"])
def test_cxx_comm_init_failures_gloo(fail):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_comm_init_worker, args=(r, 2, port, fail, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=240) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    if fail == "none":
        assert out == {0: ("ok", 1000), 1: ("ok", 1001)}
        return
    for r in (0, 1):
        assert out[r][0] == "Mi355Error" and out[r][1] == -6, out
    if fail == "uid":
        assert all("unique id" in out[r][2] for r in (0, 1))
    else:
        assert "this rank" in out[1][2] and "some rank" in out[0][2]


def test_non_power_of_two_world_rejected():
    from sgxamd.dist import _log2_exact

    assert _log2_exact(8) == 3
    with pytest.raises(ValueError):
        _log2_exact(6)
