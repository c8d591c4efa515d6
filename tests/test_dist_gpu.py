"""Single-GPU rehearsal of the multi-rank path: world_size 2 and 4 processes share
cuda:0 and exchange over gloo (device tensors staged through host memory), running
the product's shard partition and pipelined local join kernels (sgxamd.dist).  The
RCCL transport itself needs one GPU per rank and only runs in the 8-GPU bench."""
import os
import socket

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, workload, q):
    import sys

    from conftest import PKG

    sys.path.insert(0, os.path.join(PKG, "python"))
    import torch
    import torch.distributed as dist

    import sgxamd
    from sgxamd.dist import sharded_rho_join

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    stream = torch.cuda.current_stream().cuda_stream
    gR = gS = n * world
    R = torch.empty(n, dtype=torch.int64, device="cuda")
    S = torch.empty(n, dtype=torch.int64, device="cuda")
    sgxamd.gen_pk_dev(R, n, rank * n, gR, 11111, stream)
    if workload == "zipf":
        sgxamd.gen_zipf_dev(S, n, rank * n, gR, 0.75, 22222, stream)
    else:
        sgxamd.gen_fk_dev(S, n, rank * n, gR, 22222, stream)
    torch.cuda.synchronize()
    out = []
    for _ in range(2):  # twice: the library's grow-only workspace is reused
        res = sharded_rho_join(R, S)
        out.append((res.matches, res.recv_r, res.recv_s))
    q.put((rank, out, gS))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n,workload", [(2, 1 << 20, "fk"), (4, 1 << 18, "zipf")])
def test_sharded_join_on_gpu_over_gloo(world, n, workload):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, workload, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=100) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    recv_r = [0, 0]
    recv_s = [0, 0]
    for rank, out, expected in outs:
        for i, (m, rr, rs) in enumerate(out):
            assert m == expected, (rank, m, expected)  # every S tuple matches one R tuple
            recv_r[i] += rr
            recv_s[i] += rs
    assert recv_r == [n * world] * 2 and recv_s == [n * world] * 2
