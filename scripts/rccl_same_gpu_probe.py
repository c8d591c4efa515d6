"""Probe: can two RCCL ranks share one GPU on this box?  (torchrun --nproc-per-node 2,
both ranks on cuda:0, backend nccl; then the C++ path's communicator on the same GPU.)"""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "sgxv2-analytical-query-processing-benchmarks_amd", "python"))
rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
t = torch.ones(4, device="cuda") * (rank + 1)
dist.all_reduce(t)
print(f"rank {rank}: torch nccl all_reduce -> {t.tolist()}", flush=True)
import numpy as np  # noqa: E402

import sgxamd  # noqa: E402

R, S = sgxamd.reference_relations(1 << 16, 1 << 16)
n = len(R) // 2
dR = torch.from_numpy(R.view(np.int64)[rank * n:(rank + 1) * n]).cuda()
dS = torch.from_numpy(S.view(np.int64)[rank * n:(rank + 1) * n]).cuda()
os.environ["SGXAMD_DIST_IMPL"] = "cxx"
from sgxamd.dist import sharded_rho_join  # noqa: E402

res = sharded_rho_join(dR, dS)
print(f"rank {rank}: sharded join matches {res.matches} impl {res.ms.get('impl', 'python')}", flush=True)
dist.destroy_process_group()
