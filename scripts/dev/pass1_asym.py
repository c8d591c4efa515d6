"""Development: where the S / R pass-1 asymmetry of the c2 bench comes from.  Times the
pass-1 scatter of both roles with the relations swapped, S copied to a fresh allocation,
and two pk relations (no fk).  usage: python scripts/dev/pass1_asym.py [reps]"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..",
                                "sgxv2-analytical-query-processing-benchmarks_amd", "python"))
import sgxamd  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
n = 1 << 28
R = torch.empty(n, dtype=torch.int64, device="cuda")
S = torch.empty(n, dtype=torch.int64, device="cuda")
sgxamd.gen_pk_dev(R, n, 0, n, 11111)
sgxamd.gen_fk_dev(S, n, 0, n, 22222)
torch.cuda.synchronize()
stream = torch.cuda.current_stream().cuda_stream
sgxamd.set_stream(stream)
sgxamd.timing_enable(True)


def run(name, A, B):
    per = {}
    for i in range(reps + 1):
        sgxamd.rho_join(A, n, B, n)
        if i == 0:
            continue
        for k, ms in sgxamd.timings():
            per.setdefault(k, []).append(ms)
    print(name, {k: round(statistics.mean(v), 4) for k, v in per.items() if "pass1_scatter" in k}, flush=True)


run("R=pk S=fk", R, S)
run("R=fk S=pk (swapped)", S, R)
S2 = S.clone()
torch.cuda.synchronize()
run("R=pk S=fk copy", R, S2)
P2 = torch.empty(n, dtype=torch.int64, device="cuda")
sgxamd.gen_pk_dev(P2, n, 0, n, 33333)
torch.cuda.synchronize()
run("R=pk S=pk2", R, P2)
run("R=fk S=fk", S, S2)
