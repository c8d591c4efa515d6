"""Development: per-join time of one workload over forced radix plans (HIP events around
the library call, device-resident inputs).  Usage: python scripts/dev/bits_sweep.py c4 14 15 16"""
import sys, os, statistics
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "sgxv2-analytical-query-processing-benchmarks_amd", "python"))
import torch
import sgxamd

wl = sys.argv[1]
bits = [int(b) for b in sys.argv[2:]] or [0]
nR, nS = {"c2": (1 << 28, 1 << 28), "c4": (1 << 27, 1 << 30)}[wl]
dev = torch.device("cuda:0")
R = torch.empty(nR, dtype=torch.int64, device=dev)
S = torch.empty(nS, dtype=torch.int64, device=dev)
sgxamd.gen_pk_dev(R, nR, 0, nR, 11111)
sgxamd.gen_fk_dev(S, nS, 0, nR, 22222)
torch.cuda.synchronize()
for rep in range(2):
    for b in bits:
        kw = {"radix_bits": b, "passes": 2} if b else {}
        res = sgxamd.rho_join(R, nR, S, nS, **kw)
        assert res.matches == nS, (b, res.matches)
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            sgxamd.rho_join(R, nR, S, nS, **kw)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        print(wl, "bits", b or "default", "rep", rep, "ms median", round(statistics.median(ts), 3), flush=True)
