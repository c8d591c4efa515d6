"""Development: 2^20 x 2^20 joins (BASELINE config 1 shape, device generators) for a
rocprofv3 kernel-trace of the small-join path.  Usage: python scripts/dev/c1_prof.py [joins]"""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "sgxv2-analytical-query-processing-benchmarks_amd", "python"))
import torch
import sgxamd

n = 1 << 20
R = torch.empty(n, dtype=torch.int64, device="cuda:0")
S = torch.empty(n, dtype=torch.int64, device="cuda:0")
sgxamd.gen_pk_dev(R, n, 0, n, 11111)
sgxamd.gen_fk_dev(S, n, 0, n, 22222)
torch.cuda.synchronize()
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 50):
    assert sgxamd.rho_join(R, n, S, n).matches == n
print("ok")
