"""Development: per-kernel times of the 2^28 counting join without the count check (for
ablation builds loaded through SGXAMD_LIB_PATH)."""
import os, sys, statistics
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "../../sgxv2-analytical-query-processing-benchmarks_amd/python")]
import torch
import sgxamd
n = 1 << 28
torch.cuda.set_device(0)
s = torch.cuda.current_stream().cuda_stream
sgxamd.set_stream(s)
sgxamd.timing_enable(True)
R = torch.empty(n, dtype=torch.int64, device="cuda"); S = torch.empty(n, dtype=torch.int64, device="cuda")
sgxamd.gen_pk_dev(R, n, 0, n, 11111, s); sgxamd.gen_fk_dev(S, n, 0, n, 22222, s); torch.cuda.synchronize()
acc = {}
for i in range(6):
    r = sgxamd.rho_join(R, n, S, n)
    if i:
        for k, v in sgxamd.timings(): acc.setdefault(k, []).append(v)
print(os.environ.get("SGXAMD_LIB_PATH", "base"), "matches", r.matches, {k: round(statistics.mean(v), 4) for k, v in acc.items() if "scatter" in k or "join_b" in k or "hist" in k})
