"""Development: pass-2 scatter kernel time at 2^28 (counts not checked: ablation
builds write nothing).  Run once per SGXAMD_SORT2 value (read once per process)."""
import os
import statistics
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "../../sgxv2-analytical-query-processing-benchmarks_amd/python")]
import torch  # noqa: E402

import sgxamd as sgx  # noqa: E402

n = 1 << 28
R = torch.empty(n, dtype=torch.int64, device="cuda")
S = torch.empty(n, dtype=torch.int64, device="cuda")
sgx.gen_pk_dev(R, n, 0, n, 11111)
sgx.gen_fk_dev(S, n, 0, n, 22222)
sgx.timing_enable(True)
t = {}
for i in range(7):
    m = sgx.rho_join(R, n, S, n).matches
    if i:
        for name, ms in sgx.timings():
            t.setdefault(name, []).append(ms)
print(os.environ.get("SGXAMD_SORT2", "-"), m == n,
      {x: round(statistics.median(t[x]), 4) for x in t if "pass2_scatter" in x}, flush=True)
