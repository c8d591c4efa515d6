"""Development: BASELINE config 4 over 8 RCCL-double ranks on one GPU, the tail after S's
last piece (ms_tail) of several consecutive joins, beside the one-GPU join's S side
(tests/test_rccl_double_gpu.py::test_inprocess_config4_full_size's bound is 1.5x it).
Usage: python scripts/dev/c4_double_tail.py [joins]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sgxv2-analytical-query-processing-benchmarks_amd", "python"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

import sgxamd  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
sgxamd.multi_set_rccl_library(os.path.join(ROOT, "tests", "rccl_double", "librccl_double.so"))
nR, nS = 1 << 27, 1 << 30
R = torch.empty(nR, dtype=torch.int64, device="cuda:0")
S = torch.empty(nS, dtype=torch.int64, device="cuda:0")
sgxamd.gen_pk_dev(R, nR, 0, nR, 11111)
sgxamd.gen_fk_dev(S, nS, 0, nR, 22222)
torch.cuda.synchronize()
sgxamd.timing_enable(True)
assert sgxamd.rho_join(R, nR, S, nS).matches == nS
s_side = sum(ms for name, ms in sgxamd.timings() if name.startswith("S_") or name.startswith("join"))
sgxamd.timing_enable(False)
tails = []
for _ in range(n):
    res = sgxamd.rho_join_multi(R, nR, S, nS, 8, transport="rccl")
    assert res.matches == nS
    tails.append(round(res.stats["ms_tail"], 2))
print("s_side", round(s_side, 2), "bound", round(1.5 * s_side, 2), "tails", tails, flush=True)
