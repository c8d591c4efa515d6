"""Development: host time around one config-2 join (2^28 x 2^28 on one GPU), per step,
for the call paths bench.py and the library offer: sharded_rho_join (bench.py's step),
rho_join_begin + rho_join_finish, and rho_join (one call); with and without sparse
timing.  Usage: python scripts/dev/host_gap.py [steps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sgxv2-analytical-query-processing-benchmarks_amd", "python")]
import torch  # noqa: E402

import sgxamd  # noqa: E402
from sgxamd.dist import sharded_rho_join  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
n = 1 << 28
R = torch.empty(n, dtype=torch.int64, device="cuda:0")
S = torch.empty(n, dtype=torch.int64, device="cuda:0")
sgxamd.gen_pk_dev(R, n, 0, n, 11111)
sgxamd.gen_fk_dev(S, n, 0, n, 22222)
torch.cuda.synchronize()
stream = torch.cuda.current_stream().cuda_stream
sgxamd.set_stream(stream)
paths = {
    "sharded": lambda: sharded_rho_join(R, S).matches,
    "begin_finish": lambda: (sgxamd.rho_join_begin(R, n, n, stream=stream),
                             sgxamd.rho_join_finish(S, n, stream=stream).matches)[1],
    "one_call": lambda: sgxamd.rho_join(R, n, S, n, stream=stream).matches,
}
for timing in (False, "sparse"):
    sgxamd.timing_enable(timing)
    for name, f in paths.items():
        for _ in range(3):
            assert f() == n
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            f()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / K * 1e3
        print(f"timing={timing!s:6s} {name:13s} {dt:.4f} ms/step", flush=True)
