"""Host-path stamps of the config-2 step (development; needs the temporary dev_stamp
build): Python perf_counter_ns around bench.py's step next to the library's
steady_clock stamps (both CLOCK_MONOTONIC)."""
import os, sys, time
os.environ["SGXAMD_DEV_STAMPS"] = "1"
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "sgxv2-analytical-query-processing-benchmarks_amd", "python"))
import torch
import sgxamd
from sgxamd.dist import sharded_rho_join
dev = torch.device("cuda:0")
stream = torch.cuda.current_stream(dev).cuda_stream
n = 1 << 28
R = torch.empty(n, dtype=torch.int64, device=dev)
S = torch.empty(n, dtype=torch.int64, device=dev)
sgxamd.gen_pk_dev(R, n, 0, n, 11111, stream)
sgxamd.gen_fk_dev(S, n, 0, n, 22222, stream)
torch.cuda.synchronize()
for _ in range(3):
    sharded_rho_join(R, S)
sgxamd.timing_enable("sparse")
for mode in ("bench", "direct"):
    for i in range(8):
        a = time.perf_counter_ns()
        if mode == "bench":
            res = sharded_rho_join(R, S)
            t = sgxamd.timings()
        else:
            res = sgxamd.rho_join(R, n, S, n, stream=stream)
        b = time.perf_counter_ns()
        print("PY", mode, a, b, flush=True)
        sys.stderr.flush()
