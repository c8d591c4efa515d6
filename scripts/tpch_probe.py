"""Development probe: run one TPC-H query repeatedly on device tables (for rocprofv3 traces)."""
import sys
import time

sys.path.insert(0, "sgxv2-analytical-query-processing-benchmarks_amd/python")
import torch  # noqa: E402
import sgxamd.tpch as T  # noqa: E402

q = int(sys.argv[1]) if len(sys.argv) > 1 else 3
sm = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
tb = T.generate_dev(sm, 42, device="cuda")
torch.cuda.synchronize()
for _ in range(reps):
    t0 = time.perf_counter()
    r = T.QUERIES[q](tb)
    print(q, round((time.perf_counter() - t0) * 1e3, 3), "ms wall", {k: r[k] for k in ("result", "filtered", "join_matches", "ms_selection", "ms_join", "ms_copy", "ms_total")})
