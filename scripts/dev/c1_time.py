"""Development: BASELINE config 1 (2^20 x 2^20, device generators) on the small-join
path, per-call device span (the kernels' wall clock) and host wall time, medians of
`joins` calls.  SGXAMD_LIB_PATH selects a library variant.  Usage: python c1_time.py [joins]"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "sgxv2-analytical-query-processing-benchmarks_amd",
                                "python"))
import torch  # noqa: E402
import sgxamd  # noqa: E402

n = 1 << 20
R = torch.empty(n, dtype=torch.int64, device="cuda:0")
S = torch.empty(n, dtype=torch.int64, device="cuda:0")
sgxamd.gen_pk_dev(R, n, 0, n, 11111)
sgxamd.gen_fk_dev(S, n, 0, n, 22222)
torch.cuda.synchronize()
k = int(sys.argv[1]) if len(sys.argv) > 1 else 300
dev, wall = [], []
for i in range(k + 20):
    t0 = time.perf_counter()
    r = sgxamd.rho_join(R, n, S, n)
    t1 = time.perf_counter()
    assert r.matches == n
    if i >= 20:
        dev.append(r.stats["ms_total"] * 1000)
        wall.append((t1 - t0) * 1e6)
print(f"{os.environ.get('SGXAMD_LIB_PATH', 'base')}: device median {statistics.median(dev):.1f} us "
      f"(min {min(dev):.1f}), wall median {statistics.median(wall):.1f} us, plan {r.stats['radix_bits']} bits "
      f"{r.stats['passes']} passes", flush=True)
