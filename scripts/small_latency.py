"""Small-join latency (BASELINE config 1's shape and below): per-kernel device times and
wall time per call for device-resident pk/fk relations, on one GPU."""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "sgxv2-analytical-query-processing-benchmarks_amd", "python"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import sgxamd  # noqa: E402

torch.cuda.set_device(0)
stream = torch.cuda.current_stream().cuda_stream
sgxamd.set_stream(stream)
sgxamd.timing_enable(os.environ.get("SMALL_TIMING", "1") == "1")
for lg in [int(x) for x in os.environ.get("SMALL_LGS", "14,16,18,20,22").split(",")]:
    n = 1 << lg
    R, S = sgxamd.reference_relations(n, n) if lg <= 20 else (None, None)
    if R is not None:
        dR = torch.from_numpy(R.view(np.int64)).cuda()
        dS = torch.from_numpy(S.view(np.int64)).cuda()
    else:
        dR = torch.empty(n, dtype=torch.int64, device="cuda")
        dS = torch.empty(n, dtype=torch.int64, device="cuda")
        sgxamd.gen_pk_dev(dR, n, 0, n, 11111, stream)
        sgxamd.gen_fk_dev(dS, n, 0, n, 22222, stream)
    torch.cuda.synchronize()
    for _ in range(5):
        assert sgxamd.rho_join(dR, n, dS, n, stream=stream).matches == n
    per = {}
    walls = []
    for _ in range(30):
        t0 = time.perf_counter()
        res = sgxamd.rho_join(dR, n, dS, n, stream=stream)
        walls.append(time.perf_counter() - t0)
        for k, ms in sgxamd.timings():
            per.setdefault(k, []).append(ms)
    ks = {k: round(statistics.median(v) * 1e3, 1) for k, v in per.items()}
    print(f"2^{lg}: wall median {statistics.median(walls) * 1e6:.1f} us, kernel sum {sum(ks.values()):.1f} us, "
          f"bits {res.stats['radix_bits']} passes {res.stats['passes']}: {ks}", flush=True)
