"""Development: uint8 scan kernels at 2^32 entries (the reference's shapes): count,
bitvector (1 %) and index list (10 %) kernel times, against the int32 count at 2^30."""
import os
import statistics
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "../../sgxv2-analytical-query-processing-benchmarks_amd/python")]
import torch  # noqa: E402

import sgxamd as sgx  # noqa: E402

sgx.timing_enable(True)


def kt(fn, k=7):
    t = {}
    for i in range(k):
        fn()
        if i:
            for name, ms in sgx.timings():
                t.setdefault(name, []).append(ms)
    return {x: round(statistics.median(v), 4) for x, v in t.items()}


nu = 1 << 32
col = torch.empty(nu, dtype=torch.uint8, device="cuda")
sgx.gen_scan_dev(col, nu, 0, 0, "u8")
bv = torch.empty(nu // 64, dtype=torch.int64, device="cuda")
k10 = nu // 256 * 27
idx = torch.empty(k10, dtype=torch.int64, device="cuda")
for name, fn, byts in (
        ("u8 count [0,3]", lambda: sgx.scan_count(0, 3, col, nu, "u8"), nu),
        ("u8 bitvector [0,3]", lambda: sgx.scan_bitvector(0, 3, col, nu, bv, "u8"), nu + nu // 8),
        ("u8 index [0,26]", lambda: sgx.scan_index(0, 26, col, nu, idx, k10, "u8"), nu + 8 * k10)):
    t = kt(fn)
    main = max(t, key=t.get)
    print(name, t, f"{byts / (t[main] * 1e-3) / 1e12:.2f} TB/s", flush=True)
del col, bv, idx
ns = 1 << 30
c32 = torch.empty(ns, dtype=torch.int32, device="cuda")
sgx.gen_scan_dev(c32, ns, 0, 0, "i32")
t = kt(lambda: sgx.scan_count(0, 26, c32, ns))
print("i32 count", t, f"{4 * ns / (t['scan_count'] * 1e-3) / 1e12:.2f} TB/s", flush=True)
bv32 = torch.empty(ns // 64, dtype=torch.int64, device="cuda")
t = kt(lambda: sgx.scan_bitvector(0, 26, c32, ns, bv32))
print("i32 bitvector", t, f"{(4 * ns + ns // 8) / (t['scan_bitvector'] * 1e-3) / 1e12:.2f} TB/s", flush=True)
