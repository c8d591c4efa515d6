"""Development: does a pass-1 scatter's time follow its data or its buffers?  The same
2^28 join on device-generated relations, then (workspace released) on the reference's
host-generated relations, then on the device relations again; S / R pass-1 times."""
import os
import statistics
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "../../sgxv2-analytical-query-processing-benchmarks_amd/python")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import sgxamd as sgx  # noqa: E402

n = 1 << 28
sgx.timing_enable(True)


def run(tag, R, S, k=6):
    t = {}
    for _ in range(k):
        assert sgx.rho_join(R, n, S, n).matches == n
        for name, ms in sgx.timings():
            t.setdefault(name, []).append(ms)
    print(tag, {x: round(statistics.median(t[x]), 4) for x in t if "pass1_scatter" in x or "build" in x}, flush=True)


Rd = torch.empty(n, dtype=torch.int64, device="cuda")
Sd = torch.empty(n, dtype=torch.int64, device="cuda")
sgx.gen_pk_dev(Rd, n, 0, n, 11111)
sgx.gen_fk_dev(Sd, n, 0, n, 22222)
run("device", Rd, Sd)
Rh, Sh = sgx.reference_relations(n, n)
Rr = torch.from_numpy(Rh.view(np.int64)).cuda()
Sr = torch.from_numpy(Sh.view(np.int64)).cuda()
run("reference (same workspace)", Rr, Sr)
run("device (same workspace)", Rd, Sd)
sgx.release_workspace()
run("reference (fresh workspace)", Rr, Sr)
run("device (fresh workspace)", Rd, Sd)
run("S=device R=reference", Rr, Sd)
run("S=reference R=device", Rd, Sr)
# the same S data in a fresh allocation
Sd2 = Sd.clone()
del Sd
run("device S cloned", Rd, Sd2)
