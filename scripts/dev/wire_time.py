"""Development: BASELINE config 4 / config 2-per-rank joins through the 8-rank rehearsal
(one GPU), u16 wire on or off (SGXAMD_WIRE16), to profile the sender-side passes and the
gather kernels (run under rocprofv3 --kernel-trace --stats).  The rehearsal's "wire" is
device memory, so the totals say nothing about xGMI; the kernel times do.
usage: python scripts/dev/wire_time.py [c4|c2] [reps] [G]   (c2: 2^28 R and S keys per rank)"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..",
                                "sgxv2-analytical-query-processing-benchmarks_amd", "python"))
import sgxamd  # noqa: E402

work = sys.argv[1] if len(sys.argv) > 1 else "c4"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
g = int(sys.argv[3]) if len(sys.argv) > 3 else 8
nR, nS = ((1 << 27), (1 << 30)) if work == "c4" else ((g << 28), (g << 28))
R = torch.empty(nR, dtype=torch.int64, device="cuda")
S = torch.empty(nS, dtype=torch.int64, device="cuda")
sgxamd.gen_pk_dev(R, nR, 0, nR, 11111)
sgxamd.gen_fk_dev(S, nS, 0, nR, 22222)
torch.cuda.synchronize()
for i in range(reps):
    t0 = time.perf_counter()
    res = sgxamd.rho_join_multi(R, nR, S, nS, g, transport="rehearsal")
    dt = (time.perf_counter() - t0) * 1e3
    st = res.stats
    assert res.matches == nS, res.matches
    print(f"{work} G={g} wire16={os.environ.get('SGXAMD_WIRE16', '1')} rep {i}: {dt:.1f} ms wall, "
          f"ms_total {st['ms_total']:.2f} post {st['ms_exchange_post']:.2f} local {st['ms_local']:.2f} "
          f"tail {st['ms_tail']:.2f} elem {st['elem_bytes']} sent {st['sent_bytes'] / 1e9:.3f} GB "
          f"bits {st['local']['radix_bits']}", flush=True)
sgxamd.multi_release()
