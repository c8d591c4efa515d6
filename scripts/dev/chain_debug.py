"""Development: chain-histogram plans under skew, GPU count vs the sort counter, for
several hot-digit fractions (SGXAMD_POOL_SEGS / SGXAMD_CHAIN_HIST from the environment)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sgxv2-analytical-query-processing-benchmarks_amd", "python"),
                os.path.join(ROOT, "oracle")]
import oracle  # noqa: E402
import sgxamd  # noqa: E402

dt = np.dtype([("key", "<u4"), ("payload", "<u4")])
rng = np.random.default_rng(3)
R = np.zeros(1 << 20, dtype=dt)
R["key"] = rng.permutation(1 << 20).astype(np.uint32)
for frac in (0.0, 0.05, 0.2, 0.4, 0.6, 0.9, 1.0):
    for umax in (1 << 20, 1 << 21):
        S = np.zeros(1 << 22, dtype=dt)
        S["key"] = np.where(rng.random(len(S)) < frac, rng.integers(0, 8192, len(S)) * 128 + 9,
                            rng.integers(0, umax, len(S))).astype(np.uint32)
        exp = oracle.count_join_sort(R, S)
        r = sgxamd.rho_join(R, len(R), S, len(S), radix_bits=14, passes=2)
        print(f"frac {frac} umax {umax}: gpu {r.matches} exp {exp} {'OK' if r.matches == exp else 'MISMATCH'} "
              f"layout {r.stats['layout']} tasks {r.stats['num_tasks']} maxS {r.stats['max_part_s']}", flush=True)
