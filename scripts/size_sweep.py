"""RHO throughput against relation size (|R| = |S| = n, pk/fk, device-resident), and
at the largest sizes the radix-bit splits the planner could take, to check that the
plan chosen past 2^28 is the fastest one.  Development measurement, not a bench input:

    python3 scripts/size_sweep.py [--auto] [log2 sizes ...]   (default 24 26 28 29 30 31)
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "sgxv2-analytical-query-processing-benchmarks_amd",
                                "python"))
import torch  # noqa: E402

import sgxamd  # noqa: E402


def timed(R, S, n, reps, **kw):
    res = sgxamd.rho_join(R, n, S, n, **kw)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        r = sgxamd.rho_join(R, n, S, n, **kw)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) * 1e3 / reps
    assert r.matches == n, (n, kw, r.matches)
    return ms, res.stats


def main():
    auto_only = "--auto" in sys.argv
    logs = [int(a) for a in sys.argv[1:] if a != "--auto"] or [24, 26, 28, 29, 30, 31]
    for lg in logs:
        n = 1 << lg
        R = torch.empty(n, dtype=torch.int64, device="cuda")
        S = torch.empty(n, dtype=torch.int64, device="cuda")
        sgxamd.gen_pk_dev(R, n, 0, n, 11111)
        sgxamd.gen_fk_dev(S, n, 0, n, 22222)
        reps = max(3, min(20, (1 << 30) // n))
        plans = [{}]
        if os.environ.get("SWEEP_BITS"):  # e.g. SWEEP_BITS=13,14,15,16
            plans += [{"radix_bits": int(b), "passes": 2} for b in os.environ["SWEEP_BITS"].split(",")]
        elif lg >= 29 and not auto_only:
            plans += [{"radix_bits": b, "passes": 2} for b in (16, 17, 18)]
        for kw in plans:
            ms, st = timed(R, S, n, reps, **kw)
            print(f"n=2^{lg} plan={kw or 'auto'} bits={st['radix_bits']} passes={st['passes']} "
                  f"{ms:.3f} ms  {n / ms / 1e3:.0f} M S-tuples/s", flush=True)
        del R, S
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
