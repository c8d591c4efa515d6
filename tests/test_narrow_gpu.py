"""Narrow key partitions (rho_kernels.hip k_sort_blk / k_join_x, rho_host.cpp plan_join):
a counting RHO join over key partitions with the 16,384-key table writes its final
partitions as u16 residuals (key >> radix bits) when every key of the relation leaves a
residual below 2^16 (the key OR that pass 1 computes).  Within one partition the
residuals of two keys are equal exactly when the keys are (the partition fixes the low
radix bits), so the count is unchanged: each case runs against the oracle's sort-based
counter, with the widths the join took (stats["narrow"]: bit 0 R, bit 1 S).

The plans here are 9 = 5 + 4 bits over ~5 M R keys (about 10,000 R keys per partition:
the 16,384-key table), so the residual bound is 2^(9 + 16) = 2^25."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

DT = np.dtype([("key", "<u4"), ("payload", "<u4")])
BITS = 9
BOUND = 1 << (BITS + 16)  # first key whose residual needs 17 bits
CAP = (1 << 14) + 64  # k_join_n's counters (rho_kernels.hip kNarrowCap)


def rel(keys):
    x = np.empty(len(keys), dtype=DT)
    x["key"] = keys
    x["payload"] = np.arange(len(keys), dtype=np.uint32)
    return x


def keys_below(rng, n, hi):
    return rng.integers(0, hi, n, dtype=np.uint64).astype(np.uint32)


def case_relations(case, rng):
    nR, nS = 5_000_011, 5_200_003
    if case == "narrow":  # duplicates on both sides, every residual below 2^16
        R = keys_below(rng, nR, BOUND // 4)
        S = keys_below(rng, nS, BOUND // 4)
        return R, S, 3
    if case == "uneven":  # both narrow, R's residuals 9 bits wide, S's 16: S keys above R's range skip
        R = keys_below(rng, nR, 1 << (BITS + 9))
        S = np.concatenate([keys_below(rng, nS // 2, BOUND), keys_below(rng, nS - nS // 2, 1 << (BITS + 9))])
        return R, S, 3
    if case == "boundary":  # the largest narrow key on both sides (residual 0xFFFF)
        R = keys_below(rng, nR, BOUND)
        S = np.concatenate([keys_below(rng, nS - 3, BOUND), np.full(3, BOUND - 1, np.uint32)])
        R[:5] = BOUND - 1
        return R, S, 3
    if case == "cap":  # residuals up to k_join_n's table end (kNarrowCap - 1: the fast body)
        R = keys_below(rng, nR, CAP << BITS)
        S = keys_below(rng, nS, CAP << BITS)
        R[:3] = (CAP << BITS) - 1
        S[:2] = (CAP << BITS) - 1
        return R, S, 3
    if case == "cap_over":  # one residual past the table on both sides: two windows
        R = keys_below(rng, nR, CAP << BITS)
        S = keys_below(rng, nS, CAP << BITS)
        R[7] = CAP << BITS
        S[11:14] = CAP << BITS
        return R, S, 3
    if case == "hot_r":  # an R partition of four 16,384-key chunks (40,000 copies of one key, hot in S too)
        R = keys_below(rng, nR, BOUND // 4)
        S = keys_below(rng, nS, BOUND // 4)
        R[:40_000] = 77 << BITS | 5
        S[:3000] = 77 << BITS | 5
        return R, S, 3
    if case == "wide_s":
        # R narrow, S holds keys of 17+ bit residuals: among them, for R keys of sparse
        # partitions (few R keys: a short table, whose 16-bit tags stop below the top
        # residual bits), keys that share the bucket and the tag of an R key and differ
        # only in bit 31 — a tag match the build/probe must reject against R's residual
        # dense: partitions 0..255 (the low 9 bits below 256); sparse: 256..511
        dense = keys_below(rng, nR - 4000, BOUND) & np.uint32(~0x1FF & 0xFFFFFFFF)
        dense |= rng.integers(0, 256, len(dense)).astype(np.uint32)
        sparse = keys_below(rng, 4000, BOUND)
        sparse = (sparse & np.uint32(~0x1FF & 0xFFFFFFFF)) | (256 + rng.integers(0, 256, 4000)).astype(np.uint32)
        R = np.concatenate([dense, sparse])
        S = np.concatenate([keys_below(rng, nS - 8000, BOUND), sparse, sparse[:4000] | np.uint32(1 << 31)])
        return R, S, 1
    if case == "wide_r":  # one R key at the bound makes R wide; S stays narrow
        R = keys_below(rng, nR, BOUND)
        R[12345] = BOUND
        S = keys_below(rng, nS, BOUND)
        return R, S, 2
    assert case == "wide"  # full-range keys on both sides
    R = rng.integers(0, 2**32, nR, dtype=np.uint64).astype(np.uint32)
    S = np.concatenate([rng.integers(0, 2**32, nS - 100_000, dtype=np.uint64).astype(np.uint32),
                        R[:100_000]])
    return R, S, 0


CASES = ["narrow", "uneven", "boundary", "cap", "cap_over", "hot_r", "wide_s", "wide_r", "wide"]


@pytest.mark.parametrize("case", CASES)
def test_narrow_partitions_match_oracle(sgx, orc, gpu, case):
    rng = np.random.default_rng(40 + CASES.index(case))  # (seeds of the first three kept from round 4)
    Rk, Sk, narrow = case_relations(case, rng)
    R, S = rel(Rk), rel(Sk)
    exp = orc.count_join_sort(R, S)
    res = sgx.rho_join(R, len(R), S, len(S), radix_bits=BITS, passes=2)
    assert res.stats["max_part_r"] > 8192  # the 16,384-key table
    assert res.stats["narrow"] == narrow, (case, res.stats["narrow"])
    assert res.matches == exp, (case, res.matches, exp)
    # RHT over the same plan keeps 4-byte key partitions
    rht = sgx.rho_join(R, len(R), S, len(S), radix_bits=BITS, passes=2, algorithm="RHT")
    assert rht.matches == exp and rht.stats["narrow"] == 0


NARROW_POOL_CHILD = r"""
import sys
import numpy as np
import sgxamd, oracle
sys.path.insert(0, sys.argv[1])
import test_narrow_gpu as T
for i, case in enumerate(T.CASES):
    Rk, Sk, narrow = T.case_relations(case, np.random.default_rng(40 + i))
    R, S = T.rel(Rk), T.rel(Sk)
    res = sgxamd.rho_join(R, len(R), S, len(S), radix_bits=T.BITS, passes=2)
    assert res.stats["narrow"] == narrow and res.stats["layout"] == 4, (case, res.stats["narrow"], res.stats["layout"])
    assert res.matches == oracle.count_join_sort(R, S), case
print("narrow pool ok")
"""


def test_narrow_pool_matches_oracle():
    """SGXAMD_NARROW_POOL=1 (opt-in): pass 1 writes the narrow pool (16-bit residuals and
    their digit bytes), k_place_seg reads it; a relation with a residual past 16 bits
    (wide_s, wide_r, wide) repeats pass 1 as 4-byte keys behind the guards.  Every case
    above, in a child process (the switch is read once per process)."""
    import os
    import subprocess
    import sys

    from conftest import PKG, ROOT

    here = os.path.dirname(os.path.abspath(__file__))
    e = dict(os.environ, SGXAMD_NARROW_POOL="1")
    e["PYTHONPATH"] = os.pathsep.join([os.path.join(PKG, "python"), os.path.join(ROOT, "oracle"), here,
                                       e.get("PYTHONPATH", "")])
    r = subprocess.run([sys.executable, "-c", NARROW_POOL_CHILD, here], env=e, capture_output=True, text=True,
                       timeout=110)
    assert r.returncode == 0 and "narrow pool ok" in r.stdout, (r.stdout[-2000:], r.stderr[-2000:])

