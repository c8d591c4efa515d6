"""Pin the CPU oracle (test infrastructure) before trusting it.

Join: no reference test or golden vector exists for any join and
running the reference was denied, so the restatement is pinned by the analytical
known-answer tests derived from the reference's generators and by an independent
sort-merge cardinality counter.  Scan: pinned by the reference's own Catch2 KATs
(testsimdscan.cpp:8-53: over the i % 256 column, a [lo, hi] predicate matches
N/256 * (hi - lo + 1) rows, in row order).
"""
import numpy as np
import pytest

DT = np.dtype([("key", "<u4"), ("payload", "<u4")])


def test_radix_bit_policy_matches_reference_formula(orc):
    # radix_join.cpp:295-329 with L2 1280 KiB / 4 -> 40960 tuples per partition
    assert orc.calc_num_radix_bits(1 << 20, 2) == 5      # C1
    assert orc.calc_num_radix_bits(1 << 28, 16) == 13    # C2 / C5
    assert orc.calc_num_radix_bits(1 << 27, 16) == 12    # C4
    assert orc.calc_num_radix_bits(13_107_200, 16) == 9  # paper shape
    assert orc.calc_num_radix_bits(100, 16) == 4         # max(required, nthreads)
    assert orc.calc_num_passes(13) == 1 and orc.calc_num_passes(14) == 2


@pytest.mark.parametrize("n,threads,two", [(1 << 10, 1, False), (1 << 16, 4, False), (1 << 16, 3, True),
                                           (1 << 20, 2, False), (100_003, 5, True)])
def test_pk_fk_kat(sgx, orc, n, threads, two):
    R, S = sgx.reference_relations(n, n)
    m, t = orc.rho_join(R, S, threads, two)
    assert m == n  # every S key is a primary key of R
    assert t["passes"] == (2 if two else orc.calc_num_passes(t["radix_bits"]))


def test_fk_multiple_copies_kat(sgx, orc):
    # C4 shape scaled down: |S| = 8 |R| -> 8 shuffled copies of 1..|R|
    R, S = sgx.reference_relations(1 << 14, 1 << 17)
    assert orc.rho_join(R, S, 4)[0] == 1 << 17


@pytest.mark.parametrize("sel", [50, 10, 1])
def test_fk_sel_kat(sgx, orc, sel):
    n = 1 << 14
    R, S = sgx.reference_relations(n, n, selectivity=sel)
    maxid = 100 * n // sel
    jump = maxid // n
    expected = len([k for k in range(n) if 1 + k * jump <= n])
    assert orc.rho_join(R, S, 2)[0] == expected


def test_zipf_kat(sgx, orc):
    n = 1 << 15
    R, S = sgx.reference_relations(n, n, skew=0.75)
    assert orc.rho_join(R, S, 4)[0] == n  # alphabet = 1..|R|


def test_against_sort_counter_with_duplicates(orc):
    rng = np.random.default_rng(7)
    for nR, nS, kmax in [(5000, 7000, 300), (1 << 14, 1 << 12, 1 << 12), (3, 5, 2), (1, 1, 1)]:
        R = np.empty(nR, dtype=DT)
        S = np.empty(nS, dtype=DT)
        R["key"] = rng.integers(1, kmax + 1, nR)
        S["key"] = rng.integers(1, kmax + 1, nS)
        R["payload"] = np.arange(nR)
        S["payload"] = np.arange(nS)
        exp = orc.count_join_sort(R, S)
        kr = np.bincount(R["key"], minlength=kmax + 1).astype(np.int64)
        ks = np.bincount(S["key"], minlength=kmax + 1).astype(np.int64)
        assert exp == int((kr * ks).sum())
        for threads, two in ((1, False), (3, False), (2, True)):
            assert orc.rho_join(R, S, threads, two)[0] == exp


def test_oracle_partition_is_stable_and_grouped(orc):
    rng = np.random.default_rng(1)
    n = 10_000
    x = np.empty(n, dtype=DT)
    x["key"] = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    x["payload"] = np.arange(n)
    out, starts = orc.radix_partition(x, 3, 4, 6)
    bins = (out["key"] >> 4) & 63
    assert np.all(np.diff(bins.astype(np.int64)) >= 0)
    for b in range(64):
        seg = out[int(starts[b]):int(starts[b + 1])]
        ref = x[((x["key"] >> 4) & 63) == b]
        assert np.array_equal(seg, ref)  # stable: input order inside each bin


# ------------------------------------------------------------------ scans ---
def u8_column(n):
    return (np.arange(n) % 256).astype(np.uint8)  # Allocator.hpp:94-110


@pytest.mark.parametrize("lo,hi,width", [(0, 100, 101), (1, 100, 100), (0, 26, 27), (0, 3, 4), (5, 5, 1),
                                         (0, 255, 256), (200, 100, 0)])
def test_scan_count_reference_kats(orc, lo, hi, width):
    n = 1 << 20
    col = u8_column(n)
    # testsimdscan.cpp:8-28 (count = N/256 * 101) and :30-53 (N/256 * 100)
    assert orc.scan("count", "u8", lo, hi, col) == n // 256 * width
    assert orc.scan("count", "i32", lo, hi, col.astype(np.int32)) == n // 256 * width


def test_scan_index_and_values_first_entries(orc):
    # testsimdscan.cpp:50-53: predicate [1, 100] -> values 1..100 then 1 again
    col = u8_column(1 << 16)
    vals = orc.scan("values", "u8", 1, 100, col)
    assert vals[:100].tolist() == list(range(1, 101)) and vals[100] == 1
    idx = orc.scan("index", "u8", 1, 100, col)
    assert idx[:3].tolist() == [1, 2, 3] and idx[100] == 257


def test_scan_bitvector_pattern(orc):
    # [0, 26] over i % 256: word w covers rows 64w..64w+63; the pattern repeats every 4 words
    col = u8_column(1 << 12)
    bv = orc.scan("bitvector", "u8", 0, 26, col)
    assert bv[0] == (1 << 27) - 1 and bv[1] == 0 and bv[2] == 0 and bv[3] == 0
    assert np.array_equal(bv[4:8], bv[0:4])


def test_scan_signed_i32(orc):
    col = np.array([-5, -1, 0, 3, 2**31 - 1, -(2**31)], dtype=np.int32)
    assert orc.scan("count", "i32", -1, 3, col) == 3
    assert orc.scan("index", "i32", -(2**31), -1, col).tolist() == [0, 1, 5]


def test_oracle_materialize_vs_pair_enumeration():
    """oracle_rho_join_mat (radix_join.cpp:437-446) emits exactly the equi-join pairs."""
    import oracle

    rng = np.random.default_rng(3)
    dt = np.dtype([("key", "<u4"), ("payload", "<u4")])
    for nR, nS, kmax in [(3000, 4000, 500), (1 << 14, 1 << 12, 1 << 20)]:
        R = np.empty(nR, dt)
        S = np.empty(nS, dt)
        R["key"] = rng.integers(0, kmax, nR)
        S["key"] = rng.integers(0, kmax, nS)
        R["payload"] = np.arange(nR)
        S["payload"] = np.arange(nS)
        got = oracle.rho_join_triples(R, S, 3)
        # independent: for each S row all R rows with the same key
        order = np.argsort(R["key"], kind="stable")
        rk = R["key"][order]
        lo = np.searchsorted(rk, S["key"], "left")
        hi = np.searchsorted(rk, S["key"], "right")
        exp = [(S["key"][j], order[i], j) for j in range(nS) for i in range(lo[j], hi[j])]
        exp = np.array(exp, dtype=np.uint32).reshape(-1, 3)
        key = lambda t: t[np.lexsort((t[:, 2], t[:, 1], t[:, 0]))]
        assert got.shape == exp.shape
        assert np.array_equal(key(got), key(exp))


def test_oracle_rht_equals_rho_and_sort_counter():
    """RHT (histogram_join) and RHO (bucket chaining) count the same equi-join."""
    import oracle

    rng = np.random.default_rng(9)
    dt = np.dtype([("key", "<u4"), ("payload", "<u4")])
    for nR, nS, kmax in [(5000, 9000, 700), (1 << 15, 1 << 15, 1 << 31), (3, 7, 2)]:
        R = np.zeros(nR, dt)
        S = np.zeros(nS, dt)
        R["key"] = rng.integers(0, kmax, nR)
        S["key"] = rng.integers(0, kmax, nS)
        exp = oracle.count_join_sort(R, S)
        for threads, two in [(1, False), (4, False), (3, True)]:
            assert oracle.rht_join(R, S, threads, two) == exp
            assert oracle.rho_join(R, S, threads, two)[0] == exp


def test_oracle_dict_scan_reference_kats():
    """oracle_dict_scan against every dictionary-scan KAT of testsimdscan.cpp."""
    import oracle
    from dict_kats import cases

    for name, codes, dictionary, lo, hi, size, probes in cases():
        got = oracle.dict_scan(lo, hi, dictionary, codes)
        assert len(got) == size, name
        for i, v in probes.items():
            assert got[i] == v, (name, i)


def test_oracle_dict_scan_wraps_like_reference():
    """Predicates outside the dictionary wrap through the reference's casts
    (SIMD512.cpp:297-305): no value >= lo -> code range [0, 255] for 8-bit codes."""
    import oracle

    d = np.arange(256, dtype=np.int64)
    codes = (np.arange(4096) % 256).astype(np.uint8)
    assert len(oracle.dict_scan(1000, 2000, d, codes)) == 4096
    assert len(oracle.dict_scan(-100, -50, d, codes)) == 4096  # hi below dict[0]: high index -1 -> 255
    assert oracle.scan_sum_u8(0, 26, codes) == 16 * sum(range(27))


@pytest.mark.parametrize("dtype,threads", [("u8", 1), ("u8", 3), ("i32", 4), ("i32", 5)])
def test_cpu_scan_baseline_matches_scalar_oracle(orc, dtype, threads):
    """The timed CPU scan baseline (cpu_baseline.c, AVX-512 where the host has it) counts
    what the scalar oracle counts over each thread's slice (N/T rows, the first
    multiple of 64 of them: multithreadedscan.cpp slicing, SIMD512's input_size/64)."""
    rng = np.random.default_rng(threads)
    n = 300_007
    if dtype == "u8":
        col = rng.integers(0, 256, n, dtype=np.uint8)
        lo, hi = 17, 200
    else:
        col = rng.integers(-2**31, 2**31, n, dtype=np.int64).astype(np.int32)
        lo, hi = -2**30, 12345
    per = n // threads
    exp = sum(orc.scan("count", dtype, lo, hi, col[t * per: t * per + per // 64 * 64]) for t in range(threads))
    for kind in ("count", "bitvector", "index"):
        secs, m = orc.cpu_scan_bench(kind, col, lo, hi, threads, reps=2)
        assert m == exp and secs > 0, kind
