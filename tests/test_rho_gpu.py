"""RHO join on the MI355X vs the CPU oracle: bit-exact match counts.

The oracle (oracle/rho_oracle.c) restates radix_join.cpp; relations come from the
restated reference generators (native.cpp:62-101 seeds and shapes)."""
import os
import subprocess

import numpy as np
import pytest

from conftest import PKG

pytestmark = pytest.mark.gpu

DT = np.dtype([("key", "<u4"), ("payload", "<u4")])


def rel(keys):
    x = np.empty(len(keys), dtype=DT)
    x["key"] = keys
    x["payload"] = np.arange(len(keys), dtype=np.uint32)
    return x


def gpu_join(sgx, R, S, **kw):
    return sgx.rho_join(R, len(R), S, len(S), **kw)


@pytest.mark.parametrize("n", [1 << 10, 1 << 16, 1 << 20])
def test_reference_pk_fk(sgx, orc, gpu, n):
    R, S = sgx.reference_relations(n, n)
    exp, _ = orc.rho_join(R, S, 4)
    assert exp == n
    res = gpu_join(sgx, R, S)
    assert res.matches == exp
    assert res.stats["ms_total"] > 0


def test_config1_native_cpu_shape(sgx, orc, gpu):
    # BASELINE config 1: |R| = |S| = 2^20 uniform; reference policy 5 bits / 1 pass
    R, S = sgx.reference_relations(1 << 20, 1 << 20)
    exp, t = orc.rho_join(R, S, 2)
    assert (t["radix_bits"], t["passes"]) == (5, 1)
    for bits, passes in [(0, 0), (5, 1), (8, 1), (9, 1), (12, 2), (16, 2), (18, 2)]:
        assert gpu_join(sgx, R, S, radix_bits=bits, passes=passes).matches == exp, (bits, passes)


@pytest.mark.parametrize("sel", [50, 10, 1])
def test_fk_sel(sgx, orc, gpu, sel):
    R, S = sgx.reference_relations(1 << 18, 1 << 18, selectivity=sel)
    assert gpu_join(sgx, R, S).matches == orc.rho_join(R, S, 4)[0]


def test_fk_multiple_copies(sgx, orc, gpu):
    R, S = sgx.reference_relations(1 << 16, 1 << 19)
    assert gpu_join(sgx, R, S).matches == 1 << 19


def test_zipf(sgx, orc, gpu):
    n = 1 << 18
    R, S = sgx.reference_relations(n, n, skew=0.75)
    res = gpu_join(sgx, R, S)
    assert res.matches == orc.rho_join(R, S, 4)[0] == n
    assert res.stats["max_part_s"] > 1.5 * (n >> res.stats["radix_bits"])  # skew reaches the partitions


@pytest.mark.parametrize("seed,nR,nS,kmax", [(1, 5000, 7000, 300), (2, 1 << 17, 1 << 15, 1 << 12),
                                             (3, 100_003, 77_777, 2**32 - 1), (4, 3, 5, 2)])
def test_random_with_duplicates(sgx, orc, gpu, seed, nR, nS, kmax):
    rng = np.random.default_rng(seed)
    R = rel(rng.integers(0, kmax + 1, nR, dtype=np.uint64).astype(np.uint32))
    S = rel(rng.integers(0, kmax + 1, nS, dtype=np.uint64).astype(np.uint32))
    exp = orc.count_join_sort(R, S)
    for bits, passes in [(0, 0), (4, 1), (14, 2)]:
        assert gpu_join(sgx, R, S, radix_bits=bits, passes=passes).matches == exp


@pytest.mark.parametrize("case", ["edge_fit", "edge_over", "dups_multichunk", "s_above_r"])
def test_small_join_direct_table(sgx, orc, gpu, case):
    """Small one-pass joins count a chunk in a direct table of u16 counters when R's
    largest residual (key >> radix bits) is below 2 x the chain table's capacity (8192 at
    4096 R keys per partition, 8 bits over 2^20 R keys): at the edge (residuals up to
    8191), one past it (8192: the chain table), R duplicates with partitions above the
    table (several R chunks per partition), and S keys above R's range (no counter)."""
    rng = np.random.default_rng(31)
    n = 1 << 20
    if case == "edge_fit":
        rk = rng.integers(0, 8192 << 8, n)
        rk[0] = (8192 << 8) - 1
        sk = rng.integers(0, 8192 << 8, n)
    elif case == "edge_over":
        rk = rng.integers(0, 8192 << 8, n)
        rk[0] = 8192 << 8
        sk = rng.integers(0, (8192 << 8) + 1, n)
    elif case == "dups_multichunk":
        rk = np.concatenate([rng.integers(0, 1000 << 8, n - 20000), np.full(20000, 77 << 8)])
        sk = rng.integers(0, 1000 << 8, n)
    else:
        rk = rng.integers(0, 4000 << 8, n)
        sk = rng.integers(0, 2**32, n)
        sk[: n // 2] = rng.integers(0, 4000 << 8, n // 2)
    R, S = rel(rk.astype(np.uint32)), rel(sk.astype(np.uint32))
    exp = orc.count_join_sort(R, S)
    res = gpu_join(sgx, R, S, radix_bits=8, passes=1)
    assert res.matches == exp, (case, res.matches, exp)


@pytest.mark.parametrize("bits,kmax", [(6, 1 << 22), (5, 2**32 - 1), (4, 1 << 19), (1, 1 << 12)])
def test_big_table_partitions(sgx, orc, gpu, bits, kmax):
    """Partitions above 8192 R tuples take the 16,384-tuple counting tables (RHO's chain
    table k_join_x, RHT's bucket table k_join_hist_big; 32,768-tuple S chunks): |R| = 2^20 over 2^bits
    partitions gives 16,384 (one table, ragged), 32,768 (two), 65,536 (four, duplicate
    keys) and 2^19 (32 tables, long chains, 16 S chunks per partition) R tuples per
    partition; the materialising join of the same plan keeps 8192-tuple chunks."""
    rng = np.random.default_rng(bits)
    nR, nS = 1 << 20, (1 << 20) + 777
    R = rel(rng.integers(0, kmax + 1, nR, dtype=np.uint64).astype(np.uint32))
    S = rel(rng.integers(0, kmax + 1, nS, dtype=np.uint64).astype(np.uint32))
    exp = orc.count_join_sort(R, S)
    passes = 1 if bits <= 8 else 2
    res = gpu_join(sgx, R, S, radix_bits=bits, passes=passes)
    assert res.matches == exp
    assert res.stats["max_part_r"] > 8192
    # RHT's 16,384-key bucket table (k_join_hist_big): full and ragged chunks
    assert gpu_join(sgx, R, S, radix_bits=bits, passes=passes, algorithm="RHT").matches == exp
    if bits == 6:
        got = gpu_triples(sgx, R, S, radix_bits=bits, passes=passes)
        assert np.array_equal(sorted_triples(got), sorted_triples(orc.rho_join_triples(R, S, 4)))


@pytest.mark.parametrize("case", ["one_region", "hot_s", "ragged", "dense_dups"])
def test_pooled_two_pass_layouts(sgx, orc, gpu, case):
    """Two-pass plans take the pooled pass 1 (per-workgroup block chains, no pass-1
    histogram) and the block-list pass 2: every tuple of one pass-1 digit (one region,
    chains of thousands of blocks), a hot S key (one region far above the rest), ragged
    sizes (partial tiles, chains ending inside a block) and dense duplicates, over the
    plans 10 = 5 + 5, 14 = 7 + 7 and 17 = 9 + 8 bits, counts and materialised triples."""
    rng = np.random.default_rng(11)
    if case == "one_region":  # low 9 bits zero: one digit in pass 1 of every plan
        R = rel(rng.integers(0, 1 << 20, 300_000).astype(np.uint32) << 9)
        S = rel(rng.integers(0, 1 << 20, 400_000).astype(np.uint32) << 9)
    elif case == "hot_s":
        R = rel(rng.permutation(np.arange(1, 200_001, dtype=np.uint32)))
        S = rel(np.concatenate([np.full(150_000, 4242, np.uint32),
                                rng.integers(1, 200_001, 250_000).astype(np.uint32)]))
    elif case == "ragged":
        R = rel(rng.integers(0, 2**32, 123_457, dtype=np.uint64).astype(np.uint32) % 1_000_003)
        S = rel(rng.integers(0, 2**32, 98_765, dtype=np.uint64).astype(np.uint32) % 1_000_003)
    else:
        R = rel(rng.integers(0, 5000, 70_001).astype(np.uint32))
        S = rel(rng.integers(0, 5000, 65_537).astype(np.uint32))
    exp = orc.count_join_sort(R, S)
    for bits in (10, 14, 17):
        res = gpu_join(sgx, R, S, radix_bits=bits, passes=2)
        assert res.matches == exp, (case, bits, res.matches, exp)
        # RHT counts over the same key partitions (histogram build/probe with KS = 1)
        rht = gpu_join(sgx, R, S, radix_bits=bits, passes=2, algorithm="RHT")
        assert rht.matches == exp and rht.stats["layout"] in (2, 3), (case, bits, rht.matches, exp)
    if case != "dense_dups":
        got = gpu_triples(sgx, R, S, radix_bits=14, passes=2)
        assert np.array_equal(sorted_triples(got), sorted_triples(orc.rho_join_triples(R, S, 4)))


def test_key_layout_switch(sgx, orc, gpu):
    """mi355_set_key_layout: counting joins (RHO and RHT) move 4-byte keys (layout 3 at 14 =
    7 + 7 bits: keys with chain histograms) or whole tuples (layout 1) after the input read;
    the counts are identical, materialising joins keep tuples either way."""
    rng = np.random.default_rng(21)
    R = rel(rng.integers(0, 1 << 21, 400_001).astype(np.uint32))
    S = rel(rng.integers(0, 1 << 21, 300_007).astype(np.uint32))
    exp = orc.count_join_sort(R, S)
    try:
        for on, layout in ((True, 3), (False, 1), (True, 3)):
            sgx.set_key_layout(on)
            for alg in ("RHO", "RHT"):
                res = gpu_join(sgx, R, S, radix_bits=14, passes=2, algorithm=alg)
                assert res.matches == exp and res.stats["layout"] == layout, alg
                assert res.stats["elem_bytes"] == (4 if on else 8)
    finally:
        sgx.set_key_layout(True)
    got = gpu_triples(sgx, R, S, radix_bits=14, passes=2)
    assert len(got) == exp


def test_extreme_keys(sgx, orc, gpu):
    # 0 and 0xFFFFFFFF (the LDS empty marker) must join like any other key
    keys = np.array([0, 0xFFFFFFFF, 0xFFFFFFFF, 1, 0x80000000, 0xFFFFFFFE] * 50, dtype=np.uint32)
    R = rel(keys)
    S = rel(np.concatenate([keys[::-1], np.array([0xFFFFFFFF] * 7, dtype=np.uint32)]))
    exp = orc.count_join_sort(R, S)
    for bits in (0, 3, 10):
        assert gpu_join(sgx, R, S, radix_bits=bits).matches == exp


def test_skewed_build_side_chunks(sgx, orc, gpu):
    # one R partition far larger than an LDS table (R chunking) plus a hot S key
    R = rel(np.concatenate([np.full(20_000, 7, np.uint32), np.arange(1, 5001, dtype=np.uint32)]))
    S = rel(np.concatenate([np.full(1000, 7, np.uint32), np.arange(1, 90_001, dtype=np.uint32)]))
    exp = orc.count_join_sort(R, S)
    assert exp == 20_001 * 1_001 + 4_999  # key 7 also occurs once in each arange
    assert gpu_join(sgx, R, S).matches == exp
    assert gpu_join(sgx, R, S, radix_bits=2).matches == exp


@pytest.mark.parametrize("nR,nS", [(0, 10), (10, 0), (1, 1), (63, 2049), (2049, 63)])
def test_empty_and_ragged(sgx, orc, gpu, nR, nS):
    R, _ = sgx.reference_relations(max(nR, 1), 1)
    R = R[:nR]
    S = rel(np.arange(1, nS + 1, dtype=np.uint32) % max(nR, 1) + 1)
    exp = orc.count_join_sort(R, S) if nR and nS else 0
    assert gpu_join(sgx, R, S).matches == exp


def test_device_resident_inputs(sgx, orc, gpu):
    import torch

    R, S = sgx.reference_relations(1 << 18, 1 << 18)
    dR = torch.from_numpy(R.view(np.int64)).to(gpu)
    dS = torch.from_numpy(S.view(np.int64)).to(gpu)
    res = sgx.rho_join(dR, len(R), dS, len(S))
    assert res.matches == 1 << 18 and res.stats["ms_h2d"] == 0.0
    # inputs are const: untouched
    assert np.array_equal(dR.cpu().numpy().view(DT), R)


def test_dropin_table_api(sgx, gpu):
    R, S = sgx.reference_relations(1 << 16, 1 << 16)
    out = sgx.rho_join_tables(R, len(R), S, len(S), nthreads=16)
    assert out.totalresults == 1 << 16
    assert out.nthreads == 16 and out.materialized == 0 and out.result_type == 0
    assert out.throughput > 0


def test_shard_partition_matches_radix_partition(sgx, orc, gpu):
    """Same bins with the same tuples as the reference's radix partition (radix_join.cpp:851-931).
    Inside a bin the GPU keeps arrival order of its LDS atomics, so bins are compared as multisets."""
    import torch

    rng = np.random.default_rng(5)
    x = rel(rng.integers(0, 2**32, 300_001, dtype=np.uint64).astype(np.uint32))
    dx = torch.from_numpy(x.view(np.int64)).to(gpu)
    out = torch.empty_like(dx)
    for shift, bits in [(0, 3), (0, 1), (5, 9), (2, 8)]:
        counts = sgx.shard_partition(dx, len(x), shift, bits, out)
        ref, starts = orc.radix_partition(x, 1, shift, bits)
        assert counts == np.diff(starts).tolist()
        got = out.cpu().numpy()
        exp = ref.view(np.int64)
        for b in range(1 << bits):
            lo, hi = int(starts[b]), int(starts[b + 1])
            assert np.array_equal(np.sort(got[lo:hi]), np.sort(exp[lo:hi])), (shift, bits, b)


def test_full_size_config2_property(sgx, gpu):
    """BASELINE config 2 size (|R| = |S| = 2^28) on device-generated pk/fk: matches == |S|."""
    import torch

    n = 1 << 28
    R = torch.empty(n, dtype=torch.int64, device=gpu)
    S = torch.empty(n, dtype=torch.int64, device=gpu)
    sgx.gen_pk_dev(R, n, 0, n, 11111)
    sgx.gen_fk_dev(S, n, 0, n, 22222)
    res = sgx.rho_join(R, n, S, n)
    assert res.matches == n
    # 2^14 partitions of 16,384 R tuples (7 + 7 bits), one 16,384-tuple table each
    assert res.stats["radix_bits"] == 14 and res.stats["passes"] == 2
    # keys 1..2^28: residuals above 14 bits fit 16 bits, both final partitions are u16
    assert res.stats["narrow"] == 3
    del R, S
    torch.cuda.empty_cache()


def test_config4_full_size(sgx, gpu):
    """BASELINE config 4 at its size on one GPU: pk(2^27, seed 11111) join fk(2^30,
    maxid 2^27, seed 22222) = 8 shuffled copies of 1..2^27 (native.cpp:62-101 shapes,
    device generators).  matches == |S|; the planner sizes partitions for one 65,536-key
    S task each (ceil(log2(2^30 / 65,536)) = 14 bits, 7 + 7): every R partition then holds
    exactly 2^27 / 2^14 = 8192 keys and every S partition its 8 copies, 65,536 tuples,
    probed in one task."""
    import torch

    nR, nS = 1 << 27, 1 << 30
    R = torch.empty(nR, dtype=torch.int64, device=gpu)
    S = torch.empty(nS, dtype=torch.int64, device=gpu)
    sgx.gen_pk_dev(R, nR, 0, nR, 11111)
    sgx.gen_fk_dev(S, nS, 0, nR, 22222)
    res = sgx.rho_join(R, nR, S, nS)
    assert res.matches == nS
    st = res.stats
    assert (st["radix_bits"], st["passes"], st["num_partitions"]) == (14, 2, 1 << 14)
    assert st["max_part_r"] == 8192 and st["max_part_s"] == 65536
    assert st["num_tasks"] == 1 << 14  # one 65,536-key S chunk per partition
    # a hot S key: 2^23 tuples of S take R key 12345 (still one R match each), so its
    # partition holds > 2^23 tuples and is split into 65,536-key tasks
    hot = S[: 1 << 23]
    hot.copy_((hot & ~0xFFFFFFFF) | 12345)
    res = sgx.rho_join(R, nR, S, nS)
    assert res.matches == nS
    st = res.stats
    assert st["max_part_s"] > 1 << 23 and st["num_tasks"] >= (1 << 14) + (1 << 23) // 65536 - 1
    del R, S, hot
    torch.cuda.empty_cache()


def test_config5_full_size_host_zipf(sgx, orc, gpu):
    """BASELINE config 5 at its size: pk(2^28) join Zipf(theta = 0.75) over 1..2^28 from
    the host mt19937_64 seed-22222 stream (generator.cpp restating genzipf.cpp:87-144,
    BASELINE.md row 5), staged once to HBM.  The count equals an independent
    sum_k cnt_R(k) * cnt_S(k) over the same buffers (numpy bincount) and |S|; the
    partitions are skewed (the hottest key alone is ~0.2 % of S) and the hot ones are
    split into several build/probe tasks.  The device Zipf generator gives the same count."""
    import torch

    n = 1 << 28
    R = torch.empty(n, dtype=torch.int64, device=gpu)
    sgx.gen_pk_dev(R, n, 0, n, 11111)
    host = np.empty(n, dtype=np.int64)
    sgx.gen_zipf(host, n, n, 0.75, 22222, 16)
    S = torch.from_numpy(host).to(gpu)
    res = sgx.rho_join(R, n, S, n)
    rk = (R.cpu().numpy() & 0xFFFFFFFF).astype(np.uint32)
    sk = (host & 0xFFFFFFFF).astype(np.uint32)
    del host
    cr = np.bincount(rk, minlength=n + 1)
    cs = np.bincount(sk, minlength=n + 1)
    exp = int(np.dot(cr[: n + 1].astype(np.int64), cs[: n + 1].astype(np.int64)))
    assert len(cr) == len(cs) == n + 1  # every key in 1..2^28
    assert res.matches == exp == n
    st = res.stats
    mean_s = n >> st["radix_bits"]
    assert st["max_part_s"] > 20 * mean_s  # per-partition skew reaches the join (33x at 14 bits)
    assert st["num_tasks"] > st["num_partitions"]  # hot partitions split into tasks
    assert cs.max() > 500_000  # the hottest key (~0.197 % of S)
    sgx.gen_zipf_dev(S, n, 0, n, 0.75, 22222)
    assert sgx.rho_join(R, n, S, n).matches == n
    del R, S
    torch.cuda.empty_cache()


def test_max_size_pk_fk(sgx, gpu):
    """|R| = |S| = 2^31 + 12,345 (ragged, 8x the headline size, 17 GB per relation):
    the planner goes past 16 radix bits (17: average partitions of 16,384 R tuples in
    the big counting table); an explicit 18-bit plan runs the 9-bit pass-2 digit,
    which does not fit the side stream, through the tuple histogram at scale.
    matches == |S|, and with foreign keys drawn from [1, 1.5 |R|] exactly the ones that
    fall inside R's key range."""
    import torch

    n = (1 << 31) + 12_345
    R = torch.empty(n, dtype=torch.int64, device=gpu)
    S = torch.empty(n, dtype=torch.int64, device=gpu)
    sgx.gen_pk_dev(R, n, 0, n, 11111)
    sgx.gen_fk_dev(S, n, 0, n, 22222)
    res = sgx.rho_join(R, n, S, n)
    assert res.matches == n
    assert res.stats["passes"] == 2 and res.stats["radix_bits"] == 17
    assert sgx.rho_join(R, n, S, n, radix_bits=18, passes=2).matches == n
    sgx.gen_fk_dev(S, n, 0, n + n // 2, 33333)
    m = sgx.rho_join(R, n, S, n).matches
    assert m == int(((S & 0xFFFFFFFF) <= n).sum()) and n // 2 < m < n
    del R, S
    torch.cuda.empty_cache()


@pytest.mark.parametrize("alg,extra", [("RHO", []), ("RHT", []), ("RHO", ["-m"]), ("RHT", ["-m", "-l", "50"])])
def test_native_driver_binary(gpu, alg, extra):
    exe = os.path.join(PKG, "bin", "native_mi355")
    out = subprocess.run([exe, "-a", alg, "-r", str(1 << 20), "-s", str(1 << 20), "-n", "2"] + extra,
                         capture_output=True, text=True, timeout=300, check=True).stdout
    m = (1 << 19) if "50" in extra else (1 << 20)
    assert f"Matches = {m}" in out
    assert "Throughput (M rec/sec)" in out and f"Running {alg}" in out
    if "-m" in extra:
        assert f"Materialized {m} tuples" in out
    throughput, phases = parse_teebench_output(out)
    assert throughput > 0
    assert set(phases) == set(TEEBENCH_TIMED_PHASES), sorted(phases)
    # One Hist + One Copy = pass 1; Build + Join = the build/probe kernels inside Build+Join Overall
    assert phases["build"] > 0 and phases["probe"] > 0
    assert phases["build"] + phases["probe"] <= phases["join_total"] + 2
    assert abs(phases["partition_r"] + phases["partition_s"] - phases["partition_1"]) <= 2 + phases["partition_1"] // 100
    assert phases["total"] >= phases["partition"] + phases["join_total"] - 2


# The phase keys the reference's harness extracts from print_timing
# (SGXv2Scripts/scripts/helpers/runner.py:14-55; its "Partition One Hist/Copy" lines
# land in partition_r / partition_s).  The regexes below restate that parser.
TEEBENCH_TIMED_PHASES = ["total", "partition", "partition_1", "partition_r", "partition_s", "partition_2",
                         "partition_2_h", "partition_2_c", "join_total", "build", "probe"]
_PHASE_LINES = [("Total Join Time (cycles)", "total"), ("Partition Overall (cycles)", "partition"),
                ("Partition Pass One (cycles)", "partition_1"), ("Partition One Hist (cycles)", "partition_r"),
                ("Partition One Copy (cycles)", "partition_s"), ("Partition Pass Two (cycles)", "partition_2"),
                ("Partition Two Hist (cycles)", "partition_2_h"), ("Partition Two Copy (cycles)", "partition_2_c"),
                ("Build+Join Overall (cycles)", "join_total"), ("Build (cycles)", "build"),
                ("Join (cycles)", "probe")]


def parse_teebench_output(stdout):
    import re

    phases, throughput = {}, 0.0
    for line in stdout.splitlines():
        if "Throughput" in line:
            throughput = float(re.findall(r"\d+\.\d+", line)[1])
            continue
        for text, key in _PHASE_LINES:  # first match wins, like runner.py's elif chain
            if text in line:
                phases[key] = int(re.findall(r"\d+", line)[-2])  # -2: the colour reset ends in 0
                break
    return throughput, phases


# ---------------------------------------------------------------- materialisation
def sorted_triples(t):
    t = np.asarray(t, dtype=np.uint32).reshape(-1, 3)
    return t[np.lexsort((t[:, 2], t[:, 1], t[:, 0]))]


def gpu_triples(sgx, R, S, **kw):
    m = sgx.rho_join(R, len(R), S, len(S)).matches
    out = np.zeros((max(m, 1), 3), dtype=np.uint32)
    res = sgx.rho_join(R, len(R), S, len(S), out=out, out_capacity=m, **kw)
    assert res.matches == m
    return out[:m]


@pytest.mark.parametrize("case", ["pk_fk_sel50", "fk_copies", "dups", "hot_key"])
def test_materialize_matches_oracle(sgx, orc, gpu, case):
    """MATERIALIZE = 1 (radix_join.cpp:437-446): the same multiset of {key, R payload, S payload}."""
    rng = np.random.default_rng(11)
    if case == "pk_fk_sel50":
        R, S = sgx.reference_relations(1 << 16, 1 << 16, selectivity=50)
    elif case == "fk_copies":
        R, S = sgx.reference_relations(1 << 14, 1 << 17)
    elif case == "dups":
        R = rel(rng.integers(0, 3000, 20_000).astype(np.uint32))
        S = rel(rng.integers(0, 3000, 30_000).astype(np.uint32))
    else:  # hot S key split over several build/probe tasks, duplicated R key
        R = rel(np.concatenate([np.full(3, 9, np.uint32), np.arange(100, 20_100, dtype=np.uint32)]))
        S = rel(np.concatenate([np.full(40_000, 9, np.uint32), rng.integers(0, 30_000, 50_000).astype(np.uint32)]))
    exp = orc.rho_join_triples(R, S, 4)
    for bits, passes in [(0, 0), (6, 1), (14, 2)]:
        got = gpu_triples(sgx, R, S, radix_bits=bits, passes=passes)
        assert got.shape == exp.shape
        assert np.array_equal(sorted_triples(got), sorted_triples(exp)), (case, bits, passes)


def test_materialize_capacity_and_device_output(sgx, gpu):
    import torch

    R, S = sgx.reference_relations(1 << 15, 1 << 15)
    with pytest.raises(sgx.Mi355Error) as ei:
        sgx.rho_join(R, len(R), S, len(S), out=np.zeros((10, 3), np.uint32), out_capacity=10)
    assert ei.value.code == -5 and str(1 << 15) in str(ei.value)
    d = torch.zeros((1 << 15) * 3, dtype=torch.int32, device=gpu)
    res = sgx.rho_join(R, len(R), S, len(S), out=d, out_capacity=1 << 15)
    t = d.cpu().numpy().view(np.uint32).reshape(-1, 3)
    assert res.matches == 1 << 15
    assert (R["key"][t[:, 1]] == t[:, 0]).all() and (S["key"][t[:, 2]] == t[:, 0]).all()
    assert np.array_equal(np.sort(t[:, 2]), np.arange(1 << 15, dtype=np.uint32))


def test_dropin_materialize_chunked_table(sgx, orc, gpu):
    R, S = sgx.reference_relations(1 << 12, 1 << 13, selectivity=50)
    res = sgx.rho_join_tables(R, len(R), S, len(S), nthreads=4, materialize=True)
    try:
        assert res.materialized == 1 and res.result_type == 1
        got = sgx.chunked_table_triples(res)
        exp = orc.rho_join_triples(R, S, 4)
        assert res.totalresults == len(exp) == len(got)
        assert np.array_equal(sorted_triples(got), sorted_triples(exp))
    finally:
        sgx.free_result(res)


def test_skew_splits_hot_partition(sgx, orc, gpu):
    """A hot S partition (200k copies of one key) is split over several build/probe tasks."""
    R = rel(np.concatenate([np.full(2, 5, np.uint32), np.arange(1000, 60_000, dtype=np.uint32)]))
    S = rel(np.concatenate([np.full(200_000, 5, np.uint32), np.arange(1000, 50_000, dtype=np.uint32)]))
    res = gpu_join(sgx, R, S)
    assert res.matches == orc.count_join_sort(R, S) == 2 * 200_000 + 49_000
    assert res.stats["num_tasks"] >= res.stats["num_partitions"] + 200_000 // 8192


def test_full_size_materialize_property(sgx, gpu):
    """|R| = |S| = 2^26 device pk/fk, materialised on the device: every S row matches once,
    and each triple's payloads point at rows holding its key."""
    import torch

    n = 1 << 26
    R = torch.empty(n, dtype=torch.int64, device=gpu)
    S = torch.empty(n, dtype=torch.int64, device=gpu)
    sgx.gen_pk_dev(R, n, 0, n, 11111)
    sgx.gen_fk_dev(S, n, 0, n, 22222)
    out = torch.empty(n * 3, dtype=torch.int32, device=gpu)
    assert sgx.rho_join(R, n, S, n, out=out, out_capacity=n).matches == n
    t = out.view(n, 3).to(torch.int64) & 0xFFFFFFFF
    rk, sk = R & 0xFFFFFFFF, S & 0xFFFFFFFF
    assert torch.equal(rk[t[:, 1]], t[:, 0]) and torch.equal(sk[t[:, 2]], t[:, 0])
    assert torch.equal(torch.sort(t[:, 2]).values, torch.arange(n, device=gpu))
    del R, S, out, t, rk, sk
    torch.cuda.empty_cache()


# ------------------------------------------------------------------ RHT
@pytest.mark.parametrize("case", ["pk_fk", "sel10", "dups", "hot_key"])
def test_rht_matches_oracle(sgx, orc, gpu, case):
    """RHT (histogram_join, radix_join.cpp:463-612): counts and triples equal the oracle's RHT."""
    rng = np.random.default_rng(7)
    if case == "pk_fk":
        R, S = sgx.reference_relations(1 << 18, 1 << 18)
    elif case == "sel10":
        R, S = sgx.reference_relations(1 << 16, 1 << 16, selectivity=10)
    elif case == "dups":
        R = rel(rng.integers(0, 5000, 30_000).astype(np.uint32))
        S = rel(rng.integers(0, 5000, 20_000).astype(np.uint32))
    else:
        R = rel(np.concatenate([np.full(4, 3, np.uint32), np.arange(10, 40_010, dtype=np.uint32)]))
        S = rel(np.concatenate([np.full(30_000, 3, np.uint32), rng.integers(0, 50_000, 40_000).astype(np.uint32)]))
    exp = orc.rht_join(R, S, 4)
    assert exp == orc.count_join_sort(R, S)
    for bits, passes in [(0, 0), (5, 1), (13, 2), (2, 1), (1, 1)]:  # (2, 1) / (1, 1): 16,384-key tables
        assert gpu_join(sgx, R, S, radix_bits=bits, passes=passes, algorithm="RHT").matches == exp
    if len(R) <= 1 << 16:
        got = gpu_triples(sgx, R, S, algorithm="RHT")
        assert np.array_equal(sorted_triples(got), sorted_triples(orc.rht_join_triples(R, S, 4)))


def test_rht_dropin_and_full_size(sgx, gpu):
    import torch

    R, S = sgx.reference_relations(1 << 16, 1 << 16)
    out = sgx.rho_join_tables(R, len(R), S, len(S), nthreads=8, algorithm="RHT")
    assert out.totalresults == 1 << 16 and out.result_type == 0
    n = 1 << 28
    dR = torch.empty(n, dtype=torch.int64, device=gpu)
    dS = torch.empty(n, dtype=torch.int64, device=gpu)
    sgx.gen_pk_dev(dR, n, 0, n, 11111)
    sgx.gen_fk_dev(dS, n, 0, n, 22222)
    assert sgx.rho_join(dR, n, dS, n, algorithm="RHT").matches == n
    del dR, dS
    torch.cuda.empty_cache()


@pytest.mark.parametrize("case", ["pk_fk", "dups"])
def test_partition_overlap_same_result(sgx, orc, gpu, case):
    """Two-stream partition chains (default) and one stream give the same join."""
    rng = np.random.default_rng(5)
    if case == "pk_fk":
        R, S = sgx.reference_relations(1 << 18, 1 << 19)
    else:
        R = rel(rng.integers(0, 5000, 60_000).astype(np.uint32))
        S = rel(rng.integers(0, 5000, 90_000).astype(np.uint32))
    exp = orc.rho_join_triples(R, S, 4)
    got = {}
    try:
        for on in (True, False):
            sgx.set_partition_overlap(on)
            for bits, passes in [(8, 1), (14, 2)]:
                got[(on, bits)] = gpu_triples(sgx, R, S, radix_bits=bits, passes=passes)
                assert np.array_equal(sorted_triples(got[(on, bits)]), sorted_triples(exp)), (case, on, bits)
    finally:
        sgx.set_partition_overlap(True)


@pytest.mark.parametrize("case", ["pk_fk_shift", "dups", "rht"])
def test_pipelined_begin_finish(sgx, orc, gpu, case):
    """mi355_rho_join_begin + mi355_rho_join_finish == one mi355_rho_join_ex call (the
    multi-GPU path's local join, with S written to HBM only between the two calls)."""
    import torch

    rng = np.random.default_rng(9)
    shift, algo = 0, "RHO"
    if case == "pk_fk_shift":  # a shard's view: every key has the same low 2 bits
        R, S = sgx.reference_relations(1 << 18, 3 << 17)
        R = R[(R["key"] & 3) == 1]
        S = S[(S["key"] & 3) == 1]
        shift = 2
    else:
        R = rel(rng.integers(0, 7000, 70_001).astype(np.uint32))
        S = rel(rng.integers(0, 7000, 50_003).astype(np.uint32))
        algo = "RHT" if case == "rht" else "RHO"
    exp = orc.count_join_sort(R, S)
    dR = torch.from_numpy(R.view(np.int64).copy()).to(gpu)
    dS = torch.empty(len(S), dtype=torch.int64, device=gpu)
    stream = torch.cuda.current_stream().cuda_stream
    sgx.rho_join_begin(dR, len(R), len(S), key_shift=shift, stream=stream, algorithm=algo)
    dS.copy_(torch.from_numpy(S.view(np.int64).copy()))  # S lands after begin, in stream order
    res = sgx.rho_join_finish(dS, len(S), key_shift=shift, stream=stream, algorithm=algo)
    assert res.matches == exp
    assert sgx.rho_join(dR, len(R), dS, len(S), key_shift=shift, algorithm=algo).matches == exp


def test_pipelined_guards(sgx, gpu):
    import torch

    R, S = sgx.reference_relations(1 << 14, 1 << 14)
    dR = torch.from_numpy(R.view(np.int64).copy()).to(gpu)
    dS = torch.from_numpy(S.view(np.int64).copy()).to(gpu)
    with pytest.raises(sgx.Mi355Error):  # finish without begin
        sgx.rho_join_finish(dS, len(S))
    sgx.rho_join_begin(dR, len(R), len(S))
    with pytest.raises(sgx.Mi355Error):  # another join while one is pending
        sgx.rho_join(dR, len(R), dS, len(S))
    with pytest.raises(sgx.Mi355Error):  # the shard step would reuse the pending join's scratch
        sgx.shard_partition(dR, len(R), 0, 2, torch.empty_like(dR))
    with pytest.raises(sgx.Mi355Error):  # |S| differs from begin's
        sgx.rho_join_finish(dS, len(S) - 1)
    sgx.rho_join_begin(dR, len(R), len(S))
    assert sgx.rho_join_finish(dS, len(S)).matches == len(S)
    assert sgx.rho_join(dR, len(R), dS, len(S)).matches == len(S)


# ---------------------------------------------------------------- golden fixtures
def test_golden_join_counts(sgx, gpu):
    """Every committed join fixture (tests/golden/golden.json): GPU RHO and RHT counts equal
    the fixture's, with the GPU policy and a forced 2-pass plan."""
    from test_golden import GOLDEN, relation, zipf_relation

    for case in GOLDEN["joins"]:
        R, S = relation(sgx, case["R"]), relation(sgx, case["S"])
        assert gpu_join(sgx, R, S).matches == case["matches"], case
        assert gpu_join(sgx, R, S, radix_bits=10, passes=2).matches == case["matches"], case
        assert gpu_join(sgx, R, S, algorithm="RHT").matches == case["matches"], case
    z = GOLDEN["zipf"]
    Z = zipf_relation(sgx)
    R = relation(sgx, f"pk_{z['n']}_11111")
    assert gpu_join(sgx, R, Z).matches == z["pk_join_matches"]
    assert gpu_join(sgx, Z, Z).matches == z["self_join_matches"]


def test_config2_reference_relations_full_size(sgx, gpu):
    """BASELINE config 2 on the reference's own relations at full size: pk(2^28, seed
    11111) and fk(2^28, seed 22222) from the restated glibc rand() Knuth shuffles
    (native.cpp:62-101, generator.cpp:100-153), generated on the host and staged to HBM.
    matches == |S|, and the plan is the device relations' one: 14 radix bits in two
    passes, key partitions, every R and S partition exactly 2^14 keys (pk 1..2^28 and a
    permutation of it: each key's low 14 bits once per 2^14)."""
    import torch

    n = 1 << 28
    Rh, Sh = sgx.reference_relations(n, n)
    assert int(Rh["key"][:8].min()) >= 1 and int(Rh["key"].max()) == n
    R = torch.from_numpy(Rh.view(np.int64)).to(gpu)
    S = torch.from_numpy(Sh.view(np.int64)).to(gpu)
    del Rh, Sh
    try:
        res = sgx.rho_join(R, n, S, n)
        st = res.stats
        assert res.matches == n
        assert (st["radix_bits"], st["passes"], st["layout"]) == (14, 2, 3)  # keys, chain histograms
        assert st["max_part_r"] == st["max_part_s"] == 1 << 14
    finally:
        del R, S
        torch.cuda.empty_cache()
