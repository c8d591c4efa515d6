"""Predicate scan on the MI355X vs the CPU oracle (SIMD512.cpp semantics), bit-exact."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SIZES = [1, 63, 64, 65, 1000, 16384, 16385, (1 << 20) + 37, 3 << 20]
PREDS = [(0, 26), (5, 5), (200, 100), (0, 255), (1, 100)]


def column(n, dtype, kind):
    if kind == "mod":
        base = np.arange(n) % 256
    else:
        base = np.random.default_rng(n).integers(0, 256, n)
    return base.astype(np.uint8 if dtype == "u8" else np.int32)


@pytest.mark.parametrize("dtype", ["u8", "i32"])
@pytest.mark.parametrize("n", SIZES)
def test_all_outputs_match_oracle(sgx, orc, gpu, dtype, n):
    for kind in ("mod", "rand"):
        col = column(n, dtype, kind)
        for lo, hi in PREDS:
            cnt = orc.scan("count", dtype, lo, hi, col)
            assert sgx.scan_count(lo, hi, col, n, dtype) == cnt
            bv = np.full((n + 63) // 64, 0xDEADBEEF, dtype=np.uint64)
            sgx.scan_bitvector(lo, hi, col, n, bv, dtype)
            assert np.array_equal(bv, orc.scan("bitvector", dtype, lo, hi, col))
            idx = np.zeros(max(cnt, 1), dtype=np.uint64)
            assert sgx.scan_index(lo, hi, col, n, idx, cnt, dtype) == cnt
            assert np.array_equal(idx[:cnt], orc.scan("index", dtype, lo, hi, col))
            vals = np.zeros(max(cnt, 1), dtype=np.uint32 if dtype == "u8" else np.int32)
            assert sgx.scan_values(lo, hi, col, n, vals, cnt, dtype) == cnt
            assert np.array_equal(vals[:cnt], orc.scan("values", dtype, lo, hi, col))


def test_u8_predicate_sweep(sgx, orc, gpu):
    """The uint8 predicate on packed 16-bit halves ((b + 256 - lo) & (hi + 256 - b) & 0x100,
    scan_kernels.hip match_mask<uint8_t>) against the oracle for bounds on and around every
    byte-boundary case, empty ranges (lo > hi) included, on a ragged column holding every
    code at every lane and byte position: count and bitvector for all 196 (lo, hi) pairs,
    index and values for every seventh pair (SIMD512.cpp:7-32, 210-222, 251-287)."""
    import torch

    n = 3 * 65536 + 77
    col = np.random.default_rng(11).integers(0, 256, n).astype(np.uint8)
    col[:4096] = np.arange(4096) % 256  # every code at every byte of a 16-byte lane load
    d = torch.from_numpy(col).to(gpu)
    bounds = [0, 1, 2, 7, 8, 15, 16, 100, 127, 128, 129, 200, 254, 255]
    bv = torch.zeros((n + 63) // 64, dtype=torch.int64, device=gpu)
    for i, (lo, hi) in enumerate((a, b) for a in bounds for b in bounds):
        cnt = orc.scan("count", "u8", lo, hi, col)
        assert sgx.scan_count(lo, hi, d, n, "u8") == cnt, (lo, hi)
        sgx.scan_bitvector(lo, hi, d, n, bv, "u8")
        assert np.array_equal(bv.cpu().numpy().view(np.uint64), orc.scan("bitvector", "u8", lo, hi, col)), (lo, hi)
        if i % 7 == 0:
            idx = torch.zeros(max(cnt, 1), dtype=torch.int64, device=gpu)
            assert sgx.scan_index(lo, hi, d, n, idx, cnt, "u8") == cnt
            assert np.array_equal(idx.cpu().numpy().view(np.uint64)[:cnt], orc.scan("index", "u8", lo, hi, col))
            vals = np.zeros(max(cnt, 1), dtype=np.uint32)
            assert sgx.scan_values(lo, hi, col, n, vals, cnt, "u8") == cnt
            assert np.array_equal(vals[:cnt], orc.scan("values", "u8", lo, hi, col))


def test_signed_i32_full_range(sgx, orc, gpu):
    col = np.random.default_rng(3).integers(-(2**31), 2**31, 200_003, dtype=np.int64).astype(np.int32)
    for lo, hi in [(-(2**31), -1), (-1000, 1000), (0, 2**31 - 1), (-(2**31), 2**31 - 1)]:
        assert sgx.scan_count(lo, hi, col, len(col)) == orc.scan("count", "i32", lo, hi, col)
        k = orc.scan("count", "i32", lo, hi, col)
        idx = np.zeros(max(k, 1), dtype=np.uint64)
        sgx.scan_index(lo, hi, col, len(col), idx, k)
        assert np.array_equal(idx[:k], orc.scan("index", "i32", lo, hi, col))


def test_device_pointers_and_misaligned_views(sgx, orc, gpu):
    import torch

    n = (1 << 20) + 5
    col = column(n, "i32", "rand")
    d = torch.from_numpy(col).to(gpu)
    view = d[1:]  # 4 bytes past a 256-B boundary: not 16-B aligned
    ref = col[1:]
    cnt = orc.scan("count", "i32", 0, 26, ref)
    assert sgx.scan_count(0, 26, view, n - 1) == cnt
    out = torch.zeros(cnt, dtype=torch.int64, device=gpu)
    assert sgx.scan_index(0, 26, view, n - 1, out, cnt) == cnt
    assert np.array_equal(out.cpu().numpy().view(np.uint64), orc.scan("index", "i32", 0, 26, ref))
    bv = torch.zeros((n - 1 + 63) // 64, dtype=torch.int64, device=gpu)
    sgx.scan_bitvector(0, 26, view, n - 1, bv)
    assert np.array_equal(bv.cpu().numpy().view(np.uint64), orc.scan("bitvector", "i32", 0, 26, ref))


def test_capacity_error_reports_required_size(sgx, gpu):
    col = column(10_000, "u8", "mod")
    out = np.zeros(10, dtype=np.uint64)
    with pytest.raises(sgx.Mi355Error) as e:
        sgx.scan_index(0, 26, col, len(col), out, 10, "u8")
    assert e.value.code == sgx.MI355_ERR_CAPACITY
    assert out.tolist() == list(range(10))  # the first `cap` indexes are still written


def test_config3_full_size(sgx, gpu):
    """BASELINE config 3: 2^30 int32, 10 % selectivity -> [0, 26] matches 27/256 of the rows."""
    import torch

    n = 1 << 30
    col = torch.empty(n, dtype=torch.int32, device=gpu)
    sgx.gen_scan_dev(col, n, 0, 0, "i32")
    exp = n // 256 * 27
    assert exp == 113_246_208
    assert sgx.scan_count(0, 26, col, n) == exp
    idx = torch.empty(exp, dtype=torch.int64, device=gpu)
    assert sgx.scan_index(0, 26, col, n, idx, exp) == exp
    # size-independent properties: ascending, every index satisfies the predicate
    i = idx[: 1 << 22]
    assert bool((i[1:] > i[:-1]).all())
    assert bool(((i % 256) <= 26).all())
    assert int(idx[-1]) == n - 256 + 26
    bv = torch.empty(n // 64, dtype=torch.int64, device=gpu)
    sgx.scan_bitvector(0, 26, col, n, bv)
    assert int(bv[0]) == (1 << 27) - 1 and int(bv[4]) == (1 << 27) - 1 and int(bv[1]) == 0
    del col, idx, bv
    torch.cuda.empty_cache()


# ------------------------------------------------------------- dictionary scans
def test_dict_scan_reference_kats(sgx, orc, gpu):
    """dict_scan_{8,16,32}bit_64bit on the GPU == the oracle on every testsimdscan.cpp dictionary KAT."""
    from dict_kats import cases

    for name, codes, dictionary, lo, hi, size, probes in cases():
        bits = codes.dtype.itemsize * 8
        out = np.zeros(size + 16, dtype=np.int64)
        n = sgx.dict_scan(lo, hi, dictionary, codes, len(codes), out, len(out), bits, len(dictionary))
        assert n == size, name
        assert np.array_equal(out[:n], orc.dict_scan(lo, hi, dictionary, codes)), name
        for i, v in probes.items():
            assert out[i] == v, (name, i)


@pytest.mark.parametrize("bits", [8, 16, 32])
def test_dict_scan_random_vs_oracle(sgx, orc, gpu, bits, seed=3):
    import torch

    rng = np.random.default_rng(seed + bits)
    dsize = {8: 256, 16: 1 << 16, 32: 70_000}[bits]
    dt = {8: np.uint8, 16: np.uint16, 32: np.uint32}[bits]
    dictionary = rng.integers(-10**12, 10**12, dsize)  # unsorted: find_if semantics, not a sorted range
    dictionary[: dsize // 2].sort()
    n = 1_000_003
    codes = rng.integers(0, dsize, n).astype(dt)
    dcodes = torch.from_numpy(codes.view(np.int8 if bits == 8 else (np.int16 if bits == 16 else np.int32))).to(gpu)
    for lo, hi in [(-10**11, 3 * 10**11), (0, 10**12), (10**13, 10**14), (-10**13, -10**12 - 1), (5, 5)]:
        exp = orc.dict_scan(lo, hi, dictionary, codes)
        out = torch.zeros(len(exp) + 1, dtype=torch.int64, device=gpu)
        k = sgx.dict_scan(lo, hi, dictionary, dcodes, n, out, len(exp) + 1, bits, dsize)
        assert k == len(exp)
        assert np.array_equal(out[:k].cpu().numpy(), exp), (bits, lo, hi)
    with pytest.raises(sgx.Mi355Error):
        sgx.dict_scan(-10**13, 10**13, dictionary, codes, n, np.zeros(10, np.int64), 10, bits, dsize)


def test_scan_sum_u8(sgx, orc, gpu):
    col = (np.arange((1 << 20) + 77) % 256).astype(np.uint8)
    for lo, hi in [(0, 26), (0, 255), (200, 255), (7, 7), (9, 3)]:
        assert sgx.scan_sum_u8(lo, hi, col, len(col)) == orc.scan_sum_u8(lo, hi, col)


# ------------------------------------------------- one-pass selection (k_select)
def test_select_lookback_sparse_and_empty_chunks(sgx, orc, gpu):
    """Index / value outputs when whole 65,536-row chunks have no match (zero aggregates
    in the look-back), when only one middle chunk and the ragged last chunk match, and
    when every row matches (dense staging rounds) — against the oracle."""
    import torch

    n = (1 << 22) + 5
    col = np.full(n, 1000, dtype=np.int32)
    col[37 * 65536 + 11: 37 * 65536 + 5000] = 7
    col[-3:] = 7
    d = torch.from_numpy(col).to(gpu)
    for lo, hi in [(7, 7), (0, 2000), (5000, 6000)]:
        cnt = orc.scan("count", "i32", lo, hi, col)
        out = torch.zeros(max(cnt, 1), dtype=torch.int64, device=gpu)
        assert sgx.scan_index(lo, hi, d, n, out, cnt) == cnt
        assert np.array_equal(out[:cnt].cpu().numpy().view(np.uint64), orc.scan("index", "i32", lo, hi, col))


def test_select_repeated_full_size_calls(sgx, gpu):
    """20 back-to-back 2^26-row index scans (1,024 chunks each): the ticket and the
    status words are re-armed per call, and every call ends with the exact count."""
    import torch

    n = 1 << 26
    col = torch.empty(n, dtype=torch.int32, device=gpu)
    sgx.gen_scan_dev(col, n, 0, 0, "i32")
    exp = n // 256 * 27
    idx = torch.empty(exp, dtype=torch.int64, device=gpu)
    for _ in range(20):
        assert sgx.scan_index(0, 26, col, n, idx, exp) == exp
    assert int(idx[-1]) == n - 256 + 26 and int(idx[27]) == 256
    del col, idx


def test_scan_beyond_2pow32_rows(sgx, gpu):
    """Maximum sizes: a u8 column of 2^32 + 4,099 rows (row ids past 32 bits, ragged
    tail).  Count / index / bitvector against torch's own predicate on the device:
    the index list is strictly ascending, every entry satisfies the predicate and the
    count equals torch's, which together pin the exact set; bitvector words across the
    2^32 boundary and at the tail match the predicate bit for bit."""
    import torch

    n = (1 << 32) + 4099
    col = torch.empty(n, dtype=torch.uint8, device=gpu)
    sgx.gen_scan_dev(col, n, 1, 77, "u8")
    lo, hi = 3, 5
    exp = int(((col >= lo) & (col <= hi)).sum())
    assert sgx.scan_count(lo, hi, col, n, "u8") == exp
    idx = torch.empty(exp, dtype=torch.int64, device=gpu)
    assert sgx.scan_index(lo, hi, col, n, idx, exp, "u8") == exp
    assert bool((idx[1:] > idx[:-1]).all())
    v = col[idx]
    assert bool(((v >= lo) & (v <= hi)).all())
    assert int(idx[-1]) < n and int((idx >= (1 << 32)).sum()) > 0
    del v, idx
    nwords = (n + 63) // 64
    bv = torch.empty(nwords, dtype=torch.int64, device=gpu)
    sgx.scan_bitvector(lo, hi, col, n, bv, "u8")
    weights = torch.tensor([1 << b for b in range(63)] + [-(1 << 63)], dtype=torch.int64, device=gpu)
    for w0 in ((1 << 26) - 8, nwords - 8):
        rows = col[w0 * 64: min((w0 + 8) * 64, n)]
        bits = ((rows >= lo) & (rows <= hi)).to(torch.int64)
        bits = torch.nn.functional.pad(bits, (0, 8 * 64 - len(bits)))
        words = (bits.view(8, 64) * weights).sum(1)
        assert torch.equal(bv[w0: w0 + 8], words[: nwords - w0]), w0
    del col, bv
    torch.cuda.empty_cache()


# ------------------------------------------------------- explicit index scan
@pytest.mark.parametrize("n", [64, 1000, 16384, (1 << 20) + 37])
def test_explicit_index_scan_matches_oracle(sgx, orc, gpu, n):
    """SIMD512::explicit_index_scan (SIMD512.cpp:152-208): row r emits the index entry
    8*(r/64 + (r%64)/8) + r%8 (the reference's index_compressed[i + j])."""
    rng = np.random.default_rng(n)
    L = orc.explicit_index_len(n)
    index = rng.integers(0, 2**63, L, dtype=np.int64).astype(np.uint64)
    for kind in ("mod", "rand"):
        col = column(n, "u8", kind)
        for lo, hi in PREDS:
            exp = orc.explicit_index_scan(lo, hi, index, col)
            out = np.zeros(max(len(exp), 1), dtype=np.uint64)
            assert sgx.scan_explicit_index(lo, hi, index, L, col, n, out, len(exp)) == len(exp)
            assert np.array_equal(out[: len(exp)], exp)


def test_explicit_index_scan_short_index_fails_loudly(sgx, gpu):
    col = column(4096, "u8", "mod")
    index = np.arange(100, dtype=np.uint64)
    out = np.zeros(4096, dtype=np.uint64)
    with pytest.raises(sgx.Mi355Error) as e:
        sgx.scan_explicit_index(0, 255, index, len(index), col, len(col), out, len(out))
    assert e.value.code == sgx.MI355_ERR_INVALID
    # a predicate whose matches stay inside the index array is fine: rows 0..3 -> entries 0..3
    assert sgx.scan_explicit_index(0, 3, index, len(index), col[:64], 64, out, 64) == 4
    assert out[:4].tolist() == [0, 1, 2, 3]


# ----------------------------------------------- SIMD512:: adapter, compiled caller
def _self_alloc_size(size, blocks, before_last):
    """SIMD512.cpp:262-266 growth rule restated: the vector size the reference ends with."""
    if blocks == 0:
        return size
    while before_last + 64 > size:
        size = (64 + size) * 3
    return size


def test_simd512_adapter_binary(orc, gpu, tmp_path):
    """bin/simd512_check calls every SIMD512:: function through sgxamd/SIMD512_mi355.hpp with a
    64-B aligned CacheAlignedVector, like the reference's drivers and Catch2 tests; every
    output equals the oracle's on the reference's n / 64 whole blocks."""
    import os
    import subprocess

    from conftest import PKG

    n = (1 << 18) + 100  # the adapter drops the n % 64 tail, like the reference
    m = n // 64 * 64
    rng = np.random.default_rng(5)
    col = rng.integers(0, 256, n).astype(np.uint8)
    col[: 1 << 16] = np.arange(1 << 16) % 256  # the i % 256 column of Allocator.hpp:94-110
    index = rng.integers(0, 2**63, 8 * (m // 64 + 7), dtype=np.int64).astype(np.uint64)
    dict8 = np.sort(rng.integers(-1000, 1000, 256)).astype(np.int64)
    codes16 = rng.integers(0, 65536, n).astype(np.uint16)
    dict16 = np.sort(rng.integers(-50_000, 50_000, 65536)).astype(np.int64)
    codes32 = rng.integers(0, 3000, n).astype(np.uint32)
    dict32 = np.sort(rng.integers(-5000, 5000, 3000)).astype(np.int64)
    preds = [(0, 26), (7, 7), (1, 100), (0, 255), (200, 100)]
    sizes = [0, 5, 10_000, 1 << 20]
    for name, a in [("col_u8", col), ("index_u64", index), ("dict8", dict8), ("codes16", codes16),
                    ("dict16", dict16), ("codes32", codes32), ("dict32", dict32)]:
        a.tofile(tmp_path / f"{name}.bin")
    (tmp_path / "preds.txt").write_text("".join(f"{lo} {hi}\n" for lo, hi in preds))
    (tmp_path / "self_alloc.txt").write_text("".join(f"{s}\n" for s in sizes))
    (tmp_path / "out").mkdir()
    exe = os.path.join(PKG, "bin", "simd512_check")
    subprocess.run([exe, str(tmp_path)], check=True, timeout=120, capture_output=True)
    res = dict(line.split() for line in (tmp_path / "out" / "results.txt").read_text().splitlines())
    o = tmp_path / "out"
    cw = col[:m]
    for k, (lo, hi) in enumerate(preds):
        cnt = orc.scan("count", "u8", lo, hi, cw)
        assert int(res[f"p{k}_count"]) == cnt
        assert int(res[f"p{k}_sum"]) == orc.scan_sum_u8(lo, hi, cw)
        assert np.array_equal(np.fromfile(o / f"p{k}_bitvector.bin", np.uint64), orc.scan("bitvector", "u8", lo, hi, cw))
        idx = orc.scan("index", "u8", lo, hi, cw)
        assert np.array_equal(np.fromfile(o / f"p{k}_implicit.bin", np.uint64)[:cnt], idx)
        assert np.array_equal(np.fromfile(o / f"p{k}_explicit.bin", np.uint64)[:cnt],
                              orc.explicit_index_scan(lo, hi, index, cw))
        assert int(res[f"p{k}_scan"]) == cnt
        assert np.array_equal(np.fromfile(o / f"p{k}_scan.bin", np.uint32), orc.scan("values", "u8", lo, hi, cw))
        before_last = int((idx < m - 64).sum())
        for j, s0 in enumerate(sizes):
            assert int(res[f"p{k}_self_alloc_{j}_1"]) == cnt
            assert np.array_equal(np.fromfile(o / f"p{k}_self_alloc_{j}.bin", np.uint64), idx)
            assert int(res[f"p{k}_self_alloc_{j}_0"]) == _self_alloc_size(s0, m // 64, before_last)
        assert np.array_equal(np.fromfile(o / f"p{k}_dict8.bin", np.int64), orc.dict_scan(lo, hi, dict8, cw))
        assert np.array_equal(np.fromfile(o / f"p{k}_dict16.bin", np.int64),
                              orc.dict_scan(lo, hi, dict16, codes16[: n // 32 * 32]))
        assert np.array_equal(np.fromfile(o / f"p{k}_dict32.bin", np.int64),
                              orc.dict_scan(lo, hi, dict32, codes32[: n // 16 * 16]))


def test_golden_scan_fixtures(sgx, orc, gpu):
    """Every committed scan fixture (tests/golden/golden.json): GPU outputs hash to the fixture."""
    from test_golden import GOLDEN, explicit_index, scan_columns, sha

    cols = scan_columns()
    for e in GOLDEN["scans"]:
        c = cols[e["column"]]
        c = c if e["dtype"] == "u8" else c.astype(np.int32)
        lo, hi, dt, n, k = e["lo"], e["hi"], e["dtype"], len(c), e["count"]
        assert sgx.scan_count(lo, hi, c, n, dt) == k
        bv = np.zeros((n + 63) // 64, dtype=np.uint64)
        sgx.scan_bitvector(lo, hi, c, n, bv, dt)
        assert sha(bv) == e["bitvector_sha256"]
        idx = np.zeros(max(k, 1), dtype=np.uint64)
        assert sgx.scan_index(lo, hi, c, n, idx, k, dt) == k
        assert sha(idx[:k]) == e["index_sha256"]
        vals = np.zeros(max(k, 1), dtype=np.uint32 if dt == "u8" else np.int32)
        assert sgx.scan_values(lo, hi, c, n, vals, k, dt) == k
        assert sha(vals[:k]) == e["values_sha256"]
        if dt == "u8":
            assert sgx.scan_sum_u8(lo, hi, c, n) == e["sum"]
            ix = explicit_index(orc, n)
            assert sgx.scan_explicit_index(lo, hi, ix, len(ix), c, n, idx, k) == k
            assert sha(idx[:k]) == e["explicit_index_sha256"]


# ----------------------------------------------------- SimdScanMulti driver
def test_simdmulti_driver_csv(gpu, tmp_path):
    """bin/simdmulti_mi355 takes SimdScanMulti's flags (flags.hpp:8-40), enumerates the same
    configuration spectrum (types.hpp:140-190), maps selectivity to [0, round(sel/100*255)]
    (types.hpp:125,134) and prints CSV rows results/plot.py reads (plot.py:20-24)."""
    import io
    import os
    import subprocess

    import pandas as pd

    from conftest import PKG

    exe = os.path.join(PKG, "bin", "simdmulti_mi355")
    args = ["--mode=noIndex,bitvector,dict,scalar", "--min_entries_exp=16", "--max_entries_exp=20",
            "--min_selectivity=1", "--max_selectivity=10", "--step_selectivity=9", "--num_reruns=2",
            "--unique_data=b", "--num_runs=3", "--num_warmup_runs=1", "--min_threads=1", "--max_threads=2"]
    out = subprocess.run([exe] + args, capture_output=True, text=True, timeout=300, check=True).stdout
    df = pd.read_csv(io.StringIO(out), header=0, skipinitialspace=True)
    # 4 modes x unique {f, t} x threads {1, 2} x entries {2^16 .. 2^20} x selectivity {1, 10}
    assert len(df) == 4 * 2 * 2 * 5 * 2
    for col in ("entries", "numRuns", "numThreads", "reruns", "selectivity", "writeMode", "enclaveMode",
                "dataLoading", "datasizeKiB", "timeMicroSec", "cpuCycles", "unique", "warmup"):
        assert col in df.columns, col
    assert set(df["writeMode"]) == {"bitvector", "noindex", "dict", "scalar"}
    hi = (df["selectivity"] * 255).round().astype(int)  # 1 % -> 3, 10 % -> 26
    assert set(hi) == {3, 26}
    # the column is i % 256: every rerun of `entries` rows matches entries / 256 * (hi + 1)
    assert (df["matches"] == df["entries"] // 256 * (hi + 1)).all()
    assert ((df["numRuns"] == 1) == (df["unique"] == 1)).all()
    # plot.py's throughput formula is finite and positive
    time_s = df["cpuCycles"] / df["reruns"] / 2.9e9
    gib = df["entries"] * df["numRuns"] / time_s / 2**30
    assert (gib > 0).all() and (df["deviceMicroSec"] > 0).all()
