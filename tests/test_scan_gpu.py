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
