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
