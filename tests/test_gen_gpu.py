"""Device generators: pk/fk shapes (shuffled 1..n / copies of 1..maxid), slice-consistent."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

DT = np.dtype([("key", "<u4"), ("payload", "<u4")])


@pytest.mark.parametrize("n", [1, 2, 1000, 1 << 20, (1 << 20) + 12345])
def test_pk_dev_is_permutation_and_sliceable(sgx, gpu, n):
    import torch

    R = torch.empty(n, dtype=torch.int64, device=gpu)
    sgx.gen_pk_dev(R, n, 0, n, 11111)
    keys = (R & 0xFFFFFFFF).sort().values
    assert torch.equal(keys, torch.arange(1, n + 1, device=gpu, dtype=torch.int64))
    assert torch.equal(R >> 32, torch.arange(n, device=gpu, dtype=torch.int64))  # payload = row id
    half = n // 2
    P = torch.empty(n - half, dtype=torch.int64, device=gpu)
    sgx.gen_pk_dev(P, n - half, half, n, 11111)
    assert torch.equal(P, R[half:])


def test_fk_dev_copies(sgx, gpu):
    import torch

    maxid, copies = 100_000, 5
    S = torch.empty(maxid * copies + 777, dtype=torch.int64, device=gpu)
    sgx.gen_fk_dev(S, S.numel(), 0, maxid, 22222)
    k = S & 0xFFFFFFFF
    for c in range(copies):
        blk = k[c * maxid:(c + 1) * maxid].sort().values
        assert torch.equal(blk, torch.arange(1, maxid + 1, device=gpu, dtype=torch.int64))
    assert not torch.equal(k[:maxid], k[maxid:2 * maxid])  # independent shuffles


def test_scan_column_dev(sgx, gpu):
    import torch

    n = 100_000
    c = torch.empty(n, dtype=torch.int32, device=gpu)
    sgx.gen_scan_dev(c, n, 0, 0, "i32")
    assert torch.equal(c, (torch.arange(n, device=gpu) % 256).to(torch.int32))
    u = torch.empty(n, dtype=torch.uint8, device=gpu)
    sgx.gen_scan_dev(u, n, 0, 0, "u8")
    assert torch.equal(u.to(torch.int32), c)


def test_zipf_dev_shape_and_kat(sgx, orc, gpu):
    """Device Zipf (genzipf.cpp:87-144): keys in 1..N, slices of one global relation,
    pk(1..N) join Zipf = |S| (the BASELINE config 5 KAT), GPU join == oracle join."""
    import torch

    N, n, theta = 1 << 16, 1 << 18, 0.75
    S = torch.empty(n, dtype=torch.int64, device=gpu)
    sgx.gen_zipf_dev(S, n, 0, N, theta, 22222)
    s = S.cpu().numpy().view(DT)
    assert s["key"].min() >= 1 and s["key"].max() <= N
    assert np.array_equal(s["payload"], np.arange(n, dtype=np.uint32))
    # two slices == one call
    S2 = torch.empty(n, dtype=torch.int64, device=gpu)
    sgx.gen_zipf_dev(S2[: n // 3], n // 3, 0, N, theta, 22222)
    sgx.gen_zipf_dev(S2[n // 3:], n - n // 3, n // 3, N, theta, 22222)
    assert torch.equal(S, S2)
    # frequency of the most common key ~ 1 / H(N, theta)
    h = np.sum(1.0 / np.arange(1, N + 1, dtype=np.float64) ** theta)
    top = np.bincount(s["key"]).max() / n
    assert abs(top - 1.0 / h) < 0.1 / h, (top, 1.0 / h)
    R = torch.empty(N, dtype=torch.int64, device=gpu)
    sgx.gen_pk_dev(R, N, 0, N, 11111)
    r = R.cpu().numpy().view(DT)
    res = sgx.rho_join(R, N, S, n)
    assert res.matches == n == orc.rho_join(r, s, 4)[0]
