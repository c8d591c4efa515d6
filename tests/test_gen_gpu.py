"""Device generators: pk/fk shapes (shuffled 1..n / copies of 1..maxid), slice-consistent."""
import pytest

pytestmark = pytest.mark.gpu


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
