"""The HBM ceiling probes (mi355_stream_probe) that bench.py prices the kernels against:
the copy moves exactly the bytes, the write fills its pattern, the read leaves its
buffer alone, and bad arguments are refused."""
import pytest

pytestmark = pytest.mark.gpu


def test_stream_probe_copy_read_write(sgx):
    import torch

    n = (1 << 22) + 16  # bytes: a ragged tail past the grid's stride
    src = torch.randint(0, 2**31 - 1, (n // 4,), dtype=torch.int32, device="cuda")
    for ntl, nts, u, grid in ((True, True, 4, 0), (False, False, 8, 7), (True, False, 1, 3), (False, True, 2, 4096)):
        dst = torch.zeros_like(src)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        sgx.stream_probe("copy", src, dst, n, nt_load=ntl, nt_store=nts, loads_in_flight=u, grid=grid,
                         stream=s.cuda_stream)
        s.synchronize()
        assert torch.equal(dst, src), (ntl, nts, u, grid)
    w = torch.zeros(n // 4, dtype=torch.int32, device="cuda")
    sgx.stream_probe("write", None, w, n, loads_in_flight=4)
    torch.cuda.synchronize()
    v = w.view(-1, 4).cpu()
    assert torch.equal(v[:, 1], torch.ones(n // 16, dtype=torch.int32))
    assert torch.equal(v[:, 0], torch.arange(n // 16, dtype=torch.int32))
    word = torch.zeros(4, dtype=torch.int32, device="cuda")
    before = src.clone()
    sgx.stream_probe("read", src, word, n, loads_in_flight=8)
    torch.cuda.synchronize()
    assert torch.equal(src, before)


def test_stream_probe_rejects_bad_arguments(sgx):
    import torch

    a = torch.zeros(64, dtype=torch.int32, device="cuda")
    with pytest.raises(sgx.Mi355Error):
        sgx.stream_probe("copy", a, a, 100)  # not a multiple of 16
    with pytest.raises(sgx.Mi355Error):
        sgx.stream_probe("copy", a, a, 64, loads_in_flight=3)  # 1, 2, 4 or 8
