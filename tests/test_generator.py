"""Host generators restate the reference's (generator.cpp, genzipf.cpp) bit for bit."""
import ctypes as C
import ctypes.util

import numpy as np
import pytest

DT = np.dtype([("key", "<u4"), ("payload", "<u4")])


def test_glibc_rand_restatement_matches_libc(sgx):
    libc = C.CDLL(ctypes.util.find_library("c"))
    libc.rand.restype = C.c_int
    for seed in (0, 1, 11111, 22222, 2**31 - 1, 4000000000):
        libc.srand(C.c_uint(seed))
        sgx.gen_seed(seed)
        ref = [libc.rand() for _ in range(5000)]
        got = [sgx.lib.mi355_gen_rand() for _ in range(5000)]
        assert ref == got, seed


def _libc_knuth_pk(n, seed):
    """random_unique_gen + knuth_shuffle (generator.cpp:100-153) driven by the real libc rand()."""
    libc = C.CDLL(ctypes.util.find_library("c"))
    libc.rand.restype = C.c_int
    libc.srand(C.c_uint(seed))
    keys = list(range(1, n + 1))
    for i in range(n - 1, 0, -1):
        j = int(float(libc.rand()) / (2147483647.0 + 1.0) * float(i))
        keys[i], keys[j] = keys[j], keys[i]
    return keys


@pytest.mark.parametrize("n", [1, 2, 3, 1000, 4096])
def test_pk_matches_libc_driven_shuffle(sgx, n):
    R = np.empty(n, dtype=DT)
    sgx.gen_seed(11111)
    sgx.gen_pk(R, n)
    assert R["key"].tolist() == _libc_knuth_pk(n, 11111)
    assert R["payload"].tolist() == list(range(n))


def test_pk_is_permutation(sgx):
    n = 1 << 18
    R = np.empty(n, dtype=DT)
    sgx.gen_seed(11111)
    sgx.gen_pk(R, n)
    assert np.array_equal(np.sort(R["key"]), np.arange(1, n + 1, dtype=np.uint32))


def test_fk_is_shuffled_copies(sgx):
    # create_relation_fk(n, maxid): n / maxid copies of 1..maxid, then a shuffled 1..(n % maxid)
    n, maxid = 10_000, 3_000
    S = np.empty(n, dtype=DT)
    sgx.gen_seed(22222)
    sgx.gen_fk(S, n, maxid)
    for c in range(3):
        blk = S["key"][c * maxid:(c + 1) * maxid]
        assert np.array_equal(np.sort(blk), np.arange(1, maxid + 1))
    assert np.array_equal(np.sort(S["key"][9000:]), np.arange(1, 1001))


def test_fk_sel_integer_jump(sgx):
    # native.cpp:96 maxid = 100 * |R| / sel; random_unique_gen_maxid uses jump = maxid / n (integer)
    n = 4096
    maxid = 100 * n // 50
    S = np.empty(n, dtype=DT)
    sgx.gen_seed(22222)
    sgx.gen_fk_sel(S, n, maxid)
    assert np.array_equal(np.sort(S["key"]), np.arange(1, 2 * n, 2, dtype=np.uint32))


def test_zipf_deterministic_and_in_alphabet(sgx):
    n, alpha = 50_000, 4096
    A = np.empty(n, dtype=DT)
    B = np.empty(n, dtype=DT)
    sgx.gen_zipf(A, n, alpha, 0.75, 22222, 1)
    sgx.gen_zipf(B, n, alpha, 0.75, 22222, 7)  # thread count must not change the result
    assert np.array_equal(A["key"], B["key"])
    assert A["key"].min() >= 1 and A["key"].max() <= alpha
    # skewed: the hottest key is much more frequent than average
    counts = np.bincount(A["key"], minlength=alpha + 1)
    assert counts.max() > 20 * (n / alpha)


def test_reference_relations_helper(sgx):
    R, S = sgx.reference_relations(1 << 12, 1 << 13)
    assert np.array_equal(np.sort(R["key"]), np.arange(1, (1 << 12) + 1))
    assert np.array_equal(np.bincount(S["key"])[1:], np.full(1 << 12, 2))
