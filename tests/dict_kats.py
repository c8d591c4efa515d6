"""The dictionary-scan known-answer cases of the reference's Catch2 suite
(Scan-Micro-Benchmarks/shared_libraries/SimdScan/tests/testsimdscan.cpp, [main]
cases :8-245 and :478-529), as (name, code dtype, codes, dictionary, lo, hi,
expected size, {index: value}) built with the reference allocator's rule
(Allocator.hpp:94-117: uint8 i % 256, other types i % (max + 1); a generator
where the test passes one).  Shared by the CPU oracle test and the GPU test."""
import numpy as np

N = 1 << 20


def _default(dtype, n):
    dt = np.dtype(dtype)
    if dt == np.uint8:
        return (np.arange(n) % 256).astype(np.uint8)
    return (np.arange(n, dtype=np.uint64) % (np.iinfo(dt).max + 1)).astype(dt)


def cases():
    d256 = np.arange(256, dtype=np.int64)
    u8 = _default(np.uint8, N)
    yield "dict8 test1 :8-28", u8, d256, 0, 100, N // 256 * 101, {}
    yield "dict8 test2 :30-54", u8, d256, 1, 100, N // 256 * 100, {**{i: i + 1 for i in range(100)}, 100: 1}
    yield "dict8 test3 :56-84", u8, d256 * 2, 0, 98, N // 256 * 50, {**{i: 2 * i for i in range(50)}, 99: 98, 100: 0}
    yield "dict8 test4 :86-113", (np.arange(N) & 3).astype(np.uint8), d256, 0, 2, N // 4 * 3, {0: 0, 1: 1, 2: 2, 3: 0}
    yield "dict8 test5 :115-138", u8, d256, 100, 199, N // 256 * 100, {0: 100, 99: 199}
    yield "dict8 test6 :140-165", u8, d256 - 128, -10, 0, N // 256 * 11, {0: -10, 10: 0}
    yield ("dict16 test1 :167-190", _default(np.uint16, N), np.arange(1 << 16, dtype=np.int64), 0, 299,
           N // (1 << 16) * 300, {i: i % 300 for i in range(0, N // (1 << 16) * 300, 97)})
    d20 = np.arange(1 << 20, dtype=np.int64)
    yield "dict32 test1 :192-215", (np.arange(N) & 255).astype(np.uint32), d20, 0, 299, N, {}
    yield "dict32 sg test1 :478-502", (np.arange(N) & 255).astype(np.uint32), d20, 0, 299, N, {}
    yield "dict32 sg test2 :504-529", _default(np.uint32, N), d20, 0, 99, 100, {0: 0, 10: 10}
