"""ctypes wrapper of liboracle.so — the CPU restatement of the reference's RHO join
and predicate scans (oracle/rho_oracle.c, oracle/scan_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, as the checker / the timed CPU baseline.  The
product (libsgxamd.so and its Python binding) never imports this module.
Parity pinning: see oracle.h and DESIGN.md ("Oracle").
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def _load() -> C.CDLL:
    if not os.path.exists(LIB):
        build()
    lib = C.CDLL(LIB)
    P = C.c_void_p
    U64P = C.POINTER(C.c_uint64)

    class Timing(C.Structure):
        _fields_ = [("radix_bits", C.c_uint32), ("passes", C.c_uint32), ("join_tasks", C.c_uint64),
                    ("s_total", C.c_double), ("s_partition", C.c_double), ("s_pass1", C.c_double),
                    ("s_pass2", C.c_double), ("s_join", C.c_double)]

    lib.Timing = Timing
    sig = {
        "oracle_calc_num_radix_bits": (C.c_uint32, [C.c_uint64, C.c_uint64]),
        "oracle_calc_num_passes": (C.c_uint32, [C.c_uint32]),
        "oracle_rho_join": (C.c_int64, [P, C.c_uint64, P, C.c_uint64, C.c_int, C.c_int, C.POINTER(Timing)]),
        "oracle_rho_join_mat": (C.c_int64, [P, C.c_uint64, P, C.c_uint64, C.c_int, C.c_int, P, C.c_uint64]),
        "oracle_rht_join": (C.c_int64, [P, C.c_uint64, P, C.c_uint64, C.c_int, C.c_int, P, C.c_uint64]),
        "oracle_count_join_sort": (C.c_int64, [P, C.c_uint64, P, C.c_uint64]),
        "oracle_radix_partition": (None, [P, C.c_uint64, C.c_int, C.c_uint32, C.c_uint32, P, U64P]),
        "oracle_scan_count_u8": (C.c_uint64, [C.c_uint8, C.c_uint8, P, C.c_size_t]),
        "oracle_scan_count_i32": (C.c_uint64, [C.c_int32, C.c_int32, P, C.c_size_t]),
        "oracle_scan_bitvector_u8": (None, [C.c_uint8, C.c_uint8, P, C.c_size_t, P]),
        "oracle_scan_bitvector_i32": (None, [C.c_int32, C.c_int32, P, C.c_size_t, P]),
        "oracle_scan_index_u8": (C.c_uint64, [C.c_uint8, C.c_uint8, P, C.c_size_t, P]),
        "oracle_scan_index_i32": (C.c_uint64, [C.c_int32, C.c_int32, P, C.c_size_t, P]),
        "oracle_scan_values_u8": (C.c_uint64, [C.c_uint8, C.c_uint8, P, C.c_size_t, P]),
        "oracle_scan_explicit_index_u8": (C.c_uint64, [C.c_uint8, C.c_uint8, P, P, C.c_size_t, P]),
        "oracle_scan_values_i32": (C.c_uint64, [C.c_int32, C.c_int32, P, C.c_size_t, P]),
        "oracle_scan_count_i32_mt": (C.c_uint64, [C.c_int32, C.c_int32, P, C.c_size_t, C.c_int]),
        "oracle_cpu_scan_bench": (C.c_double, [C.c_int, C.c_int, C.c_int64, C.c_int64, P, C.c_size_t, C.c_int,
                                               C.POINTER(C.c_int), C.c_int, U64P]),
        "oracle_scan_sum_u8": (C.c_uint64, [C.c_uint8, C.c_uint8, P, C.c_size_t]),
        "oracle_dict_scan": (C.c_uint64, [C.c_int64, C.c_int64, P, C.c_uint64, P, C.c_int, C.c_size_t, P]),
        "oracle_tpch_filter": (C.c_uint64, [C.c_int, C.c_int, P, P, P, P, P]),
        "oracle_tpch_q3": (C.c_int64, [P, P, P, C.c_int, C.c_int, U64P]),
        "oracle_tpch_q10": (C.c_int64, [P, P, P, P, C.c_int, C.c_int, U64P]),
        "oracle_tpch_q12": (C.c_int64, [P, P, C.c_int, C.c_int, U64P]),
        "oracle_tpch_q19": (C.c_int64, [P, P, C.c_int, C.c_int, U64P]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def _p(a) -> int:
    if hasattr(a, "data_ptr"):
        return a.data_ptr()
    return a.ctypes.data


def rho_join(R, S, nthreads: int = 1, force_two_passes: bool = False) -> tuple[int, dict]:
    """Reference RHO (count-only) on numpy row_t arrays; returns (matches, timing)."""
    t = lib.Timing()
    m = lib.oracle_rho_join(_p(R), len(R), _p(S), len(S), nthreads, 1 if force_two_passes else 0, C.byref(t))
    return int(m), {f: getattr(t, f) for f, _ in t._fields_}


def rho_join_triples(R, S, nthreads: int = 1, force_two_passes: bool = False):
    """Materialising RHO (radix_join.cpp:437-446): (n, 3) uint32 {key, R payload,
    S payload} in the restatement's per-thread order."""
    m = lib.oracle_rho_join(_p(R), len(R), _p(S), len(S), nthreads, 1 if force_two_passes else 0, None)
    out = np.zeros((max(m, 1), 3), dtype=np.uint32)
    got = lib.oracle_rho_join_mat(_p(R), len(R), _p(S), len(S), nthreads, 1 if force_two_passes else 0, _p(out), m)
    assert got == m
    return out[:m]


def rht_join(R, S, nthreads: int = 1, force_two_passes: bool = False) -> int:
    """RHT (histogram_join) match count."""
    return int(lib.oracle_rht_join(_p(R), len(R), _p(S), len(S), nthreads, 1 if force_two_passes else 0, None, 0))


def rht_join_triples(R, S, nthreads: int = 1, force_two_passes: bool = False):
    m = rht_join(R, S, nthreads, force_two_passes)
    out = np.zeros((max(m, 1), 3), dtype=np.uint32)
    got = lib.oracle_rht_join(_p(R), len(R), _p(S), len(S), nthreads, 1 if force_two_passes else 0, _p(out), m)
    assert got == m
    return out[:m]


def count_join_sort(R, S) -> int:
    return int(lib.oracle_count_join_sort(_p(R), len(R), _p(S), len(S)))


def calc_num_radix_bits(num_r: int, nthreads: int) -> int:
    return int(lib.oracle_calc_num_radix_bits(num_r, nthreads))


def calc_num_passes(bits: int) -> int:
    return int(lib.oracle_calc_num_passes(bits))


def radix_partition(inp, nthreads: int, shift: int, bits: int):
    import numpy as np

    out = np.empty_like(inp)
    starts = np.zeros((1 << bits) + 1, dtype=np.uint64)
    lib.oracle_radix_partition(_p(inp), len(inp), nthreads, shift, bits, _p(out),
                               starts.ctypes.data_as(C.POINTER(C.c_uint64)))
    return out, starts


def scan(kind: str, dtype: str, lo: int, hi: int, col):
    """kind in count/bitvector/index/values; dtype u8/i32; col a numpy array."""
    import numpy as np

    n = len(col)
    fn = getattr(lib, f"oracle_scan_{kind}_{dtype}")
    if kind == "count":
        return int(fn(lo, hi, _p(col), n))
    if kind == "bitvector":
        out = np.zeros((n + 63) // 64, dtype=np.uint64)
        fn(lo, hi, _p(col), n, _p(out))
        return out
    if kind == "index":
        out = np.empty(max(n, 1), dtype=np.uint64)
        k = fn(lo, hi, _p(col), n, _p(out))
        return out[:k]
    out = np.empty(max(n, 1), dtype=np.uint32 if dtype == "u8" else np.int32)
    k = fn(lo, hi, _p(col), n, _p(out))
    return out[:k]


def explicit_index_scan(lo: int, hi: int, index, col):
    """SIMD512::explicit_index_scan restated: uint64 index entries of the matching u8 rows."""
    idx = np.ascontiguousarray(index, dtype=np.uint64)
    c = np.ascontiguousarray(col, dtype=np.uint8)
    out = np.empty(max(len(c), 1), dtype=np.uint64)
    k = lib.oracle_scan_explicit_index_u8(lo, hi, _p(idx), _p(c), len(c), _p(out))
    return out[:k]


def explicit_index_len(n: int) -> int:
    """Index entries row n-1 can reach (8*((n-1)/64 + 7) + 8): what a caller allocates."""
    return 0 if n == 0 else 8 * ((n - 1) // 64 + 7) + 8


def scan_count_mt(lo: int, hi: int, col, nthreads: int) -> int:
    return int(lib.oracle_scan_count_i32_mt(lo, hi, _p(col), len(col), nthreads))


def cpu_scan_bench(kind: str, col, lo: int, hi: int, nthreads: int, cpus=None, reps: int = 1) -> tuple[float, int]:
    """The timed CPU scan baseline (cpu_baseline.c): per-call seconds averaged over
    `nthreads` threads (pinned one per core to `cpus` if given) and the total matches."""
    k = {"count": 0, "bitvector": 1, "index": 2}[kind]
    width = col.dtype.itemsize
    cp = (C.c_int * nthreads)(*cpus) if cpus else None
    m = C.c_uint64(0)
    s = lib.oracle_cpu_scan_bench(k, width, lo, hi, _p(col), len(col), nthreads, cp, reps, C.byref(m))
    if s < 0:
        raise RuntimeError("oracle_cpu_scan_bench failed")
    return float(s), int(m.value)


def scan_sum_u8(lo: int, hi: int, col) -> int:
    return int(lib.oracle_scan_sum_u8(lo, hi, _p(col), len(col)))


def dict_scan(lo: int, hi: int, dictionary, codes):
    """dict_scan_{8,16,32}bit_64bit restated: int64 values dict[code] of the matching rows."""
    d = np.ascontiguousarray(dictionary, dtype=np.int64)
    c = np.ascontiguousarray(codes)
    k = int(lib.oracle_dict_scan(lo, hi, _p(d), len(d), _p(c), c.dtype.itemsize, len(c), None))
    out = np.zeros(max(k, 1), dtype=np.int64)
    lib.oracle_dict_scan(lo, hi, _p(d), len(d), _p(c), c.dtype.itemsize, len(c), _p(out))
    return out[:k]


# ---------------------------------------------------------------- TPC-H ---
# `tables` is any object with .struct(name) -> ctypes table struct (host columns),
# e.g. sgxamd.tpch.Tables; the structs follow sgxamd/tpch.h.
_ROW = np.dtype([("key", "<u4"), ("payload", "<u4")])


def _sp(tables, name):
    s = tables.struct(name)
    return C.addressof(s) if s is not None else None, s


def tpch_filter(query: int, which: int, tables) -> np.ndarray:
    """filter_table (filters.hpp:118-138) of one selection: rows in input order."""
    refs = [_sp(tables, t) for t in ("customer", "orders", "lineitem", "part")]
    cap = max(tables.n(t) for t in ("customer", "orders", "lineitem", "part")) + 1
    out = np.zeros(cap, dtype=_ROW)
    k = lib.oracle_tpch_filter(query, which, *[r[0] for r in refs], out.ctypes.data)
    return out[:k]


def tpch_query(query: int, tables, nthreads: int = 4, rht: bool = False) -> dict:
    """tpch.cpp's query `query` on the CPU restatement: result + per-step sizes."""
    info = (C.c_uint64 * 6)()
    names = {3: ("customer", "orders", "lineitem"), 10: ("customer", "orders", "lineitem", "nation"),
             12: ("lineitem", "orders"), 19: ("lineitem", "part")}[query]
    refs = [_sp(tables, t) for t in names]
    fn = getattr(lib, f"oracle_tpch_q{query}")
    res = fn(*[r[0] for r in refs], nthreads, 1 if rht else 0, info)
    return {"result": int(res), "filtered": [int(x) for x in info[0:3]], "join_matches": [int(x) for x in info[3:6]]}
