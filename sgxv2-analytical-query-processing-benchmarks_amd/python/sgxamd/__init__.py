"""ctypes binding of libsgxamd.so, the MI355X RHO join + predicate scan C-ABI.

This is the Python side of the drop-in boundary declared in include/sgxamd/*.h:
the same entry points a cgo / JNI / ctypes caller of the reference would bind
(see INTEGRATION.md).  Arguments are raw pointers and sizes; torch tensors and
numpy arrays are accepted and passed by address (device tensors stay in HBM).

The library is built in-tree by ``make`` in the package directory (or
``__graft_entry__.build()``).  There is no CPU fallback: if libsgxamd.so is
missing, importing this module raises, and every compute call on a host
without a gfx950 device returns MI355_ERR_NO_DEVICE (raised as Mi355Error).
"""
from __future__ import annotations

import ctypes as C
import os

PKG_DIR = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# SGXAMD_LIB_PATH: a development build of the same library (scripts/build_variant.sh)
LIB_PATH = os.environ.get("SGXAMD_LIB_PATH") or os.path.join(PKG_DIR, "libsgxamd.so")

MI355_OK = 0
MI355_ERR_INVALID = -1
MI355_ERR_NO_DEVICE = -2
MI355_ERR_HIP = -3
MI355_ERR_OOM = -4
MI355_ERR_CAPACITY = -5


class Mi355Error(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"mi355 error {code}: {msg}")
        self.code = code


class row_t(C.Structure):
    _fields_ = [("key", C.c_uint32), ("payload", C.c_uint32)]


class table_t(C.Structure):
    _fields_ = [("tuples", C.c_void_p), ("num_tuples", C.c_uint64), ("ratio_holes", C.c_int), ("sorted", C.c_int)]


class result_t(C.Structure):
    _fields_ = [
        ("totalresults", C.c_int64),
        ("nthreads", C.c_int),
        ("throughput", C.c_double),
        ("materialized", C.c_int),
        ("result", C.c_void_p),
        ("result_type", C.c_int),
    ]


class joinconfig_t(C.Structure):
    _fields_ = [
        (n, C.c_int)
        for n in (
            "NTHREADS", "PARTFANOUT", "SCALARSORT", "SCALARMERGE", "MWAYMERGEBUFFERSIZE", "NUMASTRATEGY",
            "RADIXBITS", "WRITETOFILE", "MATERIALIZE", "PRINT", "CRACKING_THRESHOLD", "ALLOC_CORE",
        )
    ]


class rho_opts(C.Structure):
    _fields_ = [
        ("radix_bits", C.c_int),
        ("passes", C.c_int),
        ("key_shift", C.c_uint32),
        ("materialize", C.c_int),
        ("timing", C.c_int),
        ("algorithm", C.c_int),
        ("stream", C.c_void_p),
        ("out", C.c_void_p),
        ("out_capacity", C.c_uint64),
    ]


class chunked_table_t(C.Structure):
    """data-types.h:86-92 (ChunkedTable.cpp): the MATERIALIZE=1 result of RHO."""
    _fields_ = [
        ("chunks", C.POINTER(C.c_void_p)),
        ("current_chunk", C.c_uint64),
        ("num_chunks", C.c_uint64),
        ("chunk_capacity", C.c_uint64),
        ("num_tuples", C.c_uint64),
    ]


TUPLES_PER_CHUNK = (16 * 1024 - 8) // 12  # data-types.h:80-81 with CSKB = 16


class rho_stats(C.Structure):
    _fields_ = [
        ("matches", C.c_uint64),
        ("radix_bits", C.c_uint32),
        ("passes", C.c_uint32),
        ("pass1_bits", C.c_uint32),
        ("pass2_bits", C.c_uint32),
        ("num_partitions", C.c_uint64),
        ("num_tasks", C.c_uint64),
        ("max_part_r", C.c_uint64),
        ("max_part_s", C.c_uint64),
        ("ms_h2d", C.c_double),
        ("ms_partition", C.c_double),
        ("ms_pass1", C.c_double),
        ("ms_pass2", C.c_double),
        ("ms_join", C.c_double),
        ("ms_total", C.c_double),
        ("ms_pass1_r", C.c_double),
        ("ms_pass1_s", C.c_double),
        ("ms_pass1_hist", C.c_double),
        ("ms_pass1_copy", C.c_double),
        ("ms_pass2_hist", C.c_double),
        ("ms_pass2_copy", C.c_double),
        ("ms_build", C.c_double),
        ("ms_probe", C.c_double),
        ("layout", C.c_uint32),
        ("elem_bytes", C.c_uint32),
        ("narrow", C.c_uint32),
        ("reserved0", C.c_uint32),
    ]

    def as_dict(self) -> dict:
        return {f: getattr(self, f) for f, _ in self._fields_}


class multi_stats(C.Structure):  # sgxamd/multi.h
    _fields_ = [
        ("matches", C.c_uint64),
        ("world", C.c_int),
        ("transport", C.c_int),
        ("pieces", C.c_int),
        ("rank", C.c_int),
        ("local_matches", C.c_uint64),
        ("recv_r_max", C.c_uint64),
        ("recv_r_min", C.c_uint64),
        ("recv_s_max", C.c_uint64),
        ("recv_s_min", C.c_uint64),
        ("max_part_s", C.c_uint64),
        ("sent_bytes", C.c_uint64),
        ("ms_total", C.c_double),
        ("ms_exchange_post", C.c_double),
        ("ms_local", C.c_double),
        ("ms_allreduce", C.c_double),
        ("local", rho_stats),
        ("elem_bytes", C.c_uint32),
        ("ms_tail", C.c_double),
    ]

    def as_dict(self) -> dict:
        d = {f: getattr(self, f) for f, _ in self._fields_ if f != "local"}
        d["local"] = self.local.as_dict()
        d["transport"] = {1: "rccl", 2: "rehearsal"}.get(self.transport, "?")
        return d


# TPC-H tables (sgxamd/tpch.h = TpcHTypes.hpp:53-87): column pointers, host or device.
class LineItemTable(C.Structure):
    _fields_ = [("numTuples", C.c_uint64), ("l_orderkey", C.c_void_p), ("l_shipdate", C.c_void_p),
                ("l_commitdate", C.c_void_p), ("l_receiptdate", C.c_void_p), ("l_shipmode", C.c_void_p),
                ("l_partkey", C.c_void_p), ("l_quantity", C.c_void_p), ("l_shipinstruct", C.c_void_p),
                ("l_returnflag", C.c_void_p)]


class OrdersTable(C.Structure):
    _fields_ = [("numTuples", C.c_uint64), ("o_orderkey", C.c_void_p), ("o_orderdate", C.c_void_p),
                ("o_custkey", C.c_void_p)]


class CustomerTable(C.Structure):
    _fields_ = [("numTuples", C.c_uint64), ("c_custkey", C.c_void_p), ("c_mktsegment", C.c_void_p),
                ("c_nationkey", C.c_void_p)]


class PartTable(C.Structure):
    _fields_ = [("numTuples", C.c_uint64), ("p_partkey", C.c_void_p), ("p_brand", C.c_void_p),
                ("p_size", C.c_void_p), ("p_container", C.c_void_p)]


class NationTable(C.Structure):
    _fields_ = [("numTuples", C.c_uint64), ("n_nationkey", C.c_void_p)]


class tpch_stats(C.Structure):
    _fields_ = [("result", C.c_uint64), ("join_matches", C.c_uint64 * 3), ("filtered", C.c_uint64 * 3),
                ("ms_selection", C.c_double * 3), ("ms_join", C.c_double * 3), ("ms_copy", C.c_double),
                ("ms_total", C.c_double), ("ms_h2d", C.c_double), ("input_tuples", C.c_uint64),
                ("column_bytes", C.c_uint64)]

    def as_dict(self) -> dict:
        out = {}
        for f, _ in self._fields_:
            v = getattr(self, f)
            out[f] = list(v) if hasattr(v, "__len__") else v
        return out


# Every symbol declared in include/sgxamd/*.h with its (restype, argtypes).
_P = C.c_void_p
_U64P = C.POINTER(C.c_uint64)
SIGNATURES = {
    # rho.h
    "mi355_device_count": (C.c_int, []),
    "mi355_last_error": (C.c_char_p, []),
    "mi355_version": (C.c_char_p, []),
    "mi355_rho_join": (C.c_int, [C.POINTER(table_t), C.POINTER(table_t), C.POINTER(joinconfig_t), C.POINTER(result_t)]),
    "mi355_rho_join_ex": (C.c_int, [_P, C.c_uint64, _P, C.c_uint64, C.POINTER(rho_opts), C.POINTER(rho_stats)]),
    "mi355_free_chunked_table": (None, [_P]),
    "mi355_rht_join": (C.c_int, [C.POINTER(table_t), C.POINTER(table_t), C.POINTER(joinconfig_t), C.POINTER(result_t)]),
    "mi355_last_join_stats": (C.c_int, [C.POINTER(rho_stats)]),
    "mi355_rho_shard_partition": (C.c_int, [_P, C.c_uint64, C.c_uint32, C.c_uint32, _P, _U64P, _P]),
    "mi355_rho_join_begin": (C.c_int, [_P, C.c_uint64, C.c_uint64, C.POINTER(rho_opts)]),
    "mi355_rho_join_finish": (C.c_int, [_P, C.c_uint64, C.POINTER(rho_opts), C.POINTER(rho_stats)]),
    "mi355_timing_enable": (None, [C.c_int]),
    "mi355_set_partition_overlap": (None, [C.c_int]),
    "mi355_set_key_layout": (None, [C.c_int]),
    "mi355_timing_get": (C.c_int, [C.POINTER(C.c_char_p), C.POINTER(C.c_double), C.c_int]),
    "mi355_set_stream": (None, [_P]),
    "mi355_stream_probe": (C.c_int, [C.c_int, _P, _P, C.c_uint64, C.c_int, C.c_int, C.c_int, C.c_uint32, _P]),
    # multi.h
    "mi355_rho_join_multi_ex": (C.c_int, [_P, C.c_uint64, _P, C.c_uint64, C.c_int, C.c_int, C.POINTER(rho_opts),
                                          C.POINTER(multi_stats)]),
    "mi355_rho_join_multi": (C.c_int, [C.POINTER(table_t), C.POINTER(table_t), C.POINTER(joinconfig_t), C.c_int,
                                       C.POINTER(result_t)]),
    "mi355_multi_unique_id": (C.c_int, [_P]),
    "mi355_multi_comm_init": (C.c_int, [_P, C.c_int, C.c_int, C.POINTER(C.c_void_p)]),
    "mi355_multi_comm_destroy": (C.c_int, [_P]),
    "mi355_rho_join_sharded": (C.c_int, [_P, _P, C.c_uint64, _P, C.c_uint64, C.POINTER(rho_opts),
                                         C.POINTER(multi_stats)]),
    "mi355_last_multi_stats": (C.c_int, [C.POINTER(multi_stats)]),
    "mi355_multi_set_pieces": (None, [C.c_int]),
    "mi355_multi_set_wire": (None, [C.c_int]),
    "mi355_multi_inject_failure": (None, [C.c_int, C.c_int]),
    "mi355_multi_set_rccl_library": (C.c_int, [C.c_char_p]),
    "mi355_multi_release": (C.c_int, []),
    "mi355_release_workspace": (C.c_int, []),
    # scan.h
    "mi355_scan_count_u8": (C.c_int, [C.c_uint8, C.c_uint8, _P, C.c_size_t, _U64P]),
    "mi355_scan_count_i32": (C.c_int, [C.c_int32, C.c_int32, _P, C.c_size_t, _U64P]),
    "mi355_scan_bitvector_u8": (C.c_int, [C.c_uint8, C.c_uint8, _P, C.c_size_t, _P]),
    "mi355_scan_bitvector_i32": (C.c_int, [C.c_int32, C.c_int32, _P, C.c_size_t, _P]),
    "mi355_scan_index_u8": (C.c_int, [C.c_uint8, C.c_uint8, _P, C.c_size_t, _P, C.c_size_t, _U64P]),
    "mi355_scan_index_i32": (C.c_int, [C.c_int32, C.c_int32, _P, C.c_size_t, _P, C.c_size_t, _U64P]),
    "mi355_scan_explicit_index_u8": (C.c_int, [C.c_uint8, C.c_uint8, _P, C.c_size_t, _P, C.c_size_t, _P,
                                               C.c_size_t, _U64P]),
    "mi355_scan_values_u8": (C.c_int, [C.c_uint8, C.c_uint8, _P, C.c_size_t, _P, C.c_size_t, _U64P]),
    "mi355_scan_values_i32": (C.c_int, [C.c_int32, C.c_int32, _P, C.c_size_t, _P, C.c_size_t, _U64P]),
    "mi355_scan_sum_u8": (C.c_int, [C.c_uint8, C.c_uint8, _P, C.c_size_t, _U64P]),
    "mi355_dict_scan_8bit_64bit": (C.c_int, [C.c_int64, C.c_int64, _P, _P, C.c_size_t, _P, C.c_size_t, _U64P]),
    "mi355_dict_scan_16bit_64bit": (C.c_int, [C.c_int64, C.c_int64, _P, _P, C.c_size_t, _P, C.c_size_t, _U64P]),
    "mi355_dict_scan_32bit_64bit": (C.c_int, [C.c_int64, C.c_int64, _P, C.c_size_t, _P, C.c_size_t, _P, C.c_size_t,
                                              _U64P]),
    # generator.h
    "mi355_gen_seed": (None, [C.c_uint]),
    "mi355_gen_rand": (C.c_int, []),
    "mi355_gen_pk": (C.c_int, [_P, C.c_uint64]),
    "mi355_gen_fk": (C.c_int, [_P, C.c_uint64, C.c_int64]),
    "mi355_gen_fk_sel": (C.c_int, [_P, C.c_uint64, C.c_int64]),
    "mi355_gen_zipf": (C.c_int, [_P, C.c_uint64, C.c_uint32, C.c_double, C.c_uint64, C.c_int]),
    "mi355_gen_scan_u8": (C.c_int, [_P, C.c_size_t]),
    "mi355_gen_scan_i32": (C.c_int, [_P, C.c_size_t]),
    "mi355_gen_pk_dev": (C.c_int, [_P, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, _P]),
    "mi355_gen_fk_dev": (C.c_int, [_P, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, _P]),
    "mi355_gen_zipf_dev": (C.c_int, [_P, C.c_uint64, C.c_uint64, C.c_uint32, C.c_double, C.c_uint64, _P]),
    "mi355_gen_scan_u8_dev": (C.c_int, [_P, C.c_size_t, C.c_int, C.c_uint64, _P]),
    "mi355_gen_scan_i32_dev": (C.c_int, [_P, C.c_size_t, C.c_int, C.c_uint64, _P]),
    # tpch.h
    "mi355_tpch_q3": (C.c_int, [C.POINTER(CustomerTable), C.POINTER(OrdersTable), C.POINTER(LineItemTable), C.c_int,
                                C.POINTER(tpch_stats)]),
    "mi355_tpch_q10": (C.c_int, [C.POINTER(CustomerTable), C.POINTER(OrdersTable), C.POINTER(LineItemTable),
                                 C.POINTER(NationTable), C.c_int, C.POINTER(tpch_stats)]),
    "mi355_tpch_q12": (C.c_int, [C.POINTER(LineItemTable), C.POINTER(OrdersTable), C.c_int, C.POINTER(tpch_stats)]),
    "mi355_tpch_q19": (C.c_int, [C.POINTER(LineItemTable), C.POINTER(PartTable), C.c_int, C.POINTER(tpch_stats),
                                 C.c_int, C.POINTER(C.c_void_p)]),
    "mi355_tpch_filter": (C.c_int, [C.c_int, C.c_int, C.POINTER(CustomerTable), C.POINTER(OrdersTable),
                                    C.POINTER(LineItemTable), C.POINTER(PartTable), _P, C.c_uint64, _U64P]),
    "mi355_tpch_load_lineitem": (C.c_int, [C.POINTER(LineItemTable), C.c_char_p, C.c_int, C.c_int, C.c_int]),
    "mi355_tpch_load_orders": (C.c_int, [C.POINTER(OrdersTable), C.c_char_p, C.c_int, C.c_int, C.c_int]),
    "mi355_tpch_load_customer": (C.c_int, [C.POINTER(CustomerTable), C.c_char_p, C.c_int, C.c_int, C.c_int]),
    "mi355_tpch_load_part": (C.c_int, [C.POINTER(PartTable), C.c_char_p, C.c_int, C.c_int, C.c_int]),
    "mi355_tpch_load_nation": (C.c_int, [C.POINTER(NationTable), C.c_char_p, C.c_int, C.c_int, C.c_int]),
    "mi355_tpch_store": (C.c_int, [C.c_char_p, C.c_int, C.POINTER(LineItemTable), C.POINTER(OrdersTable),
                                   C.POINTER(CustomerTable), C.POINTER(PartTable), C.POINTER(NationTable)]),
    "mi355_tpch_free_lineitem": (None, [C.POINTER(LineItemTable)]),
    "mi355_tpch_free_orders": (None, [C.POINTER(OrdersTable)]),
    "mi355_tpch_free_customer": (None, [C.POINTER(CustomerTable)]),
    "mi355_tpch_free_part": (None, [C.POINTER(PartTable)]),
    "mi355_tpch_free_nation": (None, [C.POINTER(NationTable)]),
    "mi355_tpch_generate": (C.c_int, [C.c_uint32, C.c_uint64, C.POINTER(LineItemTable), C.POINTER(OrdersTable),
                                      C.POINTER(CustomerTable), C.POINTER(PartTable), C.POINTER(NationTable)]),
    "mi355_tpch_sizes": (C.c_int, [C.c_uint32, C.c_uint64, _U64P, _U64P, _U64P, _U64P, _U64P]),
    "mi355_tpch_generate_dev": (C.c_int, [C.c_uint32, C.c_uint64, C.POINTER(LineItemTable), C.POINTER(OrdersTable),
                                          C.POINTER(CustomerTable), C.POINTER(PartTable), C.POINTER(NationTable),
                                          _P]),
}


def _load() -> C.CDLL:
    # PyTorch-ROCm ships its own libamdhip64 / libhsa-runtime64 (SONAME libamdhip64.so.7).
    # Loading torch first makes libsgxamd.so bind to that same HIP runtime instead of
    # /opt/rocm's, so one process never holds two HIP runtimes (torch tensors are then
    # device pointers of our runtime too).  Without torch, /opt/rocm's runtime is used.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `make -C {PKG_DIR}` or __graft_entry__.build(); "
            "there is no CPU fallback for the MI355X kernels"
        )
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def last_error() -> str:
    return (lib.mi355_last_error() or b"").decode()


def _check(rc: int) -> None:
    if rc != MI355_OK:
        raise Mi355Error(rc, last_error())


def ptr(x) -> int:
    """Address of a torch tensor, numpy array, ctypes object or int."""
    if x is None:
        return 0
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    if hasattr(x, "ctypes"):
        return x.ctypes.data
    return C.addressof(x)


def device_count() -> int:
    return lib.mi355_device_count()


def version() -> str:
    return lib.mi355_version().decode()


# ------------------------------------------------------------------ join ---
class JoinResult:
    """Match count and the call's statistics.  `stats` (a dict of the stats struct's
    fields) is built on first access: building it took ~4.5 us, a third of the Python
    overhead of a small join."""

    __slots__ = ("matches", "_raw", "_stats")

    def __init__(self, matches: int, raw):
        self.matches = matches
        self._raw = raw  # rho_stats / multi_stats, or an already built dict
        self._stats = raw if isinstance(raw, dict) else None

    @property
    def stats(self) -> dict:
        if self._stats is None:
            self._stats = self._raw.as_dict()
        return self._stats

    def stat(self, name: str):
        """One field of the stats, without building the dict."""
        return self._stats[name] if self._stats is not None else getattr(self._raw, name)

    def __repr__(self) -> str:
        return f"JoinResult(matches={self.matches}, stats={self.stats})"


ALGORITHMS = {"RHO": 0, "RHT": 1}  # MI355_ALGO_RHO / MI355_ALGO_RHT


def rho_join(R, nR: int, S, nS: int, *, radix_bits: int = 0, passes: int = 0, key_shift: int = 0,
             timing: bool = False, stream: int | None = None, out=None, out_capacity: int = 0,
             algorithm: str = "RHO") -> JoinResult:
    """RHO join of nR R-tuples and nS S-tuples (8-byte {key, payload}; host or device).

    With `out` (host or device buffer of out_capacity 12-byte triples) every match is
    materialised as {key, R payload, S payload}; a too-small buffer raises Mi355Error
    with code MI355_ERR_CAPACITY (-5)."""
    o = rho_opts(radix_bits, passes, key_shift, 1 if out is not None else 0, 1 if timing else 0,
                 ALGORITHMS[algorithm], stream or None, ptr(out) if out is not None else None, out_capacity)
    st = rho_stats()
    rc = lib.mi355_rho_join_ex(ptr(R), nR, ptr(S), nS, C.byref(o), C.byref(st))
    if rc == -5:
        raise Mi355Error(rc, f"capacity: {int(st.matches)} triples needed")
    _check(rc)
    return JoinResult(int(st.matches), st)


def rho_join_begin(R, nR: int, nS: int, *, key_shift: int = 0, stream: int | None = None,
                   algorithm: str = "RHO") -> None:
    """First half of a pipelined count join (mi355_rho_join_begin): plans both
    relations and enqueues R's partition passes on `stream`; returns at once."""
    o = rho_opts(0, 0, key_shift, 0, 0, ALGORITHMS[algorithm], stream or None, None, 0)
    _check(lib.mi355_rho_join_begin(ptr(R), nR, nS, C.byref(o)))


def rho_join_finish(S, nS: int, *, key_shift: int = 0, stream: int | None = None,
                    algorithm: str = "RHO") -> JoinResult:
    """Second half (mi355_rho_join_finish): S's passes and build/probe, after S became
    valid in the stream order; blocks and returns the count."""
    o = rho_opts(0, 0, key_shift, 0, 0, ALGORITHMS[algorithm], stream or None, None, 0)
    st = rho_stats()
    _check(lib.mi355_rho_join_finish(ptr(S), nS, C.byref(o), C.byref(st)))
    return JoinResult(int(st.matches), st)


TRANSPORTS = {"auto": 0, "rccl": 1, "rehearsal": 2}  # MI355_TRANSPORT_*


def rho_join_multi(R, nR: int, S, nS: int, ngpus: int, *, transport: str = "auto", algorithm: str = "RHO",
                   radix_bits: int = 0, passes: int = 0, out=None, out_capacity: int = 0) -> JoinResult:
    """Multi-GPU join in one process (mi355_rho_join_multi_ex): ngpus ranks, the
    radix-shard exchange over RCCL or the one-GPU rehearsal transport.  With `out`
    (host or device buffer of out_capacity 12-byte triples) the join materialises:
    every rank's triples, rank 0's first."""
    o = rho_opts(radix_bits, passes, 0, 1 if out is not None else 0, 0, ALGORITHMS[algorithm], None,
                 ptr(out) if out is not None else None, out_capacity)
    st = multi_stats()
    rc = lib.mi355_rho_join_multi_ex(ptr(R), nR, ptr(S), nS, ngpus, TRANSPORTS[transport], C.byref(o), C.byref(st))
    if rc == -5:  # MI355_ERR_CAPACITY
        raise Mi355Error(rc, f"capacity: {int(st.matches)} triples needed")
    _check(rc)
    return JoinResult(int(st.matches), st)


def multi_unique_id() -> bytes:
    """128-byte RCCL unique id (rank 0 creates it, every rank passes it to multi_comm_init)."""
    buf = C.create_string_buffer(128)
    _check(lib.mi355_multi_unique_id(buf))
    return buf.raw


def multi_comm_init(uid: bytes, nranks: int, rank: int) -> int:
    """This process's RCCL communicator on its current device (collective)."""
    h = C.c_void_p()
    buf = C.create_string_buffer(bytes(uid), 128)
    _check(lib.mi355_multi_comm_init(buf, nranks, rank, C.byref(h)))
    return h.value


def multi_comm_destroy(handle: int) -> None:
    _check(lib.mi355_multi_comm_destroy(handle))


def rho_join_sharded(handle: int, R, nR: int, S, nS: int, *, algorithm: str = "RHO", radix_bits: int = 0,
                     passes: int = 0, out=None, out_capacity: int = 0) -> JoinResult:
    """One rank's part of the multi-GPU join (collective; device-resident slices).  With
    `out` the join materialises and this rank's own triples (stats["local_matches"] of
    them) are written to it.  radix_bits / passes: the local joins' plan (every rank the
    same; 0 = from the global sizes)."""
    o = rho_opts(radix_bits, passes, 0, 1 if out is not None else 0, 0, ALGORITHMS[algorithm], None,
                 ptr(out) if out is not None else None, out_capacity)
    st = multi_stats()
    _check(lib.mi355_rho_join_sharded(handle, ptr(R), nR, ptr(S), nS, C.byref(o), C.byref(st)))
    return JoinResult(int(st.matches), st)


def multi_set_pieces(pieces: int) -> None:
    lib.mi355_multi_set_pieces(pieces)


def multi_set_wire(mode: int) -> None:
    """The u16 wire: 0 off, 1 auto (default), 2 whenever the residuals fit (mi355_multi_set_wire)."""
    lib.mi355_multi_set_wire(mode)


def release_workspace() -> None:
    """Free the current device's workspace (mi355_release_workspace)."""
    _check(lib.mi355_release_workspace())


def multi_release() -> None:
    """Free the rehearsal ranks' workspaces (mi355_multi_release)."""
    _check(lib.mi355_multi_release())


def multi_inject_failure(rank: int, step: int) -> None:
    """Test hook: `rank` fails at `step` (1 buffers, 2 a shard pass, 3 the local join, 4 no
    device context, 5 the local join's stream synchronisation) of every later
    multi-GPU join; step 0 clears it."""
    lib.mi355_multi_inject_failure(rank, step)


def multi_set_rccl_library(path: str | None) -> None:
    """Test hook (mi355_multi_set_rccl_library): load `path` instead of librccl.so.1 for
    later multi-GPU calls (None: librccl.so.1 again)."""
    _check(lib.mi355_multi_set_rccl_library(path.encode() if path else None))


def rho_join_tables(R, nR: int, S, nS: int, nthreads: int = 1, materialize: bool = False,
                    algorithm: str = "RHO") -> result_t:
    """The drop-in mi355_rho_join(table_t*, table_t*, joinconfig_t*, result_t*).

    With materialize, result.result is a chunked_table_t* (result_type 1): read it
    with chunked_table_triples() and release it with free_result()."""
    tR = table_t(ptr(R), nR, 0, 0)
    tS = table_t(ptr(S), nS, 0, 0)
    cfg = joinconfig_t()
    cfg.NTHREADS = nthreads
    cfg.MATERIALIZE = 1 if materialize else 0
    out = result_t()
    fn = lib.mi355_rht_join if algorithm == "RHT" else lib.mi355_rho_join
    _check(fn(C.byref(tR), C.byref(tS), C.byref(cfg), C.byref(out)))
    return out


def chunked_table_triples(res: result_t):
    """numpy (n, 3) uint32 array of the {key, Rpayload, Spayload} triples of a
    materialised result (chunk order)."""
    import numpy as np

    if not res.materialized or res.result_type != 1 or not res.result:
        return np.zeros((0, 3), dtype=np.uint32)
    return chunked_table_triples_ptr(res.result)


def chunked_table_triples_ptr(table_ptr: int):
    """The triples of the chunked_table_t at table_ptr, as chunked_table_triples."""
    import numpy as np

    if not table_ptr:
        return np.zeros((0, 3), dtype=np.uint32)
    t = C.cast(table_ptr, C.POINTER(chunked_table_t)).contents
    parts = []
    for c in range(t.num_chunks):
        base = t.chunks[c]
        k = C.c_uint64.from_address(base).value
        if k:
            parts.append(np.frombuffer(C.string_at(base + 8, 12 * k), dtype=np.uint32).reshape(k, 3))
    return np.concatenate(parts) if parts else np.zeros((0, 3), dtype=np.uint32)


def free_result(res: result_t) -> None:
    if res.result and res.result_type == 1:
        lib.mi355_free_chunked_table(res.result)
        res.result = None


def shard_partition(inp, n: int, key_shift: int, dest_bits: int, out, stream: int | None = None) -> list[int]:
    counts = (C.c_uint64 * (1 << dest_bits))()
    _check(lib.mi355_rho_shard_partition(ptr(inp), n, key_shift, dest_bits, ptr(out), counts, stream or None))
    return [int(c) for c in counts]


def timing_enable(on=True) -> None:
    """Per-kernel HIP events: True (every kernel), False, or "sparse" (R's pass-1 scatter
    and the build/probe only, the launches between them as one span "other")."""
    lib.mi355_timing_enable(2 if on == "sparse" else 1 if on else 0)


def set_partition_overlap(on: bool = True) -> None:
    """R/S partition chains on two streams (default) or back to back on one."""
    lib.mi355_set_partition_overlap(1 if on else 0)


def set_key_layout(on: bool = True) -> None:
    """Counting joins on this thread move 4-byte keys after the input read (default) or
    whole 8-byte tuples (the reference's data movement); counts are identical."""
    lib.mi355_set_key_layout(1 if on else 0)


def timings() -> list[tuple[str, float]]:
    cap = 256
    names = (C.c_char_p * cap)()
    ms = (C.c_double * cap)()
    n = lib.mi355_timing_get(names, ms, cap)
    return [(names[i].decode(), ms[i]) for i in range(min(n, cap))]


def set_stream(stream: int | None) -> None:
    lib.mi355_set_stream(stream or None)


# ------------------------------------------------------------------ scan ---
def _scan_fn(kind: str, dtype: str):
    return getattr(lib, f"mi355_scan_{kind}_{dtype}")


def scan_count(lo: int, hi: int, col, n: int, dtype: str = "i32") -> int:
    c = C.c_uint64()
    _check(_scan_fn("count", dtype)(lo, hi, ptr(col), n, C.byref(c)))
    return int(c.value)


def scan_bitvector(lo: int, hi: int, col, n: int, out_words, dtype: str = "i32") -> None:
    _check(_scan_fn("bitvector", dtype)(lo, hi, ptr(col), n, ptr(out_words)))


def scan_index(lo: int, hi: int, col, n: int, out, cap: int, dtype: str = "i32") -> int:
    c = C.c_uint64()
    _check(_scan_fn("index", dtype)(lo, hi, ptr(col), n, ptr(out), cap, C.byref(c)))
    return int(c.value)


def scan_explicit_index(lo: int, hi: int, index, index_len: int, col, n: int, out, cap: int) -> int:
    """SIMD512::explicit_index_scan over a u8 column: the index entries of the matching rows."""
    c = C.c_uint64()
    _check(lib.mi355_scan_explicit_index_u8(lo, hi, ptr(index), index_len, ptr(col), n, ptr(out), cap,
                                            C.byref(c)))
    return int(c.value)


def scan_values(lo: int, hi: int, col, n: int, out, cap: int, dtype: str = "i32") -> int:
    c = C.c_uint64()
    _check(_scan_fn("values", dtype)(lo, hi, ptr(col), n, ptr(out), cap, C.byref(c)))
    return int(c.value)


# ------------------------------------------------------------- generators ---
def scan_sum_u8(lo: int, hi: int, col, n: int) -> int:
    out = C.c_uint64()
    _check(lib.mi355_scan_sum_u8(lo, hi, ptr(col), n, C.byref(out)))
    return int(out.value)


def dict_scan(lo: int, hi: int, dictionary, codes, n: int, out, cap: int, code_bits: int,
              dict_size: int | None = None) -> int:
    """dict_scan_{8,16,32}bit_64bit: writes dict[code] (int64) of the matching rows to out."""
    cnt = C.c_uint64()
    if code_bits == 8:
        rc = lib.mi355_dict_scan_8bit_64bit(lo, hi, ptr(dictionary), ptr(codes), n, ptr(out), cap, C.byref(cnt))
    elif code_bits == 16:
        rc = lib.mi355_dict_scan_16bit_64bit(lo, hi, ptr(dictionary), ptr(codes), n, ptr(out), cap, C.byref(cnt))
    else:
        rc = lib.mi355_dict_scan_32bit_64bit(lo, hi, ptr(dictionary), dict_size, ptr(codes), n, ptr(out), cap,
                                             C.byref(cnt))
    _check(rc)
    return int(cnt.value)


def gen_seed(seed: int) -> None:
    lib.mi355_gen_seed(seed)


def gen_pk(out, n: int) -> None:
    _check(lib.mi355_gen_pk(ptr(out), n))


def gen_fk(out, n: int, maxid: int) -> None:
    _check(lib.mi355_gen_fk(ptr(out), n, maxid))


def gen_fk_sel(out, n: int, maxid: int) -> None:
    _check(lib.mi355_gen_fk_sel(ptr(out), n, maxid))


def gen_zipf(out, n: int, alphabet: int, theta: float, seed: int, nthreads: int = 8) -> None:
    _check(lib.mi355_gen_zipf(ptr(out), n, alphabet, theta, seed, nthreads))


def gen_pk_dev(out, count: int, first: int, n: int, seed: int, stream: int | None = None) -> None:
    _check(lib.mi355_gen_pk_dev(ptr(out), count, first, n, seed, stream or None))


def gen_fk_dev(out, count: int, first: int, maxid: int, seed: int, stream: int | None = None) -> None:
    _check(lib.mi355_gen_fk_dev(ptr(out), count, first, maxid, seed, stream or None))


def gen_zipf_dev(out, count: int, first: int, alphabet: int, theta: float, seed: int,
                 stream: int | None = None) -> None:
    """Rows [first, first+count) of a device Zipf(theta) relation over keys 1..alphabet."""
    _check(lib.mi355_gen_zipf_dev(ptr(out), count, first, alphabet, theta, seed, stream or None))


def stream_probe(kind: str, src, dst, nbytes: int, *, nt_load: bool = True, nt_store: bool = True,
                 loads_in_flight: int = 4, grid: int = 0, stream: int | None = None) -> None:
    """Enqueue one HBM ceiling probe (mi355_stream_probe): kind "copy" (src -> dst),
    "read" (src; dst a 16-byte word) or "write" (dst), 16-byte accesses."""
    k = {"copy": 0, "read": 1, "write": 2}[kind]
    _check(lib.mi355_stream_probe(k, ptr(src) if src is not None else None, ptr(dst), nbytes, int(nt_load),
                                  int(nt_store), loads_in_flight, grid, stream or None))


def gen_scan_dev(out, n: int, mode: int, seed: int, dtype: str = "i32", stream: int | None = None) -> None:
    _check(getattr(lib, f"mi355_gen_scan_{dtype}_dev")(ptr(out), n, mode, seed, stream or None))


def reference_relations(nR: int, nS: int, *, selectivity: int = 100, skew: float = 0.0,
                        r_seed: int = 11111, s_seed: int = 22222, zipf_seed: int | None = None,
                        nthreads: int = 8):
    """R and S exactly as the reference's native driver builds them (native.cpp:62-101),
    as numpy structured arrays of row_t (payload = row index)."""
    import numpy as np

    dt = np.dtype([("key", "<u4"), ("payload", "<u4")])
    R = np.empty(nR, dtype=dt)
    S = np.empty(nS, dtype=dt)
    gen_seed(r_seed)
    gen_pk(R, nR)
    gen_seed(s_seed)
    if skew > 0:
        gen_zipf(S, nS, nR, skew, s_seed if zipf_seed is None else zipf_seed, nthreads)
    elif selectivity != 100:
        maxid = (100 * nR // selectivity) & 0xFFFFFFFF if selectivity else 0
        gen_fk_sel(S, nS, maxid)
    else:
        gen_fk(S, nS, nR)
    return R, S
