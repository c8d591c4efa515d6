"""TPC-H callers of the MI355X join path (ctypes side of include/sgxamd/tpch.h).

Mirrors the reference's TPC-H app (Join-Benchmarks/App/TpcH, lib/TPCH-Queries):
tables are sets of columns (TpcHTypes.hpp:53-87), read from the binary table
directories (TpcHCommons.cpp) or generated synthetically, and the four queries
Q3/Q10/Q12/Q19 (tpch.cpp:36-309) run on the GPU.  Columns may be numpy arrays
(host; the library stages them to HBM) or torch tensors on the GPU.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import (ALGORITHMS, CustomerTable, LineItemTable, NationTable, OrdersTable, PartTable, _check, lib, ptr,
               tpch_stats)

ROW = np.dtype([("key", "<u4"), ("payload", "<u4")])

# table -> [(column, numpy dtype)]; "row" columns are row_t {key, row id}
COLUMNS = {
    "lineitem": [("l_orderkey", ROW), ("l_shipdate", np.uint64), ("l_commitdate", np.uint64),
                 ("l_receiptdate", np.uint64), ("l_shipmode", np.uint8), ("l_partkey", np.uint32),
                 ("l_quantity", np.float32), ("l_shipinstruct", np.uint8), ("l_returnflag", np.uint8)],
    "orders": [("o_orderkey", ROW), ("o_orderdate", np.uint64), ("o_custkey", np.uint32)],
    "customer": [("c_custkey", ROW), ("c_mktsegment", np.uint8), ("c_nationkey", np.uint32)],
    "part": [("p_partkey", ROW), ("p_brand", np.uint8), ("p_size", np.uint32), ("p_container", np.uint8)],
    "nation": [("n_nationkey", ROW)],
}
STRUCTS = {"lineitem": LineItemTable, "orders": OrdersTable, "customer": CustomerTable, "part": PartTable,
           "nation": NationTable}
QUERY_TABLES = {3: ("customer", "orders", "lineitem"), 10: ("customer", "orders", "lineitem", "nation"),
                12: ("lineitem", "orders"), 19: ("lineitem", "part")}
_TORCH_DTYPE = {np.dtype(np.uint64): "int64", np.dtype(np.uint32): "int32", np.dtype(np.uint8): "uint8",
                np.dtype(np.float32): "float32"}


class Tables:
    """Columns per table: {table: {column: numpy array | torch tensor}} plus row counts."""

    def __init__(self, cols: dict, sizes: dict):
        self.cols = cols
        self.sizes = sizes

    def n(self, table: str) -> int:
        return self.sizes.get(table, 0)

    def struct(self, table: str):
        """The C struct of one table (column pointers into this object's arrays)."""
        if table not in self.sizes:
            return None
        s = STRUCTS[table]()
        s.numTuples = self.sizes[table]
        for name, arr in self.cols.get(table, {}).items():
            setattr(s, name, ptr(arr))
        return s

    def structs(self, *tables):
        return [self.struct(t) for t in tables]


def _ref(s):
    return C.byref(s) if s is not None else None


def _from_c(table_struct, table: str) -> dict:
    """Copy the malloc'd columns of a C table struct into numpy arrays."""
    n = table_struct.numTuples
    out = {}
    for name, dt in COLUMNS[table]:
        p = getattr(table_struct, name)
        if not p:
            continue
        nbytes = n * np.dtype(dt).itemsize
        raw = np.ctypeslib.as_array((C.c_uint8 * max(nbytes, 1)).from_address(p))[:nbytes].copy()
        out[name] = raw.view(dt)
    return out


_FREE = {"lineitem": "mi355_tpch_free_lineitem", "orders": "mi355_tpch_free_orders",
         "customer": "mi355_tpch_free_customer", "part": "mi355_tpch_free_part", "nation": "mi355_tpch_free_nation"}


def sizes(scale_milli: int, seed: int = 0) -> dict:
    v = [C.c_uint64() for _ in range(5)]
    _check(lib.mi355_tpch_sizes(scale_milli, seed, *[C.byref(x) for x in v]))
    return dict(zip(("lineitem", "orders", "customer", "part", "nation"), (x.value for x in v)))


def generate(scale_milli: int, seed: int = 0) -> Tables:
    """Synthetic tables on the host (tpch_gen.hpp distributions), as numpy columns."""
    st = {t: STRUCTS[t]() for t in STRUCTS}
    rc = lib.mi355_tpch_generate(scale_milli, seed, C.byref(st["lineitem"]), C.byref(st["orders"]),
                                 C.byref(st["customer"]), C.byref(st["part"]), C.byref(st["nation"]))
    try:
        _check(rc)
        cols = {t: _from_c(st[t], t) for t in STRUCTS}
        return Tables(cols, {t: st[t].numTuples for t in STRUCTS})
    finally:
        for t, fn in _FREE.items():
            getattr(lib, fn)(C.byref(st[t]))


def generate_dev(scale_milli: int, seed: int = 0, device="cuda", tables=tuple(STRUCTS), stream=None) -> Tables:
    """The same synthetic tables generated directly in HBM (torch tensors)."""
    import torch

    n = sizes(scale_milli, seed)
    cols = {}
    for t in tables:
        cols[t] = {}
        for name, dt in COLUMNS[t]:
            if dt is ROW:
                cols[t][name] = torch.empty(n[t], dtype=torch.int64, device=device)
            else:
                cols[t][name] = torch.empty(n[t], dtype=getattr(torch, _TORCH_DTYPE[np.dtype(dt)]), device=device)
    tb = Tables(cols, {t: n[t] for t in tables})
    _check(lib.mi355_tpch_generate_dev(scale_milli, seed, _ref(tb.struct("lineitem")), _ref(tb.struct("orders")),
                                       _ref(tb.struct("customer")), _ref(tb.struct("part")),
                                       _ref(tb.struct("nation")), ptr(stream)))
    return tb


def to_numpy(tb: Tables) -> Tables:
    """Host copy of (device) tables, columns as the numpy dtypes of COLUMNS."""
    cols = {}
    for t, cs in tb.cols.items():
        cols[t] = {}
        for name, arr in cs.items():
            dt = dict(COLUMNS[t])[name]
            a = arr.cpu().numpy() if hasattr(arr, "cpu") else np.asarray(arr)
            cols[t][name] = a.view(dt)
    return Tables(cols, dict(tb.sizes))


_LOADERS = {"lineitem": "mi355_tpch_load_lineitem", "orders": "mi355_tpch_load_orders",
            "customer": "mi355_tpch_load_customer", "part": "mi355_tpch_load_part", "nation": "mi355_tpch_load_nation"}


def load(root: str, query: int, scale: int, csv: bool = False) -> Tables:
    """load_*_from_binary (query's columns only) or load_*_from_csv (TpcHCommons.cpp)."""
    cols, szs = {}, {}
    wanted = QUERY_TABLES.get(query, tuple(STRUCTS)) if not csv else tuple(STRUCTS)
    for t in wanted:
        s = STRUCTS[t]()
        rc = getattr(lib, _LOADERS[t])(C.byref(s), root.encode(), query, scale, 1 if csv else 0)
        try:
            if rc != 0:
                raise OSError(f"loading {t} from {root} (scale {scale}) failed")
            cols[t] = _from_c(s, t)
            szs[t] = s.numTuples
        finally:
            getattr(lib, _FREE[t])(C.byref(s))
    return Tables(cols, szs)


def store(root: str, scale: int, tb: Tables) -> None:
    """The csv_convert binary layout (host tables only)."""
    rc = lib.mi355_tpch_store(root.encode(), scale, _ref(tb.struct("lineitem")), _ref(tb.struct("orders")),
                              _ref(tb.struct("customer")), _ref(tb.struct("part")), _ref(tb.struct("nation")))
    if rc != 0:
        raise OSError(f"storing TPC-H tables under {root} failed")


def _stats(s: tpch_stats) -> dict:
    return s.as_dict()


def q3(tb: Tables, algorithm: str = "RHO") -> dict:
    st = tpch_stats()
    c, o, l = tb.structs("customer", "orders", "lineitem")
    _check(lib.mi355_tpch_q3(_ref(c), _ref(o), _ref(l), ALGORITHMS[algorithm], C.byref(st)))
    return _stats(st)


def q10(tb: Tables, algorithm: str = "RHO") -> dict:
    st = tpch_stats()
    c, o, l, n = tb.structs("customer", "orders", "lineitem", "nation")
    _check(lib.mi355_tpch_q10(_ref(c), _ref(o), _ref(l), _ref(n), ALGORITHMS[algorithm], C.byref(st)))
    return _stats(st)


def q12(tb: Tables, algorithm: str = "RHO") -> dict:
    st = tpch_stats()
    l, o = tb.structs("lineitem", "orders")
    _check(lib.mi355_tpch_q12(_ref(l), _ref(o), ALGORITHMS[algorithm], C.byref(st)))
    return _stats(st)


def q19(tb: Tables, algorithm: str = "RHO", want_join: bool = False):
    """Returns the stats, and with want_join the join-1 triples (numpy) the reference keeps in result->result."""
    from . import chunked_table_triples_ptr

    st = tpch_stats()
    l, p = tb.structs("lineitem", "part")
    jt = C.c_void_p()
    _check(lib.mi355_tpch_q19(_ref(l), _ref(p), ALGORITHMS[algorithm], C.byref(st), 1 if want_join else 0,
                              C.byref(jt)))
    if not want_join:
        return _stats(st)
    try:
        triples = chunked_table_triples_ptr(jt.value)
    finally:
        lib.mi355_free_chunked_table(jt.value)
    return _stats(st), triples


QUERIES = {3: q3, 10: q10, 12: q12, 19: q19}


def filter_rows(query: int, which: int, tb: Tables) -> np.ndarray:
    """Selection `which` of `query` on the GPU: the filtered rows in input order."""
    c, o, l, p = tb.structs("customer", "orders", "lineitem", "part")
    n = C.c_uint64()
    rc = lib.mi355_tpch_filter(query, which, _ref(c), _ref(o), _ref(l), _ref(p), None, 0, C.byref(n))
    if rc not in (0, -5):
        _check(rc)
    out = np.zeros(n.value, dtype=ROW)
    _check(lib.mi355_tpch_filter(query, which, _ref(c), _ref(o), _ref(l), _ref(p), ptr(out), n.value, C.byref(n)))
    return out[: n.value]
