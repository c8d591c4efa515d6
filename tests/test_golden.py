"""Committed fixtures (tests/golden/, written by tests/golden/make_golden.py) pin the
generators, the join oracle and the scan oracle; the GPU tests assert
the MI355X results against the same files."""
import hashlib
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = json.load(open(os.path.join(HERE, "golden", "golden.json")))
DT = np.dtype([("key", "<u4"), ("payload", "<u4")])


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def relation(sgx, name):
    """Rebuild a fixture relation with the library's host generator and check its hash."""
    g = GOLDEN["relations"][name]
    kind, rest = name.split("_", 1) if not name.startswith("fk_sel") else ("fk_sel", name[7:])
    parts = [int(x) for x in rest.split("_")]
    x = np.empty(g["n"], dtype=DT)
    sgx.gen_seed(parts[-1])
    if kind == "pk":
        sgx.gen_pk(x, g["n"])
    elif kind == "fk":
        sgx.gen_fk(x, g["n"], g["maxid"])
    else:
        sgx.gen_fk_sel(x, g["n"], g["maxid"])
    assert sha(x["key"]) == g["sha256"], name
    return x


def zipf_relation(sgx):
    z = GOLDEN["zipf"]
    x = np.empty(z["n"], dtype=DT)
    sgx.gen_zipf(x, z["n"], z["alphabet"], z["theta"], z["seed"], 4)
    assert sha(x["key"]) == z["sha256"]
    return x


def scan_columns():
    n = GOLDEN["scan_rows"]
    return {"mod": (np.arange(n) % 256).astype(np.uint8),
            "rand": np.load(os.path.join(HERE, "golden", "scan_col_rand_u8.npy"))}


def explicit_index(orc, n):
    i = np.arange(orc.explicit_index_len(n), dtype=np.uint64)
    return i * np.uint64(0x9E3779B97F4A7C15)


@pytest.mark.parametrize("name", sorted(GOLDEN["relations"]))
def test_host_generator_reproduces_fixture(sgx, name):
    relation(sgx, name)


def test_zipf_fixture(sgx, orc):
    z = GOLDEN["zipf"]
    Z = zipf_relation(sgx)
    assert int(np.bincount(Z["key"]).max()) == z["max_count"]
    n = z["n"]
    R = relation(sgx, f"pk_{n}_11111")
    assert orc.rho_join(R, Z, 4)[0] == z["pk_join_matches"] == n
    assert orc.rho_join(Z, Z, 4)[0] == z["self_join_matches"]


@pytest.mark.parametrize("j", range(len(GOLDEN["joins"])))
def test_oracle_join_counts_match_fixture(sgx, orc, j):
    case = GOLDEN["joins"][j]
    R, S = relation(sgx, case["R"]), relation(sgx, case["S"])
    assert orc.rho_join(R, S, 3)[0] == case["matches"]
    assert orc.rho_join(R, S, 1, force_two_passes=True)[0] == case["matches"]
    assert orc.count_join_sort(R, S) == case["matches"]


def test_oracle_scans_match_fixture(orc):
    cols = scan_columns()
    for e in GOLDEN["scans"]:
        c = cols[e["column"]]
        c = c if e["dtype"] == "u8" else c.astype(np.int32)
        lo, hi, dt = e["lo"], e["hi"], e["dtype"]
        assert orc.scan("count", dt, lo, hi, c) == e["count"]
        assert sha(orc.scan("bitvector", dt, lo, hi, c)) == e["bitvector_sha256"]
        assert sha(orc.scan("index", dt, lo, hi, c)) == e["index_sha256"]
        assert sha(orc.scan("values", dt, lo, hi, c)) == e["values_sha256"]
        if dt == "u8":
            assert orc.scan_sum_u8(lo, hi, c) == e["sum"]
            assert sha(orc.explicit_index_scan(lo, hi, explicit_index(orc, len(c)), c)) == e["explicit_index_sha256"]
