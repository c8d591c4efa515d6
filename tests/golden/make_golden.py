"""Writes tests/golden/golden.json (+ scan_col_rand_u8.npy): the SURVEY.md §8(c)
fixtures that pin the generators, the join oracle and the scan oracle.

Run from the repo root:  python tests/golden/make_golden.py

Relations are built twice and must agree:
  * by a Python restatement of Join-Benchmarks/lib/AppUtilities/src/generator.cpp
    (random_unique_gen :143-153, knuth_shuffle :100-109, create_relation_fk :474-512,
    random_unique_gen_maxid :156-169 with its integer jump, create_relation_fk_sel
    :515-553) driven by the SYSTEM libc's rand()/srand() through ctypes — the
    third-party generator the reference itself calls (generator.cpp:19, :75-80);
  * by the library's host generator (csrc/generator.cpp, glibc TYPE_3 restated).
Zipf (genzipf.cpp:34-144) uses libstdc++'s mt19937_64 / shuffle / uniform_real_distribution,
which have no Python twin here: its fixture is the library generator's output with a fixed
seed (the reference seeds from std::random_device, so no reference vector exists).
Join counts come from the oracle's restated RHO (oracle/rho_oracle.c) and must equal the
independent sort-merge counter and the analytical KATs; scan outputs from oracle/scan_oracle.c
and the Catch2 KATs of testsimdscan.cpp (count = N/256 * width over i % 256).
"""
import ctypes as C
import ctypes.util
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (os.path.join(ROOT, "sgxv2-analytical-query-processing-benchmarks_amd", "python"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

DT = np.dtype([("key", "<u4"), ("payload", "<u4")])
LIBC = C.CDLL(ctypes.util.find_library("c"))
LIBC.rand.restype = C.c_int
RAND_MAX = 2147483647.0


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _shuffle(keys: list) -> None:  # knuth_shuffle, generator.cpp:100-109 (RAND_RANGE :19)
    for i in range(len(keys) - 1, 0, -1):
        j = int(float(LIBC.rand()) / (RAND_MAX + 1.0) * float(i))
        keys[i], keys[j] = keys[j], keys[i]


def libc_pk(n, seed):
    LIBC.srand(C.c_uint(seed))
    keys = list(range(1, n + 1))
    _shuffle(keys)
    return np.array(keys, dtype=np.uint32)


def libc_fk(n, maxid, seed):
    LIBC.srand(C.c_uint(seed))
    out = []
    for _ in range(n // maxid):
        k = list(range(1, maxid + 1))
        _shuffle(k)
        out += k
    if n % maxid:
        k = list(range(1, n % maxid + 1))
        _shuffle(k)
        out += k
    return np.array(out, dtype=np.uint32)


def libc_fk_sel(n, maxid, seed):
    LIBC.srand(C.c_uint(seed))
    maxid32 = maxid & 0xFFFFFFFF

    def chunk(m):
        jump = float(maxid32 // m)  # double jump = maxid / num_tuples: integer division
        idv = 0.0 if maxid32 == 0 else 1.0
        k = []
        for _ in range(m):
            k.append(int(idv) & 0xFFFFFFFF)
            idv += jump
        _shuffle(k)
        return k

    iters = n // maxid if maxid else 0
    out = []
    for _ in range(iters):
        out += chunk(maxid)
    rem = n % maxid if maxid else n
    if rem:
        out += chunk(rem)
    return np.array(out, dtype=np.uint32)


def rel(keys):
    x = np.empty(len(keys), dtype=DT)
    x["key"] = keys
    x["payload"] = np.arange(len(keys), dtype=np.uint32)
    return x


def main():
    import oracle
    import sgxamd

    def lib_rel(kind, n, seed, arg=0):
        x = np.empty(n, dtype=DT)
        sgxamd.gen_seed(seed)
        if kind == "pk":
            sgxamd.gen_pk(x, n)
        elif kind == "fk":
            sgxamd.gen_fk(x, n, arg)
        else:
            sgxamd.gen_fk_sel(x, n, arg)
        return x

    rels = {}
    joins = []
    for e in range(10, 17, 2):
        n = 1 << e
        for seed in (11111, 22222):
            k = libc_pk(n, seed)
            assert np.array_equal(k, lib_rel("pk", n, seed)["key"])
            rels[f"pk_{n}_{seed}"] = {"n": n, "sha256": sha(k), "first": k[:8].tolist(), "sum": int(k.sum(dtype=np.uint64))}
        R = rel(libc_pk(n, 11111))
        cases = [("fk", n, n), ("fk", n, max(n // 8, 1))] + [("fk_sel", n, 100 * n // sel) for sel in (50, 10, 1)]
        for kind, m, maxid in cases:
            for seed in (11111, 22222):
                k = libc_fk(m, maxid, seed) if kind == "fk" else libc_fk_sel(m, maxid, seed)
                assert np.array_equal(k, lib_rel(kind, m, seed, maxid)["key"]), (kind, m, maxid, seed)
                rels[f"{kind}_{m}_{maxid}_{seed}"] = {"n": m, "maxid": maxid, "sha256": sha(k), "first": k[:8].tolist(),
                                                     "sum": int(k.sum(dtype=np.uint64))}
            S = rel(libc_fk(m, maxid, 22222) if kind == "fk" else libc_fk_sel(m, maxid, 22222))
            cnt, _ = oracle.rho_join(R, S, 4)
            assert cnt == oracle.count_join_sort(R, S) == oracle.rht_join(R, S, 2)
            if kind == "fk":
                assert cnt == m
            else:  # keys {1 + k * jump}: matches = #{1 + k * jump <= n}
                jump = maxid // m
                assert cnt == sum(1 for i in range(m) if 1 + i * jump <= n)
            joins.append({"R": f"pk_{n}_11111", "S": f"{kind}_{m}_{maxid}_22222", "matches": cnt})

    # seeded Zipf 2^16 over 1..2^16, theta 0.75 (genzipf.cpp:87-144; mt19937_64 seed 22222)
    n = 1 << 16
    Z = np.empty(n, dtype=DT)
    sgxamd.gen_zipf(Z, n, n, 0.75, 22222, 1)
    zk = Z["key"]
    cnts = np.bincount(zk).astype(np.uint64)
    R = rel(libc_pk(n, 11111))
    m, _ = oracle.rho_join(R, Z, 4)
    assert m == n == oracle.count_join_sort(R, Z)
    self_cnt, _ = oracle.rho_join(Z, Z, 4)
    assert self_cnt == int((cnts * cnts).sum()) == oracle.count_join_sort(Z, Z)
    zipf = {"n": n, "alphabet": n, "theta": 0.75, "seed": 22222, "sha256": sha(zk), "first": zk[:8].tolist(),
            "max_count": int(cnts.max()), "pk_join_matches": m, "self_join_matches": self_cnt}

    # scan columns at 2^16: i % 256 (Allocator.hpp:94-110) and a seeded uniform u8 column (stored)
    n = 1 << 16
    rand_col = np.random.default_rng(42).integers(0, 256, n).astype(np.uint8)
    np.save(os.path.join(HERE, "scan_col_rand_u8.npy"), rand_col)
    cols = {"mod": (np.arange(n) % 256).astype(np.uint8), "rand": rand_col}
    index = explicit_index_array(n)
    scans = []
    for name, c8 in cols.items():
        for lo, hi in [(0, 26), (0, 3), (5, 5), (1, 100), (200, 100)]:
            for dt, c in (("u8", c8), ("i32", c8.astype(np.int32))):
                cnt = oracle.scan("count", dt, lo, hi, c)
                if name == "mod":
                    assert cnt == n // 256 * max(hi - lo + 1, 0)  # testsimdscan.cpp KAT
                e = {"column": name, "dtype": dt, "lo": lo, "hi": hi, "count": cnt,
                     "bitvector_sha256": sha(oracle.scan("bitvector", dt, lo, hi, c)),
                     "index_sha256": sha(oracle.scan("index", dt, lo, hi, c)),
                     "values_sha256": sha(oracle.scan("values", dt, lo, hi, c))}
                if dt == "u8":
                    e["sum"] = oracle.scan_sum_u8(lo, hi, c)
                    e["explicit_index_sha256"] = sha(oracle.explicit_index_scan(lo, hi, index, c))
                scans.append(e)
    out = {"about": __doc__.strip().splitlines()[0], "relations": rels, "joins": joins, "zipf": zipf,
           "scans": scans, "scan_rows": n}
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(f"wrote {len(rels)} relations, {len(joins)} joins, {len(scans)} scans")


def explicit_index_array(n):
    """Index entries for the explicit index scan fixture: entry i = i * 0x9E3779B97F4A7C15 mod 2^64."""
    import oracle

    i = np.arange(oracle.explicit_index_len(n), dtype=np.uint64)
    return i * np.uint64(0x9E3779B97F4A7C15)


if __name__ == "__main__":
    main()
