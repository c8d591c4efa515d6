"""The development A/B switches select alternative kernel paths with identical results:
SGXAMD_DIGIT_SIDE=0 (pass-2 histograms over the tuples instead of the digit side
stream), SGXAMD_BIG_JOIN=0 (R partitions above 8192 tuples in 8192-tuple chain tables
instead of the 16,384-tuple counting table; the 5-bit plan below has 32,768-tuple
partitions), SGXAMD_SMALL_JOIN=0
(small one-pass joins on the regular launch sequence instead of the three-launch path:
the (5, 1) plan and the full-range cases below take it), SGXAMD_SMALL_DIRECT=0 (their
build/probe keeps the chain table where the direct count table fits), SGXAMD_POOL=0 (two-pass plans
with a pass-1 histogram and cursors instead of the pooled pass 1 and block-list pass 2;
SGXAMD_POOL_SEGS sets the pooled pass-1 workgroups: 3 gives large pools, 100000 one
tile per segment), SGXAMD_KEYS=0 (counting joins move whole tuples instead of keys),
SGXAMD_SORT2=0 (pass 2 of key partitions with the write-combining scatter instead of
the LDS counting sort), SGXAMD_CHAIN_HIST=0 (the digit side stream and its histogram
pass instead of the chain histograms counted in pass 1),
SGXAMD_NARROW=0 (key partitions stay 4-byte keys where u16 residuals would fit),
SGXAMD_JOIN_N=0 (narrow relations' build/probe in k_join_x's direct table, one
workgroup per CU, instead of k_join_n, one task per workgroup), SGXAMD_PLACE=0 (narrow
relations' pass 2 as k_sort_blk's tile sort instead of k_place_seg's segment
placement), SGXAMD_NARROW_POOL=1 (narrow plans' pass 1 writes the narrow pool of 16-bit
residuals and their digits instead of 4-byte keys; opt-in).  The switches are read
once per process, so each setting runs in a child process against the oracle (the
TPC-H selections ride along: they share the library's workspace)."""
import os
import subprocess
import sys

import pytest

from conftest import PKG, ROOT

pytestmark = pytest.mark.gpu

CHILD = r"""
import sys
import numpy as np
import sgxamd, oracle
R, S = sgxamd.reference_relations(1 << 20, 1 << 20, selectivity=50)
exp, _ = oracle.rho_join(R, S, 2)
for bits, passes in [(12, 2), (13, 2), (14, 2), (16, 2), (18, 2), (5, 1)]:
    got = sgxamd.rho_join(R, len(R), S, len(S), radix_bits=bits, passes=passes).matches
    assert got == exp, (bits, passes, got, exp)
rng = np.random.default_rng(5)
# full-range keys with duplicates: big-table partitions whose 8-bit tags are not the whole
# remaining key (hash_shift + log2 N + 8 < 32), confirmed against the R keys
dt = np.dtype([("key", "<u4"), ("payload", "<u4")])
for kmax, bits in ((2**32 - 1, 5), (1 << 22, 4)):
    R2 = np.zeros(1 << 20, dtype=dt); R2["key"] = rng.integers(0, kmax + 1, 1 << 20)
    S2 = np.zeros((1 << 20) + 99, dtype=dt); S2["key"] = rng.integers(0, kmax + 1, (1 << 20) + 99)
    got = sgxamd.rho_join(R2, len(R2), S2, len(S2), radix_bits=bits, passes=1).matches
    assert got == oracle.count_join_sort(R2, S2), (kmax, bits, got)
for n in (1, 1000, 65536, 65537, (1 << 20) + 37):
    col = rng.integers(0, 256, n).astype(np.int32)
    for lo, hi in [(0, 26), (0, 255), (7, 7), (200, 100)]:
        cnt = oracle.scan("count", "i32", lo, hi, col)
        assert sgxamd.scan_count(lo, hi, col, n) == cnt
        bv = np.zeros((n + 63) // 64, dtype=np.uint64)
        sgxamd.scan_bitvector(lo, hi, col, n, bv)
        assert np.array_equal(bv, oracle.scan("bitvector", "i32", lo, hi, col)), (n, lo, hi)
        c8 = col.astype(np.uint8)
        assert sgxamd.scan_count(lo, hi, c8, n, "u8") == oracle.scan("count", "u8", lo, hi, c8)
        bv8 = np.zeros((n + 63) // 64, dtype=np.uint64)
        sgxamd.scan_bitvector(lo, hi, c8, n, bv8, "u8")
        assert np.array_equal(bv8, oracle.scan("bitvector", "u8", lo, hi, c8)), (n, lo, hi)
        idx = np.zeros(max(cnt, 1), dtype=np.uint64)
        assert sgxamd.scan_index(lo, hi, col, n, idx, cnt) == cnt
        assert np.array_equal(idx[:cnt], oracle.scan("index", "i32", lo, hi, col)), (n, lo, hi)
        vals = np.zeros(max(cnt, 1), dtype=np.int32)
        assert sgxamd.scan_values(lo, hi, col, n, vals, cnt) == cnt
        assert np.array_equal(vals[:cnt], oracle.scan("values", "i32", lo, hi, col)), (n, lo, hi)
dictionary = np.sort(rng.integers(-10**9, 10**9, 256))
codes = rng.integers(0, 256, 300_001).astype(np.uint8)
ref = oracle.dict_scan(-10**8, 5 * 10**8, dictionary, codes)
out = np.zeros(len(ref) + 1, dtype=np.int64)
k = sgxamd.dict_scan(-10**8, 5 * 10**8, dictionary, codes, len(codes), out, len(out), 8, 256)
assert k == len(ref) and np.array_equal(out[:k], ref)
import sgxamd.tpch as T
tb = T.generate(20, 5)  # SF 0.02
for q, w in [(3, 1), (3, 2), (3, 3), (10, 1), (10, 2), (12, 1), (19, 1), (19, 2)]:
    assert np.array_equal(T.filter_rows(q, w, tb), oracle.tpch_filter(q, w, tb)), (q, w)
print("paths ok")
"""


@pytest.mark.parametrize("env", [{"SGXAMD_DIGIT_SIDE": "0", "SGXAMD_BIG_JOIN": "0"},
                                 {"SGXAMD_DIGIT_SIDE": "1", "SGXAMD_BIG_JOIN": "1"},
                                 {"SGXAMD_SMALL_JOIN": "0"}, {"SGXAMD_SMALL_DIRECT": "0"},
                                 {"SGXAMD_POOL": "0"}, {"SGXAMD_POOL_SEGS": "3"}, {"SGXAMD_POOL_SEGS": "100000"},
                                 {"SGXAMD_KEYS": "0"}, {"SGXAMD_SORT2": "0"}, {"SGXAMD_NARROW": "0"}, {"SGXAMD_JOIN_N": "0"}, {"SGXAMD_PLACE": "0"}, {"SGXAMD_NARROW_POOL": "1"},
                                 {"SGXAMD_NARROW_POOL": "1", "SGXAMD_PLACE": "0"}, {"SGXAMD_CHAIN_HIST": "0"},
                                 {"SGXAMD_CHAIN_HIST": "0", "SGXAMD_POOL_SEGS": "3"}])
def test_switch_paths_match_oracle(env):
    e = dict(os.environ, **env)
    e["PYTHONPATH"] = os.pathsep.join([os.path.join(PKG, "python"), os.path.join(ROOT, "oracle"),
                                       e.get("PYTHONPATH", "")])
    r = subprocess.run([sys.executable, "-c", CHILD], env=e, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "paths ok" in r.stdout, (env, r.stdout[-2000:], r.stderr[-2000:])


# The multi-GPU u16 wire under the switches that change the sender's passes or the
# receiver's build/probe (rehearsal transport, 4 ranks, a 14-bit plan): exact counts;
# SGXAMD_WIRE16=0 (and SGXAMD_NARROW=0, which it needs) fall back to 4-byte keys.
WIRE_CHILD = r"""
import os
import numpy as np
import sgxamd, oracle
dt = np.dtype([("key", "<u4"), ("payload", "<u4")])
rng = np.random.default_rng(9)
R = np.zeros(200_003, dtype=dt); R["key"] = rng.integers(0, 2**32, len(R), dtype=np.uint64).astype(np.uint32)
S = np.zeros(300_007, dtype=dt); S["key"] = rng.integers(0, 2**32, len(S), dtype=np.uint64).astype(np.uint32)
S[:70_000] = R[:70_000]
Pk, Fk = sgxamd.reference_relations(1 << 20, 1 << 20, selectivity=50)
off = os.environ.get("SGXAMD_WIRE16") == "0" or os.environ.get("SGXAMD_NARROW") == "0"
if os.environ.get("SGXAMD_WIRE16") != "0":
    sgxamd.multi_set_wire(2)  # whenever the residuals fit (these relations are small)
for A, B in ((R, S), (Pk, Fk)):
    for g in (4, 8):
        r = sgxamd.rho_join_multi(A, len(A), B, len(B), g, transport="rehearsal", radix_bits=14, passes=2)
        assert r.matches == oracle.count_join_sort(A, B), (g, r.matches)
        assert r.stats["elem_bytes"] == (4 if off else 2), r.stats["elem_bytes"]
print("wire ok")
"""


@pytest.mark.parametrize("env", [{"SGXAMD_WIRE16": "0"}, {"SGXAMD_NARROW": "0"}, {"SGXAMD_PLACE": "0"},
                                 {"SGXAMD_WIRE_GATHER": "1"},
                                 {"SGXAMD_JOIN_N": "0"}, {"SGXAMD_CHAIN_HIST": "0"}, {"SGXAMD_PASS1_BITS": "6"},
                                 {"SGXAMD_POOL_SEGS": "3"}])
def test_wire16_switches(env):
    e = dict(os.environ, **env)
    e["PYTHONPATH"] = os.pathsep.join([os.path.join(PKG, "python"), os.path.join(ROOT, "oracle"),
                                       e.get("PYTHONPATH", "")])
    r = subprocess.run([sys.executable, "-c", WIRE_CHILD], env=e, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "wire ok" in r.stdout, (env, r.stdout[-2000:], r.stderr[-2000:])


# Chain histograms under skew (rho_kernels.hip k_hist_chain): every S key has the same
# pass-1 digit, so with 8 pass-1 workgroups each chain holds 2^19 keys (u16 counts wrap)
# and every pass-2 segment lies inside one chain (counted from its keys); with 512 a
# segment holds whole chains of that digit and cut ones at both ends.
CHAIN_CHILD = r"""
import numpy as np
import sgxamd, oracle
dt = np.dtype([("key", "<u4"), ("payload", "<u4")])
rng = np.random.default_rng(3)
R = np.zeros(1 << 20, dtype=dt); R["key"] = rng.permutation(1 << 20).astype(np.uint32)
S = np.zeros((1 << 22) + 777, dtype=dt); S["key"] = (rng.integers(0, 8192, len(S)) * 128 + 5).astype(np.uint32)
for bits in (13, 14):
    for algo in ("RHO", "RHT"):
        r = sgxamd.rho_join(R, len(R), S, len(S), radix_bits=bits, passes=2, algorithm=algo)
        assert r.matches == len(S), (bits, algo, r.matches)
        assert r.stats["layout"] == 3, r.stats["layout"]
# and two hot digits among uniform ones, against the sort counter
S2 = np.zeros(1 << 22, dtype=dt)
S2["key"] = np.where(rng.random(len(S2)) < 0.6, rng.integers(0, 8192, len(S2)) * 128 + 9,
                     rng.integers(0, 1 << 21, len(S2))).astype(np.uint32)
assert sgxamd.rho_join(R, len(R), S2, len(S2), radix_bits=14, passes=2).matches == oracle.count_join_sort(R, S2)
print("chain ok")
"""


@pytest.mark.parametrize("segs", ["8", "512"])
def test_chain_histograms_skewed(segs):
    e = dict(os.environ, SGXAMD_POOL_SEGS=segs, SGXAMD_CHAIN_HIST="1")
    e["PYTHONPATH"] = os.pathsep.join([os.path.join(PKG, "python"), os.path.join(ROOT, "oracle"),
                                       e.get("PYTHONPATH", "")])
    r = subprocess.run([sys.executable, "-c", CHAIN_CHILD], env=e, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "chain ok" in r.stdout, (segs, r.stdout[-2000:], r.stderr[-2000:])


# Chain histograms (layout 3) with narrow partitions: BASELINE config 2's 2^28 pk/fk keys
# over the 14 = 7 + 7-bit plan, pass 2 writing 2-byte residuals.
CHAIN_NARROW_CHILD = r"""
import torch
import sgxamd
n = 1 << 28
R = torch.empty(n, dtype=torch.int64, device="cuda:0")
S = torch.empty(n, dtype=torch.int64, device="cuda:0")
sgxamd.gen_pk_dev(R, n, 0, n, 11111)
sgxamd.gen_fk_dev(S, n, 0, n, 22222)
r = sgxamd.rho_join(R, n, S, n)
assert r.matches == n, r.matches
assert r.stats["layout"] == 3 and r.stats["narrow"] == 3, (r.stats["layout"], r.stats["narrow"])
print("chain narrow ok")
"""


def test_chain_histograms_narrow_full_size():
    e = dict(os.environ, SGXAMD_CHAIN_HIST="1")
    e["PYTHONPATH"] = os.pathsep.join([os.path.join(PKG, "python"), e.get("PYTHONPATH", "")])
    r = subprocess.run([sys.executable, "-c", CHAIN_NARROW_CHILD], env=e, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "chain narrow ok" in r.stdout, (r.stdout[-2000:], r.stderr[-2000:])
