"""Multi-GPU RHO in C++ (sgxamd/multi.h) on one MI355X through the rehearsal transport:
G logical ranks with their own streams and workspaces, the radix-shard exchange done by
device-to-device copies.  The same rank pipeline (pieced shard partition, count
exchange, tuple exchange on a communication stream, pipelined local join with
key_shift = log2 G, all-reduce) runs over RCCL when G GPUs are visible.

Counts are compared bit-exactly with the oracle's restated RHO (radix_join.cpp) on
the reference's relations (native.cpp:62-101) and with the sort counter."""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import PKG

pytestmark = pytest.mark.gpu

DT = np.dtype([("key", "<u4"), ("payload", "<u4")])


def rel(keys):
    x = np.empty(len(keys), dtype=DT)
    x["key"] = keys
    x["payload"] = np.arange(len(keys), dtype=np.uint32)
    return x


def multi(sgx, R, S, g, **kw):
    return sgx.rho_join_multi(R, len(R), S, len(S), g, transport="rehearsal", **kw)


@pytest.fixture
def wire16(sgx):
    """The u16 wire whenever the residuals fit (mode 2), not only where the local plan
    is the narrow 16,384-key-table plan anyway (the default, mode 1: relations of
    2^27+ keys per rank)."""
    sgx.multi_set_wire(2)
    yield
    sgx.multi_set_wire(1)


@pytest.mark.parametrize("g", [2, 4, 8])
def test_reference_pk_fk(sgx, orc, gpu, g):
    n = 1 << 18
    R, S = sgx.reference_relations(n, n)
    res = multi(sgx, R, S, g)
    assert res.matches == orc.rho_join(R, S, 4)[0] == n
    st = res.stats
    assert st["world"] == g and st["transport"] == "rehearsal" and st["pieces"] == 4
    # every key lands on the rank of its low log2(g) bits: pk keys 1..n spread evenly
    assert st["recv_r_min"] == st["recv_r_max"] == n // g
    assert 0 < st["sent_bytes"] <= 8 * 2 * n


@pytest.mark.parametrize("seed,nR,nS,kmax,g", [(1, 5000, 7001, 300, 4), (2, 100_003, 77_777, 2**32 - 1, 8),
                                               (3, 3, 5, 2, 4), (4, 1 << 17, 1 << 16, 1 << 10, 2)])
def test_random_with_duplicates(sgx, orc, gpu, seed, nR, nS, kmax, g):
    rng = np.random.default_rng(seed)
    R = rel(rng.integers(0, kmax + 1, nR, dtype=np.uint64).astype(np.uint32))
    S = rel(rng.integers(0, kmax + 1, nS, dtype=np.uint64).astype(np.uint32))
    exp = orc.count_join_sort(R, S)
    assert multi(sgx, R, S, g).matches == exp
    assert multi(sgx, R, S, g, algorithm="RHT").matches == exp
    assert multi(sgx, R, S, g, radix_bits=12, passes=2).matches == exp


def test_zipf_and_sel(sgx, orc, gpu):
    n = 1 << 18
    R, S = sgx.reference_relations(n, n, skew=0.75)
    res = multi(sgx, R, S, 8)
    assert res.matches == orc.rho_join(R, S, 4)[0] == n
    assert res.stats["recv_s_max"] < 1.2 * n / 8  # hot keys spread over the ranks by the alphabet shuffle
    R, S = sgx.reference_relations(n, n, selectivity=10)
    assert multi(sgx, R, S, 4).matches == orc.rho_join(R, S, 4)[0]


@pytest.mark.parametrize("g,n,kw", [(2, 1 << 23, {}), (4, 1 << 23, {}), (8, 1 << 21, {"radix_bits": 14, "passes": 2}),
                                    (4, 1 << 20, {"radix_bits": 10, "passes": 2})])
def test_keys_only_exchange(sgx, orc, gpu, wire16, g, n, kw):
    """Counting joins whose local plan takes the pooled keys layout exchange 4-byte keys:
    the default policy from the mean local sizes (2^23 over 2 / 4 ranks: 10 / 9 bits, two
    passes) or a forced two-pass plan.  Exact counts, half the bytes of the tuple
    exchange on the wire (SGXAMD_KEYS=0 in test_paths_gpu keeps tuples)."""
    R, S = sgx.reference_relations(n, n)  # pk / fk: every rank receives R and S tuples
    exp = orc.count_join_sort(R, S)
    res = multi(sgx, R, S, g, **kw)
    assert res.matches == exp
    st = res.stats
    # S as 2-byte residuals when its keys' residuals above the shard and partition bits
    # fit 16 bits (u16 wire forced: mode 2), else 4-byte keys
    wire16 = (int(S["key"].max()) >> ((g.bit_length() - 1) + st["local"]["radix_bits"])) < 2**16
    assert st["elem_bytes"] == (2 if wire16 else 4) and st["local"]["layout"] in (2, 3, 4)
    # every key of a rank except those it keeps goes out once
    assert st["sent_bytes"] == _exchange_bytes(st, _keys_out(R, g), _keys_out(S, g), g)
    # RHT counts over key partitions too (SGXAMD_KEYS=0 in test_paths_gpu keeps tuples)
    rht = multi(sgx, R, S, g, algorithm="RHT", **kw)
    assert rht.matches == exp and rht.stats["elem_bytes"] == 4


@pytest.mark.parametrize("pieces", [1, 3, 7])
def test_pieces(sgx, orc, gpu, pieces):
    R, S = sgx.reference_relations(100_000, 150_001, selectivity=50)
    exp = orc.rho_join(R, S, 4)[0]
    sgx.multi_set_pieces(pieces)
    try:
        res = multi(sgx, R, S, 4)
    finally:
        sgx.multi_set_pieces(4)
    assert res.matches == exp and res.stats["pieces"] == pieces


@pytest.mark.parametrize("nR,nS,g", [(0, 100, 4), (100, 0, 4), (3, 1000, 8), (1000, 5, 8), (1, 1, 2)])
def test_empty_and_tiny_slices(sgx, orc, gpu, nR, nS, g):
    R = rel(np.arange(1, nR + 1, dtype=np.uint32))
    S = rel((np.arange(nS, dtype=np.uint32) % max(nR, 1)) + 1)
    exp = orc.count_join_sort(R, S) if nR and nS else 0
    assert multi(sgx, R, S, g).matches == exp


def test_device_resident_and_repeat(sgx, orc, gpu):
    import torch

    R, S = sgx.reference_relations(1 << 17, (1 << 17) + 33)
    dR = torch.from_numpy(R.view(np.int64)).to(gpu)
    dS = torch.from_numpy(S.view(np.int64)).to(gpu)
    exp = orc.rho_join(R, S, 4)[0]
    for g in (4, 2, 4, 1):  # workspaces are reused across calls and world sizes
        assert sgx.rho_join_multi(dR, len(R), dS, len(S), g, transport="rehearsal").matches == exp
    assert np.array_equal(dR.cpu().numpy().view(DT), R)  # inputs untouched


def test_dropin_table_api(sgx, gpu):
    import ctypes as C

    R, S = sgx.reference_relations(1 << 16, 1 << 16)
    tR = sgx.table_t(R.ctypes.data, len(R), 0, 0)
    tS = sgx.table_t(S.ctypes.data, len(S), 0, 0)
    cfg = sgx.joinconfig_t()
    cfg.NTHREADS = 8
    out = sgx.result_t()
    os.environ["SGXAMD_MULTI_TRANSPORT"] = "rehearsal"
    try:
        rc = sgx.lib.mi355_rho_join_multi(C.byref(tR), C.byref(tS), C.byref(cfg), 4, C.byref(out))
    finally:
        del os.environ["SGXAMD_MULTI_TRANSPORT"]
    assert rc == 0, sgx.last_error()
    assert out.totalresults == 1 << 16 and out.nthreads == 8 and out.throughput > 0


def test_native_driver_multi_gpu_rehearsal(gpu):
    """The reference driver's call chain (native.cpp:137 -> run_join -> RHO) with
    SGXAMD_GPUS=4: RHO() takes the radix-shard exchange; the count is exact and the
    reference's timing lines are all there."""
    exe = os.path.join(PKG, "bin", "native_mi355")
    env = dict(os.environ, SGXAMD_GPUS="4", SGXAMD_MULTI_TRANSPORT="rehearsal")
    out = subprocess.run([exe, "-a", "RHO", "-r", "1000000", "-s", "3000000"], capture_output=True, text=True,
                         env=env, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "Radix-shard exchange over 4 GPUs (one-GPU rehearsal" in out.stdout
    assert "Matches = 3000000" in out.stdout
    for key in ("Partition Overall (cycles)", "Build+Join Overall (cycles)", "Throughput (M rec/sec)"):
        assert key in out.stdout


def test_rccl_comm_single_rank(sgx, orc, gpu):
    """One-process-per-GPU entry points on a world of one: RCCL loads, the unique id and
    communicator are created, and the sharded join of the slice is the local join."""
    import torch

    uid = sgx.multi_unique_id()
    assert len(uid) == 128
    h = sgx.multi_comm_init(uid, 1, 0)
    try:
        R, S = sgx.reference_relations(1 << 16, 1 << 16, selectivity=50)
        dR = torch.from_numpy(R.view(np.int64)).to(gpu)
        dS = torch.from_numpy(S.view(np.int64)).to(gpu)
        res = sgx.rho_join_sharded(h, dR, len(R), dS, len(S))
        assert res.matches == orc.rho_join(R, S, 4)[0]
        assert res.stats["transport"] == "rccl" and res.stats["world"] == 1
    finally:
        sgx.multi_comm_destroy(h)


def sorted_triples(t):
    t = np.asarray(t, dtype=np.uint32).reshape(-1, 3)
    return t[np.lexsort((t[:, 2], t[:, 1], t[:, 0]))]


def materialize_cases(sgx):
    rng = np.random.default_rng(17)
    dt = np.dtype([("key", "<u4"), ("payload", "<u4")])
    R1, S1 = sgx.reference_relations(1 << 16, 1 << 16, selectivity=50)
    R2 = np.empty(30_000, dtype=dt)
    R2["key"] = rng.integers(0, 5000, len(R2))
    R2["payload"] = np.arange(len(R2))
    S2 = np.empty(40_003, dtype=dt)
    S2["key"] = rng.integers(0, 5000, len(S2))
    S2["payload"] = np.arange(len(S2)) + 7
    return [(R1, S1), (R2, S2)]


@pytest.mark.parametrize("g", [2, 4, 8])
def test_materialize_multi_matches_oracle(sgx, orc, gpu, g):
    """Multi-GPU MATERIALIZE (radix_join.cpp:437-446): tuples (with their payloads) on the
    wire, every rank's triples concatenated into the caller's buffer: the same multiset
    of {key, R payload, S payload} as the oracle's restated RHO; too small a buffer is a
    capacity error that reports the triples needed."""
    import torch

    for R, S in materialize_cases(sgx):
        exp = orc.rho_join_triples(R, S, 4)
        out = np.zeros((len(exp) + 3, 3), dtype=np.uint32)
        res = multi(sgx, R, S, g, out=out, out_capacity=len(out))
        assert res.matches == len(exp)
        assert res.stats["elem_bytes"] == 8  # the payloads travel
        assert np.array_equal(sorted_triples(out[:len(exp)]), sorted_triples(exp))
        with pytest.raises(sgx.Mi355Error, match=f"{len(exp)} triples needed"):
            multi(sgx, R, S, g, out=out, out_capacity=len(exp) - 1)
    # device output, device-resident inputs
    R, S = materialize_cases(sgx)[0]
    exp = orc.rho_join_triples(R, S, 4)
    dR = torch.from_numpy(R.view(np.int64)).to(gpu)
    dS = torch.from_numpy(S.view(np.int64)).to(gpu)
    dout = torch.zeros((len(exp), 3), dtype=torch.int32, device=gpu)
    assert multi(sgx, dR, S=dS, g=g, out=dout, out_capacity=len(exp)).matches == len(exp)
    assert np.array_equal(sorted_triples(dout.cpu().numpy().view(np.uint32)), sorted_triples(exp))


def test_rccl_single_rank_local_failure_keeps_handle(sgx, orc, gpu):
    """A world of one has no collective to leave: a local failure (injected at the local
    join) returns that error and leaves the communicator usable, so the next sharded
    join on the same handle is exact (the handle is not marked broken)."""
    import torch

    h = sgx.multi_comm_init(sgx.multi_unique_id(), 1, 0)
    try:
        R, S = sgx.reference_relations(1 << 16, 1 << 16, selectivity=50)
        dR = torch.from_numpy(R.view(np.int64)).to(gpu)
        dS = torch.from_numpy(S.view(np.int64)).to(gpu)
        sgx.multi_inject_failure(0, 3)
        try:
            with pytest.raises(sgx.Mi355Error, match="injected failure"):
                sgx.rho_join_sharded(h, dR, len(R), dS, len(S))
        finally:
            sgx.multi_inject_failure(-1, 0)
        res = sgx.rho_join_sharded(h, dR, len(R), dS, len(S))
        assert res.matches == orc.rho_join(R, S, 4)[0]
        assert res.stats["ms_tail"] == -1  # nothing exchanged: no tail measured
    finally:
        sgx.multi_comm_destroy(h)


@pytest.mark.parametrize("kw", [{}, {"radix_bits": 14, "passes": 2}], ids=["keys", "wire16"])
@pytest.mark.parametrize("step", [1, 2, 3])
def test_failure_on_one_rank(sgx, orc, gpu, wire16, step, kw):
    """A rank that fails (exchange buffers, a shard pass of S, its local join) flags it in
    the next collective: every rank leaves the join at the same step, the call returns
    the failed rank's own error (no rank is left waiting in a collective), and the next
    join on the same transport is exact.  Also on the u16 wire (a 14-bit plan over 4
    ranks), whose sender-side passes and gathers take the local join's place."""
    R, S = sgx.reference_relations(1 << 17, (1 << 17) + 5)
    exp = orc.rho_join(R, S, 4)[0]
    sgx.multi_inject_failure(2, step)
    try:
        with pytest.raises(sgx.Mi355Error, match="rank 2: injected failure"):
            multi(sgx, R, S, 4, **kw)
    finally:
        sgx.multi_inject_failure(-1, 0)
    res = multi(sgx, R, S, 4, **kw)
    assert res.matches == exp and (res.stats["elem_bytes"] == 2 or not kw)


def _keys_out(rel_, g):
    """Keys of a host relation that leave their rank's slice (_slices_sent, one per key)."""
    import torch

    keys = rel_["key"] if rel_.dtype.names else rel_ & 0xFFFFFFFF
    return _slices_sent(torch.from_numpy(np.asarray(keys, dtype=np.int64)), g, 1)


def _exchange_bytes(st, out_r, out_s, g):
    """sent_bytes of a counting join's keys exchange over all ranks of one process: 4 bytes
    per key that leaves its rank, except that on the u16 wire S's keys go as 2-byte
    residuals plus, per peer, the sender's counts row (P partition counts, P partition
    starts and its largest key, 8 bytes each); the padding of each run's slot (its
    partitions on 16-byte boundaries, read in place) is not counted."""
    if st["elem_bytes"] == 2:
        p = 1 << st["local"]["radix_bits"]
        return 4 * out_r + 2 * out_s + g * (g - 1) * (2 * p + 1) * 8
    assert st["elem_bytes"] == 4
    return 4 * (out_r + out_s)


@pytest.mark.parametrize("g", [2, 4, 8])
def test_wire16_exchange(sgx, orc, gpu, wire16, g):
    """The u16 wire: with log2 g + the local radix bits >= 16, every
    sender runs the receiver's two passes on the S keys it sends each rank, and 2-byte
    residuals travel with one counts row per peer (R's keys as 4 bytes, partitioned by
    the receiver while S is on the wire); each receiver gathers a partition's g pieces
    (one per sender) and runs the narrow build/probe.  Exact counts
    against the sort counter on pk / fk, on random keys with duplicates over the whole
    u32 range (residuals up to 2^16: the windowed direct table), on a hot key, and on
    sizes that leave some (sender, destination) runs empty; the exact bytes."""
    bits = 16 - (g.bit_length() - 1)
    rng = np.random.default_rng(g)
    cases = [sgx.reference_relations(1 << 20, 1 << 20),
             (rel(rng.integers(0, 2**32, 300_001, dtype=np.uint64).astype(np.uint32)),
              rel(rng.integers(0, 2**32, 200_003, dtype=np.uint64).astype(np.uint32))),
             (rel(rng.integers(0, 5000, 70_000, dtype=np.uint64).astype(np.uint32) * 8),
              rel(np.full(90_000, 4096 * 8, dtype=np.uint32))),
             (rel(np.arange(1, 3 * g + 1, dtype=np.uint32)), rel(np.arange(1, 2 * g + 2, dtype=np.uint32)))]
    for R, S in cases:
        R = np.concatenate([R, R[: len(R) // 3]])  # duplicate R keys too
        exp = orc.count_join_sort(R, S)
        res = multi(sgx, R, S, g, radix_bits=bits, passes=2)
        st = res.stats
        assert res.matches == exp, (g, len(R), len(S))
        assert st["elem_bytes"] == 2 and st["local"]["radix_bits"] == bits
        assert st["sent_bytes"] == _exchange_bytes(st, _keys_out(R, g), _keys_out(S, g), g)
        assert 0 <= st["ms_tail"] <= st["ms_total"]


def test_wire16_largest_key_check(sgx, orc, gpu, wire16):
    """2 ranks and a 14-bit plan: log2 G + bits = 15 < 16, so the residuals fit 16 bits
    only when S's keys allow.  The senders run their passes, then S's largest key over
    the ranks decides: 2-byte residuals for keys below 2^31 (pk / fk), else S goes as
    4-byte keys (its shard scatter reused) and the local join takes the 4-byte plan --
    exact either way, and the bytes say which."""
    R, S = sgx.reference_relations(1 << 20, 1 << 20)
    res = multi(sgx, R, S, 2, radix_bits=14, passes=2)
    assert res.matches == orc.count_join_sort(R, S) and res.stats["elem_bytes"] == 2
    assert res.stats["sent_bytes"] == _exchange_bytes(res.stats, _keys_out(R, 2), _keys_out(S, 2), 2)
    rng = np.random.default_rng(77)
    R2 = rel(rng.integers(0, 2**32, 200_001, dtype=np.uint64).astype(np.uint32))
    S2 = rel(np.concatenate([rng.integers(0, 2**32, 150_000, dtype=np.uint64).astype(np.uint32),
                             R2["key"][:60_000], np.array([2**32 - 1], dtype=np.uint32)]))
    res = multi(sgx, R2, S2, 2, radix_bits=14, passes=2)
    assert res.matches == orc.count_join_sort(R2, S2) and res.stats["elem_bytes"] == 4
    assert res.stats["sent_bytes"] == 4 * (_keys_out(R2, 2) + _keys_out(S2, 2))


def _slices_sent(keys, g, elem):
    """Bytes a rank-sliced relation sends to other ranks: per slice (radix_join.cpp:1488-1499
    slicing), every element whose low log2(g) key bits name another rank."""
    import torch

    n = keys.numel()
    per = n // g
    kept = 0
    for r in range(g):
        a, b = r * per, (n if r == g - 1 else (r + 1) * per)
        kept += int(((keys[a:b] & (g - 1)) == r).sum().item())
    return (n - kept) * elem


def test_config4_rehearsal_full_size(sgx, gpu):
    """BASELINE config 4 at its size through the 8-rank pipeline (rehearsal transport on one
    MI355X): pk(2^27) join fk(2^30, maxid 2^27), device generators (native.cpp:62-101
    shapes).  Exercises the receive capacity G*K*ceil(m/K) = 2^30 keys per rank (4 GiB,
    byte offsets past 2^32), the keys-only plan decision and the local S-heavy plan with
    key_shift 3.  matches == |S|; every rank receives exactly 2^24 R and 2^27 S keys (8
    copies of its 1/8 of 1..2^27); 4-byte keys on the wire, the exact bytes."""
    import torch

    nR, nS, g = 1 << 27, 1 << 30, 8
    R = torch.empty(nR, dtype=torch.int64, device=gpu)
    S = torch.empty(nS, dtype=torch.int64, device=gpu)
    sgx.gen_pk_dev(R, nR, 0, nR, 11111)
    sgx.gen_fk_dev(S, nS, 0, nR, 22222)
    try:
        res = sgx.rho_join_multi(R, nR, S, nS, g, transport="rehearsal")
        st = res.stats
        assert res.matches == nS
        assert st["world"] == g and st["elem_bytes"] in (2, 4) and st["local"]["layout"] in (2, 3, 4)
        assert st["recv_r_max"] == st["recv_r_min"] == nR // g
        assert st["recv_s_max"] == st["recv_s_min"] == nS // g
        out_r, out_s = _slices_sent(R & 0xFFFFFFFF, g, 1), _slices_sent(S & 0xFFFFFFFF, g, 1)
        assert st["sent_bytes"] == _exchange_bytes(st, out_r, out_s, g)
        assert abs(out_r + out_s - (nR + nS) * 7 / 8) < (nR + nS) * 0.001
        # S's pass 1 ran per landed piece: the device time after S's last piece is a part
        # of the local join (the rehearsal's ranks share one GPU, so only its presence is
        # checked, not its size)
        assert 0 < st["ms_tail"] <= st["ms_total"]
        print(f"c4 rehearsal G=8: {st['ms_total']:.2f} ms (after S landed: {st['ms_tail']:.2f} ms), local plan "
              f"{st['local']['radix_bits']} bits, sent {st['sent_bytes'] / 1e9:.3f} GB")
    finally:
        del R, S
        sgx.multi_release()
        torch.cuda.empty_cache()


def test_config5_rehearsal_full_size(sgx, gpu):
    """BASELINE config 5 at its size through the 8-rank pipeline: pk(2^28) join the host
    mt19937_64 seed-22222 Zipf(0.75) stream over 1..2^28 (generator.cpp restating
    genzipf.cpp:87-144), staged once to HBM.  matches == |S| (every Zipf key is an R key);
    the load report: the hot keys land where their low 3 bits say, so the received S
    per rank is uneven (reported as max / mean)."""
    import torch

    n, g = 1 << 28, 8
    R = torch.empty(n, dtype=torch.int64, device=gpu)
    sgx.gen_pk_dev(R, n, 0, n, 11111)
    host = np.empty(n, dtype=np.int64)
    sgx.gen_zipf(host, n, n, 0.75, 22222, 16)
    S = torch.from_numpy(host).to(gpu)
    del host
    try:
        res = sgx.rho_join_multi(R, n, S, n, g, transport="rehearsal")
        st = res.stats
        assert res.matches == n
        assert st["elem_bytes"] == 4  # 2^25 keys per rank: not the narrow local plan (mode 1)
        assert st["recv_r_max"] == st["recv_r_min"] == n // g
        per_rank = torch.bincount((S & (g - 1)).to(torch.int64), minlength=g)
        assert st["recv_s_max"] == int(per_rank.max()) and st["recv_s_min"] == int(per_rank.min())
        print(f"c5 rehearsal G=8: {st['ms_total']:.2f} ms, recv_s max/mean "
              f"{st['recv_s_max'] / (n / g):.3f}, max S partition {st['max_part_s']}")
    finally:
        del R, S
        sgx.multi_release()
        torch.cuda.empty_cache()


LATE_CHILD = r"""
import numpy as np
import sgxamd, oracle
# unpooled local plans (one-pass, 2^16 per rank) and pooled key plans (2^21 per rank)
for n, g in ((1 << 18, 4), (1 << 23, 4)):
    R, S = sgxamd.reference_relations(n, n + 17)
    exp = oracle.count_join_sort(R, S)
    res = sgxamd.rho_join_multi(R, len(R), S, len(S), g, transport="rehearsal")
    assert res.matches == exp, (n, g, res.matches, exp)
    assert res.stats["ms_tail"] > 0
print("late ok")
"""


def test_late_pieces(gpu):
    """Every piece lands 3 ms late (SGXAMD_DEBUG_EXCHANGE_DELAY_US holds the communication
    stream before each post): the local passes that read a received piece must wait for
    its event, S's per-piece pass 1 (pooled plans) as much as the whole-relation passes
    (one-pass plans), or they read a receive buffer that has not landed yet."""
    e = dict(os.environ, SGXAMD_DEBUG_EXCHANGE_DELAY_US="3000")
    e["PYTHONPATH"] = os.pathsep.join([os.path.join(PKG, "python"), os.path.join(os.path.dirname(PKG), "oracle"),
                                       e.get("PYTHONPATH", "")])
    r = subprocess.run([sys.executable, "-c", LATE_CHILD], env=e, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "late ok" in r.stdout, (r.stdout[-2000:], r.stderr[-2000:])
