"""RcclTransport (csrc/multi_host.cpp) at G = 2 / 4 / 8 on ONE MI355X, through the RCCL
test double of tests/rccl_double (loaded with mi355_multi_set_rccl_library).

RCCL refuses two ranks on one GPU, so without the double the transport's grouped
Send/Recv offsets, its ncclUint32 key typing, the count all-gather on the split
communicator (recv[q] = h[w1 + q*w1 + rank]) and its all-reduces would first run at
G > 1 on the driver's 8-GPU node.  Here they run with the product's own code:
  - single process (mi355_rho_join_multi_ex, transport "rccl"): ncclCommInitAll
    communicators, the tuples through ncclSend/ncclRecv, counts through the host table;
  - one process per GPU (mi355_multi_comm_init + mi355_rho_join_sharded): G Python
    threads stand in for the G processes, each with its own communicator pair
    (ncclCommInitRank + ncclCommSplit), the count all-gathers and all-reduces through
    RCCL calls.
Counts are compared bit-exactly with the oracle's restated RHO (radix_join.cpp) and the
sort counter; the reference's cross-thread prefix (radix_join.cpp:897-915) is what the
exchange replaces."""
import ctypes as C
import os
import threading

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

DOUBLE = os.path.join(ROOT, "tests", "rccl_double", "librccl_double.so")
DT = np.dtype([("key", "<u4"), ("payload", "<u4")])


def rel(keys):
    x = np.empty(len(keys), dtype=DT)
    x["key"] = keys
    x["payload"] = np.arange(len(keys), dtype=np.uint32)
    return x


@pytest.fixture
def dbl(sgx, gpu):
    assert os.path.exists(DOUBLE), "build tests/rccl_double (make -C tests/rccl_double or __graft_entry__.build())"
    sgx.multi_set_rccl_library(DOUBLE)
    lib = C.CDLL(DOUBLE)  # the same instance libsgxamd.so loaded (fault injection, timeout)
    lib.rccl_double_set_timeout_ms(20000)
    try:
        yield lib
    finally:
        lib.rccl_double_fail(-1, 0)
        for r in range(8):
            lib.rccl_double_fail(r, 0)
        sgx.multi_inject_failure(-1, 0)
        sgx.multi_set_rccl_library(None)
        sgx.multi_release()


def multi(sgx, R, S, g, **kw):
    return sgx.rho_join_multi(R, len(R), S, len(S), g, transport="rccl", **kw)


# ---------------------------------------------------------------- single process
@pytest.mark.parametrize("g", [2, 4, 8])
def test_inprocess_reference_pk_fk(sgx, orc, dbl, g):
    n = 1 << 18
    R, S = sgx.reference_relations(n, n)
    res = multi(sgx, R, S, g)
    assert res.matches == orc.rho_join(R, S, 4)[0] == n
    st = res.stats
    assert st["world"] == g and st["transport"] == "rccl"
    assert st["recv_r_min"] == st["recv_r_max"] == n // g


@pytest.mark.parametrize("seed,nR,nS,kmax,g", [(1, 5000, 7001, 300, 4), (2, 100_003, 77_777, 2**32 - 1, 8),
                                               (3, 3, 5, 2, 4), (5, 1 << 20, 1 << 20, 1 << 19, 8)])
def test_inprocess_random_with_duplicates(sgx, orc, dbl, seed, nR, nS, kmax, g):
    """Duplicates over the full u32 range, tiny slices (empty pieces skipped on both sides
    of the send/recv pairs), tuples (one-pass plans) and keys (two-pass plans) on the wire."""
    rng = np.random.default_rng(seed)
    R = rel(rng.integers(0, kmax + 1, nR, dtype=np.uint64).astype(np.uint32))
    S = rel(rng.integers(0, kmax + 1, nS, dtype=np.uint64).astype(np.uint32))
    exp = orc.count_join_sort(R, S)
    assert multi(sgx, R, S, g).matches == exp
    assert multi(sgx, R, S, g, algorithm="RHT").matches == exp
    keys = multi(sgx, R, S, g, radix_bits=14, passes=2)
    assert keys.matches == exp


@pytest.mark.parametrize("step", [1, 2, 3, 4, 5])
def test_inprocess_failure_on_one_rank(sgx, orc, dbl, step):
    """A rank that fails (buffers, a shard pass, the local join, no context, the local
    join's stream sync) flags it at the next collective; every rank leaves together and
    the communicators stay usable: the next join is exact."""
    R, S = sgx.reference_relations(1 << 17, (1 << 17) + 5)
    exp = orc.rho_join(R, S, 4)[0]
    sgx.multi_inject_failure(2, step)
    want = "hipStreamSynchronize \\(local join\\)" if step == 5 else "injected failure"
    try:
        with pytest.raises(sgx.Mi355Error, match="rank 2: " + want):
            multi(sgx, R, S, 4)
    finally:
        sgx.multi_inject_failure(-1, 0)
    assert multi(sgx, R, S, 4).matches == exp


def test_inprocess_transport_failure(sgx, orc, dbl):
    """An RCCL call fails on one rank: it leaves the collective sequence, the other rank
    threads are released (host waits aborted; the double's waits time out), the call
    returns MI355_ERR_COMM naming that rank, and the next call builds new communicators."""
    R, S = sgx.reference_relations(1 << 16, 1 << 16)
    exp = orc.rho_join(R, S, 4)[0]
    dbl.rccl_double_set_timeout_ms(3000)
    dbl.rccl_double_fail(1, 3)  # rank 1's third Send/Recv
    with pytest.raises(sgx.Mi355Error) as ei:
        multi(sgx, R, S, 4)
    assert ei.value.code == -6 and "rank 1:" in str(ei.value)
    dbl.rccl_double_set_timeout_ms(20000)
    assert multi(sgx, R, S, 4).matches == exp


@pytest.mark.parametrize("g", [2, 4, 8])
def test_inprocess_materialize(sgx, orc, dbl, g):
    """Multi-GPU MATERIALIZE through RcclTransport (tuples with payloads as ncclUint64 on
    the wire): the ranks' triples equal the oracle's as a multiset."""
    from test_multi_gpu import materialize_cases, sorted_triples

    for R, S in materialize_cases(sgx):
        exp = orc.rho_join_triples(R, S, 4)
        out = np.zeros((len(exp), 3), dtype=np.uint32)
        res = multi(sgx, R, S, g, out=out, out_capacity=len(out))
        assert res.matches == len(exp) and res.stats["transport"] == "rccl"
        assert np.array_equal(sorted_triples(out), sorted_triples(exp))


def test_inprocess_config4_full_size(sgx, dbl, gpu):
    """BASELINE config 4 at its size over 8 RCCL ranks (the double on one GPU): pk(2^27)
    join fk(2^30): matches == 2^30, 4-byte keys as ncclUint32 on the wire, exactly 2^24 R
    and 2^27 S keys received per rank, and the sent bytes of every key whose low 3 bits
    name another rank (counted on the device)."""
    import torch

    from test_multi_gpu import _exchange_bytes, _slices_sent

    nR, nS, g = 1 << 27, 1 << 30, 8
    R = torch.empty(nR, dtype=torch.int64, device=gpu)
    S = torch.empty(nS, dtype=torch.int64, device=gpu)
    sgx.gen_pk_dev(R, nR, 0, nR, 11111)
    sgx.gen_fk_dev(S, nS, 0, nR, 22222)
    torch.cuda.synchronize()
    try:
        # the same join on one GPU without an exchange: its S side (S's passes and the
        # build/probe, the work that follows S's arrival) is what the tail may cost
        sgx.timing_enable(True)
        assert sgx.rho_join(R, nR, S, nS).matches == nS
        s_side = sum(ms for name, ms in sgx.timings() if name.startswith("S_") or name.startswith("join"))
        # (the first call allocates every rank's workspace between its launches, and that
        # host time would show in its tail: three warm calls follow it)
        tails = []
        for i in range(4):
            res = sgx.rho_join_multi(R, nR, S, nS, g, transport="rccl")
            st = res.stats
            assert res.matches == nS
            if i:
                tails.append(st["ms_tail"])
        assert st["transport"] == "rccl" and st["world"] == g and st["elem_bytes"] in (2, 4)
        assert st["recv_r_max"] == st["recv_r_min"] == nR // g
        assert st["recv_s_max"] == st["recv_s_min"] == nS // g
        out_r, out_s = _slices_sent(R & 0xFFFFFFFF, g, 1), _slices_sent(S & 0xFFFFFFFF, g, 1)
        assert st["sent_bytes"] == _exchange_bytes(st, out_r, out_s, g)
        # the double's transfers are kernels on the communication streams (k_copy), so an
        # exchange starved of CUs by the join's own grids shows up here as time: the tail
        # after S's last piece landed (the 8 ranks' S-side work, on this one GPU) stays
        # within 1.75x the one-GPU join's S side in the best of three warm joins and within
        # 2.5x in every one -- S's pass 1 runs per piece as pieces land, so most of it is
        # hidden behind the exchange.  (The eight ranks share one GPU, and their host threads
        # the box's 16 CPUs: from join to join the tail varies by 1-3 ms -- 6.4-10.7 ms
        # against a 4.8-5.2-ms S side in round 6, scripts/dev/c4_double_tail.py,
        # profiles/r06zg_c4_double_tails.log -- while the S side itself shrank with every
        # faster single-GPU kernel, so round 5's 1.5x on one join failed one run in three.)
        assert 0 < min(tails) <= 1.75 * s_side and max(tails) <= 2.5 * s_side, (tails, s_side, st["ms_total"])
        print(f"c4 rccl-double G=8: {st['ms_total']:.2f} ms, tail {st['ms_tail']:.2f} ms (one-GPU S side "
              f"{s_side:.2f} ms), sent {st['sent_bytes'] / 1e9:.3f} GB")
    finally:
        del R, S
        sgx.multi_release()
        torch.cuda.empty_cache()


# ---------------------------------------------------------------- one "process" per GPU
def sharded(sgx, R, S, g, *, handles=None, algorithm="RHO", timeout=120, outs=None, **kw_plan):
    """Rank r's slice of the device tensors R and S (radix_join.cpp:1488-1499 slicing)
    joined by G threads, each standing for one process with its own communicator
    (created here unless `handles` are given).  Returns (results, errors, handles)."""
    import torch

    torch.cuda.synchronize()
    own = handles is None
    if own:
        uid = sgx.multi_unique_id()
        handles = [None] * g
    res, errs = [None] * g, [None] * g
    nR, nS = R.numel(), S.numel()

    def body(r):
        try:
            if own:
                handles[r] = sgx.multi_comm_init(uid, g, r)
            ra, rb = r * (nR // g), (nR if r == g - 1 else (r + 1) * (nR // g))
            sa, sb = r * (nS // g), (nS if r == g - 1 else (r + 1) * (nS // g))
            kw = {} if outs is None else {"out": outs[r], "out_capacity": outs[r].shape[0]}
            res[r] = sgx.rho_join_sharded(handles[r], R[ra:rb], rb - ra, S[sa:sb], sb - sa, algorithm=algorithm,
                                          **kw, **kw_plan)
        except Exception as e:  # noqa: BLE001 - every rank's outcome is checked by the caller
            errs[r] = e

    th = [threading.Thread(target=body, args=(r,)) for r in range(g)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout)
        assert not t.is_alive(), "a rank thread hung"
    return res, errs, handles


def destroy(sgx, handles):
    for h in handles:
        if h:
            sgx.multi_comm_destroy(h)


@pytest.mark.parametrize("g", [2, 4, 8])
def test_sharded_materialize_chunks(sgx, orc, dbl, gpu, g):
    """One process per GPU, MATERIALIZE: every rank writes its own output chunk (its
    local_matches triples, device memory); the chunks together equal the oracle's
    triples as a multiset and their sizes add up to the global count."""
    import torch

    from test_multi_gpu import materialize_cases, sorted_triples

    R, S = materialize_cases(sgx)[1]
    exp = orc.rho_join_triples(R, S, 4)
    dR = torch.from_numpy(R.view(np.int64)).to(gpu)
    dS = torch.from_numpy(S.view(np.int64)).to(gpu)
    outs = [torch.zeros((len(exp), 3), dtype=torch.int32, device=gpu) for _ in range(g)]
    res, errs, handles = sharded(sgx, dR, dS, g, outs=outs)
    try:
        assert errs == [None] * g, errs
        loc = [r.stats["local_matches"] for r in res]
        assert all(r.matches == len(exp) for r in res) and sum(loc) == len(exp)
        got = np.concatenate([o[:n].cpu().numpy().view(np.uint32) for o, n in zip(outs, loc)])
        assert np.array_equal(sorted_triples(got), sorted_triples(exp))
    finally:
        destroy(sgx, handles)


@pytest.mark.parametrize("g", [2, 4, 8])
def test_sharded_reference_pk_fk(sgx, orc, dbl, gpu, g):
    import torch

    n = 1 << 18
    Rh, Sh = sgx.reference_relations(n, n)
    R = torch.from_numpy(Rh.view(np.int64)).to(gpu)
    S = torch.from_numpy(Sh.view(np.int64)).to(gpu)
    res, errs, hs = sharded(sgx, R, S, g)
    try:
        assert errs == [None] * g, errs
        exp = orc.rho_join(Rh, Sh, 4)[0]
        assert [r.matches for r in res] == [exp] * g
        for r, x in enumerate(res):
            st = x.stats
            assert st["transport"] == "rccl" and st["world"] == g and st["rank"] == r
            assert st["recv_r_max"] == n // g  # every rank's own receive: 1/g of 1..n
        assert sum(x.stats["local_matches"] for x in res) == exp
    finally:
        destroy(sgx, hs)


@pytest.mark.parametrize("g,kmax", [(4, 1000), (8, 2**32 - 1)])
def test_sharded_random_with_duplicates_and_rht(sgx, orc, dbl, gpu, g, kmax):
    import torch

    rng = np.random.default_rng(g)
    Rh = rel(rng.integers(0, kmax + 1, 300_001, dtype=np.uint64).astype(np.uint32))
    Sh = rel(rng.integers(0, kmax + 1, 200_003, dtype=np.uint64).astype(np.uint32))
    R = torch.from_numpy(Rh.view(np.int64)).to(gpu)
    S = torch.from_numpy(Sh.view(np.int64)).to(gpu)
    exp = orc.count_join_sort(Rh, Sh)
    res, errs, hs = sharded(sgx, R, S, g)
    try:
        assert errs == [None] * g, errs
        assert {r.matches for r in res} == {exp}
        res2, errs2, _ = sharded(sgx, R, S, g, handles=hs, algorithm="RHT")  # communicators reused
        assert errs2 == [None] * g, errs2
        assert {r.matches for r in res2} == {exp}
    finally:
        destroy(sgx, hs)


def test_sharded_keys_exchange_exact_bytes(sgx, dbl, gpu):
    """pk(2^24) join fk(2^25) over 8 ranks: the keys-only plan (elem_bytes 4) and every
    rank's sent bytes = 4 x its keys whose low 3 bits name another rank."""
    import torch

    g, nR, nS = 8, 1 << 24, 1 << 25
    R = torch.empty(nR, dtype=torch.int64, device=gpu)
    S = torch.empty(nS, dtype=torch.int64, device=gpu)
    sgx.gen_pk_dev(R, nR, 0, nR, 11111)
    sgx.gen_fk_dev(S, nS, 0, nR, 22222)
    res, errs, hs = sharded(sgx, R, S, g)
    try:
        assert errs == [None] * g, errs
        assert {r.matches for r in res} == {nS}
        for r, x in enumerate(res):
            st = x.stats
            assert st["elem_bytes"] in (2, 4)
            out = []
            for X in (R, S):
                n = X.numel()
                a, b = r * (n // g), (n if r == g - 1 else (r + 1) * (n // g))
                k = X[a:b] & 0xFFFFFFFF
                out.append(int(((k & (g - 1)) != r).sum().item()))
            # u16 wire: S as 2 bytes per key and a counts row (2 P + 1 words) per peer
            rows = (g - 1) * (2 * (1 << st["local"]["radix_bits"]) + 1) * 8  # counts, starts, largest key
            assert st["sent_bytes"] == (4 * out[0] + 2 * out[1] + rows if st["elem_bytes"] == 2
                                        else 4 * (out[0] + out[1]))
            assert st["recv_r_max"] == nR // g and st["recv_s_max"] == nS // g
    finally:
        destroy(sgx, hs)
        del R, S
        torch.cuda.empty_cache()


@pytest.mark.parametrize("g", [2, 4, 8])
def test_wire16_rccl(sgx, orc, dbl, gpu, g):
    """The u16 wire (forced: mode 2) through RcclTransport (S's residuals as ncclUint8
    pairs, its counts rows as ncclUint64, R's keys as ncclUint32), in one process and one
    "process" per rank: exact counts against the sort counter on random keys with
    duplicates over the whole u32 range and on pk / fk, the exact bytes."""
    sgx.multi_set_wire(2)
    try:
        _wire16_rccl(sgx, orc, gpu, g)
    finally:
        sgx.multi_set_wire(1)


def _wire16_rccl(sgx, orc, gpu, g):
    import torch

    from test_multi_gpu import _exchange_bytes, _keys_out

    bits = 16 - (g.bit_length() - 1)
    rng = np.random.default_rng(100 + g)
    Rh = rel(rng.integers(0, 2**32, 300_001, dtype=np.uint64).astype(np.uint32))
    Sh = rel(rng.integers(0, 2**32, 200_003, dtype=np.uint64).astype(np.uint32))
    Sh = np.concatenate([Sh, Rh[:50_000]])  # matches and duplicates
    exp = orc.count_join_sort(Rh, Sh)
    res = multi(sgx, Rh, Sh, g, radix_bits=bits, passes=2)
    st = res.stats
    assert res.matches == exp and st["transport"] == "rccl" and st["elem_bytes"] == 2
    assert st["sent_bytes"] == _exchange_bytes(st, _keys_out(Rh, g), _keys_out(Sh, g), g)
    if g == 2:  # log2 G + 14 bits < 16: S's largest key decides (here: too large, keys)
        res = multi(sgx, Rh, Sh, g, radix_bits=14, passes=2)
        assert res.matches == exp and res.stats["elem_bytes"] == 4
    Pk, Fk = sgx.reference_relations(1 << 20, 1 << 20)
    R = torch.from_numpy(Pk.view(np.int64)).to(gpu)
    S = torch.from_numpy(Fk.view(np.int64)).to(gpu)
    out, errs, hs = sharded(sgx, R, S, g, radix_bits=bits, passes=2)
    try:
        assert errs == [None] * g, errs
        assert {r.matches for r in out} == {1 << 20}
        assert all(r.stats["elem_bytes"] == 2 for r in out)
        assert sum(r.stats["local_matches"] for r in out) == 1 << 20
    finally:
        destroy(sgx, hs)


@pytest.mark.parametrize("step", [1, 2, 3, 4, 5])
def test_sharded_failure_on_one_rank(sgx, orc, dbl, gpu, step):
    """One process per GPU: rank 2 fails at `step`; every rank raises at the same
    collective (rank 2 its own error, the others MI355_ERR_COMM 'another rank failed'),
    no rank hangs, the communicators are not aborted, and the next join is exact."""
    import torch

    Rh, Sh = sgx.reference_relations(1 << 17, (1 << 17) + 5)
    R = torch.from_numpy(Rh.view(np.int64)).to(gpu)
    S = torch.from_numpy(Sh.view(np.int64)).to(gpu)
    exp = orc.rho_join(Rh, Sh, 4)[0]
    uid = sgx.multi_unique_id()
    hs = [None] * 4

    def init(r):
        hs[r] = sgx.multi_comm_init(uid, 4, r)

    th = [threading.Thread(target=init, args=(r,)) for r in range(4)]
    [t.start() for t in th]
    [t.join(60) for t in th]
    try:
        sgx.multi_inject_failure(2, step)
        try:
            res, errs, _ = sharded(sgx, R, S, 4, handles=hs)
        finally:
            sgx.multi_inject_failure(-1, 0)
        assert all(isinstance(e, sgx.Mi355Error) for e in errs), errs
        want = "hipStreamSynchronize (local join)" if step == 5 else "injected failure"
        assert want in str(errs[2])
        for r in (0, 1, 3):
            assert errs[r].code == -6 and "another rank failed" in str(errs[r])
        res, errs, _ = sharded(sgx, R, S, 4, handles=hs)
        assert errs == [None] * 4 and {x.matches for x in res} == {exp}
    finally:
        destroy(sgx, hs)


@pytest.mark.parametrize("nth", [1, 4])
def test_sharded_transport_failure(sgx, orc, dbl, gpu, nth):
    """An RCCL call fails on rank 1 (its 1st: the sizes all-reduce; its 4th: a count
    all-gather): rank 1 leaves the sequence and aborts its communicators, the peers'
    waits in RCCL are released with an error, every rank raises MI355_ERR_COMM, the
    handles refuse further joins, and new communicators join exactly."""
    import torch

    Rh, Sh = sgx.reference_relations(1 << 16, 1 << 16)
    R = torch.from_numpy(Rh.view(np.int64)).to(gpu)
    S = torch.from_numpy(Sh.view(np.int64)).to(gpu)
    exp = orc.rho_join(Rh, Sh, 4)[0]
    uid = sgx.multi_unique_id()
    hs = [None] * 4
    th = [threading.Thread(target=lambda r: hs.__setitem__(r, sgx.multi_comm_init(uid, 4, r)), args=(r,))
          for r in range(4)]
    [t.start() for t in th]
    [t.join(60) for t in th]
    try:
        dbl.rccl_double_set_timeout_ms(5000)
        dbl.rccl_double_fail(1, nth)
        res, errs, _ = sharded(sgx, R, S, 4, handles=hs)
        assert all(isinstance(e, sgx.Mi355Error) and e.code == -6 for e in errs), errs
        assert "injected" in str(errs[1]) or "system error" in str(errs[1])
        res, errs, _ = sharded(sgx, R, S, 4, handles=hs)
        assert all("communicator was aborted" in str(e) for e in errs), errs
    finally:
        dbl.rccl_double_set_timeout_ms(20000)
        destroy(sgx, hs)
    res, errs, hs = sharded(sgx, R, S, 4)
    try:
        assert errs == [None] * 4 and {x.matches for x in res} == {exp}
    finally:
        destroy(sgx, hs)


# ------------------------------------------------------------ rank processes (round 6)
def test_bench_rank_processes_on_double(sgx, gpu):
    """bench.py --gpus 2 as two rank PROCESSES sharing this GPU (its own rank launcher,
    gloo for the bench's barriers and the unique id's broadcast) on the RCCL test double
    in its cross-process mode (RCCL_DOUBLE_XPROC=1: shared-memory communicators, IPC-mapped
    buffers): mi355_multi_comm_init with rank 0's broadcast unique id, the split count
    communicator and mi355_rho_join_sharded run exactly as in the 8-GPU driver run.  The
    line says n_gpus 2, the join is exact (bench asserts every step's count), and each
    rank's sent bytes equal the bytes of its keys whose low bit names the other rank,
    counted here on the device from the same generators."""
    import json
    import subprocess
    import sys

    import torch

    log2n, g = 22, 2
    env = dict(os.environ, SGXAMD_DIST_IMPL="cxx-any", SGXAMD_RCCL_LIBRARY=DOUBLE, RCCL_DOUBLE_XPROC="1")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(g), "--dist-backend", "gloo",
           "--log2n", str(log2n), "--steps", "3", "--warmup", "1", "--no-scan", "--no-tpch", "--no-cpu-baseline",
           "--no-paper", "--no-configs", "--no-tuple-layout"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == g and line["rho"]["matches_ok"]
    m = line["multi"]
    assert m["world"] == g and m["transport"] == "rccl" and "cxx-rccl" in line["config"]["exchange"]
    # the same relations, generated here: every rank's slice of pk / fk over g * 2^log2n
    n = 1 << log2n
    gR = gS = n * g
    for pr in m["per_rank"]:
        rk = pr["rank"]
        R = torch.empty(n, dtype=torch.int64, device=gpu)
        S = torch.empty(n, dtype=torch.int64, device=gpu)
        sgx.gen_pk_dev(R, n, rk * n, gR, 11111)
        sgx.gen_fk_dev(S, n, rk * n, gR, 22222)
        out_r = int(((R & 0xFFFFFFFF) % g != rk).sum())
        out_s = int(((S & 0xFFFFFFFF) % g != rk).sum())
        # 4 bytes per key that leaves; on the u16 wire S's keys as 2-byte residuals and a
        # counts row of 2 P + 1 words per peer
        per_rank = 4 * (out_r + out_s) if m["elem_bytes"] == 4 else (
            4 * out_r + 2 * out_s + (g - 1) * (2 * (1 << line["rho"]["radix_bits"]) + 1) * 8)
        assert m["elem_bytes"] in (2, 4) and pr["sent_bytes"] == per_rank, (rk, pr["sent_bytes"], per_rank)
        assert pr["recv_r"] + pr["recv_s"] > 0
    print(f"bench --gpus 2 on the double (processes): {line['value']:.1f} M/s, elem {m['elem_bytes']} B, "
          f"sent {m['sent_bytes_total'] / 1e6:.1f} MB")
