"""TPC-H callers on the CPU side: the synthetic generator, the binary/text table
loaders (TpcHCommons.cpp) and the oracle's query restatement (tpch.cpp), the
latter pinned against an independent numpy formulation of each query.

The reference holds no TPC-H data or expected query answers (dbgen output is not
in the repository), so TPC-H parity is pinned by that independent restatement:
the oracle follows tpch.cpp step by step (filter_table, RHO joins with
MATERIALIZE, result transforms), numpy evaluates each query as set arithmetic."""
import os

import numpy as np
import pytest

import sgxamd.tpch as T
import oracle as O

DAY = 86400


@pytest.fixture(scope="module")
def tb():
    return T.generate(50, 11)  # SF 0.05


def test_generator_shapes_and_rules(tb):
    n = T.sizes(50, 11)
    assert tb.sizes == n
    assert n["customer"] == 7500 and n["orders"] == 75000 and n["part"] == 10000 and n["nation"] == 25
    assert 75000 <= n["lineitem"] <= 7 * 75000
    o, l, c = tb.cols["orders"], tb.cols["lineitem"], tb.cols["customer"]
    ok = o["o_orderkey"]["key"].astype(np.int64)
    i = np.arange(n["orders"])
    assert np.array_equal(ok, (i // 8) * 32 + (i % 8) + 1)  # sparse keys (8 of every 32)
    assert np.array_equal(o["o_orderkey"]["payload"], i)
    assert (o["o_custkey"] % 3 != 0).all() and o["o_custkey"].max() <= n["customer"]
    day = o["o_orderdate"] // DAY
    assert day.min() >= 8035 and day.max() <= 10591 - 151
    # lineitem rows belong to their orders in order; date rules of clause 4.2.3
    lk = l["l_orderkey"]["key"]
    assert (np.diff(lk.astype(np.int64)) >= 0).all()
    pos = np.searchsorted(ok, lk)
    od = o["o_orderdate"][pos] // DAY
    ship, commit, receipt = (l[k] // DAY for k in ("l_shipdate", "l_commitdate", "l_receiptdate"))
    assert ((ship - od >= 1) & (ship - od <= 121)).all()
    assert ((commit - od >= 30) & (commit - od <= 90)).all()
    assert ((receipt - ship >= 1) & (receipt - ship <= 30)).all()
    rf = l["l_returnflag"]
    assert set(np.unique(rf[receipt > 9298])) == {ord("N")}
    assert set(np.unique(rf[receipt <= 9298])) <= {ord("R"), ord("A")}
    assert set(np.unique(l["l_shipmode"])) == {0, 1, 2, 3}  # REG AIR encodes to 0, as the reference loader does
    assert set(np.unique(c["c_mktsegment"])) == {0, 1}


def test_generator_deterministic_and_seeded():
    a, b, c = T.generate(5, 1), T.generate(5, 1), T.generate(5, 2)
    for t in T.STRUCTS:
        for k in a.cols[t]:
            assert np.array_equal(a.cols[t][k], b.cols[t][k])
    assert not np.array_equal(a.cols["lineitem"]["l_shipdate"][:100], c.cols["lineitem"]["l_shipdate"][:100])


def test_binary_store_load_roundtrip(tb, tmp_path):
    T.store(str(tmp_path), 1, tb)
    assert (tmp_path / "scale001" / "lineitem.tbl.dir" / "size").read_text() == str(tb.n("lineitem"))
    for q, tables in T.QUERY_TABLES.items():
        got = T.load(str(tmp_path), q, 1)
        assert set(got.sizes) == set(tables)
        for t in tables:
            assert got.n(t) == tb.n(t)
            for k, v in got.cols[t].items():  # only the query's columns (TpcHCommons.cpp per-query loads)
                assert np.array_equal(v, tb.cols[t][k]), (q, t, k)
    q12 = T.load(str(tmp_path), 12, 1)
    assert set(q12.cols["lineitem"]) == {"l_orderkey", "l_shipdate", "l_commitdate", "l_receiptdate", "l_shipmode"}
    with pytest.raises(OSError):
        T.load(str(tmp_path), 3, 2)  # no scale002


def test_csv_loader_encodings(tmp_path):
    d = tmp_path / "scale001"
    d.mkdir()
    (d / "lineitem.tbl").write_text(
        "1|155190|7706|1|17|21168.23|0.04|0.02|N|O|1996-03-13|1996-02-12|1996-03-22|DELIVER IN PERSON|TRUCK|egular|\n"
        "1|67310|7311|2|36|45983.16|0.09|0.06|R|F|1994-04-12|1994-02-28|1994-04-20|TAKE BACK RETURN|MAIL|ly final|\n"
        "3|4297|1798|1|45|54058.05|0.06|0.00|A|F|1994-02-02|1994-01-04|1994-02-23|NONE|REG AIR|ongside|\n"
        "7|1|1|1|8|1.0|0.0|0.0|R|F|1970-01-02|1970-01-03|1970-01-04|DELIVER IN PERSON|AIR REG|x|\n")
    (d / "orders.tbl").write_text("1|36901|O|173665.47|1996-01-02|5-LOW|Clerk#1|0|nstructions|\n"
                                  "2|78002|O|46929.18|1996-12-01|1-URGENT|Clerk#2|0|foxes|\n")
    (d / "customer.tbl").write_text("1|Customer#1|addr|15|25-989|711.56|BUILDING|comment|\n"
                                    "2|Customer#2|addr|13|23-768|121.65|AUTOMOBILE|comment|\n")
    (d / "part.tbl").write_text("1|goldenrod|Manufacturer#1|Brand#13|PROMO BURNISHED COPPER|7|JUMBO PKG|901.00|ly|\n"
                                "2|blush|Manufacturer#1|Brand#23|LARGE BRUSHED BRASS|1|MED PACK|902.00|lar|\n")
    (d / "nation.tbl").write_text("0|ALGERIA|0|haggle|\n1|ARGENTINA|1|al foxes|\n")
    tb = T.load(str(tmp_path), 0, 1, csv=True)
    l = tb.cols["lineitem"]
    assert tb.n("lineitem") == 4
    assert list(l["l_orderkey"]["key"]) == [1, 1, 3, 7] and list(l["l_orderkey"]["payload"]) == [0, 1, 2, 3]
    assert list(l["l_shipmode"]) == [0, 1, 0, 4]  # TRUCK, MAIL, REG AIR (unmatched), "AIR REG"
    assert list(l["l_shipinstruct"]) == [1, 0, 0, 1]
    assert bytes(l["l_returnflag"]) == b"NRAR"
    assert list(l["l_partkey"]) == [155190, 67310, 4297, 1]
    assert list(l["l_quantity"]) == [17.0, 36.0, 45.0, 8.0]
    assert l["l_shipdate"][1] == 766108800  # 1994-04-12 00:00 UTC
    assert list(l["l_shipdate"][3:]) == [DAY] and list(l["l_receiptdate"][3:]) == [3 * DAY]
    o = tb.cols["orders"]
    assert list(o["o_custkey"]) == [36901, 78002] and o["o_orderdate"][0] == 820540800  # 1996-01-02
    c = tb.cols["customer"]
    assert list(c["c_mktsegment"]) == [1, 0] and list(c["c_nationkey"]) == [15, 13]
    p = tb.cols["part"]
    assert list(p["p_brand"]) == [0, 2] and list(p["p_container"]) == [0, 8] and list(p["p_size"]) == [7, 1]
    assert list(tb.cols["nation"]["n_nationkey"]["key"]) == [0, 1]


# ---- independent numpy formulation of each query (set arithmetic, no joins code shared)
TS = {"1995-03-15": 795225600, "1995-03-16": 795312000, "1993-10-01": 749433600, "1994-01-01": 757382400,
      "1995-01-01": 788918400}


def np_q3(tb):
    c, o, l = tb.cols["customer"], tb.cols["orders"], tb.cols["lineitem"]
    building = set(c["c_custkey"]["key"][c["c_mktsegment"] == 1].tolist())
    osel = o["o_orderdate"] < TS["1995-03-15"]
    okeys = o["o_orderkey"]["key"][osel][np.isin(o["o_custkey"][osel], list(building))]
    lsel = l["l_shipdate"] >= TS["1995-03-16"]
    return int(np.isin(l["l_orderkey"]["key"][lsel], okeys).sum())


def np_q10(tb):
    o, l = tb.cols["orders"], tb.cols["lineitem"]
    d = o["o_orderdate"]
    osel = (d >= TS["1993-10-01"]) & (d < TS["1994-01-01"])
    # every filtered order has a customer (custkeys exist) and every customer a nation: 1 row per order
    okeys = o["o_orderkey"]["key"][osel]
    return int(np.isin(l["l_orderkey"]["key"][l["l_returnflag"] == ord("R")], okeys).sum())


def np_q12(tb):
    l = tb.cols["lineitem"]
    m, s, cm, r = l["l_shipmode"], l["l_shipdate"], l["l_commitdate"], l["l_receiptdate"]
    sel = ((m == 1) | (m == 2)) & (cm < r) & (s < cm) & (r >= TS["1994-01-01"]) & (r < TS["1995-01-01"])
    return int(sel.sum())  # every lineitem's order exists exactly once


def np_q19(tb):
    l, p = tb.cols["lineitem"], tb.cols["part"]
    q, m, ins = l["l_quantity"], l["l_shipmode"], l["l_shipinstruct"]
    lsel = (q >= 1) & (q <= 30) & ((m == 3) | (m == 4)) & (ins == 1)
    pk = l["l_partkey"][lsel].astype(np.int64) - 1  # p_partkey = row + 1
    qq = q[lsel]
    b, k, sz = p["p_brand"][pk], p["p_container"][pk], p["p_size"][pk]
    p1 = (b == 1) & (k >= 1) & (k <= 4) & (sz >= 1) & (sz <= 5) & (qq >= 1) & (qq <= 11)
    p2 = (b == 2) & (k >= 5) & (k <= 8) & (sz >= 1) & (sz <= 10) & (qq >= 10) & (qq <= 20)
    p3 = (b == 3) & (k >= 9) & (k <= 12) & (sz >= 1) & (sz <= 15) & (qq >= 20) & (qq <= 30)
    return int((p1 | p2 | p3).sum())


@pytest.mark.parametrize("q,fn", [(3, np_q3), (10, np_q10), (12, np_q12), (19, np_q19)])
def test_oracle_queries_match_numpy(tb, q, fn):
    r = O.tpch_query(q, tb, nthreads=4)
    assert r["result"] == fn(tb)
    assert O.tpch_query(q, tb, nthreads=1, rht=True) == r


def test_oracle_filters_keep_input_order(tb):
    o = tb.cols["orders"]
    rows = O.tpch_filter(3, 2, tb)
    sel = o["o_orderdate"] < TS["1995-03-15"]
    assert np.array_equal(rows["key"], o["o_custkey"][sel])
    assert np.array_equal(rows["payload"], o["o_orderkey"]["key"][sel])
    rows = O.tpch_filter(19, 2, tb)
    l = tb.cols["lineitem"]
    assert np.array_equal(rows["key"], l["l_partkey"][
        (l["l_quantity"] >= 1) & (l["l_quantity"] <= 30) & np.isin(l["l_shipmode"], [3, 4]) & (l["l_shipinstruct"] == 1)])
