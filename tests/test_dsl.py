"""The DSL / SQL-dispatch mirror (hstream_amd/processing.py, sql.py).
CPU: interval refinement, key equality, window-key serdes.
GPU: the reference's SQL-level tests driven through the mirror."""
import numpy as np
import pytest

import pyoracle
from hstream_amd import abi, processing as P, sql
from hstream_amd.columnar import OpSpec


def test_interval_refinement_keeps_reference_quirks():
    # AST.hs:66-74: SECOND / MINUTE right, DAY = 60*24 seconds (sic)
    assert sql.refine_interval(10, "SECOND") == 10
    assert sql.refine_interval(10, "MINUTE") == 600
    assert sql.refine_interval(1, "DAY") == 1440
    assert sql.refine_interval(1, "WEEK") == 1440 * 7
    assert sql.refine_interval(1, "MONTH") == 1440 * 30
    assert sql.refine_interval(1, "YEAR") == 1440 * 365
    with pytest.raises(ValueError):
        sql.refine_interval(0, "SECOND")


def test_parse_refine_tumbling_10s_is_10000ms():
    # ParseRefineSpec.hs:55-56: TUMBLING (INTERVAL 10 SECOND) -> RTumblingWindow 10
    w = sql.RTumblingWindow(sql.refine_interval(10, "SECOND"))
    tw = P.mkTumblingWindow(sql.diff_time_to_ms(w.seconds))
    assert tw == P.TimeWindows(10000, 10000, 86400000)


def test_key_equality_follows_aeson_numbers():
    d = P.KeyDict()
    assert d.encode(1) == d.encode(1.0)
    assert d.encode("1") != d.encode(1)
    assert d.encode({"a": 1}) == d.encode({"a": 1.0})
    assert d.encode(True) != d.encode(1)


def test_window_key_serdes_round_trip():
    w = P.TimeWindow(45000, 105000)
    b = P.time_window_key_bytes(b'"k"', w)
    assert b[:16] == (45000).to_bytes(8, "big") + bytes(8)
    key, w2 = P.time_window_key_from_bytes(b, 60000)
    assert key == b'"k"' and w2 == w
    bs = P.time_window_key_bytes(b'"k"', P.TimeWindow(3, 9), session=True)
    assert P.time_window_key_from_bytes(bs, 0, session=True)[1] == P.TimeWindow(3, 9)


@pytest.fixture(scope="module")
def eng():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs the GPU")
    from hstream_amd.engine import Engine
    e = Engine(device=0, batch_capacity=1 << 16)
    yield e
    e.close()


def _rec(ts, **value):
    return {"timestamp": ts, "value": value}


@pytest.mark.gpu
def test_sql_session_sum_regression_394(eng):
    """RegressionSpec.hs:42-56: SUM(a) GROUP BY b, SESSION(10 MINUTE) -> 1,2,3,4."""
    t = sql.gen_group_by_node(eng, [("SUM", "a")], sql.RGroupBy("b", sql.RSessionWindow(sql.refine_interval(10, "MINUTE"))))
    _, rows = t.process([_rec(1000 + i, a=1, b=4) for i in range(4)])
    assert [v["SUM(a)"] for _, v in rows] == [1, 2, 3, 4]
    assert all(k.twkKey == 4 for k, _ in rows)


@pytest.mark.gpu
def test_sql_non_windowed_sum_runsql(eng):
    """RunSQLSpec.hs:66-83: SELECT SUM(a) AS result ... GROUP BY b -> 1, 3, 6, 4."""
    t = sql.gen_group_by_node(eng, [("SUM", "a", "result")], sql.RGroupBy("b"))
    _, rows = t.process([_rec(1, a=1, b=2), _rec(2, a=2, b=2), _rec(3, a=3, b=2), _rec(4, a=4, b=3)])
    assert [v["result"] for _, v in rows] == [1, 3, 6, 4]


@pytest.mark.gpu
def test_sql_raw_403_count_sum_passthrough(eng):
    """RegressionSpec.hs:58-74: SUM(a), a + 1 (host-evaluated), COUNT(*) AS result, b."""
    t = sql.gen_group_by_node(eng, [("SUM", "a"), ("COL", "a+1"), ("COUNT(*)", "result"), ("COL", "b")],
                              sql.RGroupBy("b"))
    _, rows = t.process([_rec(10 + i, **{"a": 1, "a+1": 2, "b": 4}) for i in range(4)])
    assert [(v["result"], v["a+1"], v["b"], v["SUM(a)"]) for _, v in rows] == [(i, 2, 4, i) for i in range(1, 5)]


@pytest.mark.gpu
def test_dsl_hopping_count_like_stream_example2(eng):
    """StreamExample2.hs:100-108: groupBy . timeWindowedBy (mkHoppingWindow 3000 1000) . count."""
    rng = np.random.default_rng(3)
    recs = [_rec(int(1000 * i + rng.integers(0, 900)), key=["a", "b", "c"][int(rng.integers(0, 3))])
            for i in range(200)]
    t = P.groupBy(eng, "key").timeWindowedBy(P.mkHoppingWindow(3000, 1000)).count(P.Materialized())
    _, rows = t.process(recs)
    # the oracle on the same columns
    keys, ts, cols, valid = t.columns(recs)
    o = pyoracle.OracleOp(OpSpec(abi.HSG_HOPPING, abi.HSG_EMIT_PER_RECORD, size_ms=3000, advance_ms=1000,
                                 aggs=[(abi.HSG_COUNT_ALL, 0)]))
    o.push(keys, ts, [], None)
    exp = o.drain()
    assert len(rows) == len(exp)
    for (k, v), i in zip(rows, range(len(exp))):
        assert t.mat.keys.encode(k.twkKey) == exp.key_id[i]
        assert (k.twkWindow.tWindowStart, k.twkWindow.tWindowEnd) == (exp.win_start[i], exp.win_end[i])
        assert v["count"] == exp.aggs[0][i]


@pytest.mark.gpu
def test_type_error_record_only_moves_stream_time(eng):
    """SUM over a non-number throws before any window is updated (Codegen.hs:430-431);
    the record still advanced stream time (Processor.hs:139)."""
    t = P.groupBy(eng, "k").timeWindowedBy(P.mkTumblingWindow(1000)).aggregate([P.SUM("v")], P.Materialized())
    wm, rows = t.process([_rec(5, k=1, v=2), _rec(900_000_000, k=1, v="x"), _rec(7, k=1, v=3)])
    assert wm == 900_000_000
    # the third record's window [0, 1000) is > 24 h behind stream time: skipped
    assert [v["SUM(v)"] for _, v in rows] == [2]


@pytest.mark.gpu
@pytest.mark.parametrize("window", ["tumbling", "session"])
def test_json_poll_batch_through_native_ingest(eng, window):
    """A poll batch of raw JSON values (SourceRecord srcValue) decoded by the
    native ingest straight into the GPU op: the changelog equals the same
    records run through the Python columnariser into the CPU oracle
    (pyoracle, the checker); the keys come back as the values the records
    spelled (1 and 1.0 are one key)."""
    import json
    from hstream_amd import ingest
    rng = np.random.default_rng(17)
    vals, recs = [], []
    for i in range(3000):
        k = [1, 1.0, "a", "b", 7, {"x": 1}][int(rng.integers(0, 6))]
        v = {"k": k, "v": int(rng.integers(-1000, 1000)), "pad": "z" * int(rng.integers(0, 20))}
        if rng.random() < 0.05:
            v["v"] = "oops"           # SUM over a string: the record only moves stream time
        if rng.random() < 0.05:
            del v["k"]                # no GROUP BY field
        ts = 10_000 + 37 * i + int(rng.integers(0, 500))
        vals.append(json.dumps(v).encode())
        recs.append(_rec(ts, **v))
    ts = np.array([r["timestamp"] for r in recs], np.int64)
    buf, off = ingest.pack_records(vals)

    class OracleEngine:  # the Table's operator factory, on the CPU restatement
        def op(self, spec):
            return pyoracle.OracleOp(spec)

    def table(keys, engine):
        g = P.groupBy(engine, "k")
        w = g.timeWindowedBy(P.mkTumblingWindow(2000)) if window == "tumbling" else \
            g.sessionWindowedBy(P.mkSessionWindows(300))
        return w.aggregate([P.COUNT_ALL("n"), P.SUM("v", "s"), P.MAX("v", "m")], P.Materialized(keys=keys))

    tn = table(ingest.KeyDict(), eng)
    wm_n, rows_n = tn.process_json(buf, off, ts, threads=4)
    tp = table(P.KeyDict(), OracleEngine())
    wm_p, rows_p = tp.process(recs)
    assert wm_n == wm_p == int(ts.max())
    assert len(rows_n) == len(rows_p)
    for (kn, vn), (kp, vp) in zip(rows_n, rows_p):
        assert kn.twkWindow == kp.twkWindow and vn == vp
        assert P._canon(kn.twkKey) == P._canon(kp.twkKey)
    tn.close()
    tp.close()
