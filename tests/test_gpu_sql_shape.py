"""GPU: the SQL drop-in's op shape on the fast pipelines, at a BASELINE
config's size.

Every windowed GROUP BY that hstream-sql's genGroupByNode dispatches
(Codegen.hs:479-521) carries Scientific literals to an objectSerde sink
(Boilerplate.hs:32-37): its MIN / MAX fold with `min n x` / `max n x`
(Codegen.hs:436-461), its SUM prints as an integer only when every literal
that reached it was integral, and every non-aggregate SELECT column is a
passthrough holding the group's last record's value (Codegen.hs:463-469). In
this engine that is an op with HSG_OPF_LITERAL_FORMS and an HSG_LAST output.
Here C2's query in that shape -- `SELECT v, COUNT(*), SUM(v), AVG(v), MIN(v),
MAX(v) ... GROUP BY key, TUMBLING (60 s)` -- runs over >= 1M records per
batch sequence with many ties (a narrow value range) and decimal literals,
in both emit modes:

  * values, windows, keys, row order: the oracle (oracle/hsoracle.cpp, the
    reference's fold restated), bit-exact for integers, f64 within F64_RTOL;
  * literal forms (hsg_rows.form, 2 bits per output): a vectorised
    restatement of the reference's sequential fold below -- a SUM is
    integral iff no decimal literal reached it, a MIN keeps the earliest
    literal among equal minima, a MAX the latest among equal maxima, a
    passthrough its last present record's literal, an aggregate no present
    record reached its initial value;
  * the path: per batch, every batch on the SQL lean kernels (k_agg_sql /
    k_sql_apply: hsg_stats lean_batches, no replay onto the record kernels);
    EMIT CHANGES, the partitioned per-record pipeline (k_pr_bucket).
"""
import numpy as np
import pytest

from hstream_amd import abi
from hstream_amd.columnar import OpSpec
from util import F64_RTOL, rows_equal

pytestmark = pytest.mark.gpu

TS0 = 1_700_000_000_000
# SELECT v, COUNT(*), SUM(v), AVG(v), MIN(v), MAX(v): the passthrough first
AGGS = [(abi.HSG_LAST, 0), (abi.HSG_COUNT_ALL, 0), (abi.HSG_SUM, 0), (abi.HSG_AVG, 0), (abi.HSG_MIN, 0),
        (abi.HSG_MAX, 0)]
FORM = {abi.HSG_LAST: "last", abi.HSG_SUM: "sum", abi.HSG_MIN: "min", abi.HSG_MAX: "max"}


def _gen(seed, n, start, total, nkeys, f64, absent=0.03, dec=0.3, vr=40):
    rng = np.random.default_rng([seed, start])
    key = rng.integers(0, nkeys, size=n).astype(np.uint32)
    i = np.arange(start, start + n, dtype=np.int64)
    ts = TS0 + (i * 600_000) // total + rng.integers(0, 2000, size=n)  # 10 minutes: 10 windows
    if f64:
        v = rng.integers(-vr, vr + 1, size=n).astype(np.float64) / 4.0
    else:
        v = rng.integers(-vr, vr + 1, size=n).astype(np.int64)
    present = rng.random(n) >= absent
    decimal = present & (rng.random(n) < dec)
    valid = (present.astype(np.uint8) | (decimal.astype(np.uint8) << 1)).astype(np.uint8)
    return key, ts.astype(np.int64), v, valid


def _prefix_forms(gid, v, valid, f64, aggs=AGGS):
    """Literal-form word (hsg_rows.form) of each record's group right after
    the record, in arrival order: the reference's sequential fold."""
    import pandas as pd
    n = len(gid)
    present = (valid & 1) != 0
    dec = (valid & 2) != 0
    idx = np.arange(n)
    hi, lo = (np.inf, -np.inf) if f64 else (np.iinfo(np.int64).max, np.iinfo(np.int64).min)
    df = pd.DataFrame({"g": gid, "i": idx, "p": present, "d": dec & present,
                       "vmin": np.where(present, v, hi), "vmax": np.where(present, v, lo)})
    df = df.sort_values(["g", "i"], kind="stable")
    gb = df.groupby("g", sort=False)
    sum_dec = gb["d"].cumsum().to_numpy()
    run_min = gb["vmin"].cummin()
    prev_min = run_min.groupby(df["g"]).shift(1).fillna(hi).to_numpy()
    run_max = gb["vmax"].cummax()
    prev_max = run_max.groupby(df["g"]).shift(1).fillna(lo).to_numpy()
    p = df["p"].to_numpy()
    i_s = df["i"].to_numpy()
    new_min = p & (df["vmin"].to_numpy() < prev_min)   # min n x = n: a tie keeps the earlier literal
    new_max = p & (df["vmax"].to_numpy() >= prev_max)  # max n x = x: a tie takes the later one
    tmp = pd.DataFrame({"g": df["g"].to_numpy(), "a": np.where(new_min, i_s, -1), "b": np.where(new_max, i_s, -1),
                        "c": np.where(p, i_s, -1)})
    g2 = tmp.groupby("g", sort=False)
    tmin = g2["a"].cummax().to_numpy()
    tmax = g2["b"].cummax().to_numpy()
    tlast = g2["c"].cummax().to_numpy()
    integral = ~dec

    def bits(t):  # the winning literal's "prints as an integer" bit; 3 = the initial value
        return np.where(t < 0, 3, integral[np.maximum(t, 0)].astype(np.int64))

    per = {"sum": (sum_dec == 0).astype(np.int64), "min": bits(tmin), "max": bits(tmax), "last": bits(tlast)}
    word = np.zeros(n, np.int64)
    for j, (k, _c) in enumerate(aggs):
        if k in FORM:
            word |= per[FORM[k]] << (2 * j)
    out = np.empty(n, np.uint32)
    out[i_s] = word.astype(np.uint32)
    return out


@pytest.mark.parametrize("f64", [False, True], ids=["i64", "f64"])
@pytest.mark.parametrize("emit", [abi.HSG_EMIT_PER_BATCH, abi.HSG_EMIT_PER_RECORD], ids=["per_batch", "changes"])
def test_sql_shape_c2_reduced(emit, f64):
    import pyoracle
    from hstream_amd.engine import Engine
    nb, per = 3, 700_000  # 2.1M records
    total = nb * per
    nkeys = 8192
    ct = abi.HSG_F64 if f64 else abi.HSG_I64
    spec = OpSpec(abi.HSG_TUMBLING, emit, size_ms=60_000, col_types=[ct], aggs=AGGS, flags=abi.HSG_OPF_LITERAL_FORMS)
    batches = [_gen(7 + f64, per, b * per, total, nkeys, f64) for b in range(nb)]
    key = np.concatenate([b[0] for b in batches])
    ts = np.concatenate([b[1] for b in batches])
    v = np.concatenate([b[2] for b in batches])
    valid = np.concatenate([b[3] for b in batches])
    gid = key.astype(np.int64) * 1_000_000 + (ts // 60_000 - TS0 // 60_000)
    fw = _prefix_forms(gid, v, valid, f64)
    eng = Engine(device=0, batch_capacity=1 << 20)
    g = eng.op(spec)
    o = pyoracle.OracleOp(spec)
    f64s = spec.agg_is_f64()
    wg = wo = -1
    for bi, (k, t, c, va) in enumerate(batches):
        wg = g.push(k, t, [c], [va], watermark=wg)
        wo = o.push(k, t, [c], [va], watermark=wo)
        assert wg == wo
        a, b = g.drain(), o.drain()
        base = bi * per
        if emit == abi.HSG_EMIT_PER_RECORD:
            rows_equal(a, b, f64s, ordered=True, what=f"batch {bi}")
            assert len(a) == per
            np.testing.assert_array_equal(a.form, fw[a.src_index], err_msg=f"batch {bi}: forms")
        else:
            rows_equal(a, b, f64s, what=f"batch {bi}")
            # a touched group's row: its state after its last record of the batch
            hi = base + per
            sel = np.arange(base, hi)
            lastrec = {}
            for i, gg in zip(sel, gid[base:hi]):
                lastrec[gg] = i
            a = a.sorted()
            want = np.array([fw[lastrec[int(kk) * 1_000_000 + (int(ws) // 60_000 - TS0 // 60_000)]]
                             for kk, ws in zip(a.key_id, a.win_start)], np.uint32)
            np.testing.assert_array_equal(a.form, want, err_msg=f"batch {bi}: forms")
    rows_equal(g.dump_state(), o.dump_state(), f64s, what="state")
    st = g.stats()
    if emit == abi.HSG_EMIT_PER_BATCH:
        # every batch on the SQL lean kernels, none run again on the record kernels
        assert st["lean_batches"] == nb and st["replays"] == 0, st
    g.close()
    eng.close()


# BASELINE C5's query in the SQL shape, `SELECT v, SUM(v), MAX(v)` (a baked
# slot program of its own in k_agg_sql)
AGGS_C5 = [(abi.HSG_LAST, 0), (abi.HSG_SUM, 0), (abi.HSG_MAX, 0)]


@pytest.mark.parametrize("query", ["c2", "c5"])
@pytest.mark.parametrize("f64", [False, True], ids=["i64", "f64"])
def test_sql_shape_hot_keys_and_full_tables(f64, query):
    """The SQL shape on skewed keys (BASELINE C5's shape, reduced): a hot key
    whose bucket is split over several aggregation workgroups, and buckets
    with more groups than a chunk's LDS table holds (each such record a
    partial of its own). Both meet in k_sql_apply under the rows' locks, in
    any order; the changelog then comes from the touched list. Every batch
    stays on the SQL lean kernels; values, forms and ties match the oracle
    and the reference's sequential fold. Both the C2 query and C5's."""
    import pyoracle
    from hstream_amd.engine import Engine
    nb, per = 2, 1_500_000
    total = nb * per
    ct = abi.HSG_F64 if f64 else abi.HSG_I64
    aggs = AGGS if query == "c2" else AGGS_C5
    spec = OpSpec(abi.HSG_TUMBLING, abi.HSG_EMIT_PER_BATCH, size_ms=60_000, col_types=[ct], aggs=aggs,
                  flags=abi.HSG_OPF_LITERAL_FORMS)
    rng = np.random.default_rng(11 + f64)
    batches = []
    for b in range(nb):
        _k, t, c, va = _gen(21 + f64, per, b * per, total, 4096, f64)
        z = rng.zipf(1.2, size=per)
        key = np.where(z <= 400_000, z, rng.integers(1, 400_000, size=per)).astype(np.uint32)
        batches.append((key, t, c, va))
    key = np.concatenate([b[0] for b in batches])
    ts = np.concatenate([b[1] for b in batches])
    v = np.concatenate([b[2] for b in batches])
    valid = np.concatenate([b[3] for b in batches])
    gid = key.astype(np.int64) * 1_000_000 + (ts // 60_000 - TS0 // 60_000)
    fw = _prefix_forms(gid, v, valid, f64, aggs)
    eng = Engine(device=0, batch_capacity=per)
    g = eng.op(spec)
    o = pyoracle.OracleOp(spec)
    f64s = spec.agg_is_f64()
    wg = wo = -1
    for bi, (k, t, c, va) in enumerate(batches):
        wg = g.push(k, t, [c], [va], watermark=wg)
        wo = o.push(k, t, [c], [va], watermark=wo)
        assert wg == wo
        a, b = g.drain(), o.drain()
        rows_equal(a, b, f64s, what=f"batch {bi}")
        base = bi * per
        gg = gid[base:base + per]
        # the state after a group's last record of the batch: its last index
        order = np.argsort(gg, kind="stable")
        last_of = {}
        sg = gg[order]
        ends = np.r_[np.nonzero(sg[1:] != sg[:-1])[0], len(sg) - 1]
        for e in ends:
            last_of[int(sg[e])] = base + int(order[e])
        a = a.sorted()
        want = np.array([fw[last_of[int(kk) * 1_000_000 + (int(ws) // 60_000 - TS0 // 60_000)]]
                         for kk, ws in zip(a.key_id, a.win_start)], np.uint32)
        np.testing.assert_array_equal(a.form, want, err_msg=f"batch {bi}: forms")
    rows_equal(g.dump_state(), o.dump_state(), f64s, what="state")
    st = g.stats()
    assert st["lean_batches"] == nb, st
    g.close()
    eng.close()


@pytest.mark.parametrize("shape", ["sql", "sql_c5", "plain"])
def test_per_record_hot_key_chunked(shape):
    """EMIT CHANGES of a one-window op with a hot key (its partition bucket far
    over kPrHot records): the batch takes the chunked path (chunks of the
    bucket in parallel, carries in order) instead of one workgroup walking
    the bucket. Every row, in arrival order, against the oracle; forms of
    the SQL shape against the reference's sequential fold."""
    import pyoracle
    from hstream_amd.engine import Engine
    nb, per = 2, 1_000_000
    total = nb * per
    aggs = {"sql": AGGS, "sql_c5": AGGS_C5}.get(shape, [(abi.HSG_COUNT_ALL, 0), (abi.HSG_SUM, 0), (abi.HSG_MAX, 0)])
    flags = abi.HSG_OPF_LITERAL_FORMS if shape != "plain" else 0
    spec = OpSpec(abi.HSG_TUMBLING, abi.HSG_EMIT_PER_RECORD, size_ms=60_000, col_types=[abi.HSG_I64], aggs=aggs,
                  flags=flags)
    rng = np.random.default_rng(31)
    batches = []
    for b in range(nb):
        _k, t, c, va = _gen(41, per, b * per, total, 4096, False)
        z = rng.zipf(1.2, size=per)
        key = np.where(z <= 200_000, z, rng.integers(1, 200_000, size=per)).astype(np.uint32)
        batches.append((key, t, c, va))
    eng = Engine(device=0, batch_capacity=per)
    g = eng.op(spec)
    o = pyoracle.OracleOp(spec)
    f64s = spec.agg_is_f64()
    fw = None
    if shape != "plain":
        key = np.concatenate([b[0] for b in batches])
        ts = np.concatenate([b[1] for b in batches])
        gid = key.astype(np.int64) * 1_000_000 + (ts // 60_000 - TS0 // 60_000)
        fw = _prefix_forms(gid, np.concatenate([b[2] for b in batches]), np.concatenate([b[3] for b in batches]),
                           False, aggs)
    wg = wo = -1
    for bi, (k, t, c, va) in enumerate(batches):
        wg = g.push(k, t, [c], [va], watermark=wg)
        wo = o.push(k, t, [c], [va], watermark=wo)
        assert wg == wo
        a, b = g.drain(), o.drain()
        rows_equal(a, b, f64s, ordered=True, what=f"batch {bi}")
        if fw is not None:
            np.testing.assert_array_equal(a.form, fw[a.src_index], err_msg=f"batch {bi}: forms")
    rows_equal(g.dump_state(), o.dump_state(), f64s, what="state")
    g.close()
    eng.close()
