"""Shared test helpers: seeded small inputs, row comparison, KAT runner."""
import json
import math
import os

import numpy as np

from hstream_amd import abi
from hstream_amd.columnar import OpSpec, Rows

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
F64_RTOL = 1e-6  # north_star: floating-point SUM/AVG within 1e-6 relative


def load_kat():
    with open(os.path.join(GOLDEN, "reference_kat.json")) as f:
        return json.load(f)


def spec_from_json(d):
    return OpSpec(window_kind=d["window_kind"], emit_mode=d["emit_mode"], size_ms=d.get("size_ms", 0),
                  advance_ms=d.get("advance_ms", 0), gap_ms=d.get("gap_ms", 0),
                  grace_ms=d.get("grace_ms", abi.HSG_DEFAULT_GRACE_MS),
                  col_types=d.get("col_types", []), aggs=[tuple(a) for a in d["aggs"]],
                  state_capacity=d.get("state_capacity", 0), out_capacity=d.get("out_capacity", 0))


def batch_arrays(b, col_types):
    key = np.asarray(b["key_id"], dtype=np.uint32)
    ts = np.asarray(b["ts"], dtype=np.int64)
    cols = [np.asarray(c, dtype=np.float64 if t == abi.HSG_F64 else np.int64) for c, t in zip(b["cols"], col_types)]
    valid = None
    if b.get("valid") is not None:
        valid = [None if v is None else np.asarray(v, dtype=np.uint8) for v in b["valid"]]
    return key, ts, cols, valid


def gen_small(seed, n, nkeys, col_types=(abi.HSG_I64,), late_frac=0.02, neg_frac=0.01, none_frac=0.02,
              absent_frac=0.05, span=200_000, base=1_000_000, very_late=True):
    """Seeded messy batch: near-sorted ts with jitter, some records far in the
    past (late by more than grace), negative ts, HSG_KEY_NONE records and
    absent fields."""
    rng = np.random.default_rng(seed)
    key = rng.integers(0, nkeys, size=n).astype(np.uint32)
    ts = base + (np.arange(n) * span) // max(1, n) + rng.integers(0, 3000, size=n)
    if very_late:
        late = rng.random(n) < late_frac
        ts = np.where(late, ts - abi.HSG_DEFAULT_GRACE_MS - rng.integers(0, 200_000, size=n), ts)
    neg = rng.random(n) < neg_frac
    ts = np.where(neg, -rng.integers(1, 50_000, size=n), ts).astype(np.int64)
    none = rng.random(n) < none_frac
    key = np.where(none, np.uint32(abi.HSG_KEY_NONE), key).astype(np.uint32)
    cols, valid = [], []
    for t in col_types:
        if t == abi.HSG_F64:
            cols.append(np.round(rng.uniform(-1e6, 1e6, size=n), 3))
        else:
            cols.append(rng.integers(-10**9, 10**9, size=n, dtype=np.int64))
        valid.append((rng.random(n) >= absent_frac).astype(np.uint8))
    return key, ts, cols, valid


def rows_equal(a: Rows, b: Rows, agg_f64, ordered=False, what=""):
    """Bit-exact keys/windows/integer aggregates; f64 within F64_RTOL."""
    if not ordered:
        a, b = a.sorted(), b.sorted()
    assert len(a) == len(b), f"{what}: row count {len(a)} != {len(b)}"
    np.testing.assert_array_equal(a.key_id, b.key_id, err_msg=f"{what}: key_id")
    np.testing.assert_array_equal(a.win_start, b.win_start, err_msg=f"{what}: win_start")
    np.testing.assert_array_equal(a.win_end, b.win_end, err_msg=f"{what}: win_end")
    if ordered:
        np.testing.assert_array_equal(a.src_index, b.src_index, err_msg=f"{what}: src_index")
    for j, f in enumerate(agg_f64):
        x, y = a.aggs[j], b.aggs[j]
        if f:
            np.testing.assert_allclose(x, y, rtol=F64_RTOL, atol=0, equal_nan=True, err_msg=f"{what}: agg {j}")
        else:
            np.testing.assert_array_equal(x, y, err_msg=f"{what}: agg {j}")


def run_kat_case(case, make_op):
    """Run one reference KAT through an op factory; returns nothing, asserts."""
    spec = spec_from_json(case["op"])
    op = make_op(spec)
    batches = case.get("batches") or [dict(case["batch"])]
    wm = -1
    changelog = []
    for b in batches:
        key, ts, cols, valid = batch_arrays(b, spec.col_types)
        wm = op.push(key, ts, cols, valid, watermark=wm)
        rows = op.drain() if spec.emit_mode != abi.HSG_EMIT_NONE else None
        if rows is not None:
            changelog.extend(rows.tuples())
        exp_state = b.get("expect_state")
        if exp_state is not None:
            st = op.dump_state().tuples()
            got = [[k, list(v)] for k, _, _, v in st]
            assert got == exp_state, f"{case['name']}: state {got} != {exp_state}"
    if "expect_changelog_aggs" in case:
        got = [list(v) for _, _, _, v in changelog]
        assert got == case["expect_changelog_aggs"], f"{case['name']}: {got}"
    if "expect_changelog" in case:
        got = [[k, s, e, list(v)] for k, s, e, v in changelog]
        assert got == case["expect_changelog"], f"{case['name']}: {got}"
    if "expect_state" in case:
        st = op.dump_state().tuples()
        got = [[k, list(v)] for k, _, _, v in st]
        assert got == case["expect_state"], f"{case['name']}: state {got}"
    op.close() if hasattr(op, "close") else None


ALL_AGG_SETS = {
    "count": [(abi.HSG_COUNT_ALL, 0)],
    "full_i64": [(abi.HSG_COUNT_ALL, 0), (abi.HSG_COUNT, 0), (abi.HSG_SUM, 0), (abi.HSG_MIN, 0), (abi.HSG_MAX, 0),
                 (abi.HSG_AVG, 0), (abi.HSG_LAST, 0)],
    "mixed": [(abi.HSG_COUNT_ALL, 0), (abi.HSG_SUM, 0), (abi.HSG_SUM, 1), (abi.HSG_MIN, 1), (abi.HSG_MAX, 1),
              (abi.HSG_AVG, 1), (abi.HSG_MAX, 0), (abi.HSG_COUNT, 1), (abi.HSG_LAST, 1)],
}


def run_join_kat(case, push_join, make_op):
    """A reference join vector: the join (push_join(batch) -> rows (this handle,
    other handle, join key, ts) of that batch, in order), then its rows through
    the GROUP BY op built from case["op"], as genStreamBuilderWithStream chains
    them (Codegen.hs:532-559). Asserts the join rows and the changelog."""
    rows = []
    for b in case["join"]["batches"]:
        rows += [tuple(int(x) for x in r) for r in push_join(b)]
    assert [list(r) for r in rows] == case["expect_join_rows"], f"{case['name']}: join rows {rows}"
    vals = case["values"]
    pick = lambda r, side, field: vals[str(r[0] if side == "this" else r[1])][field]
    gside, gfield = case["group_by"]
    dict_ids = {}
    key = np.asarray([dict_ids.setdefault(pick(r, gside, gfield), len(dict_ids)) for r in rows], dtype=np.uint32)
    ts = np.asarray([r[3] for r in rows], dtype=np.int64)
    cols = [np.asarray([pick(r, s, f) for r in rows], dtype=np.int64) for s, f in case["columns"]]
    spec = spec_from_json(case["op"])
    op = make_op(spec)
    op.push(key, ts, cols, None, watermark=-1)
    got = [list(v) for _, _, _, v in op.drain().tuples()]
    assert got == case["expect_changelog_aggs"], f"{case['name']}: {got}"
    op.close() if hasattr(op, "close") else None
