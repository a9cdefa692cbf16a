"""Stream-stream join (include/hstream_join.h) against the oracle
(oracle/joinref.py, a record-by-record restatement of joinStreamProcessor,
Stream.hs:267-300, over InMemoryTimestampedKVStore, Store.hs:316-385).

CPU: hand-derived vectors pin the oracle (window bounds, the end-point quirk
of tksRange, overwrite of an equal (key, ts), the missing-join-field abort).
GPU: batches of interleaved records compared row for row, in order.
The reference's one join vector (RegressionSpec.hs:24-40, #391_JOIN: join ->
unwindowed GROUP BY) runs through the oracle on CPU and the GPU join + GPU
op on the GPU.
"""
import numpy as np
import pytest

import joinref
import pyoracle
from joinref import NONE
from util import load_kat, run_join_kat

JOIN_KAT = load_kat()["joins"]


def _jarrays(b):
    return (np.asarray(b["side"], np.uint8), np.asarray(b["key_id"], np.uint32),
            np.asarray(b["join_key"], np.uint32), np.asarray(b["ts"], np.int64), np.asarray(b["handle"], np.uint64))


@pytest.mark.parametrize("case", JOIN_KAT, ids=lambda c: c["name"])
def test_reference_join_kat_oracle(case):
    ref = joinref.JoinRef(case["join"]["before_ms"], case["join"]["after_ms"])
    run_join_kat(case, lambda b: ref.push(*_jarrays(b)), lambda spec: pyoracle.OracleOp(spec))


@pytest.mark.gpu
@pytest.mark.parametrize("case", JOIN_KAT, ids=lambda c: c["name"])
def test_reference_join_kat_gpu(case):
    import torch
    assert torch.cuda.is_available()
    from hstream_amd.engine import Engine
    from hstream_amd.join import Join
    eng = Engine(device=0, batch_capacity=1 << 10)
    j = Join(eng, case["join"]["before_ms"], case["join"]["after_ms"], batch_capacity=1 << 10)

    def push(b):
        j.push(*_jarrays(b))
        return list(zip(*[x.tolist() for x in j.drain()]))

    run_join_kat(case, push, lambda spec: eng.op(spec))
    j.close()
    eng.close()


def _run(ref, recs):
    rows = []
    for side, key, jk, ts, h in recs:
        rows += ref.push_one(side, key, jk, ts, h)
    return rows


def test_window_and_orientation():
    # before 10, after 5: a this-record at t matches other-records in [t-10, t+5]
    r = joinref.JoinRef(10, 5)
    rows = _run(r, [(1, 7, 1, 100, 1), (1, 7, 1, 94, 2), (1, 7, 1, 106, 3), (0, 7, 1, 100, 4)])
    # endpoints 90 / 105 are not held by the other store: open interval (90, 105)
    assert rows == [(4, 2, 1, 100), (4, 1, 1, 100)]
    # an other-record at 112 matches this-records in [112-5, 112+10] = [107, 122]: none
    assert r.push_one(1, 7, 1, 112, 5) == []


def test_endpoints_need_both_ends_present():
    r = joinref.JoinRef(10, 10)
    # other store holds ts 90 and 110 (different keys fill them)
    _run(r, [(1, 7, 1, 90, 1), (1, 8, 1, 110, 2), (1, 7, 1, 95, 3)])
    # both end timestamps 90 and 110 present: inclusive -> key 7 at 90 and 95
    assert r.push_one(0, 7, 1, 100, 9) == [(9, 1, 1, 100), (9, 3, 1, 100)]
    r2 = joinref.JoinRef(10, 10)
    _run(r2, [(1, 7, 1, 90, 1), (1, 7, 1, 95, 3)])
    # only 90 present: exclusive -> 90 drops out
    assert r2.push_one(0, 7, 1, 100, 9) == [(9, 3, 1, 100)]
    # zero-width window never matches (splitLookup of the same point twice)
    r3 = joinref.JoinRef(0, 0)
    _run(r3, [(1, 7, 1, 100, 1)])
    assert r3.push_one(0, 7, 1, 100, 2) == []


def test_overwrite_and_missing_join_key():
    r = joinref.JoinRef(10, 10)
    _run(r, [(1, 7, 1, 100, 1), (1, 7, 2, 100, 2)])  # same (key, ts): the second replaces the first
    assert r.push_one(0, 7, 1, 101, 3) == []
    assert r.push_one(0, 7, 2, 101, 4) == [(4, 2, 2, 101)]
    r2 = joinref.JoinRef(10, 10)
    _run(r2, [(1, 7, 1, 95, 1), (1, 7, NONE, 97, 2), (1, 7, 1, 99, 3)])
    # ascending candidates: 95 joins, 97 has no join field -> the scan stops
    assert r2.push_one(0, 7, 1, 100, 9) == [(9, 1, 1, 100)]
    assert r2.push_one(0, 7, NONE, 100, 10) == []


def _gen(seed, n, nkeys=40, grid=5, span=40_000, none_frac=0.03):
    rng = np.random.default_rng(seed)
    side = (rng.random(n) < 0.5).astype(np.uint8)
    key = rng.integers(0, nkeys, n).astype(np.uint32)
    key[rng.random(n) < 0.01] = NONE
    jk = rng.integers(0, 3, n).astype(np.uint32)
    jk[rng.random(n) < none_frac] = NONE
    # near-sorted timestamps on a coarse grid: many equal timestamps and window end points
    ts = ((np.arange(n) * span) // n + rng.integers(0, 400, n)) // grid * grid
    ts = ts.astype(np.int64) + 1_700_000_000_000
    handle = np.arange(n, dtype=np.uint64) + (seed << 32)
    return side, key, jk, ts, handle


@pytest.mark.gpu
@pytest.mark.parametrize("before,after,grid", [(100, 50, 5), (30, 30, 10), (0, 0, 1), (250, 0, 25)])
def test_join_matches_oracle(before, after, grid):
    import torch
    assert torch.cuda.is_available()
    from hstream_amd.engine import Engine
    from hstream_amd.join import Join
    eng = Engine(device=0, batch_capacity=1 << 16)
    j = Join(eng, before, after, batch_capacity=1 << 14)
    ref = joinref.JoinRef(before, after)
    side, key, jk, ts, h = _gen(before * 7 + after + grid, 30_000, grid=grid)
    total = 0
    for s0 in range(0, len(ts), 7_000):
        sl = slice(s0, s0 + 7_000)
        j.push(side[sl], key[sl], jk[sl], ts[sl], h[sl])
        exp = ref.push(side[sl], key[sl], jk[sl], ts[sl], h[sl])
        th, oh, k, t = j.drain()
        got = list(zip(th.tolist(), oh.tolist(), k.tolist(), t.tolist()))
        assert got == exp, f"batch at {s0}: {len(got)} rows vs {len(exp)}"
        total += len(exp)
    assert j.state_rows() == ref.state_rows()
    assert total > 0 or (before == 0 and after == 0)
    j.close()
    eng.close()
