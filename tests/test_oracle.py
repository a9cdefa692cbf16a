"""CPU: the oracle against the reference's own test vectors, and the C++
restatement against the independent pure-Python one on seeded inputs."""
import numpy as np
import pytest

import pyoracle
import pyref
from hstream_amd import abi
from hstream_amd.columnar import OpSpec, Rows
from util import ALL_AGG_SETS, gen_small, load_kat, run_kat_case

KAT = load_kat()


@pytest.mark.parametrize("w", KAT["windows_for"], ids=lambda w: f"ts{w['ts']}_s{w['size']}_a{w['adv']}")
def test_windows_for_kat(w):
    got = pyoracle.windows_for(w["ts"], w["size"], w["adv"])
    assert [s for s, _ in got] == w["starts"]
    assert all(e == s + w["size"] for s, e in got)
    assert [s for s, _ in pyref.windows_for(w["ts"], w["size"], w["adv"])] == w["starts"]


@pytest.mark.parametrize("case", KAT["cases"], ids=lambda c: c["name"])
def test_reference_kat_oracle(case):
    run_kat_case(case, lambda spec: pyoracle.OracleOp(spec))


@pytest.mark.parametrize("case", KAT["cases"], ids=lambda c: c["name"])
def test_reference_kat_pyref(case):
    run_kat_case(case, lambda spec: _PyRefAdapter(spec))


class _PyRefAdapter:
    def __init__(self, spec):
        self.r = pyref.PyRefOp(spec)
        self.spec = spec

    def push(self, key, ts, cols, valid, watermark):
        return self.r.push(key, ts, cols, valid, watermark)

    def drain(self):
        return _rows(self.r.drain(), len(self.spec.aggs))

    def dump_state(self):
        return _rows(self.r.dump_state(), len(self.spec.aggs))


def _rows(tups, naggs):
    n = len(tups)
    return Rows(np.array([t[0] for t in tups], dtype=np.uint32), np.array([t[1] for t in tups], dtype=np.int64),
                np.array([t[2] for t in tups], dtype=np.int64), np.array([t[3] for t in tups], dtype=np.int64),
                [np.array([t[4][j] for t in tups]) for j in range(naggs)] if n else [np.array([]) for _ in range(naggs)])


def _specs():
    out = []
    for aggname, col_types in (("count", []), ("full_i64", [abi.HSG_I64]), ("mixed", [abi.HSG_I64, abi.HSG_F64])):
        aggs = ALL_AGG_SETS[aggname]
        for kind, kw in ((abi.HSG_TUMBLING, dict(size_ms=10_000)),
                         (abi.HSG_HOPPING, dict(size_ms=10_000, advance_ms=3_000)),
                         (abi.HSG_UNWINDOWED, {}),
                         (abi.HSG_SESSION, dict(gap_ms=2_000))):
            aggs_k = aggs
            for mode in (abi.HSG_EMIT_PER_RECORD, abi.HSG_EMIT_PER_BATCH):
                out.append(pytest.param(OpSpec(kind, mode, col_types=col_types, aggs=aggs_k, **kw),
                                        id=f"{aggname}-k{kind}-m{mode}"))
    return out


def _close(a, b):
    if isinstance(a, float) or isinstance(b, float):
        if np.isnan(a) and np.isnan(b):
            return True
        return abs(a - b) <= 1e-9 * max(1.0, abs(a), abs(b))
    return a == b


@pytest.mark.parametrize("spec", _specs())
def test_cpp_oracle_matches_pyref(spec):
    """Two independent restatements agree, batch by batch, on messy inputs."""
    ncols = len(spec.col_types)
    o = pyoracle.OracleOp(spec)
    r = pyref.PyRefOp(spec)
    wm_o = wm_r = -1
    for bi in range(3):
        key, ts, cols, valid = gen_small(100 + bi, 300, 7, col_types=spec.col_types or (abi.HSG_I64,),
                                         span=20_000, base=1_000_000 + bi * 20_000)
        cols, valid = cols[:ncols], valid[:ncols]
        wm_o = o.push(key, ts, cols, valid, watermark=wm_o)
        wm_r = r.push(key, ts, cols, valid, watermark=wm_r)
        assert wm_o == wm_r
        got = o.drain().tuples()
        exp = [(k, s, e, v) for k, s, e, _, v in r.drain()]
        if spec.emit_mode == abi.HSG_EMIT_PER_BATCH:
            got, exp = sorted(got), sorted(exp)
        assert len(got) == len(exp)
        for g, x in zip(got, exp):
            assert g[:3] == x[:3]
            assert all(_close(a, b) for a, b in zip(g[3], x[3])), (g, x)
    st = sorted(o.dump_state().tuples())
    ex = sorted((k, s, e, v) for k, s, e, _, v in r.dump_state())
    assert len(st) == len(ex)
    for g, x in zip(st, ex):
        assert g[:3] == x[:3] and all(_close(a, b) for a, b in zip(g[3], x[3]))


def test_faithful_and_fast_session_store_agree():
    spec = OpSpec(abi.HSG_SESSION, abi.HSG_EMIT_PER_RECORD, gap_ms=1_500, col_types=[abi.HSG_I64],
                  aggs=[(abi.HSG_COUNT_ALL, 0), (abi.HSG_SUM, 0), (abi.HSG_MIN, 0)])
    a = pyoracle.OracleOp(spec, faithful_sessions=True)
    b = pyoracle.OracleOp(spec, faithful_sessions=False)
    wa = wb = -1
    for bi in range(4):
        key, ts, cols, valid = gen_small(7 + bi, 2000, 50, span=60_000, base=bi * 60_000)
        wa = a.push(key, ts, cols, valid, watermark=wa)
        wb = b.push(key, ts, cols, valid, watermark=wb)
        assert a.drain().tuples() == b.drain().tuples()
    assert a.dump_state().tuples() == b.dump_state().tuples()
