"""Sink encoding (include/hstream_sink.h).

CPU: the number formatter (the host build of the device code, hsg_fmt.h)
against a restatement: int64 aggregates print as aeson prints a Scientific
with exponent 0; f64 aggregates as Scientific's formatScientific Generic of
the shortest decimal that reads back as the double (Python's repr gives that
decimal).
GPU: changelog rows of an op -> key bytes (timeWindowSerde int64BE start ++
int64BE 0 ++ encode {key_field: key}, Boilerplate.hs:60-74, TimeWindows.hs:68-73)
and value bytes (encode of the SELECT-projected object, Codegen.hs:355-369),
compared byte for byte with a Python restatement of the same serdes.

Member order: aeson writes an Object's members in its HashMap's traversal
order; restated below from hashable-1.3.0.0 / text-1.2.4.0 /
unordered-containers-0.2.10.0 (Stack lts-16.21, hstream-processing/
stack.yaml:20-21). No reference test prints an encoded object, so the order
is pinned by this restatement of the libraries' published algorithm only.
Aggregate identities (Codegen.hs:425,438,451: Number 0, minBound / maxBound
:: Int, exponent 0) print as integers: a decimal column's SUM / MAX / MIN no
value reached is "0" / "-9223372036854775808" / "9223372036854775807"
(test_sink_identity_text, hand-derived). With HSG_OPF_LITERAL_FORMS every
SUM / MIN / MAX prints as the reference's Scientific does (an exponent >= 0 as
an integer), and under EMIT CHANGES each row's key prints in its record's own
spelling: test_sink_literal_forms_and_key_spellings, against a restatement of
Data.Scientific's sum / min / max and aeson's number encoding.
"""
import json
import math
import random
import struct
from decimal import Decimal

import numpy as np
import pytest

from hstream_amd import abi
from hstream_amd.sink import format_number


def generic(d: Decimal) -> str:
    """formatScientific Generic (scientific-0.3.6) of a decimal."""
    sign, digits, exp = d.normalize().as_tuple()
    s = "".join(map(str, digits)).rstrip("0")
    if not s or s == "0":
        return "0.0"
    e = exp + (len("".join(map(str, digits))) - len(s))
    E = len(s) + e
    pre = "-" if sign else ""
    if E < 0 or E > 7:
        return pre + s[0] + "." + (s[1:] or "0") + "e" + str(E - 1)
    if E == 0:
        return pre + "0." + s
    return pre + (s + "0" * E)[:E] + "." + (s[E:] or "0")


def ref_f64(v: float, agg: str = "") -> str:
    if math.isnan(v) or math.isinf(v):
        return "null"
    # the identities of the f64 slots (a SUM nothing was added to is -0.0 on
    # the device, MIN / MAX +-2^63): the reference's Number 0 / maxBound /
    # minBound, exponent 0, printed as integers; any other value exactly
    if agg == "sum" and v == 0.0 and math.copysign(1.0, v) < 0:
        return "0"
    if agg == "min" and v == 2.0 ** 63:
        return str((1 << 63) - 1)
    if agg == "max" and v == -(2.0 ** 63):
        return str(-(1 << 63))
    if v == 0.0:
        return "0.0"  # (a Scientific has no negative zero)
    return generic(Decimal(repr(v)))


_M64 = (1 << 64) - 1


def aeson_key_hash(alias: str) -> int:
    """hashable-1.3.0.0 hashWithSalt defaultSalt (Text): FNV-1 over the UTF-16
    code units' little-endian bytes, seeded with combine defaultSalt len."""
    u = alias.encode("utf-16-le")
    h = ((0xDC36D1615B7400A4 * 16777619) & _M64) ^ (len(u) // 2)
    for b in u:
        h = ((h * 16777619) & _M64) ^ b
    return h


def aeson_member_order(aliases):
    """Traversal order of a HashMap Text (unordered-containers-0.2.10.0: 4-bit
    subkeys from the low bits of the hash, children in subkey order)."""
    def digits(h):
        return [(h >> (4 * k)) & 15 for k in range(16)]
    return sorted(range(len(aliases)), key=lambda m: (digits(aeson_key_hash(aliases[m])), m))


def test_int64_text():
    for v in [0, 1, -1, 42, -(1 << 63), (1 << 63) - 1, 10 ** 18, -10 ** 18 + 7]:
        assert format_number(v, False) == str(v)


def test_f64_text_known():
    cases = {0.0: "0.0", 1.0: "1.0", 4.0: "4.0", 2.5: "2.5", 0.1: "0.1", 0.25: "0.25",
             0.001: "1.0e-3", 1234567.5: "1234567.5", 12345678.5: "1.23456785e7", 1e7: "1.0e7", 1e22: "1.0e22",
             -3.75: "-3.75", 1 / 3: "0.3333333333333333", 5e-324: "5.0e-324", 1.7976931348623157e308:
             "1.7976931348623157e308", 0.30000000000000004: "0.30000000000000004", 100.0: "100.0"}
    for v, t in cases.items():
        assert format_number(v, True) == t, v
        assert ref_f64(v) == t, v
    assert format_number(float("nan"), True) == "null"


def test_sink_identity_text():
    """Hand-derived from Codegen.hs:423-461 and aeson's Scientific encoding: a
    group whose decimal field was absent in every record keeps the initial
    values Number 0 / minBound / maxBound (exponent 0), printed as integers."""
    assert format_number(-0.0, True, "sum") == "0"                       # SUM: Number 0
    assert format_number(-(2.0 ** 63), True, "max") == "-9223372036854775808"  # MAX: minBound :: Int
    assert format_number(2.0 ** 63, True, "min") == "9223372036854775807"      # MIN: maxBound :: Int
    # the same values as other aggregates (or plain numbers) print exactly
    for v, agg in ((2.0 ** 63, ""), (2.0 ** 63, "sum"), (2.0 ** 63, "max"), (-(2.0 ** 63), "min"),
                   (-(2.0 ** 63), ""), (-0.0, "min")):
        assert format_number(v, True, agg) == ref_f64(v), (v, agg)


def test_member_order_restatement():
    """The encoder's member order (sink.cpp, hsg_sink_member_order) equals the
    independent Python restatement of the HashMap traversal."""
    from hstream_amd.sink import member_order
    rng = random.Random(11)
    pool = ["cnt", "total", "avg_x", "k", "max_x", "min v", "SUM(a)", "a", "b", "s1.a", "s2.b", "result",
            "COUNT(*)", "é", "𝄞x", "a+1", "winStart", "key1", "key2", "key3"]
    for _ in range(200):
        names = rng.sample(pool, rng.randrange(1, 12))
        assert member_order(names) == aeson_member_order(names), names


def test_f64_text_random_bits():
    rng = random.Random(5)
    for _ in range(20000):
        bits = rng.getrandbits(64)
        v = struct.unpack("<d", struct.pack("<Q", bits))[0]
        assert format_number(v, True) == ref_f64(v), (hex(bits), v)


def test_f64_text_decimal_like_values():
    rng = random.Random(6)
    for _ in range(20000):
        v = round(rng.uniform(-1e7, 1e7), rng.randrange(0, 7))
        assert format_number(v, True) == ref_f64(v), v
    for k in range(-30, 30):
        for m in (1, 3, 7, 9, 5):
            v = m * 10.0 ** k
            assert format_number(v, True) == ref_f64(v), v


# ---------------------------------------------------------------------------
# GPU: whole records
# ---------------------------------------------------------------------------
def _ref_record(key_text, key_field, ws, members, windowed):
    key_obj = "{" + json.dumps(key_field) + ":" + key_text + "}"
    kb = (struct.pack(">qq", ws, 0) if windowed else b"") + key_obj.encode()
    parts = []
    for alias, text in members:
        parts.append(json.dumps(alias, ensure_ascii=False) + ":" + text)
    return kb, ("{" + ",".join(parts) + "}").encode()


@pytest.mark.gpu
@pytest.mark.parametrize("windowed", [True, False], ids=["tumbling", "unwindowed"])
def test_sink_records_match_serdes(windowed):
    import torch
    assert torch.cuda.is_available()
    from hstream_amd.columnar import OpSpec
    from hstream_amd.engine import Engine
    from hstream_amd.ingest import Decoder, KeyDict, pack_records
    from hstream_amd.sink import Sink
    eng = Engine(device=0, batch_capacity=1 << 16)
    kind = abi.HSG_TUMBLING if windowed else abi.HSG_UNWINDOWED
    spec = OpSpec(kind, abi.HSG_EMIT_PER_RECORD, size_ms=5000, col_types=[abi.HSG_I64, abi.HSG_F64],
                  aggs=[(abi.HSG_COUNT_ALL, 0), (abi.HSG_SUM, 0), (abi.HSG_AVG, 1), (abi.HSG_MAX, 1),
                        (abi.HSG_MIN, 0)])
    op = eng.op(spec)
    rng = np.random.default_rng(3)
    keyvals = [1, "a\"b", 2.5, {"z": [1, 2]}, "é", -7, True]
    vals, ts = [], []
    for i in range(4000):
        k = keyvals[int(rng.integers(0, len(keyvals)))]
        vals.append(json.dumps({"k": k, "v": int(rng.integers(-10 ** 12, 10 ** 12)),
                                "x": round(float(rng.uniform(-1e4, 1e4)), 3)}).encode())
        ts.append(1_000_000 + 25 * i)
    keys = KeyDict()
    dec = Decoder("k", [("v", abi.HSG_I64, True), ("x", abi.HSG_F64, True)])
    buf, off = pack_records(vals)
    kid, t, cols, valid, st, rej = dec.decode(keys, buf, off, np.array(ts, np.int64))
    assert rej == 0
    op.push(kid, t, cols, valid)
    rows = op.drain()
    members = [("cnt", 0), ("total", 1), ("avg_x", 2), ("k", -1), ("max_x", 3), ("min v", 4)]
    sink = Sink(op, keys, "k", members, windowed=windowed)
    written = [members[m] for m in aeson_member_order([a for a, _ in members])]
    got = sink.encode(rows)
    assert len(got) == len(rows) > 0
    f64 = spec.agg_is_f64()
    for i, (kb, vb) in enumerate(got):
        ktext = keys.text(int(rows.key_id[i]))
        mem = []
        for alias, j in written:
            if j < 0:
                mem.append((alias, ktext))
            else:
                v = rows.aggs[j][i]
                kind = {abi.HSG_SUM: "sum", abi.HSG_MIN: "min", abi.HSG_MAX: "max"}.get(spec.aggs[j][0], "")
                mem.append((alias, ref_f64(float(v), kind) if f64[j] else str(int(v))))
        ek, ev = _ref_record(ktext, "k", int(rows.win_start[i]), mem, windowed)
        assert kb == ek, (i, kb, ek)
        assert vb == ev, (i, vb, ev)
    # the value bytes parse as JSON with the projected members
    assert set(json.loads(got[0][1].decode())) == {a for a, _ in members}
    sink.close()
    op.close()
    eng.close()


# ---------------------------------------------------------------------------
# GPU: literal forms and key spellings (HSG_OPF_LITERAL_FORMS,
# hsg_decode_json_spelled, hsg_sink_encode_spelled) against a restatement of
# Data.Scientific arithmetic and aeson's number encoding
# ---------------------------------------------------------------------------
def sci_parse(text: str):
    """A JSON number literal as Data.Scientific keeps it: (coefficient,
    exponent), not normalised (2.50 is 250e-2)."""
    t = text.lower()
    mant, _, ex = t.partition("e")
    ip, _, fp = mant.partition(".")
    neg = ip.startswith("-")
    digits = ip.lstrip("-") + fp
    c = int(digits) * (-1 if neg else 1)
    return c, (int(ex) if ex else 0) - len(fp)


def sci_add(a, b):
    e = min(a[1], b[1])
    return a[0] * 10 ** (a[1] - e) + b[0] * 10 ** (b[1] - e), e


def sci_val(a):
    from fractions import Fraction
    return Fraction(a[0]) * Fraction(10) ** a[1]


def aeson_sci(a) -> str:
    """aeson 1.4's Number encoding: exponent in [0, 1024] as an integer, else
    formatScientific Generic."""
    c, e = a
    if 0 <= e <= 1024:
        return str(c * 10 ** e)
    return generic(Decimal(c).scaleb(e))


MAXB, MINB = ((1 << 63) - 1, 0), (-(1 << 63), 0)  # maxBound / minBound :: Int (Codegen.hs:438,451)
ZERO = (0, 0)                                      # Number 0 (Codegen.hs:406,425,466)


_TIES = [0]  # folds / merges of equal MIN / MAX values with different literal forms


def _tie(a, b):
    if sci_val(a) == sci_val(b) and (a[1] >= 0) != (b[1] >= 0):
        _TIES[0] += 1


def _init(kind):
    return {"cnt": 0, "sum": ZERO, "min": MAXB, "max": MINB, "last": ZERO}[kind]


def _fold(kind, n, x):
    """aggregateF of one component (Codegen.hs:404-469) on a present literal
    x (None: the field is absent). Haskell's min n x = if n <= x then n else
    x, max n x = if n <= x then x else n: on equal values MIN keeps the
    earlier literal, MAX takes the later."""
    if kind == "cnt":
        return n + 1
    if x is None:
        return n
    if kind == "sum":
        return sci_add(n, x)
    if kind in ("min", "max"):
        _tie(n, x)
    if kind == "min":
        return n if sci_val(n) <= sci_val(x) else x
    if kind == "max":
        return x if sci_val(n) <= sci_val(x) else n
    return x  # last: the record's own value (HM.adjust updateV)


def _merge(kind, n1, n2):
    """aggregateMergeF (Codegen.hs:409-469): n1 = the merged side (the new
    record and the sessions merged so far), n2 = the next overlapped session
    (SessionWindowedStream.hs:100-114)."""
    if kind == "cnt":
        return n1 + n2
    if kind == "sum":
        return sci_add(n1, n2)
    if kind in ("min", "max"):
        _tie(n1, n2)
    if kind == "min":
        return n1 if sci_val(n1) <= sci_val(n2) else n2
    if kind == "max":
        return n2 if sci_val(n1) <= sci_val(n2) else n1
    return n2  # passthrough: o2


def _lit(vals, col):
    x = vals.get(col) if col else None
    return None if x is None else sci_parse(x)


def _text(kind, v):
    return str(v) if kind == "cnt" else aeson_sci(v)


def _group_key(key_text):
    """Aeson Value equality of a key: numbers by their Scientific value."""
    key = json.loads(key_text)
    return float(key) if isinstance(key, (int, float)) and not isinstance(key, bool) else json.dumps(key)


def _ref_literal_rows(recs, comps, window, emit, batches):
    """The reference's fold over literal records (key text, ts, {column:
    literal or None}), one changelog row per record (EMIT CHANGES) or, per
    batch, the state after the batch of every group it touched. Rows:
    (record index or -1, key text, window start, {alias: text}).
    window = ("tumbling", size) (TimeWindowedStream.hs:86-103) or
    ("session", gap) (SessionWindowedStream.hs:84-118, findSessions order:
    end, then start, ascending, Store.hs:243-272)."""
    kind, size = window
    state = {}   # tumbling: (group, ws) -> comps state; session: group -> [[start, end, state], ...]
    first_text = {}
    out = []
    rec_at = 0
    for nb in batches:
        touched = {}
        for r in range(rec_at, rec_at + nb):
            key_text, ts, vals = recs[r]
            gk = _group_key(key_text)
            first_text.setdefault(gk, key_text)
            if kind == "tumbling":
                ws = (ts // size) * size
                st = state.setdefault((gk, ws), {a: _init(k) for a, k, _ in comps})
                for a, k, col in comps:
                    st[a] = _fold(k, st[a], _lit(vals, col))
                row_key, row_st = (gk, ws), st
            else:
                sess = state.setdefault(gk, [])
                acc = {a: _fold(k, _init(k), _lit(vals, col)) for a, k, col in comps}
                s0 = e0 = ts
                over = sorted((x for x in sess if x[1] >= ts - size and x[0] <= ts + size), key=lambda x: (x[1], x[0]))
                for cur in over:
                    acc = {a: _merge(k, acc[a], cur[2][a]) for a, k, _ in comps}
                    s0, e0 = min(s0, cur[0]), max(e0, cur[1])
                    sess.remove(cur)
                sess.append([s0, e0, acc])
                ws, row_st = s0, acc
                row_key = (gk, s0)
                for o in over:  # merged sessions are gone from this batch's rows
                    touched.pop((gk, o[0]), None)
            texts = {a: _text(k, row_st[a]) for a, k, _ in comps}
            if emit == abi.HSG_EMIT_PER_RECORD:
                own = json.dumps(json.loads(key_text)) if key_text.startswith('"') else aeson_sci(sci_parse(key_text))
                out.append((r, own, ws, texts))
            else:
                touched[row_key] = (-1, first_text[gk], ws, texts)
        rec_at += nb
        if emit != abi.HSG_EMIT_PER_RECORD:
            out.append(sorted(touched.values(), key=lambda x: (x[1], x[2])))
    return out


def _first_text(kt):
    return json.dumps(json.loads(kt)) if kt.startswith('"') else aeson_sci(sci_parse(kt))


LITERAL_CASES = {
    # tumbling, EMIT CHANGES: the changelog, key spellings per record
    "tumbling_changes": (("tumbling", 5000), abi.HSG_EMIT_PER_RECORD, 2),
    # tumbling, per batch: the last row of each group the batch touched
    "tumbling_batch": (("tumbling", 5000), abi.HSG_EMIT_PER_BATCH, 2),
    # four value columns (each aggregated), per batch and EMIT CHANGES
    "tumbling_changes_4col": (("tumbling", 5000), abi.HSG_EMIT_PER_RECORD, 4),
    "tumbling_batch_4col": (("tumbling", 5000), abi.HSG_EMIT_PER_BATCH, 4),
    # sessions: record folds and session merges (min n1 n2 / max n1 n2)
    "session_changes": (("session", 900), abi.HSG_EMIT_PER_RECORD, 2),
    "session_batch": (("session", 900), abi.HSG_EMIT_PER_BATCH, 4),
}


@pytest.mark.gpu
@pytest.mark.parametrize("case", sorted(LITERAL_CASES))
def test_sink_literal_forms_and_key_spellings(case):
    """Decimal columns fed integral literals print integers ("6" for 2 + 4),
    mixed 2 / 2.0 / 25e-1 / 1e1 spellings follow the Scientific exponent
    rules (a SUM's exponent is the smaller one; a MIN / MAX reached by equal
    values spelled differently keeps the literal the reference's fold keeps:
    min n x = n, max n x = x, and on session merges min n1 n2 / max n1 n2),
    absent fields leave the reference's initial values (0, maxBound,
    minBound), an i64 column fed 20e-1 prints "2.0", a passthrough column
    prints its last literal; keys 1 / 1.0 / 1e0 / 10e-1 are one group whose
    EMIT CHANGES rows print each record's own spelling ("1" or "1.0"). Every
    row is compared with the restatement, ties included."""
    import torch
    assert torch.cuda.is_available()
    from hstream_amd.columnar import OpSpec
    from hstream_amd.engine import Engine
    from hstream_amd.ingest import Decoder, KeyDict, pack_records
    from hstream_amd.sink import Sink
    window, emit, ncols = LITERAL_CASES[case]
    rng = random.Random(17 + ncols + 7 * (window[0] == "session") + emit)
    keylits = ["1", "1.0", "1e0", "10e-1", '"a"', "2.5", "25e-1"]
    ilits = ["5", "-3", "20e-1", "2e1", "7", "7.0", "70e-1", "-1", "-1.0", "2"]           # integral values
    flits = ["2", "2.0", "4", "25e-1", "2.50", "1e1", "-4", "-4.0", "0.5", "7", "7.0", "3.25", None, None]
    cols = [("v", abi.HSG_I64, ilits), ("x", abi.HSG_F64, flits)]
    if ncols == 4:
        cols += [("y", abi.HSG_F64, ["1", "1.0", "10e-1", "0.25", "-2", "-2.00", None]),
                 ("z", abi.HSG_I64, ["3", "3.0", "30e-1", "-8", "-8.0", "0", "0.0", None])]
    comps = [("cnt", "cnt", None)]
    # (24 state slots at most: a SUM / MIN / MAX with forms takes two, a passthrough three)
    per_col = {"v": ("sum", "min", "max"), "x": ("sum", "min", "max"), "y": ("sum", "max"), "z": ("min", "sum")}
    for name, _t, _l in cols:
        comps += [(k + "_" + name, k, name) for k in per_col[name]]
    comps.append(("last_v", "last", "v"))
    kinds = {"cnt": abi.HSG_COUNT_ALL, "sum": abi.HSG_SUM, "min": abi.HSG_MIN, "max": abi.HSG_MAX,
             "last": abi.HSG_LAST}
    colidx = {name: c for c, (name, _t, _l) in enumerate(cols)}
    aggs = [(kinds[k], colidx[col] if col else 0) for _a, k, col in comps]
    n = 3000
    recs, vals, ts = [], [], []
    t = 1_000_000
    for i in range(n):
        kt = rng.choice(keylits)
        # ~3-4 records per (key, window); sessions: gaps around the 900 ms
        # gap and some records out of order, so merges of several sessions
        t += rng.randrange(0, 400)
        tt = t - (rng.randrange(0, 3000) if rng.random() < 0.15 else 0)
        v = {name: rng.choice(lits) for name, _t, lits in cols}
        v["v"] = v["v"] or "1"
        recs.append((kt, tt, v))
        body = '{"k":' + kt + "".join(f',"{c}":{x}' for c, x in v.items() if x is not None) + "}"
        vals.append(body.encode())
        ts.append(tt)
    batches = [1000, 1200, 800]
    eng = Engine(device=0, batch_capacity=1 << 14)
    wk = abi.HSG_TUMBLING if window[0] == "tumbling" else abi.HSG_SESSION
    spec = OpSpec(wk, emit, size_ms=window[1] if wk == abi.HSG_TUMBLING else 0,
                  gap_ms=window[1] if wk == abi.HSG_SESSION else 0, col_types=[ty for _n, ty, _l in cols],
                  aggs=aggs, flags=abi.HSG_OPF_LITERAL_FORMS)
    op = eng.op(spec)
    keys = KeyDict()
    dec = Decoder("k", [(name, ty, True) for name, ty, _l in cols], literal_forms=True)
    members = [(a, j) for j, (a, _k, _c) in enumerate(comps)] + [("k", -1)]
    sink = Sink(op, keys, "k", members, windowed=True)
    written = [members[m] for m in aeson_member_order([a for a, _ in members])]
    _TIES[0] = 0
    ref = _ref_literal_rows(recs, comps, window, emit, batches)
    at = 0
    wm = -1
    for bi, nb in enumerate(batches):
        buf, off = pack_records(vals[at:at + nb])
        kid, tb, cs, valid, _st, rej, spell = dec.decode(keys, buf, off, np.array(ts[at:at + nb], np.int64),
                                                          spellings=True)
        assert rej == 0
        wm = op.push(kid, tb, cs, valid, watermark=wm)
        rows = op.drain()
        assert rows.form is not None
        if emit == abi.HSG_EMIT_PER_RECORD:
            got = sink.encode(rows, spellings=spell, src_base=at)
            assert len(got) == nb
            want = {x[0]: x for x in ref if at <= x[0] < at + nb}
            for i, (kb, vb) in enumerate(got):
                r = int(rows.src_index[i])
                _r, own, ws, texts = want[r]
                mem = [(a, own if j < 0 else texts[a]) for a, j in written]
                ek, ev = _ref_record(own, "k", ws, mem, True)
                assert kb == ek, (case, i, r, kb, ek)
                assert vb == ev, (case, i, r, recs[r], vb, ev)
        else:
            got = sink.encode(rows)
            exp = ref[bi]
            assert len(got) == len(exp), (case, bi, len(got), len(exp))
            mine = sorted(got)
            exp_b = []
            for _r, ktext, ws, texts in exp:
                own = _first_text(ktext)
                mem = [(a, own if j < 0 else texts[a]) for a, j in written]
                ek, ev = _ref_record(own, "k", ws, mem, True)
                exp_b.append((ek, ev))
            exp_b.sort()
            for g, e in zip(mine, exp_b):
                assert g == e, (case, bi, g, e)
        at += nb
    # folds and merges that met equal MIN / MAX values spelled both ways
    assert _TIES[0] > 0, case
    sink.close()
    op.close()
    eng.close()
