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
(test_sink_identity_text, hand-derived). Known divergence, parity
unpinned: a decimal aggregate whose value came only from integer JSON
literals (Scientific exponent >= 0) prints "6" in the reference and "6.0"
here (the f64 column keeps no exponent).
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


def ref_f64(v: float) -> str:
    if math.isnan(v) or math.isinf(v):
        return "null"
    # the identities of the f64 slots (a SUM nothing was added to is -0.0 on
    # the device, MIN / MAX +-2^63): the reference's Number 0 / maxBound /
    # minBound, exponent 0, printed as integers
    if v == 0.0 and math.copysign(1.0, v) < 0:
        return "0"
    if v == 2.0 ** 63:
        return str((1 << 63) - 1)
    if v == -(2.0 ** 63):
        return str(-(1 << 63))
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
    assert format_number(-0.0, True) == "0"                       # SUM: Number 0
    assert format_number(-(2.0 ** 63), True) == "-9223372036854775808"  # MAX: minBound :: Int
    assert format_number(2.0 ** 63, True) == "9223372036854775807"      # MIN: maxBound :: Int


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
                mem.append((alias, ref_f64(float(v)) if f64[j] else str(int(v))))
        ek, ev = _ref_record(ktext, "k", int(rows.win_start[i]), mem, windowed)
        assert kb == ek, (i, kb, ek)
        assert vb == ev, (i, vb, ev)
    # the value bytes parse as JSON with the projected members
    assert set(json.loads(got[0][1].decode())) == {a for a, _ in members}
    sink.close()
    op.close()
    eng.close()
