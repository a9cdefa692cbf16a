"""CPU: host ingest (include/hstream_ingest.h) against a Python restatement.

The restatement parses with exact decimals (json + decimal.Decimal keeps the
literal's coefficient and exponent, as Data.Scientific does) and follows:
  value decode           Processor.hs:192-204 (non-object / malformed: dropped)
  GROUP BY key           Codegen.hs:485-487 + getFieldByName (Internal/Codegen.hs:41-49)
  key identity           Aeson Value equality (Scientific numbers, maps, arrays)
  field reads            Codegen.hs:412-461 (absent: left alone; COUNT(col): any
                         present value; SUM/MIN/MAX: a Number or the record aborts)
  key text               aeson-1.4 encode: integer print when the literal's
                         exponent is in [0, 1024], else formatScientific Generic
Records dropped by the reference carry HSG_KEY_NONE (they still move stream
time); integral columns reject non-integral or out-of-int64 numbers.
"""
import json
import random
from decimal import Decimal

import numpy as np
import pytest

from hstream_amd import abi
from hstream_amd.ingest import Decoder, KeyDict, pack_records


# ---------------------------------------------------------------------------
# restatement
# ---------------------------------------------------------------------------
def _load(b):
    return json.loads(b, parse_float=Decimal, parse_int=Decimal)


def canon(v):
    if v is None:
        return ("z",)
    if v is True:
        return ("t",)
    if v is False:
        return ("f",)
    if isinstance(v, Decimal):
        return ("n", v)  # Decimal equality / hash = Scientific equality
    if isinstance(v, str):
        return ("s", v)
    if isinstance(v, list):
        return ("a", tuple(canon(x) for x in v))
    return ("o", frozenset((k, canon(x)) for k, x in v.items()))


def aeson_num(d: Decimal) -> str:
    sign, digits, exp = d.as_tuple()
    coef = int("".join(map(str, digits)) or "0")
    if 0 <= exp <= 1024:
        return str(-coef * 10 ** exp if sign else coef * 10 ** exp)
    if coef == 0:
        return "0.0"
    s = str(coef)
    ds = s.rstrip("0")
    e = exp + (len(s) - len(ds))
    E = len(ds) + e
    pre = "-" if sign else ""
    if E < 0 or E > 7:
        return pre + ds[0] + "." + (ds[1:] or "0") + "e" + str(E - 1)
    if E == 0:
        return pre + "0." + ds
    return pre + (ds + "0" * E)[:E] + "." + (ds[E:] or "0")


def aeson_str(s: str) -> str:
    out = ['"']
    for ch in s:
        o = ord(ch)
        if ch == "\\":
            out.append("\\\\")
        elif ch == '"':
            out.append('\\"')
        elif o >= 0x20:
            out.append(ch)
        elif ch == "\n":
            out.append("\\n")
        elif ch == "\r":
            out.append("\\r")
        elif ch == "\t":
            out.append("\\t")
        else:
            out.append("\\u%04x" % o)
    out.append('"')
    return "".join(out)


def aeson_text(v) -> str:
    if v is None:
        return "null"
    if v is True:
        return "true"
    if v is False:
        return "false"
    if isinstance(v, Decimal):
        return aeson_num(v)
    if isinstance(v, str):
        return aeson_str(v)
    if isinstance(v, list):
        return "[" + ",".join(aeson_text(x) for x in v) + "]"
    return "{" + ",".join(aeson_str(k) + ":" + aeson_text(v[k]) for k in sorted(v)) + "}"


def ref_decode(values, key_field, cols):
    """-> key ids, cols, valid, status, {id: text} (ids in first-seen order)."""
    n = len(values)
    ids, texts = {}, {}
    key = np.full(n, abi.HSG_KEY_NONE, np.uint32)
    out = [np.zeros(n, np.float64 if t == abi.HSG_F64 else np.int64) for _, t, _ in cols]
    valid = [np.zeros(n, np.uint8) for _ in cols]
    status = np.zeros(n, np.uint8)
    for i, b in enumerate(values):
        try:
            obj = _load(b)
        except ValueError:
            status[i] = abi.HSG_DEC_NOT_OBJECT
            continue
        if not isinstance(obj, dict):
            status[i] = abi.HSG_DEC_NOT_OBJECT
            continue
        if key_field not in obj:
            status[i] = abi.HSG_DEC_NO_KEY
            continue
        st, vals = abi.HSG_DEC_OK, []
        for c, (f, t, numeric) in enumerate(cols):
            if f not in obj:
                vals.append(None)
                continue
            v = obj[f]
            if not numeric:
                vals.append(0)
                continue
            if not isinstance(v, Decimal):
                st = abi.HSG_DEC_TYPE
                break
            if t == abi.HSG_F64:
                vals.append(float(v))
                continue
            if v != v.to_integral_value():
                st = abi.HSG_DEC_NOT_INTEGRAL
                break
            iv = int(v)
            if not -(1 << 63) <= iv < (1 << 63):
                st = abi.HSG_DEC_RANGE
                break
            vals.append(iv)
        status[i] = st
        if st != abi.HSG_DEC_OK:
            continue
        c0 = canon(obj[key_field])
        if c0 not in ids:
            ids[c0] = len(ids)
            texts[ids[c0]] = aeson_text(obj[key_field])
        key[i] = ids[c0]
        for c, v in enumerate(vals):
            if v is not None:
                out[c][i] = v
                valid[c][i] = 1
    return key, out, valid, status, texts


# ---------------------------------------------------------------------------
# inputs
# ---------------------------------------------------------------------------
EDGE = [
    b'{"k": 1, "v": 5, "x": 2.5}',
    b'{"k": 1.0, "v": -5, "x": 1e2}',          # same key as 1
    b'{"k": 10e-1, "v": 7}',                     # same key as 1
    b'{"k": 1E0, "v": 0}',                       # same key as 1
    b'{"k": "1", "v": 1}',                       # a string: another key
    b'{"k": -0, "v": 1}',                        # -0 == 0
    b'{"k": 0.0, "v": 1}',                       # == 0
    b'{"k": 0.000, "v": 1}',
    b'{"k": {"a": 1, "b": [1, 2.0]}, "v": 1}',
    b'{"k": {"b": [1.0, 2], "a": 1.00}, "v": 1}',  # the same object
    b'{"k": "\\u0041b", "v": 3}',                # escapes: "Ab"
    b'{"k": "Ab", "v": 4}',
    b'{"k": "tab\\there\\n", "v": 1}',
    b'{"k": "\\ud83d\\ude00", "v": 1}',          # surrogate pair
    b'{"k": null, "v": 1}',
    b'{"k": true, "v": 1}',
    b'{"k": [true, false, null], "v": 1}',
    b'{"v": 1}',                                 # no GROUP BY field
    b'{"k": 2, "v": "a"}',                       # SUM over a string
    b'{"k": 2, "v": null}',                      # SUM over null
    b'{"k": 2, "v": 2.5}',                       # not integral
    b'{"k": 2, "v": 2.50e1}',                    # 25: integral
    b'{"k": 2, "v": 9223372036854775807}',
    b'{"k": 2, "v": -9223372036854775808}',
    b'{"k": 2, "v": 9223372036854775808}',       # out of int64
    b'{"k": 2, "v": 1e30}',
    b'{"k": 2, "c": "anything"}',                # COUNT(c) counts any value
    b'{"k": 2, "c": null}',
    b'{"k": 2, "v": 1, "v": 2}',                 # duplicate member: last wins
    b'[1, 2]',                                   # not an object
    b'{"k": 1',                                  # malformed
    b'{"k": 1,}',
    b'',
    b'  {"k" : 3 , "v" : 4 }  ',
    b'{"k": 123456789.5, "v": 1}',
    b'{"k": 0.001, "v": 1}',
    b'{"k": 1.5e-7, "v": 1}',
    b'{"k": 12345678.25, "v": 1}',
    b'{"k": 1e3, "v": 1}',
    b'{"k": 1000.0, "v": 1}',
    b'{"k": 2e1025, "v": 1}',
    b'{"k": "\\"q\\\\", "v": 1}',
    b'{"k": "\\u0001", "v": 1}',
    b'{"nest": {"k": 9}, "k": 4, "v": 1}',       # nested members are not the field
]
COLS = [("v", abi.HSG_I64, True), ("x", abi.HSG_F64, True), ("c", abi.HSG_I64, False)]


def _random_values(seed, n):
    rng = random.Random(seed)
    keys = [1, 2, "a", "b", 3.0, 3, "3", None, True, [1, 2], {"z": 1, "y": [2]}, 0.5, -7, "é", "x\"y"]
    out = []
    for i in range(n):
        d = {}
        r = rng.random()
        if r > 0.03:
            d["k"] = rng.choice(keys) if rng.random() < 0.6 else rng.randrange(5000)
        if rng.random() > 0.1:
            d["v"] = rng.choice([rng.randrange(-10 ** 12, 10 ** 12), rng.randrange(100), "s", None, 1.5, 2.0])
        if rng.random() > 0.2:
            d["x"] = rng.choice([rng.uniform(-1e6, 1e6), rng.randrange(-100, 100), round(rng.uniform(0, 1000), 3)])
        if rng.random() > 0.5:
            d["c"] = rng.choice([1, "s", None, [1], {"a": 2}])
        d["pad%d" % (i % 7)] = {"deep": [1, {"e": "x"}], "s": "long string " * (i % 5)}
        items = list(d.items())
        rng.shuffle(items)
        out.append(json.dumps(dict(items)).encode())
    return out


def _check(values, threads):
    buf, off = pack_records(values)
    ts = np.arange(len(values), dtype=np.int64) * 7 - 3
    kd = KeyDict()
    dec = Decoder("k", COLS)
    key, ts_out, cols, valid, status, rej = dec.decode(kd, buf, off, ts, threads=threads)
    rkey, rcols, rvalid, rstatus, rtexts = ref_decode(values, "k", COLS)
    np.testing.assert_array_equal(status, rstatus)
    np.testing.assert_array_equal(key, rkey)
    np.testing.assert_array_equal(ts_out, ts)
    assert rej == int((rstatus != 0).sum())
    for c in range(len(COLS)):
        ok = rstatus == 0
        np.testing.assert_array_equal(valid[c][ok], rvalid[c][ok])
        np.testing.assert_array_equal(cols[c][ok & (rvalid[c] == 1)], rcols[c][ok & (rvalid[c] == 1)])
    assert len(kd) == len(rtexts)
    for i, t in rtexts.items():
        assert kd.text(i) == t, (i, t)
    return kd, key, status


def test_edge_cases_match_restatement():
    kd, key, status = _check(EDGE, threads=1)
    # the four spellings of 1 are one key, "1" is another
    assert key[0] == key[1] == key[2] == key[3] != key[4]
    assert key[5] == key[6] == key[7]
    assert key[8] == key[9] and key[10] == key[11]
    assert status[17] == abi.HSG_DEC_NO_KEY and status[18] == abi.HSG_DEC_TYPE and status[19] == abi.HSG_DEC_TYPE
    assert status[20] == abi.HSG_DEC_NOT_INTEGRAL and status[21] == 0
    assert status[24] == abi.HSG_DEC_RANGE and status[25] == abi.HSG_DEC_RANGE
    assert status[29] == status[30] == status[31] == status[32] == abi.HSG_DEC_NOT_OBJECT
    assert kd.text(int(key[0])) == "1" and kd.text(int(key[35])) == "1.0e-3"


@pytest.mark.parametrize("threads", [1, 4])
def test_random_batch_matches_restatement(threads):
    _check(_random_values(7, 20_000), threads)


def test_ids_are_stable_across_batches_and_threads():
    vals = _random_values(9, 12_000)
    buf, off = pack_records(vals)
    ts = np.zeros(len(vals), np.int64)
    a, b = KeyDict(), KeyDict()
    d = Decoder("k", COLS)
    ka = d.decode(a, buf, off, ts, threads=1)[0]
    kb = d.decode(b, buf, off, ts, threads=8)[0]
    np.testing.assert_array_equal(ka, kb)
    # a second batch reuses the ids of the keys it shares with the first
    ka2 = d.decode(a, buf, off, ts, threads=3)[0]
    np.testing.assert_array_equal(ka, ka2)


def test_keydict_encode_and_text():
    kd = KeyDict()
    assert kd.encode_json("1") == kd.encode_json("1.00") == kd.encode_json(" 1e0 ") == 0
    assert kd.encode_json('"1"') == 1
    assert kd.encode({"b": 2, "a": [1, 2]}) == kd.encode_json('{"a":[1.0,2],"b":2.0}') == 2
    assert kd.text(0) == "1" and kd.text(1) == '"1"' and kd.text(2) == '{"a":[1,2],"b":2}'
    with pytest.raises(abi.HStreamGpuError):
        kd.encode_json("{")
    assert len(kd) == 3


def test_literal_form_valid_bits():
    """literal_forms: a present number's valid byte is 1 for an exponent >= 0
    ("2", "1e1", "-4") and 3 for a negative one ("2.0", "25e-1", "20e-1",
    Data.Scientific keeps the literal's exponent); absent fields stay 0."""
    lits = ["2", "2.0", "25e-1", "1e1", "-4", "-4.0", "20e-1", "0.5", "1E2", None]
    vals = [("{\"k\":1" + ("" if x is None else ",\"x\":" + x + ",\"v\":" + x) + "}").encode() for x in lits]
    dec = Decoder("k", [("x", abi.HSG_F64, True), ("v", abi.HSG_I64, False)], literal_forms=True)
    buf, off = pack_records(vals)
    keys = KeyDict()
    _, _, cols, valid, st, rej = dec.decode(keys, buf, off, np.zeros(len(vals), np.int64))
    assert rej == 0
    want = [1, 3, 3, 1, 1, 3, 3, 3, 1, 0]
    assert valid[0].tolist() == want
    assert cols[0][:9].tolist() == [2.0, 2.0, 2.5, 10.0, -4.0, -4.0, 2.0, 0.5, 100.0]
    # a COUNT-only column keeps plain 0 / 1
    assert valid[1].tolist() == [1] * 9 + [0]
    # without literal_forms every present value is 1
    plain = Decoder("k", [("x", abi.HSG_F64, True)])
    _, _, _, valid2, _, _ = plain.decode(keys, buf, off, np.zeros(len(vals), np.int64))
    assert valid2[0].tolist() == [1] * 9 + [0]


def test_key_spellings():
    """Keys 1 / 1.0 / 1e0 / 10e-1 / 100e-2 are one group (Aeson Value
    equality); a record's spelling id is the key id when it prints as the
    group's text and HSG_SPELL_ALT | i for another spelling (aeson prints
    "1" for an exponent >= 0 and "1.0" for a negative one)."""
    lits = ["1", "1.0", "1e0", "10e-1", "100e-2", "\"a\"", "2.5", "25e-1", "1.0"]
    vals = [("{\"k\":" + k + "}").encode() for k in lits]
    keys = KeyDict()
    dec = Decoder("k", [])
    buf, off = pack_records(vals)
    kid, _, _, _, _, rej, spell = dec.decode(keys, buf, off, np.zeros(len(vals), np.int64), spellings=True)
    assert rej == 0
    assert len(set(kid[:5].tolist())) == 1 and kid[8] == kid[0] and kid[6] == kid[7]
    assert keys.text(int(kid[0])) == "1"
    texts = [keys.spelling_text(int(s)) for s in spell]
    assert texts == ["1", "1.0", "1", "1.0", "1.0", "\"a\"", "2.5", "2.5", "1.0"]
    assert spell[0] == kid[0] and spell[2] == kid[0]
    assert spell[1] & abi.HSG_SPELL_ALT and spell[1] == spell[3] == spell[4] == spell[8]
    # spellings across batches reuse the alternate ids
    kid2, _, _, _, _, _, spell2 = dec.decode(keys, buf, off, np.zeros(len(vals), np.int64), spellings=True)
    assert kid2.tolist() == kid.tolist() and spell2.tolist() == spell.tolist()


def _c2_like_records(rng, n, nkeys, t0, decimals=3, vmax=10**9, span=60_000):
    vals, ts = [], []
    for i in range(n):
        v = int(rng.integers(-vmax, vmax))
        x = round(float(rng.uniform(0, 1e6)), decimals)
        vals.append(json.dumps({"k": int(rng.integers(0, nkeys)), "v": v, "x": x}).encode())
        ts.append(t0 + (i * span) // n + int(rng.integers(0, 2000)))
    return vals, np.array(ts, np.int64)


@pytest.mark.parametrize("threads", [1, 4])
def test_decode_batch_narrow_equals_wide(threads):
    """hsg_decode_json_batch: the decoder picks the narrow transport per batch
    from the values it decoded (16-bit keys, TS16 frames, int32 values, DEC32
    mantissas of 3-decimal values) and the batch it hands over widens back to
    exactly the full-width decode (Processor.hs:192-204 decodes the same
    values); columns present in every record carry no valid bytes. C2's
    record: 8 bytes + 4 for the decimal column instead of 28."""
    rng = np.random.default_rng(8)
    vals, ts = _c2_like_records(rng, 20_000, 5000, 1_700_000_000_000)
    buf, off = pack_records(vals)
    cols = [("v", abi.HSG_I64, True), ("x", abi.HSG_F64, True)]
    wide_keys, nar_keys = KeyDict(), KeyDict()
    k, t, cs, valid, st, rej = Decoder("k", cols).decode(wide_keys, buf, off, ts, threads=threads)
    db = Decoder("k", cols).decode_batch(nar_keys, buf, off, ts, threads=threads)
    b = db.batch
    assert (b.key_enc, b.ts_enc, list(b.col_enc[:2])) == (abi.HSG_ENC_K16, abi.HSG_ENC_TS16,
                                                          [abi.HSG_ENC_I32, abi.HSG_ENC_DEC32])
    assert b.col_scale[1] == 3 and db.rejected == rej == 0
    assert db.bytes_per_record() < 12.01
    k2, t2, cs2, v2 = db.widen()
    assert np.array_equal(k2, k) and np.array_equal(t2, t)
    assert np.array_equal(cs2[0], cs[0])
    assert np.array_equal(cs2[1].view(np.int64), cs[1].view(np.int64))  # bit-identical doubles
    assert v2 == [None, None] and all(np.all(v == 1) for v in valid)


def test_decode_batch_keeps_what_does_not_fit():
    """Each column narrows only when lossless for every value of the batch:
    a value outside int32 keeps its i64 column wide, a -0.0 or a 12-decimal
    value keeps the f64 column wide, a rejected record (HSG_KEY_NONE) or more
    than 2^16 key ids keeps the keys wide, a frame spanning 2^16 ms or more
    falls back to TS32 and a batch spanning 2^31 ms to full ts; absent
    fields keep their valid bytes. Every batch widens back exactly."""
    cols = [("v", abi.HSG_I64, True), ("x", abi.HSG_F64, True)]
    base = [{"k": 1, "v": 5, "x": 1.5}, {"k": 2, "v": -7, "x": 2.25}, {"k": 3, "v": 0, "x": 0.0}]
    cases = [
        ([dict(base[0], v=2**31)] + base[1:], [0, 1, 2], (abi.HSG_ENC_FULL, abi.HSG_ENC_DEC32)),
        ([dict(base[0], x=-0.0)] + base[1:], [0, 1, 2], (abi.HSG_ENC_I32, abi.HSG_ENC_FULL)),
        ([dict(base[0], x=0.123456789012)] + base[1:], [0, 1, 2], (abi.HSG_ENC_I32, abi.HSG_ENC_FULL)),
        (base, [0, 70_000, 2], (abi.HSG_ENC_I32, abi.HSG_ENC_DEC32)),
        (base, [0, 2**31, 2], (abi.HSG_ENC_I32, abi.HSG_ENC_DEC32)),
        ([{"k": 1, "x": 1.5}, {"v": 1}, {"k": 3, "v": 4}], [0, 1, 2], (abi.HSG_ENC_I32, abi.HSG_ENC_DEC32)),
    ]
    for ci, (recs, ts, enc) in enumerate(cases):
        vals = [json.dumps(r).encode() for r in recs]
        buf, off = pack_records(vals)
        tsa = np.array(ts, np.int64)
        k, t, cs, valid, st, rej = Decoder("k", cols).decode(KeyDict(), buf, off, tsa)
        db = Decoder("k", cols).decode_batch(KeyDict(), buf, off, tsa)
        b = db.batch
        assert (b.col_enc[0], b.col_enc[1]) == enc, (ci, list(b.col_enc[:2]))
        want_k = abi.HSG_ENC_FULL if rej else abi.HSG_ENC_K16
        assert b.key_enc == want_k, ci
        want_t = abi.HSG_ENC_TS16 if ts[1] < 65536 else abi.HSG_ENC_TS32 if ts[1] < 2**31 else abi.HSG_ENC_FULL
        assert b.ts_enc == want_t, ci
        k2, t2, cs2, v2 = db.widen()
        assert np.array_equal(k2, k) and np.array_equal(t2, t), ci
        assert np.array_equal(cs2[0], cs[0]) and np.array_equal(cs2[1].view(np.int64), cs[1].view(np.int64)), ci
        for c in range(2):
            assert np.array_equal(v2[c] if v2[c] is not None else np.ones(3, np.uint8), valid[c]), (ci, c)
    # more than 2^16 key ids: 32-bit keys
    kd = KeyDict()
    for i in range(70_000):
        kd.encode(i)
    vals = [json.dumps({"k": 69_999, "v": 1, "x": 1.0}).encode()] * 3
    buf, off = pack_records(vals)
    db = Decoder("k", cols).decode_batch(kd, buf, off, np.zeros(3, np.int64))
    assert db.batch.key_enc == abi.HSG_ENC_FULL
    # allow = 0: full width
    db = Decoder("k", cols).decode_batch(KeyDict(), buf, off, np.zeros(3, np.int64), allow=0)
    assert (db.batch.key_enc, db.batch.ts_enc, db.batch.col_enc[0]) == (0, 0, 0)
