"""The narrow transport of a batch (include/hstream_gpu.h hsg_enc): ts as int32
offsets from a base, i64 columns as int32, f64 decimal columns as int32
mantissas. Lossless by construction, so every result must be bit-identical
to the same batches pushed at full width -- checked against the oracle fed the
full-width arrays, for host batches (synchronous and asynchronous, the latter
prestaged on the copy stream) and device batches, with absent fields,
HSG_KEY_NONE records, negative and late timestamps."""
import ctypes as C

import numpy as np
import pytest

import pyoracle
from hstream_amd import abi
from hstream_amd.columnar import OpSpec, narrow_columns, narrow_keys
from util import gen_small, rows_equal

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    import torch
    assert torch.cuda.is_available(), "GPU tests need cuda:0"
    from hstream_amd.engine import Engine
    e = Engine(device=0, batch_capacity=1 << 18)
    yield e
    e.close()


AGGS = [(abi.HSG_COUNT_ALL, 0), (abi.HSG_COUNT, 1), (abi.HSG_SUM, 0), (abi.HSG_MIN, 0), (abi.HSG_MAX, 0),
        (abi.HSG_SUM, 1), (abi.HSG_MIN, 1), (abi.HSG_MAX, 1), (abi.HSG_AVG, 1)]
SPECS = {
    "tumbling_batch": OpSpec(abi.HSG_TUMBLING, abi.HSG_EMIT_PER_BATCH, size_ms=10_000,
                             col_types=[abi.HSG_I64, abi.HSG_F64], aggs=AGGS),
    "hopping_record": OpSpec(abi.HSG_HOPPING, abi.HSG_EMIT_PER_RECORD, size_ms=20_000, advance_ms=5_000,
                             col_types=[abi.HSG_I64, abi.HSG_F64], aggs=AGGS),
    "session_batch": OpSpec(abi.HSG_SESSION, abi.HSG_EMIT_PER_BATCH, gap_ms=2_000,
                            col_types=[abi.HSG_I64, abi.HSG_F64], aggs=AGGS),
}


def _batches(seed, nb=3, n=40_000):
    out = []
    for b in range(nb):
        key, ts, cols, valid = gen_small(seed + b, n, 300, col_types=(abi.HSG_I64, abi.HSG_F64), span=60_000,
                                         base=3_000_000 + 60_000 * b)
        cols[0] = cols[0] // 2  # fits int32
        out.append((key, ts, cols, valid))
    return out


@pytest.mark.parametrize("k16", [False, True], ids=["k32", "k16"])
@pytest.mark.parametrize("mode", ["sync", "async", "device"])
@pytest.mark.parametrize("name", sorted(SPECS))
def test_narrow_equals_full_width(eng, name, mode, k16):
    import torch
    spec = SPECS[name]
    g, o = eng.op(spec), pyoracle.OracleOp(spec, faithful_sessions=False)
    f64 = spec.agg_is_f64()
    wm_o = -1
    wm_g = C.c_int64(-1)
    for bi, (key, ts, cols, valid) in enumerate(_batches(70 + len(name))):
        if k16:  # HSG_ENC_K16 needs a batch without HSG_KEY_NONE records
            key = np.where(key == np.uint32(abi.HSG_KEY_NONE), np.uint32(65535), key).astype(np.uint32)
        kn = narrow_keys(key) if k16 else key
        assert kn.dtype == (np.uint16 if k16 else np.uint32)
        t32, base, c32, enc, scale = narrow_columns(ts, cols, spec.col_types, [None, 3])
        assert base is not None and enc == [abi.HSG_ENC_I32, abi.HSG_ENC_DEC32], (base, enc)
        wm_o = o.push(key, ts, cols, valid, watermark=wm_o)
        kw = dict(ts_base=base, col_enc=enc, col_scale=scale)
        if mode == "sync":
            wm_g.value = g.push(kn, t32, c32, valid, watermark=wm_g.value, **kw)
        elif mode == "async":
            g.push_async(kn, t32, c32, valid, watermark=wm_g, **kw)
            g.wait()
        else:
            d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
            dv = [d(v) for v in valid]
            torch.cuda.synchronize()
            dk = d(kn.view(np.int16)) if k16 else d(kn.view(np.int32))
            wm_g.value = g.push(dk, d(t32), [d(c) for c in c32], dv, watermark=wm_g.value,
                                mem=abi.HSG_MEM_DEVICE, **kw)
        assert wm_g.value == wm_o, f"batch {bi}: watermark"
        rows_equal(g.drain(), o.drain(), f64, ordered=spec.emit_mode == abi.HSG_EMIT_PER_RECORD,
                   what=f"{name} {mode} changelog {bi}")
    rows_equal(g.dump_state(), o.dump_state(), f64, what=f"{name} {mode} state")
    g.close()
    o.close()


def test_bad_encodings_refused(eng):
    spec = SPECS["tumbling_batch"]
    g = eng.op(spec)
    key = np.arange(10, dtype=np.uint32)
    ts = np.arange(10, dtype=np.int32)
    cols = [np.arange(10, dtype=np.int32), np.arange(10, dtype=np.int32)]
    for enc in ([abi.HSG_ENC_DEC32, abi.HSG_ENC_FULL], [abi.HSG_ENC_FULL, abi.HSG_ENC_I32], [7, 0]):
        with pytest.raises(abi.HStreamGpuError) as ei:
            g.push(key, ts, [c if e != abi.HSG_ENC_FULL else c.astype(np.int64) for c, e in zip(cols, enc)],
                   None, watermark=-1, ts_base=0, col_enc=enc, col_scale=[2, 2])
        assert ei.value.status == abi.HSG_E_INVALID
    g.close()


@pytest.mark.parametrize("mode", ["sync", "async", "device"])
@pytest.mark.parametrize("name", ["tumbling_batch", "hopping_record"])
def test_ts16_frames_equal_full_width(eng, name, mode):
    """HSG_ENC_TS16: uint16 offsets from a base per HSG_TS16_FRAME records
    (batches of 40 000 records: the last frame is partial), with the other
    narrow columns, bit-identical to the full-width oracle."""
    import torch
    from hstream_amd.columnar import narrow_ts16
    spec = SPECS[name]
    g, o = eng.op(spec), pyoracle.OracleOp(spec)
    f64 = spec.agg_is_f64()
    wm_o = -1
    wm_g = C.c_int64(-1)
    for b in range(3):
        key, ts, cols, valid = gen_small(90 + b, 40_000, 300, col_types=(abi.HSG_I64, abi.HSG_F64), span=60_000,
                                         base=3_000_000 + 60_000 * b, very_late=False, neg_frac=0.0)
        cols[0] = cols[0] // 2
        t16, frames, c32, enc, scale = narrow_columns(ts, cols, spec.col_types, [None, 3], ts16=True)
        assert t16.dtype == np.uint16 and frames.size == -(-ts.size // abi.HSG_TS16_FRAME)
        assert np.array_equal(np.repeat(frames, abi.HSG_TS16_FRAME)[:ts.size] + t16, ts)
        assert narrow_ts16(ts) is not None
        wm_o = o.push(key, ts, cols, valid, watermark=wm_o)
        kw = dict(ts_frames=frames, col_enc=enc, col_scale=scale)
        if mode == "sync":
            wm_g.value = g.push(key, t16, c32, valid, watermark=wm_g.value, **kw)
        elif mode == "async":
            g.push_async(key, t16, c32, valid, watermark=wm_g, **kw)
            g.wait()
        else:
            d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
            kw["ts_frames"] = d(frames)
            dv = [d(v) for v in valid]
            torch.cuda.synchronize()
            wm_g.value = g.push(d(key.view(np.int32)), d(t16.view(np.int16)), [d(c) for c in c32], dv,
                                watermark=wm_g.value, mem=abi.HSG_MEM_DEVICE, **kw)
        assert wm_g.value == wm_o, f"batch {b}: watermark"
        rows_equal(g.drain(), o.drain(), f64, ordered=spec.emit_mode == abi.HSG_EMIT_PER_RECORD,
                   what=f"{name} {mode} ts16 changelog {b}")
    rows_equal(g.dump_state(), o.dump_state(), f64, what=f"{name} {mode} ts16 state")
    g.close()
    o.close()


@pytest.mark.parametrize("mode", ["sync", "async"])
@pytest.mark.parametrize("cap", [16, 64, 200])
def test_ts16_small_capacity_engine(cap, mode):
    """TS16 frame bases sit after the offsets (256-byte aligned) in the op's ts
    staging buffer: an engine whose batch capacity is a few records must size
    that buffer for them too (offsets + bases exceed 4 or 8 bytes per record
    below ~130 records). Many small batches, bit-identical to the oracle."""
    import torch
    assert torch.cuda.is_available()
    from hstream_amd.engine import Engine
    e = Engine(device=0, batch_capacity=cap)
    spec = SPECS["tumbling_batch"]
    g, o = e.op(spec), pyoracle.OracleOp(spec)
    f64 = spec.agg_is_f64()
    wm_o = -1
    wm_g = C.c_int64(-1)
    for b in range(6):
        key, ts, cols, valid = gen_small(300 + b, cap, 20, col_types=(abi.HSG_I64, abi.HSG_F64), span=30_000,
                                         base=3_000_000 + 30_000 * b, very_late=False, neg_frac=0.0)
        cols[0] = cols[0] // 2
        t16, frames, c32, enc, scale = narrow_columns(ts, cols, spec.col_types, [None, 3], ts16=True)
        wm_o = o.push(key, ts, cols, valid, watermark=wm_o)
        kw = dict(ts_frames=frames, col_enc=enc, col_scale=scale)
        if mode == "sync":
            wm_g.value = g.push(key, t16, c32, valid, watermark=wm_g.value, **kw)
        else:
            g.push_async(key, t16, c32, valid, watermark=wm_g, **kw)
            g.wait()
        assert wm_g.value == wm_o, f"batch {b}: watermark"
        rows_equal(g.drain(), o.drain(), f64, what=f"cap {cap} {mode} ts16 changelog {b}")
    rows_equal(g.dump_state(), o.dump_state(), f64, what=f"cap {cap} {mode} ts16 state")
    g.close()
    o.close()
    e.close()


@pytest.mark.parametrize("name", ["tumbling_batch", "hopping_record", "session_batch"])
def test_decoder_batches_equal_full_width(eng, name):
    """The product decoder's own transport (hsg_decode_json_batch: JSON poll
    batch -> narrowest lossless hsg_batch, 16-bit keys, TS16 frames, int32 /
    DEC32 values, no valid bytes for always-present fields) pushed as it
    comes, against the oracle fed the full-width decode of the same records."""
    import json
    from hstream_amd.ingest import Decoder, KeyDict, pack_records
    spec = SPECS[name]
    g, o = eng.op(spec), pyoracle.OracleOp(spec, faithful_sessions=False)
    f64 = spec.agg_is_f64()
    rng = np.random.default_rng(41)
    cols = [("v", abi.HSG_I64, True), ("x", abi.HSG_F64, True)]
    dec_w, dec_n = Decoder("k", cols), Decoder("k", cols)
    kw, kn = KeyDict(), KeyDict()
    wm_o = wm_g = -1
    for b in range(3):
        n = 30_000
        vals = []
        for i in range(n):
            r = {"k": int(rng.integers(0, 300))}
            if rng.random() > 0.05:
                r["v"] = int(rng.integers(-10**6, 10**6))
            if rng.random() > 0.05 or b == 1:  # batch 1: x in every record (no valid bytes for it)
                r["x"] = round(float(rng.uniform(-1e4, 1e4)), 2)
            vals.append(json.dumps(r).encode())
        ts = 3_000_000 + 60_000 * b + (np.arange(n) * 60_000) // n + rng.integers(0, 3000, n)
        buf, off = pack_records(vals)
        k, t, cs, valid, _st, _rej = dec_w.decode(kw, buf, off, ts)
        db = dec_n.decode_batch(kn, buf, off, ts)
        assert db.batch.key_enc == abi.HSG_ENC_K16 and db.batch.ts_enc == abi.HSG_ENC_TS16
        assert db.batch.col_enc[0] == abi.HSG_ENC_I32 and db.batch.col_enc[1] == abi.HSG_ENC_DEC32
        wm_o = o.push(k, t, cs, valid, watermark=wm_o)
        wm_g = g.push_batch(db.batch, watermark=wm_g)
        assert wm_g == wm_o, f"batch {b}: watermark"
        rows_equal(g.drain(), o.drain(), f64, ordered=spec.emit_mode == abi.HSG_EMIT_PER_RECORD,
                   what=f"{name} decoder batch {b}")
    rows_equal(g.dump_state(), o.dump_state(), f64, what=f"{name} decoder state")
    g.close()
    o.close()
